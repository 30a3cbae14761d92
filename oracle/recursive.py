"""Oracle of the speaker classifier and the recursive extraction loop (TEST INFRASTRUCTURE ONLY).

CPU restatement (torch-CPU, fp32 or fp64) of

* ``MIX_SPEECH_classifier`` -- ``Torch_multi/main_run_multi_selfSS_recuReal_GRID.py:178-199``,
  ``TDAA_beta/main_run_sstune_EvalVer.py:305-326``: BiLSTM(input_fre, 2*HIDDEN_UNITS = 600,
  3 layers) -> mean over t -> Linear(1200, N_lab) -> sigmoid.
* the GRID ``top_k_mask`` that also returns ``sort_index`` -- ``GRID.py:227-244``.
* the recursive extraction loop -- ``GRID.py:383-475``:
  per row (the reference runs it on row 0 of a B=1 batch):

    V0 = MIX_SPEECH(X)                                  (GRID.py:370, computed before the loop)
    step 1: p = classifier(X); sort_index = top-3 of p (alpha = -0.3)
            s1 = first id of sort_index not yet extracted
            m1 = sigmoid(V0 . emb[s1]); predict_1 = m1 X; residual R = (1 - m1) X
    step 2: p = classifier(R); V = MIX_SPEECH(R); s2 = first id of top-3 not in {s1}
            m2 = sigmoid(V . emb[s2]); predict_2 = m2 R       (num_step >= 2: stop)
    final:  masks of [s1, s2] on the ORIGINAL mixture: sigmoid(V0 . emb[s_k])
            (GRID.py:455-475 -> bss_eval_fromGenMap)

  If no probability exceeds alpha the loop stops with nothing extracted (GRID.py:237-238);
  with alpha = -0.3 below every sigmoid output this never happens.  If every one of the
  top-3 ids was already extracted the reference continues with all three and then fails
  on a reshape (GRID.py:444); this restatement (and the HIP path) marks the step invalid
  (-1) instead.  The reference uses row 0's speaker for every row of a batch; the build
  treats rows independently (identical at B = 1).
"""
import torch
from torch import nn


class Classifier(nn.Module):
    """MIX_SPEECH_classifier with the reference submodule names (``layer``, ``Linear``)."""

    def __init__(self, input_fre=129, hidden=600, num_layers=3, num_labels=101):
        super().__init__()
        self.layer = nn.LSTM(input_size=input_fre, hidden_size=hidden, num_layers=num_layers, batch_first=True,
                             bidirectional=True)
        self.Linear = nn.Linear(2 * hidden, num_labels)

    def forward(self, x):
        h, _ = self.layer(x)
        return torch.sigmoid(self.Linear(torch.mean(h, 1)))


def top_k_sort_index(prob, alpha, top_k):
    """GRID.py:227-244 restated: (mask (B,N) float, sort_index (B,top_k) long, any_above (bool,
    the reference tests row 0 only)).  Ties: lower id first (torch.sort stable descending)."""
    B, N = prob.shape
    sort_result, sort_index = torch.sort(prob, dim=1, descending=True, stable=True)
    sort_index = sort_index[:, :top_k]
    cnt = torch.sum(sort_result > alpha, 1)
    final = torch.zeros(B, N)
    for b in range(B):
        for i in sort_index[b][:int(cnt[b])]:
            final[b, int(i)] = 1
    return final, sort_index, cnt


def choose(sort_index, cnt, seen):
    """GRID.py:394-399 per row: first id of sort_index not in seen[b]; -1 if none (or no
    probability above alpha)."""
    out = []
    for b in range(sort_index.shape[0]):
        pick = -1
        if int(cnt[b]) > 0:
            for k in sort_index[b].tolist():
                if k not in seen[b]:
                    pick = int(k)
                    break
        out.append(pick)
    return out


def attention(V, q):
    """sigmoid(V (B,T,F,E) . q (B,E)) -> (B,T,F) (ATTENTION 'dot', GRID.py:412-418)."""
    return torch.sigmoid(torch.einsum("btfe,be->btf", V, q))


def recursive_extract(mix_net, classifier, emb, X, alpha=-0.3, top_k=3, max_steps=2):
    """mix_net(X) -> (V (B,T,F,E), h); classifier(X) -> prob (B,N); emb: (N, E) tensor.
    Returns dict(spk (B,max_steps) long (-1 = none), masks (B,max_steps,T,F) on the
    original mixture, step_pred (B,max_steps,T,F) = predict_multi_map of each step,
    probs [prob of each step])."""
    B = X.shape[0]
    V0, _ = mix_net(X)
    now = X
    V = V0
    seen = [[] for _ in range(B)]
    spk = torch.full((B, max_steps), -1, dtype=torch.long)
    step_pred = torch.zeros(B, max_steps, *X.shape[1:], dtype=X.dtype)
    probs = []
    for step in range(max_steps):
        prob = classifier(now)
        probs.append(prob)
        _, sidx, cnt = top_k_sort_index(prob, alpha, top_k)
        pick = choose(sidx, cnt, seen)
        nxt = now.clone()
        for b in range(B):
            if pick[b] < 0:
                continue
            seen[b].append(pick[b])
            spk[b, step] = pick[b]
            m = attention(V[b:b + 1], emb[pick[b]][None])[0]
            step_pred[b, step] = m * now[b]
            nxt[b] = (1 - m) * now[b]
        if step + 1 < max_steps:
            now = nxt
            V, _ = mix_net(now)
    masks = torch.zeros(B, max_steps, *X.shape[1:], dtype=X.dtype)
    for b in range(B):
        for k in range(max_steps):
            if spk[b, k] >= 0:
                masks[b, k] = attention(V0[b:b + 1], emb[int(spk[b, k])][None])[0]
    return dict(spk=spk, masks=masks, step_pred=step_pred, probs=probs)
