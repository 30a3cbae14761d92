"""Oracle mask network, losses and optimizer on torch-CPU (TEST INFRASTRUCTURE ONLY).

Restates, in plain torch-CPU (fp32 or fp64), the separation step of the reference:

* ``MIX_SPEECH`` BiLSTM-4L  -- ``TDAA_beta/main_run_sstune_EvalVer.py:277-303``;
  BiGRU-2L -- ``Torch_multi/main_run.py:258-282``,
  ``TDAA_beta/main_run_sstune_cRM_EvalVer.py:340-365``.
  ``nn.LSTM``/``nn.GRU`` (batch_first, bidirectional) -> ``Linear(2H, F*E)`` -> tanh
  -> view (B, T, F, E).
* ``SPEECH_EMBEDDING`` gather -- ``EvalVer.py:348-361`` (cRM width 2E:
  ``cRM_EvalVer.py:390-406``); dense-masked 101-channel form -- ``main_run.py:307-327``.
* ``ADDJUST`` -- ``EvalVer.py:363-377``: q <- q + W [mean_t h ; q] (no bias).
* ``ATTENTION`` 'dot' -- ``EvalVer.py:216-226``: mask = sigmoid(V . q);
  cRM branch -- ``cRM_EvalVer.py:259-271`` (10*tanh per half-query) and inverse
  compression ``cRM_EvalVer.py:688``: -1/C * log((K - m)/(K + m)).
* Losses -- ``EvalVer.py:641,659-666`` (MSE + 0.5 * MSE(sum_k mask, 1)),
  ``main_run.py:506`` (101-channel MSE, first term only),
  ``cRM_EvalVer.py:741-743`` (MSE(re) + MSE(im)).  PIT is a new spec (the
  reference has none): per-utterance min over K! assignments of
  the first term, ties -> lowest permutation index in itertools order; it equals
  the reference whenever the identity (label order) is optimal.
* ``top_k_mask`` -- ``EvalVer.py:390-405``.
* Adam(lr=2e-4, betas=(0.9, 0.999), eps=1e-8) -- ``EvalVer.py:538-544,673-675``.
"""
import itertools

import numpy as np
import torch
from torch import nn

CRM_K = 10.0
CRM_C = 0.1


class MixSpeech(nn.Module):
    """MIX_SPEECH with the reference's submodule names (``layer``, ``Linear``)."""

    def __init__(self, cell="lstm", input_fre=129, hidden=300, num_layers=4, emb=50):
        super().__init__()
        rnn = nn.LSTM if cell == "lstm" else nn.GRU
        self.cell = cell
        self.input_fre, self.emb = input_fre, emb
        self.layer = rnn(input_size=input_fre, hidden_size=hidden, num_layers=num_layers,
                         batch_first=True, bidirectional=True)
        self.Linear = nn.Linear(2 * hidden, input_fre * emb)

    def forward(self, x):
        h, _ = self.layer(x)
        B, T, _ = h.shape
        V = torch.tanh(self.Linear(h.reshape(B * T, -1))).view(B, T, self.input_fre, -1)
        return V, h


class Embedding(nn.Module):
    def __init__(self, num_labels=101, width=50):
        super().__init__()
        self.layer = nn.Embedding(num_labels, width)

    def forward(self, idx):
        return self.layer(idx)


class Adjust(nn.Module):
    def __init__(self, hidden_units=600, width=50):
        super().__init__()
        self.layer = nn.Linear(hidden_units + width, width, bias=False)

    def forward(self, h, q):
        B, K, _ = q.shape
        m = h.mean(dim=1, keepdim=True).expand(B, K, h.shape[2])
        return self.layer(torch.cat([m, q], dim=2))


def attention_dot(V, q):
    """V (B,T,F,E), q (B,K,E) -> mask (B,K,T,F)."""
    return torch.sigmoid(torch.einsum("btfe,bke->bktf", V, q))


def attention_crm(V, q2):
    """cRM branch: q2 (B,K,2E) split in halves -> compressed masks (B,K,T,F,2),
    then inverse compression (cRM_EvalVer.py:259-271,688)."""
    E = V.shape[-1]
    mr = CRM_K * torch.tanh(torch.einsum("btfe,bke->bktf", V, q2[..., :E]))
    mi = CRM_K * torch.tanh(torch.einsum("btfe,bke->bktf", V, q2[..., E:]))
    m = torch.stack([mr, mi], dim=-1)
    return -1.0 / CRM_C * torch.log((CRM_K - m) / (CRM_K + m))


def loss_label_ordered(mask, X, Y, sum_weight=0.5):
    """EvalVer.py:630,641,659-666: MSE(mask*X, Y) + 0.5*MSE(sum_k mask, 1)."""
    pred = mask * X[:, None]
    l1 = torch.mean((pred - Y) ** 2)
    l2 = torch.mean((mask.sum(dim=1) - 1.0) ** 2)
    return l1 + sum_weight * l2, pred


def pit_assign(mask, X, Y):
    """Per-utterance optimal assignment (new PIT spec; see module doc).
    Returns perms (B,K) int64 with perm[b][k] = target index for channel k."""
    B, K = mask.shape[:2]
    pred = mask * X[:, None]
    # pairwise cost C[b, k, j] = sum_{t,f} (pred_k - Y_j)^2
    C = ((pred[:, :, None] - Y[:, None, :]) ** 2).sum(dim=(-1, -2))
    perms = list(itertools.permutations(range(K)))
    costs = torch.stack([sum(C[:, k, p[k]] for k in range(K)) for p in perms], dim=1)
    best = torch.argmin(costs, dim=1)  # first minimum = lowest permutation index
    P = torch.tensor(perms, dtype=torch.int64)
    return P[best], best


def loss_pit(mask, X, Y, sum_weight=0.5):
    perm, _ = pit_assign(mask.detach(), X, Y)
    Yp = torch.stack([Y[b, perm[b]] for b in range(Y.shape[0])])
    return loss_label_ordered(mask, X, Yp, sum_weight)


def loss_crm(mask, Xc, Yc):
    """cRM_EvalVer.py:720-743. mask (B,K,T,F,2), Xc (B,T,F,2), Yc (B,K,T,F,2)."""
    mr, mi = mask[..., 0], mask[..., 1]
    xr, xi = Xc[:, None, ..., 0], Xc[:, None, ..., 1]
    pr = mr * xr - mi * xi
    pi = mr * xi + mi * xr
    loss = torch.mean((pr - Yc[..., 0]) ** 2) + torch.mean((pi - Yc[..., 1]) ** 2)
    return loss, torch.stack([pr, pi], dim=-1)


def loss_101(mask_all, topk, X, Y_all):
    """main_run.py:487-506: mask over all N_lab channels, multiplied by the
    multi-hot, MSE over B*N_lab*T*F elements (first term only)."""
    m = mask_all * topk[:, :, None, None]
    pred = m * X[:, None]
    return torch.mean((pred - Y_all) ** 2), pred


def top_k_mask(batch_pro, alpha, top_k):
    """EvalVer.py:390-405 restated (returns float multi-hot on CPU)."""
    size = batch_pro.shape
    final = torch.zeros(size)
    sort_result, sort_index = torch.sort(batch_pro, 1, True)
    sort_index = sort_index[:, :top_k]
    cnt = torch.sum(sort_result > alpha, 1)
    for i in range(size[0]):
        for j in sort_index[i][: int(cnt[i])]:
            final[i, int(j)] = 1
    return final


def multi_label_vector(spk_lists, dict_name2idx):
    """Torch_multi/test_multi_labels_speech.py:285-298 restated."""
    y_spk, y_aim = [], []
    L = len(dict_name2idx)
    for sample in spk_lists:
        v = [0] * L
        line = [dict_name2idx[s] for s in sample]
        for l in line:
            v[l] = 1
        y_spk.append(line)
        y_aim.append(v)
    return y_spk, np.array(y_aim, dtype=np.float32)


class SepModel(nn.Module):
    """The trainable part of one separation step (magnitude or cRM path)."""

    def __init__(self, cell="lstm", num_layers=4, hidden=300, emb=50, num_labels=101,
                 input_fre=129, crm=False, adjust=True):
        super().__init__()
        self.crm = crm
        self.use_adjust = adjust
        w = 2 * emb if crm else emb
        self.mix = MixSpeech(cell, input_fre, hidden, num_layers, emb)
        self.emb = Embedding(num_labels, w)
        self.adj = Adjust(2 * hidden, w) if adjust else None

    def queries(self, h, spk_idx):
        q = self.emb(spk_idx)
        if self.use_adjust:
            q = q + self.adj(h, q)
        return q

    def forward(self, feats, spk_idx):
        V, h = self.mix(feats)
        q = self.queries(h, spk_idx)
        mask = attention_crm(V, q) if self.crm else attention_dot(V, q)
        return mask, V, h, q


def train_step(model, opt, feats, X, Y, spk_idx, mode="label", sum_weight=0.5):
    """One reference training step: forward, loss, backward, Adam.
    mode: 'label' (reference), 'pit', or 'crm' (X/Y complex (...,2))."""
    opt.zero_grad()
    mask, V, h, q = model(feats, spk_idx)
    if mode == "crm":
        loss, pred = loss_crm(mask, X, Y)
    elif mode == "pit":
        loss, pred = loss_pit(mask, X, Y, sum_weight)
    else:
        loss, pred = loss_label_ordered(mask, X, Y, sum_weight)
    loss.backward()
    opt.step()
    return loss.detach(), mask.detach(), pred.detach()


def make_adam(model, lr=2e-4):
    return torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), eps=1e-8)
