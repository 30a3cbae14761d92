"""Parity at the FULL sizes of the other BASELINE.json configurations (the headline C2 is in
test_step_gpu.py): the HIP step vs the CPU oracle on identical synthetic mixtures.

* C1  Torch_multi/main_run.py: BiGRU-2L, B = 1, N = 40000 (5 s, T = 313), 101-channel loss,
      no ADDJUST -- fp32 parity mode and the bf16 mode.
* C3  cRM path: BiGRU-2L, B = 16, N = 32000 -- one step in fp32, and the step at which the
      reference's inverse compression (cRM_EvalVer.py:688) first turns the loss non-finite
      on a repeated batch, HIP vs oracle, on the same seed.
* C4  3 speakers (predata_multiAims_3dB gains), BiGRU-2L without ADDJUST (selfSS_dB model),
      B = 32, N = 32000 -- fp32 and bf16.
* C5  recursive extraction at N = 32000 (T = 251) vs oracle/recursive.py: fp32 speaker ids
      bit-exact, probabilities / masks as test_recursive_gpu.py; bf16 at B = 1 and B = 32 with
      unconditional decided-step asserts.
* C3's cRM mask-apply + iSTFT (dl4ss_istft_apply) at B = 16, T = 251 vs dsp.istft of the oracle's
  masked complex spectrogram.
* C1 / C3 / C4 in four modes: fp32, mixed (fp32 GEMMs + bf16 recurrent matvec), bf16s (split
  bf16 forward GEMMs, fp32 V: the mode their throughput is quoted in; masked magnitude within 1e-3)
  and all-bf16 operands (outside 1e-3 on these BiGRU nets; bound 1e-2).
* C5 in "mixed" (its quoted mode: masked magnitude within 1e-3) and all-bf16 (bound 1e-2).
"""
import numpy as np
import pytest
import torch

from oracle import model as om
from oracle import recursive as orc
from dl4ss_amd import engine, synth

from test_step_gpu import _compare_step, _oracle_features, _setup  # noqa: E402
from test_recursive_gpu import _feats, _models, _ours  # noqa: E402

pytestmark = pytest.mark.gpu

BF16 = dict(precision="bf16", tol_loss=1e-2, tol_grad=5e-2, tol_pred=1e-2)
# the mixed mode: exact fp32 GEMMs, bf16 MFMA recurrent matvec (fp32 state);
# masked magnitude within the north-star 1e-3 (the same as bf16s, at half its speed)
MIXED = dict(precision="fp32", rnn_precision="bf16", tol_loss=1e-3, tol_grad=5e-2, tol_pred=1e-3)
# The all-bf16 operand mode misses 1e-3 on the BiGRU nets (measured C1 2.1e-3, C4 2.2e-3, C3 4.4e-3;
# tools/parity_probe.py, profiles/r04_parity_configs.jsonl): checked here against its own 1e-2 bound
# and never quoted as an in-bar throughput.
# bf16s: the bf16 step with split-precision forward GEMMs and fp32 V (engine.SepTrainer); bf16
# recurrence and backward -- the mode C1 / C3 / C4 throughput is quoted in, within the 1e-3 bar
BF16S = dict(precision="bf16s", tol_loss=1e-3, tol_grad=5e-2, tol_pred=1e-3)
MODES = {"fp32": {}, "mixed": MIXED, "bf16": BF16, "bf16s": BF16S}


@pytest.mark.parametrize("mode", ["fp32", "mixed", "bf16", "bf16s"])
def test_c1_full_size(dev, mode):
    _compare_step(dev, "gru", 2, 1, 2, 40000, "label", loss_channels=101, adjust=False, **MODES[mode])


@pytest.mark.parametrize("mode", ["fp32", "mixed", "bf16", "bf16s"])
def test_c4_full_size_3spk(dev, mode):
    _compare_step(dev, "gru", 2, 32, 3, 32000, "label", adjust=False, **MODES[mode])


@pytest.mark.parametrize("mode", ["fp32", "mixed", "bf16", "bf16s"])
def test_c3_full_size_step(dev, mode):
    """The cRM step at B = 16: the masked complex spectrogram P = M (x) X within 1e-3 rel-L2 in
    fp32 (measured 1.2e-4) and mixed mode (6.1e-4); bf16 operands 4.4e-3 (bound 1e-2)."""
    kw = dict(MODES[mode])
    if mode == "fp32":
        kw["tol_grad"] = 5e-3
    _compare_step(dev, "gru", 2, 16, 2, 32000, "crm", **kw)


@pytest.mark.parametrize("mode", ["fp32", "bf16s"])
def test_c3_full_size_mask_apply_istft(dev, mode):
    """C3's "+ iSTFT" at its size (B = 16, K = 2, N = 32000, T = 251): the eval output path of
    cRM_EvalVer.py:96-99,720-728 -- P = M (x) X, then the overlap-add iSTFT -- through
    dl4ss_istft_apply, against dsp.istft(P_r + j P_i) of the oracle.
    (a) the kernel alone, on the ORACLE's cRM mask and the GPU mixture spectrum: 1e-5 of max;
    (b) the whole path, the trainer's own mask (attention COST pass) in the mode C3 is quoted in
        (bf16s) and in fp32: waveform rel-L2 within the north-star 1e-3."""
    from dl4ss_amd import _lib
    from oracle import dsp

    B, K, N = 16, 2, 32000
    kw = {k: v for k, v in MODES[mode].items() if not k.startswith("tol_")}
    net, tr, src, spk, gains, ref = _setup(dev, "gru", 2, B, K, N, "crm", **kw)
    feats, X, Y = _oracle_features(src, gains, True)
    with torch.no_grad():
        mask_ref, *_ = ref(feats, torch.from_numpy(spk))
        _, pred_ref = om.loss_crm(mask_ref, X, Y)  # (B, K, T, F, 2)
    assert torch.isfinite(pred_ref).all()
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(torch.from_numpy(src.astype(np.float32)).to(dev), torch.from_numpy(gains.astype(np.float32)).to(dev))
    tr.forward()
    T, F = tr.T, tr.F
    assert T == 251
    m = torch.empty(B, K, T * F, 2, device=dev)
    tr.attn(0, mask_out=m)
    L = 128 * (T - 1)
    y = torch.empty(B * K, L, device=dev)
    y_k = torch.empty(B * K, L, device=dev)
    mr = mask_ref.reshape(B, K, T * F, 2).contiguous().to(dev)
    for aux, out in ((m, y), (mr, y_k)):
        _lib.call("dl4ss_istft_apply", _lib.ptr(tr.Xc_mix), _lib.ptr(aux), B * K, K, T, 1, 0, _lib.ptr(out),
                  _lib.stream_ptr())
    torch.cuda.synchronize()
    tr.check()
    P = pred_ref[..., 0].numpy() + 1j * pred_ref[..., 1].numpy()
    wav_ref = np.stack([dsp.istft(P[b, k].T) for b in range(B) for k in range(K)])
    assert wav_ref.shape == (B * K, L)
    yk = y_k.cpu().numpy()
    assert np.abs(yk - wav_ref).max() / np.abs(wav_ref).max() < 1e-5
    yo = y.cpu().numpy()
    rel = float(np.linalg.norm(yo - wav_ref) / np.linalg.norm(wav_ref))
    print(f"C3 {mode}: cRM mask-apply + iSTFT waveform rel-L2 {rel:.3e}")
    assert rel < 1e-3, rel


def _c3_run(dev, seed, S, stop_at_non_finite=True):
    B, K, N = 16, 2, 32000
    net, tr, src, spk, gains, ref = _setup(dev, "gru", 2, B, K, N, "crm", seed=seed)
    feats, X, Y = _oracle_features(src, gains, True)
    idx = torch.from_numpy(spk)
    opt = om.make_adam(ref)
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    g = torch.from_numpy(gains.astype(np.float32)).to(dev)
    sp = torch.from_numpy(spk.astype(np.int32)).to(dev)
    torch.set_num_threads(16)
    first_ours = first_ref = None
    for s in range(S):
        lo = float(tr.step(raw, g, sp)[0].item())
        tr.check()
        lr = float(om.train_step(ref, opt, feats, X, Y, idx, mode="crm")[0])
        if first_ours is None and not np.isfinite(lo):
            first_ours = s
        if first_ref is None and not np.isfinite(lr):
            first_ref = s
        if first_ours is not None or first_ref is not None:
            break
        assert abs(lo - lr) <= 1e-3 * abs(lr), (s, lo, lr)
    return first_ours, first_ref


def test_c3_first_non_finite_step_matches_oracle(dev):
    """The cRM inverse compression -1/C log((K - M)/(K + M)) is infinite once a compressed
    mask reaches K (fp32 tanh(e) rounds to 1 for |e| >= 9.02).  With the
    reference's own seed (1, main_run.py:21-23) and default init (N(0,1) query embedding) the
    C3 configuration hits it at once: the HIP step and the oracle step must both report a
    non-finite loss, at the same step.  The hazard must actually occur (a run where neither side
    goes non-finite fails instead of passing vacuously: seeds 2-4, 6 and 8 stay finite for 25
    steps, 1, 5 and 7 are non-finite from the first step, measured on the oracle)."""
    first_ours, first_ref = _c3_run(dev, 1, 10)
    assert first_ref is not None, "the cRM_EvalVer.py:688 hazard did not occur"
    assert first_ours == first_ref, (first_ours, first_ref)


def test_c3_finite_window_matches_oracle(dev):
    """The same repeated-batch C3 training on a seed whose logits stay below the saturation:
    the HIP and oracle losses agree within 1e-3 at every one of 20 steps, none non-finite."""
    first_ours, first_ref = _c3_run(dev, 3, 20)
    assert first_ours is None and first_ref is None, (first_ours, first_ref)


@pytest.mark.parametrize("B", [1, 32])
def test_c5_full_length_recursive(dev, B):
    """C5 in fp32 at T = 251: speaker ids, probabilities (2e-5 abs) and masks (1e-4 abs) against
    oracle/recursive.py.  At B = 32 the H = 600 classifier's fp32 forward runs as two B = 16
    launches (its plan needs 50 workgroups per group); ids are compared on every decision whose
    probability gap exceeds 1e-4 (5x the fp32 bound), and must agree on at least 60 of the 64."""
    n, seed = 32000, 7
    mix, cls, emb = _models(seed)
    X = _feats(B, n, seed)
    T = X.shape[1]
    assert T == 251
    with torch.no_grad():
        ref = orc.recursive_extract(lambda x: mix(x), cls, emb.weight, X)
    out = _ours(dev, mix, cls, emb, B, T, "fp32").run(X.to(dev))
    torch.cuda.synchronize()
    for s in range(2):
        assert (out["probs"][s].cpu() - ref["probs"][s]).abs().max() < 2e-5
    spk, rspk = out["spk"].cpu().long(), ref["spk"]
    if B == 1:
        assert torch.equal(spk, rspk), (spk, rspk)
        assert (out["masks"].cpu() - ref["masks"]).abs().max() < 1e-4
        return
    agree = 0
    for b in range(B):
        seen = []
        for s in range(2):
            order = ref["probs"][s][b].sort(descending=True, stable=True).indices.tolist()
            rank = next(i for i, k in enumerate(order) if k not in seen)
            seen.append(order[rank])
            p = ref["probs"][s][b].sort(descending=True).values
            if bool((p[:rank + 1] - p[1:rank + 2]).min() > 1e-4):
                assert int(spk[b, s]) == int(rspk[b, s]), (b, s, spk[b], rspk[b])
            agree += int(spk[b, s]) == int(rspk[b, s])
    assert agree >= 60, agree
    rows = (spk == rspk).all(dim=1)
    assert (out["masks"][rows].cpu() - ref["masks"][rows]).abs().max() < 1e-4


# bf16 C5: the classifier probabilities' measured bf16 error is <= 9e-5 (B = 32, T = 251,
# profiles/r04_parity_configs.jsonl); a decision counts as decided when every gap between the
# consecutive sorted probabilities up to the chosen rank (+1) exceeds DECIDED = 5e-4
DECIDED = 5e-4


def _decided(prob, pick_rank):
    p = prob.sort(descending=True).values
    return bool((p[:pick_rank + 1] - p[1:pick_rank + 2]).min() > DECIDED)


def _masked_rel(out, ref, X, rows):
    """rel-L2 of the masked magnitudes on the rows whose speaker ids agree: the final masks on the
    original mixture M_k (x) |X| (GRID.py:455-475 -> bss_eval_fromGenMap) and each extraction
    step's prediction m_s (x) (residual) (GRID.py:412-430, predict_multi_map)."""
    fin = out["masks"][rows].cpu() * X[rows][:, None]
    fin_ref = ref["masks"][rows] * X[rows][:, None]
    r_fin = float((fin - fin_ref).norm() / fin_ref.norm())
    sp = out["step_pred"].cpu().transpose(0, 1)[rows]  # (S, B, T, F) -> rows of (B, S, T, F)
    sp_ref = ref["step_pred"][rows]
    r_step = float((sp - sp_ref).norm() / sp_ref.norm())
    return r_fin, r_step


# masked-magnitude rel-L2 bar per mode: "bf16s" (split-operand bf16 mask-net GEMMs, bf16 recurrences,
# bf16 classifier; the mode C5 is quoted in from round 6) and "mixed" (the same with fp32 GEMMs) must
# meet the north-star 1e-3; the all-bf16 operand
# mode misses it on this BiGRU net (random-init N(0,1) query embeddings, no ADDJUST) and is held to
# its own 1e-2 bound and never quoted as in-bar
C5_BAR = {"mixed": 1e-3, "bf16s": 1e-3, "bf16": 1e-2}


@pytest.mark.parametrize("precision", ["bf16s", "mixed", "bf16"])
@pytest.mark.parametrize("B,seed", [(1, 11), (32, 7)])
def test_c5_full_length_recursive_bf16(dev, B, seed, precision):
    """C5 at T = 251 against oracle/recursive.py in its bf16 modes, with unconditional asserts: at
    least 3/4 of the B x 2 extraction decisions are decided (margin above DECIDED), the speaker ids
    are equal on EVERY decided step (and on every step of this data, measured), probabilities
    within 5e-4 abs, and the masked magnitudes -- final masks on the mixture and every step's
    prediction -- within the mode's rel-L2 bar (C5_BAR; north-star 1e-3 for the quoted mode)."""
    mix, cls, emb = _models(seed)
    X = _feats(B, 32000, seed)
    T = X.shape[1]
    with torch.no_grad():
        ref = orc.recursive_extract(lambda x: mix(x), cls, emb.weight, X)
    out = _ours(dev, mix, cls, emb, B, T, precision).run(X.to(dev))
    torch.cuda.synchronize()
    spk, rspk = out["spk"].cpu().long(), ref["spk"]
    decided = 0
    for b in range(B):
        seen = []
        for s in range(2):
            order = ref["probs"][s][b].sort(descending=True, stable=True).indices.tolist()
            rank = next(i for i, k in enumerate(order) if k not in seen)
            seen.append(order[rank])
            if _decided(ref["probs"][s][b], rank):
                decided += 1
                assert int(spk[b, s]) == int(rspk[b, s]), (b, s, spk[b], rspk[b])
    assert decided >= (3 * 2 * B + 3) // 4, (decided, 2 * B)
    for s in range(2):
        assert (out["probs"][s].cpu() - ref["probs"][s]).abs().max() < DECIDED
    agree = spk == rspk
    rows = agree.all(dim=1)
    assert bool(rows.any())
    r_fin, r_step = _masked_rel(out, ref, X, rows)
    print(f"C5 {precision} B={B}: masked magnitude rel-L2 final {r_fin:.3e} steps {r_step:.3e}")
    assert r_fin < C5_BAR[precision] and r_step < C5_BAR[precision], (r_fin, r_step)
