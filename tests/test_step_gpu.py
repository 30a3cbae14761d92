"""End-to-end parity of one training step (HIP path) against the CPU oracle on
identical synthetic mixtures: loss, masked magnitude spectrogram, every
gradient and the Adam-updated parameters."""
import numpy as np
import pytest
import torch

from oracle import dsp, model as om
from dl4ss_amd import engine, synth

pytestmark = pytest.mark.gpu


def _oracle_features(src, gains, crm):
    B, K, N = src.shape
    feats, X, Y = [], [], []
    for b in range(B):
        srcs = [dsp.normalise_source(src[b, k].astype(np.float32), N) for k in range(K)]
        s, m = dsp.mix_sources(srcs, gains[b])
        Sm = dsp.stft_tf(m)
        feats.append(np.abs(Sm))
        if crm:
            X.append(dsp.convert2(Sm))
            Y.append(np.stack([dsp.convert2(dsp.stft_tf(s[k])) for k in range(K)]))
        else:
            X.append(np.abs(Sm))
            Y.append(np.stack([np.abs(dsp.stft_tf(s[k])) for k in range(K)]))
    t = lambda a: torch.from_numpy(np.array(a, dtype=np.float32))  # noqa: E731
    return t(feats), t(X), t(Y)


def _setup(dev, cell, L, B, K, N, mode, seed=3, adjust=True, loss_channels=None, precision="fp32", rnn_precision=None):
    crm = mode == "crm"
    net = engine.SepNet(cell=cell, num_layers=L, crm=crm, adjust=adjust, device=dev, seed=seed)
    tr = engine.SepTrainer(net, B, K, N, mode=mode, loss_channels=loss_channels, precision=precision,
                           rnn_precision=rnn_precision)
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=seed)
    src, spk, u = gen.batch(B)
    gains = synth.gains_for(u, K)
    ref = om.SepModel(cell=cell, num_layers=L, crm=crm, adjust=adjust)
    ref.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    return net, tr, src, spk, gains, ref


def _compare_step(dev, cell, L, B, K, N, mode, tol_loss=1e-4, tol_grad=2e-3, loss_channels=None, adjust=True,
                  precision="fp32", tol_pred=1e-3, rnn_precision=None):
    """One training step, HIP vs oracle: loss, masked magnitude (cRM: the masked complex
    spectrogram) rel-L2 < tol_pred, every gradient, and (fp32) the Adam-updated parameters.
    Returns {"masked_rel_l2": ...}."""
    net, tr, src, spk, gains, ref = _setup(dev, cell, L, B, K, N, mode, adjust=adjust, loss_channels=loss_channels,
                                           precision=precision, rnn_precision=rnn_precision)
    feats, X, Y = _oracle_features(src, gains, mode == "crm")
    idx = torch.from_numpy(spk)
    # --- oracle step
    opt = om.make_adam(ref)
    opt.zero_grad()
    mask, V, h, q = ref(feats, idx)
    if mode == "crm":
        loss_ref, pred_ref = om.loss_crm(mask, X, Y)
    elif mode == "pit":
        loss_ref, pred_ref = om.loss_pit(mask, X, Y)
    elif loss_channels:
        pred_ref = mask * X[:, None]
        loss_ref = torch.sum((pred_ref - Y) ** 2) / (B * loss_channels * X.shape[1] * X.shape[2])
    else:
        loss_ref, pred_ref = om.loss_label_ordered(mask, X, Y)
    loss_ref.backward()
    grads_ref = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
    opt.step()
    # --- HIP step
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    g = torch.from_numpy(gains.astype(np.float32)).to(dev)
    sp = torch.from_numpy(spk.astype(np.int32)).to(dev)
    tr.spk.copy_(sp)
    tr.features(raw, g)
    tr.forward()
    # masked magnitude spectrogram / cRM prediction from the COST pass
    T, F = tr.T, tr.F
    shape = (B, K, T * F, 2) if mode == "crm" else (B, K, T * F)
    pred = torch.empty(shape, device=dev)
    tr.attn(0, pred_out=pred)
    loss = tr.loss_and_grad()
    tr.backward()
    tr.optimizer_step()
    tr.check()
    # loss
    l = float(loss[0].cpu())
    assert abs(l - float(loss_ref)) / abs(float(loss_ref)) < tol_loss, (l, float(loss_ref))
    # masked magnitude (the north-star parity metric): relative L2 <= 1e-3 (fp32); cRM: the
    # masked complex spectrogram P = M (x) X (cRM_EvalVer.py:720-728); PIT: channel order
    # differs from the label-ordered reference, compared in _pit_full_size instead
    rel = None
    if mode in ("label", "crm"):
        pr = pred.cpu().view(pred_ref.shape)
        rel = ((pr - pred_ref).norm() / pred_ref.norm()).item()
        assert rel < tol_pred, rel
    # gradients (report every tensor's relative error on failure)
    errs = {}
    for name, gr in grads_ref.items():
        ours = net.view(name, net.grad).cpu()
        denom = gr.abs().max().item()
        errs[name] = (ours - gr).abs().max().item() / denom if denom > 0 else ours.abs().max().item()
    bad = {k: v for k, v in errs.items() if v > tol_grad}
    assert not bad, (bad, errs)
    if precision != "fp32" or tr.rnn_precision != "fp32":
        return {"masked_rel_l2": rel}  # a first Adam step is ~lr*sign(g): not comparable where bf16 moved a small gradient's sign
    _assert_adam_params_close(net, ref, grads_ref, errs)
    return {"masked_rel_l2": rel}


def _assert_adam_params_close(net, ref, grads_ref, errs, lr=2e-4, eps=1e-8):
    """The HIP Adam-updated parameters (net) against the oracle's torch.optim.Adam step (ref) after a
    first step, which moves each weight by ~lr*sign(g): a disagreeing weight must be explained by that
    tensor's measured gradient error errs[name] (relative to its largest reference gradient)."""
    for name, p in ref.named_parameters():
        ours = net.view(name).cpu()
        diff = (ours - p.detach()).abs()
        assert diff.max().item() <= 2.1 * lr, name
        moved = diff > 1e-6
        if moved.any():
            # Adam's first step is lr*g/(|g|+eps): sign-sensitive, and steep near |g| ~ eps
            # (d/dg = lr*eps/(|g|+eps)^2).  A disagreeing weight must be explained by that
            # tensor's measured gradient error err (<= tol_grad of its largest gradient): a sign
            # flip (|g| <= err), or a step change within 4 lr*err*eps/(|g|+eps)^2; and rare
            gr = grads_ref[name]
            err_abs = errs[name] * max(gr.abs().max().item(), 1e-30)
            ga = gr.abs()
            ok = (ga <= err_abs) | (diff <= 4 * lr * err_abs * eps / (ga + eps) ** 2)
            assert bool(ok[moved].all()), (name, int(moved.sum()), gr[moved & ~ok][:8])
            assert moved.float().mean().item() < 1e-2, name


def test_step_bilstm_label_order(dev):
    _compare_step(dev, "lstm", 4, 2, 2, 4000, "label")


def test_step_bilstm_full_length_b1(dev):
    _compare_step(dev, "lstm", 2, 1, 2, 32000, "label")


def test_step_bigru_pit(dev):
    _compare_step(dev, "gru", 2, 3, 2, 3000, "pit")


def test_step_bigru_3spk(dev):
    _compare_step(dev, "gru", 2, 2, 3, 3000, "label")


def test_step_crm(dev):
    _compare_step(dev, "gru", 2, 2, 2, 3000, "crm", tol_grad=5e-3)


def test_step_c1_101_channels(dev):
    # Torch_multi/main_run.py: BiGRU-2L, loss over 101 label channels, no sum term, no ADDJUST
    _compare_step(dev, "gru", 2, 1, 2, 4000, "label", loss_channels=101, adjust=False)


def test_step_bilstm_bf16(dev):
    """bf16 mode (bf16 GEMM operands + bf16 MFMA recurrence, fp32 accumulate and state)
    against the fp32 oracle: loss 1e-2 rel, masked magnitude 1e-2 rel L2, grads 5e-2 of max."""
    _compare_step(dev, "lstm", 4, 4, 2, 8000, "label", precision="bf16", tol_loss=1e-2, tol_grad=5e-2,
                  tol_pred=1e-2)


def test_step_bigru_bf16(dev):
    _compare_step(dev, "gru", 2, 3, 2, 3000, "pit", precision="bf16", tol_loss=1e-2, tol_grad=5e-2, tol_pred=1e-2)


def test_sepnet_state_dict_keys_match_oracle():
    net = engine.SepNet(cell="lstm", num_layers=4, device="cuda")
    ref = om.SepModel(cell="lstm", num_layers=4)
    assert set(net.state_dict()) == set(ref.state_dict())
    net2 = engine.SepNet(cell="gru", num_layers=2, adjust=False, device="cuda")
    ref2 = om.SepModel(cell="gru", num_layers=2, adjust=False)
    assert set(net2.state_dict()) == set(ref2.state_dict())


def test_pit_finds_swapped_targets(dev):
    net, tr, src, spk, gains, ref = _setup(dev, "gru", 1, 4, 2, 2000, "pit")
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(raw, torch.from_numpy(gains.astype(np.float32)).to(dev))
    tr.forward()
    tr.attn(0)
    from dl4ss_amd import _lib
    _lib.call("dl4ss_pit_select", _lib.ptr(tr.part_loss), tr.B, tr.K, tr.nblk, _lib.ptr(tr.perm), _lib.stream_ptr())
    p1 = tr.perm.cpu().clone()
    tr.mag_src.copy_(tr.mag_src.flip(1))
    tr.attn(0)
    _lib.call("dl4ss_pit_select", _lib.ptr(tr.part_loss), tr.B, tr.K, tr.nblk, _lib.ptr(tr.perm), _lib.stream_ptr())
    p2 = tr.perm.cpu()
    assert torch.equal(p2, 1 - p1)  # swapped targets -> swapped assignment, bit-exact


def test_step_c2_full_size_bf16_pit(dev):
    """The benchmark's own configuration (BiLSTM-4L, B = 32, N = 32000 -> T = 251,
    2-spk PIT, bf16 operands) against the fp32 oracle: loss 1e-2 rel, grads 5e-2 of max."""
    _compare_step(dev, "lstm", 4, 32, 2, 32000, "pit", precision="bf16", tol_loss=1e-2, tol_grad=5e-2)


def test_step_c2_full_size_fp32_masked_magnitude(dev):
    """C2 at full size in the fp32 parity mode, label order: the north-star bar -- masked
    magnitude spectrogram within 1e-3 relative L2 of the CPU path -- plus loss / gradients."""
    _compare_step(dev, "lstm", 4, 32, 2, 32000, "label")


@pytest.mark.parametrize("precision,mode", [("bf16", "pit"), ("fp32", "label"), ("bf16s", "pit"), ("bf16s2", "pit")])
def test_graph_step_matches_eager(dev, precision, mode):
    """SepTrainer.step_graph (STFT -> forward -> loss -> backward replayed as one HIP graph,
    mixing / Adam eager) against step() from the same state on three changing batches: for
    each batch the trainer state (parameters, Adam moments, step count) is saved, one eager
    step is taken, the state is restored and the graph step is taken on the same batch;
    losses, gradients and updated parameters must agree (the step is bitwise reproducible,
    test_step_bitwise_reproducible; the bounds here leave room for a replay-only
    reordering: loss 1e-6 relative, gradients 1e-5 of max, parameters 1e-6 absolute, up
    to lr on at most 1e-4 of the elements)."""
    B, K, N = 4, 2, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=5)
    batches = []
    for _ in range(3):
        src, spk, u = gen.batch(B)
        batches.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                        torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
                        torch.from_numpy(spk.astype(np.int32)).to(dev)))
    net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=7)
    tr = engine.SepTrainer(net, B, K, N, mode=mode, precision=precision)
    tr.step(*batches[0])  # eager warm-up step (GEMM plans, workspaces) before the capture
    for b in batches:
        state = (net.flat.detach().clone(), tr.m.clone(), tr.v.clone(), tr.step_count)
        le = float(tr.step(*b)[0].item())
        ge, pe = net.grad.detach().clone(), net.flat.detach().clone()
        net.flat.copy_(state[0]); tr.m.copy_(state[1]); tr.v.copy_(state[2]); tr.step_count = state[3]
        lg = float(tr.step_graph(*b)[0].item())
        tr.check()
        if precision in ("bf16", "bf16s", "bf16s2"):  # the throughput steps are bitwise reproducible: so must the replay be
            assert lg == le and torch.equal(net.grad, ge) and torch.equal(net.flat, pe), (lg, le)
        assert abs(lg - le) <= 1e-6 * abs(le), (lg, le)
        assert float((net.grad - ge).abs().max()) <= 1e-5 * float(ge.abs().max())
        # a near-zero gradient whose last bits differ can move its Adam step by up to lr:
        # allow that on a handful of elements, everything else within 1e-6
        dp = (net.flat - pe).abs()
        assert float(dp.max()) <= 2 * 2e-4 and int((dp > 1e-6).sum()) <= max(1, dp.numel() // 10000)


@pytest.mark.parametrize("precision,mode,B,cell,K", [("bf16", "pit", 4, "lstm", 2), ("bf16", "label", 4, "lstm", 2),
                                                     ("bf16s", "pit", 4, "gru", 3), ("bf16s", "label", 4, "lstm", 2),
                                                     ("bf16", "pit", 32, "lstm", 2), ("bf16", "pit", 4, "gru", 2),
                                                     ("bf16", "pit", 32, "gru", 3), ("bf16s2", "pit", 4, "gru", 3)])
def test_step_bitwise_reproducible(dev, precision, mode, B, cell, K):
    """The bf16 throughput step: two steps from the same saved state on the same batch give
    bit-identical losses, gradients and parameters (every reduction has a fixed order; the
    BiRNN bias gradients go through per-row partials and bias_reduce_kernel, not float
    atomics; every GEMM, the BiGRU's dW_hh included (its dGh direction columns padded to 904,
    DL4SS_RNN_DGH_PAD8), is gemm_gl's fixed-order split-K).  The fp32 parity mode is not
    covered: its split-K GEMMs (gemm.hip) and fp32 BPTT accumulate with atomics."""
    N = 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=9)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    net = engine.SepNet(cell=cell, num_layers=2, adjust=cell == "lstm", device=dev, seed=11)
    tr = engine.SepTrainer(net, B, K, N, mode=mode, precision=precision)
    tr.step(*batch)
    state = (net.flat.detach().clone(), tr.m.clone(), tr.v.clone(), tr.step_count)
    out = []
    for _ in range(2):
        net.flat.copy_(state[0]); tr.m.copy_(state[1]); tr.v.copy_(state[2]); tr.step_count = state[3]
        loss = tr.step(*batch).clone()
        tr.check()
        out.append((loss, net.grad.detach().clone(), net.flat.detach().clone()))
    (l0, g0, p0), (l1, g1, p1) = out
    assert torch.equal(l0, l1)
    diff = [n for n in net.named_parameters() if not torch.equal(net.view(n, g0), net.view(n, g1))]
    assert not diff, diff
    assert torch.equal(p0, p1)


def _pit_full_size(dev, cell, L, B, K, N, precision, adjust=True, tag="c2", tol_pred=1e-3, rnn_precision=None):
    """PIT at full size: the permutation indices the HIP step selects (dl4ss_pit_select over
    all K! assignments) against the oracle's om.pit_assign, bit-exactly on every utterance
    whose best and second-best assignment costs are not tied within the mode's arithmetic
    error (relative cost margin > 1e-4 fp32 / 5e-4 bf16), and the masked magnitude
    spectrogram (channel order, before the assignment) within tol_pred rel-L2 (the north-star
    bar, 1e-3, unless the caller states otherwise).  Returns the record (also written to $DL4SS_PARITY_OUT when set)."""
    import itertools
    import json
    import os

    net, tr, src, spk, gains, ref = _setup(dev, cell, L, B, K, N, "pit", precision=precision, adjust=adjust,
                                           rnn_precision=rnn_precision)
    feats, X, Y = _oracle_features(src, gains, False)
    with torch.no_grad():
        mask, V, h, q = ref(feats, torch.from_numpy(spk))
    perm_ref, _ = om.pit_assign(mask, X, Y)
    pred_ref = (mask * X[:, None]).double()
    C = ((pred_ref[:, :, None] - Y.double()[:, None, :]) ** 2).sum(dim=(-1, -2))  # (B, k, j)
    perms = list(itertools.permutations(range(K)))
    costs = torch.stack([sum(C[:, k, p[k]] for k in range(K)) for p in perms], dim=1)
    srt = torch.sort(costs, dim=1).values
    margin = ((srt[:, 1] - srt[:, 0]) / srt[:, 0]).numpy()
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(torch.from_numpy(src.astype(np.float32)).to(dev), torch.from_numpy(gains.astype(np.float32)).to(dev))
    tr.forward()
    pred = torch.empty(B, K, tr.T * tr.F, device=dev)
    tr.attn(0, pred_out=pred)
    tr.loss_and_grad()
    tr.check()
    perm = tr.perm.cpu().long()
    pred = pred.cpu().view(B, K, tr.T, tr.F)
    rel = float((pred - pred_ref.float()).norm() / pred_ref.float().norm())
    tie = 1e-4 if precision == "fp32" else 5e-4
    decided = margin > tie
    agree = (perm == perm_ref).all(dim=1).numpy()
    ident = torch.arange(K).expand(B, K)
    rec = {"config": tag, "cell": cell, "layers": L, "K": K, "permutations": len(perms), "precision": precision,
           "rnn_precision": tr.rnn_precision,
           "masked_magnitude_rel_l2": rel, "perm_agree": int(agree.sum()), "B": B, "N": N,
           "decided": int(decided.sum()), "agree_on_decided": int(agree[decided].sum()),
           "min_margin": float(margin.min()), "median_margin": float(np.median(margin)),
           "tie_threshold": tie, "n_non_identity_ref": int((perm_ref != ident).any(dim=1).sum()),
           "masked_magnitude_bar": tol_pred}
    out = os.environ.get("DL4SS_PARITY_OUT")
    if out:
        suffix = precision if tr.rnn_precision == precision else f"{precision}_rnn{tr.rnn_precision}"
        with open(out.replace(".json", f"_{tag}_{suffix}.json"), "w") as f:
            json.dump(rec, f)
    print(json.dumps(rec))
    assert agree[decided].all(), rec
    assert rel < tol_pred, rec
    return rec


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_step_c2_full_size_pit_indices(dev, precision):
    """The benchmark's configuration (C2: BiLSTM-4L, B = 32, N = 32000, 2-spk PIT) in both the
    fp32 parity mode and the benched bf16 mode (_pit_full_size): every utterance of this batch
    is decided (smallest margin 9.1e-4; 13 of the 32 choose the swapped assignment), and the
    masked magnitude is within 1e-3 rel-L2 in BOTH modes (measured: fp32 1.5e-7, bf16 3.2e-4)."""
    rec = _pit_full_size(dev, "lstm", 4, 32, 2, 32000, precision, tag="c2")
    assert rec["decided"] == rec["B"], rec


# (precision, rnn_precision): fp32 parity mode; the mixed mode (fp32 GEMMs, bf16 MFMA recurrent
# matvec) that C1 / C3 / C4 throughput is quoted in; the all-bf16 operand mode
C4_MODES = [("fp32", "fp32"), ("fp32", "bf16"), ("bf16s", None), ("bf16s2", None),
            pytest.param("bf16", "bf16", marks=pytest.mark.xfail(
                strict=True, reason="bf16 GEMM operands on the BiGRU nets: 2.2e-3 > the 1e-3 bar "
                                    "(tests/test_bf16_budget_cpu.py reproduces it by emulation)"))]


@pytest.mark.parametrize("precision,rnn_precision", C4_MODES)
def test_step_c4_full_size_pit_3spk_indices(dev, precision, rnn_precision):
    """K = 3 PIT (6 assignments, pit_select_kernel<3> / finalize_kernel<3>) at the full C4 size:
    3-spk mixed-SNR gains (predata_multiAims_3dB), BiGRU-2L without ADDJUST (the selfSS_dB
    model), B = 32, N = 32000.  Under the identity assignment the PIT loss is the reference's
    3-spk loss (Torch_multi/main_run_multi_selfSS_dB.py:513-521); here the chosen assignment
    must equal om.pit_assign on every decided utterance and most utterances must be decided
    (measured: 32 / 32 decided and equal, 25 of them a non-identity assignment), and the masked
    magnitude must be within the north-star 1e-3 (measured: fp32 3.2e-7, mixed 2.9e-4).

    The all-bf16 operand mode misses the bar on this model (2.2e-3, strict xfail): every bf16
    operand of the non-recurrent GEMMs costs ~1e-3 here (features 0.7e-3, W_ih 1.5e-3, the Linear's
    h 0.9e-3 and W 0.9e-3, V 0.9e-3), the bf16 recurrent matvec only 0.3e-3
    (tools/bf16_budget.py, tests/test_bf16_budget_cpu.py) -- so the mixed mode keeps the
    recurrence on bf16 MFMA and the GEMMs exact."""
    rec = _pit_full_size(dev, "gru", 2, 32, 3, 32000, precision, adjust=False, tag="c4", tol_pred=1e-3,
                         rnn_precision=rnn_precision)
    assert rec["decided"] >= rec["B"] * 3 // 4, rec


def test_step_c4_pit_3spk_gradients(dev):
    """The K = 3 PIT step's loss and every gradient (GRAD pass under the chosen permutation,
    finalize_kernel<3>) against the oracle's loss_pit at a reduced C4 shape, fp32."""
    _compare_step(dev, "gru", 2, 4, 3, 8000, "pit", adjust=False)


@pytest.mark.parametrize("precision,mode,cell", [("fp32", "label", "lstm"), ("bf16", "pit", "lstm"),
                                                 ("bf16", "pit", "gru")])
def test_dp_scaled_adam_on_summed_half_batches_equals_full_batch_step(dev, precision, mode, cell):
    """The data-parallel step's N > 1 arithmetic through the shipped kernels, on one GPU: two
    "ranks" take half-batch steps on the same weights (each scaling its loss by its LOCAL batch,
    s1 = 1/(B_local K T F), s2 = 0.5/(B_local T F)) and write their status flag into the slot in front
    of the flat gradient (dl4ss_status_flag); the element-wise sum of the two extended gradients is
    what the SUM all-reduce leaves on every rank; SepTrainer.optimizer_step at world 2 applies it with
    gscale = 1/2 inside the guarded Adam (dl4ss_adam_guarded_dp_scaled[_bf16]).  Checked against
      - the same Adam at world 1 on the pre-halved gradient: bitwise parameters, moments and (bf16)
        the Adam-kept bf16 weight copies, themselves bitwise a fresh conversion of the new weights;
      - the full-batch step at world 1: gradient, first moment and parameters (first Adam step);
      - fp32: the oracle's global-batch torch.optim.Adam step (the reference's objective, the mean
        loss over the whole batch: TDAA_beta/main_run_sstune_EvalVer.py:641,673-675);
    and a summed flag of 1 (one peer's hand-off timed out) refuses the update on every rank."""
    from dl4ss_amd import _lib

    B, K, N, L, seed = 4, 2, 8000, 2, 13
    adjust = cell == "lstm"
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=21)
    src, spk, u = gen.batch(B)
    gains = synth.gains_for(u, K)
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    g = torch.from_numpy(gains.astype(np.float32)).to(dev)
    sp = torch.from_numpy(spk.astype(np.int32)).to(dev)

    def new_net():
        return engine.SepNet(cell=cell, num_layers=L, adjust=adjust, device=dev, seed=seed)

    def grad_step(net, lo, hi):
        """One rank's forward + backward on utterances [lo, hi); returns (trainer, its grad_ext)."""
        tr = engine.SepTrainer(net, hi - lo, K, N, mode=mode, precision=precision)
        tr.spk.copy_(sp[lo:hi])
        tr.features(raw[lo:hi].contiguous(), g[lo:hi].contiguous())
        tr.forward()
        tr.loss_and_grad()
        tr.backward()
        # the rank's status flag in front of its gradient (the trainer writes it only with a process group)
        _lib.call("dl4ss_status_flag", _lib.ptr(tr.status), _lib.ptr(net.dp_flag), _lib.stream_ptr())
        torch.cuda.synchronize()
        tr.check()
        return tr, net.grad_ext.detach().clone()

    # --- two ranks, one SUM all-reduce, Adam at world 2 (gscale 1/2)
    net = new_net()
    tr0, g0 = grad_step(net, 0, B // 2)
    _, g1 = grad_step(net, B // 2, B)
    summed = g0 + g1
    assert float(summed[0]) == 0.0  # no rank timed out
    net.grad_ext.copy_(summed)
    tr0.world = 2
    tr0.optimizer_step()
    tr0.check()
    assert tr0.step_count == 1

    # --- the same Adam at world 1 on the pre-halved sum: bitwise (x 0.5 is exact in fp32)
    netx = new_net()
    trx, _ = grad_step(netx, 0, B // 2)
    netx.grad_ext.copy_(summed * 0.5)
    trx.optimizer_step()
    trx.check()
    torch.cuda.synchronize()
    assert torch.equal(net.flat, netx.flat)
    assert torch.equal(tr0.m, trx.m) and torch.equal(tr0.v, trx.v)
    if tr0.fast:
        assert tr0._shadow_on and not tr0._wb_stale()  # the copies Adam kept are trusted ...

        def fresh(x, like):
            y = torch.zeros_like(like)
            _lib.call("dl4ss_f32_to_bf16_2d", _lib.ptr(x), x.stride(0), x.shape[0], x.shape[1], _lib.ptr(y),
                      y.stride(0), _lib.stream_ptr())
            return y

        torch.cuda.synchronize()
        for l in range(L):  # ... and are bitwise a fresh conversion of the updated weights
            w = net.cat_view("weight_ih", l)
            assert torch.equal(tr0.wb_ih[l][:, :w.shape[1]], fresh(w, tr0.wb_ih[l])[:, :w.shape[1]]), l
            assert torch.equal(tr0.wb_ih[l], trx.wb_ih[l]), l
        assert torch.equal(tr0.wb_lin, trx.wb_lin)

    # --- the full-batch step at world 1
    netf = new_net()
    trf, gf = grad_step(netf, 0, B)
    trf.optimizer_step()
    trf.check()
    mean = 0.5 * summed
    err = float((mean[4:] - gf[4:]).abs().max() / gf[4:].abs().max())
    assert err < (1e-5 if precision == "fp32" else 1e-3), err
    merr = float((tr0.m - trf.m).abs().max() / trf.m.abs().max())
    assert merr < (1e-5 if precision == "fp32" else 1e-3), merr
    dpar = (net.flat - netf.flat).abs()
    assert float(dpar.max()) <= 2.1 * tr0.lr
    # a first Adam step moves each weight by ~lr sign(g): disagreements only where g is at rounding level
    flip = dpar > 1e-6
    tiny = gf[4:].abs() <= (1e-5 if precision == "fp32" else 1e-3) * gf[4:].abs().max()
    assert bool(tiny[flip].all()), int((flip & ~tiny).sum())

    # --- fp32: against the oracle's global-batch Adam step
    if precision == "fp32":
        ref = om.SepModel(cell=cell, num_layers=L, adjust=adjust)
        ref.load_state_dict({k: v.cpu() for k, v in new_net().state_dict().items()})
        feats, X, Y = _oracle_features(src, gains, False)
        opt = om.make_adam(ref)
        opt.zero_grad()
        mask, _, _, _ = ref(feats, torch.from_numpy(spk))
        loss_ref, _ = om.loss_label_ordered(mask, X, Y)
        loss_ref.backward()
        grads_ref = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
        opt.step()
        errs = {}
        for name, gr in grads_ref.items():
            ours = net.view(name, mean[4:]).cpu()
            errs[name] = (ours - gr).abs().max().item() / max(gr.abs().max().item(), 1e-30)
        assert max(errs.values()) < 2e-3, errs
        _assert_adam_params_close(net, ref, grads_ref, errs)

    # --- one peer's hand-off timed out: its flag sums to 1 and every rank refuses the update
    before = net.flat.detach().clone()
    m_before = tr0.m.detach().clone()
    net.grad_ext.copy_(summed)
    net.grad_ext[0] = 1.0
    tr0.optimizer_step()
    torch.cuda.synchronize()
    assert torch.equal(net.flat, before) and torch.equal(tr0.m, m_before)
    assert torch.isnan(tr0.loss[0]).item() and int(tr0.status[1]) == 1
    with pytest.raises(RuntimeError, match="peer"):
        tr0.check()
    assert tr0.step_count == 1  # the refused step is taken back out of the bias corrections


@pytest.mark.parametrize("precision,mode,B,cell,K,L,side,lc", [("bf16", "pit", 4, "lstm", 2, 2, "0", None),
                                                            ("bf16", "pit", 4, "gru", 3, 2, "0", None),
                                                            ("bf16s", "label", 4, "lstm", 2, 2, "0", None),
                                                            ("bf16s", "crm", 4, "gru", 2, 2, "0", None),
                                                            ("bf16s", "label", 1, "gru", 2, 2, "0", 101),
                                                            ("bf16", "pit", 32, "lstm", 2, 4, "1", None)])
def test_step_without_gradient_zeroing_bitwise_equals_zeroed(dev, monkeypatch, precision, mode, B, cell, K, L, side,
                                                             lc):
    """zero_free (the grouped bf16 backward's writers overwrite their gradient regions: beta-0 GEMMs,
    bias reduce, colsum / row sums, query backward zeroing the embedding rows no speaker owns) against
    the zeroed-buffer form (DL4SS_GRAD_ZERO=1) from the same state: bitwise equal losses, gradients and
    parameters -- with the flat gradient filled with NaN before the zero-free step, so a region read
    or left unwritten shows.  side "1": the Linear's gradients on the side stream (DL4SS_SIDE_DWLIN)."""
    N = 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=13)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    monkeypatch.setenv("DL4SS_SIDE_DWLIN", side)
    out = {}
    for zero in ("1", "0"):
        monkeypatch.setenv("DL4SS_GRAD_ZERO", zero)
        net = engine.SepNet(cell=cell, num_layers=L, adjust=cell == "lstm", crm=mode == "crm", device=dev, seed=17)
        if mode == "crm":  # logits below the cRM saturation (the reference's N(0,1) embedding saturates at once)
            net.view("emb.layer.weight").mul_(0.1)
        tr = engine.SepTrainer(net, B, K, N, mode=mode, precision=precision, loss_channels=lc)
        assert tr.zero_free == (zero == "0") and bool(tr.side) == (side == "1")
        for n in net.named_parameters():  # every parameter's region (the 16-B padding between them is
            net.view(n, net.grad).fill_(float("nan"))  # never written by anyone: it stays zero)
        loss = tr.step(*batch).clone()
        tr.check()
        out[zero] = (loss, net.grad.detach().clone(), net.flat.detach().clone())
        del tr
    (l0, g0, p0), (l1, g1, p1) = out["1"], out["0"]
    bad = [n for n in net.named_parameters() if not torch.isfinite(net.view(n, g1)).all()]
    assert not bad, bad  # a region no writer covered (or one that read the buffer)
    diff = [n for n in net.named_parameters() if not torch.equal(net.view(n, g0), net.view(n, g1))]
    assert not diff, diff
    assert torch.equal(l0, l1) and torch.equal(g0, g1) and torch.equal(p0, p1)


def test_adam_bf16_shadow_copies_equal_fresh_conversion(dev):
    """The bf16 weight copies the step's forward reads (every layer's W_ih, the Linear) are kept by
    Adam (dl4ss_adam_guarded_dp_scaled_bf16) instead of a conversion launch per step: after eager and
    graph steps they are bitwise a fresh dl4ss_f32_to_bf16_2d of the updated parameters (padding
    columns zero), and a torch in-place change of the parameters (version counter) is picked up."""
    from dl4ss_amd import _lib

    B, K, N = 4, 2, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=21)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=23)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    assert tr._shadow_on

    def fresh(x, like):
        y = torch.empty_like(like)
        _lib.call("dl4ss_f32_to_bf16_2d", _lib.ptr(x), x.stride(0), x.shape[0], x.shape[1], _lib.ptr(y), y.stride(0),
                  _lib.stream_ptr())
        return y

    def check():
        torch.cuda.synchronize()
        for l in range(net.L):
            assert torch.equal(tr.wb_ih[l], fresh(net.cat_view("weight_ih", l), tr.wb_ih[l])), l
        assert torch.equal(tr.wb_lin, fresh(net.view("mix.Linear.weight"), tr.wb_lin))

    for _ in range(2):
        tr.step(*batch)
    tr.check()
    check()
    tr.step_graph(*batch)
    tr.step_graph(*batch)
    tr.check()
    check()
    with torch.no_grad():
        net.flat.mul_(0.5)  # outside Adam: the next step converts again
    tr.step_graph(*batch)
    tr.check()
    check()


def test_two_trainers_on_one_net_never_read_stale_bf16_copies(dev, monkeypatch):
    """the bf16 weight copies a trainer's Adam keeps are trusted only while the net's
    (generation, version) is what that Adam left -- another trainer's Adam on the same SepNet (which
    bypasses torch's version counter) bumps the generation.  Two trainers (different batch sizes)
    stepping one net alternately, eager and graph steps, are bitwise the same run with a conversion
    every step (DL4SS_ADAM_SHADOW=0)."""
    B, K, N = 4, 2, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=37)
    batches = []
    for _ in range(3):
        src, spk, u = gen.batch(B)
        batches.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                        torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
                        torch.from_numpy(spk.astype(np.int32)).to(dev)))
    half = [tuple(t[:2].contiguous() for t in b) for b in batches]
    out = {}
    for shadow in ("0", "1"):
        monkeypatch.setenv("DL4SS_ADAM_SHADOW", shadow)
        net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=41)
        ta = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
        tb = engine.SepTrainer(net, 2, K, N, mode="pit", precision="bf16")
        assert ta._shadow_on == tb._shadow_on == (shadow == "1")
        losses = []
        for i in range(3):
            losses.append(ta.step(*batches[i]).clone())
            losses.append(tb.step(*half[i]).clone())
        for i in range(3):
            losses.append(ta.step_graph(*batches[i]).clone())
            losses.append(tb.step_graph(*half[i]).clone())
        ta.check()
        tb.check()
        out[shadow] = (torch.stack(losses), net.flat.detach().clone())
        del ta, tb
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])


@pytest.mark.parametrize("cell,K", [("lstm", 2), ("gru", 3)])
def test_workspace_reuse_without_fill_bitwise_equals_fill(dev, monkeypatch, cell, K):
    """The recurrence workspaces are zeroed once and reused as the previous launch left them (no
    per-step fill; release_start puts the start counters / placement granules back) against a fill
    before every step (DL4SS_WS_FILL=1): bitwise equal losses, gradients and parameters over eager
    and graph steps; a forced hand-off timeout in between (check() refills) does not leak into the
    next step."""
    B, N = 32, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=29)
    batches = []
    for _ in range(3):
        src, spk, u = gen.batch(B)
        batches.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                        torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
                        torch.from_numpy(spk.astype(np.int32)).to(dev)))
    from dl4ss_amd import _lib

    out = {}
    for fill in ("1", "0"):
        monkeypatch.setenv("DL4SS_WS_FILL", fill)
        net = engine.SepNet(cell=cell, num_layers=3, adjust=cell == "lstm", device=dev, seed=31)
        tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
        assert tr._ws_fill == (fill == "1")
        losses = [float(tr.step(*b)[0].item()) for b in batches]
        tr.check()
        _lib.lib().dl4ss_debug_set_spin_limit(1)  # a timed-out step, refused ...
        try:
            tr.step(*batches[0])
            torch.cuda.synchronize()
        finally:
            _lib.lib().dl4ss_debug_set_spin_limit(0)
        with pytest.raises(RuntimeError, match="timed out"):
            tr.check()
        losses += [float(tr.step_graph(*b)[0].item()) for b in batches]  # ... and steps after it
        tr.check()
        out[fill] = (losses, net.grad.detach().clone(), net.flat.detach().clone())
        del tr, net
    (l0, g0, p0), (l1, g1, p1) = out["1"], out["0"]
    assert all(np.isfinite(l0)) and l0 == l1
    assert torch.equal(g0, g1) and torch.equal(p0, p1)
