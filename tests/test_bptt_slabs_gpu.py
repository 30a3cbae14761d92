"""The BPTT reading dOut as split-K slabs (DL4SS_RNN_DOUT_SLABS, round 6): the top layer's BPTT of the
bf16 step sums the dH GEMM's S fp32 slabs (gemm_gl DL4SS_EPI_SPLIT_SLABS) as it loads them, instead of a
combine launch in front of it.  The sum is formed in slab order from zero, so every output -- fp32 and bf16
dG / dGh, the fused bias partials -- must be BITWISE the launch on the combined array.  And the trainer's
dH GEMM leaves exactly the slabs the combine would have added."""
import ctypes

import pytest
import torch

from dl4ss_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _slabs(n, S):  # DL4SS_RNN_DOUT_SLABS(S)
    return ((S - 1) & 3) << 12


def _fwd(dev, cell, B, T, H, g):
    ng = 4 if cell == "lstm" else 3
    NGH = ng * H
    cellid = 0 if cell == "lstm" else 1
    G = (torch.randn(B, T, 2, NGH, generator=g) * 0.5).to(dev)
    whh = (torch.randn(2, NGH, H, generator=g) / H ** 0.5).to(dev)
    bhh = (torch.randn(2, NGH, generator=g) * 0.1).to(dev)
    o = torch.empty(B, T, 2 * H, device=dev)
    hp = torch.empty_like(o)
    act = torch.empty(B, T, 2, 4 * H, device=dev)
    cs = torch.empty(B, T, 2, H, device=dev)
    ws = _lib.query("dl4ss_birnn_workspace_bytes", cellid, B, H)
    wsb = torch.zeros((ws + 7) // 8, dtype=torch.int64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_fwd", cellid, 1, B, T, H, _lib.ptr(G), _lib.ptr(whh), _lib.ptr(bhh), _lib.ptr(o),
              _lib.ptr(hp), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    return cellid, NGH, whh, o, hp, act, cs, ws, st


def _bwd(dev, cellid, B, T, H, NGH, dout, flags, whh, act, cs, hp, ws, st, bcast):
    dG = torch.full((B * T, 2 * NGH), float("nan"), device=dev)
    dGh = torch.full_like(dG, float("nan"))
    dGb = torch.empty(B * T, 2 * NGH, device=dev, dtype=torch.bfloat16)
    dbi = torch.zeros(2 * NGH, device=dev)
    dbh = torch.zeros(2 * NGH, device=dev)
    wsb = torch.zeros((ws + 7) // 8, dtype=torch.int64, device=dev)
    _lib.call("dl4ss_birnn_bwd_ex", cellid, 1 | flags, B, T, H, _lib.ptr(dout), _lib.ptr(bcast), _lib.ptr(whh),
              _lib.ptr(act), _lib.ptr(cs), _lib.ptr(hp), _lib.ptr(dG), _lib.ptr(dGh) if cellid == 1 else None,
              _lib.ptr(dGb), None, _lib.ptr(dbi), _lib.ptr(dbh), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    return [dG, dGb, dbi, dbh] + ([dGh] if cellid == 1 else [])


def _bits(t):
    return t.view(torch.int16) if t.dtype == torch.bfloat16 else t.view(torch.int32)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("S", [2, 3, 4])
def test_bptt_dout_slabs_bitwise(dev, cell, S):
    """B = 32 (batch chunks of 4: the packed BPTT's step-factor prefetch), H = 300, ragged T; the slabs
    include exact zeros and negative zeros (0 + -0 = +0 in the combine, so the sum must start from zero)."""
    B, T, H = 32, 11, 300
    g = torch.Generator().manual_seed(100 + S)
    cellid, NGH, whh, o, hp, act, cs, ws, st = _fwd(dev, cell, B, T, H, g)
    sl = torch.randn(S, B, T, 2 * H, generator=g)
    sl[0, :, :, :7] = -0.0
    sl[1:, :, :, :7] = 0.0
    sl = sl.to(dev).contiguous()
    comb = torch.zeros(B, T, 2 * H, device=dev)
    for z in range(S):
        comb = comb + sl[z]
    bcast = torch.randn(B, 2 * H, generator=g).to(dev)
    ref = _bwd(dev, cellid, B, T, H, NGH, comb, 0, whh, act, cs, hp, ws, st, bcast)
    got = _bwd(dev, cellid, B, T, H, NGH, sl, _slabs(None, S), whh, act, cs, hp, ws, st, bcast)
    for a, b in zip(ref, got):
        assert torch.equal(_bits(a), _bits(b))


def test_bptt_dout_slabs_refused_below_chunk_4(dev):
    """Batch chunks < 4 (B = 4 here) have no step-factor prefetch to sum slabs in: refused."""
    B, T, H = 4, 5, 300
    g = torch.Generator().manual_seed(3)
    info = (ctypes.c_int * 5)()
    _lib.call("dl4ss_birnn_plan_info", 0, B, H, 1, 0, info)
    assert info[0] < 4
    cellid, NGH, whh, o, hp, act, cs, ws, st = _fwd(dev, "lstm", B, T, H, g)
    sl = torch.zeros(2, B, T, 2 * H, device=dev)
    with pytest.raises(RuntimeError):
        _bwd(dev, cellid, B, T, H, NGH, sl, _slabs(None, 2), whh, act, cs, hp, ws, st, None)


def test_gemm_split_slabs_are_the_combine_terms(dev):
    """dl4ss_gemm_bf16_gl with DL4SS_EPI_SPLIT_SLABS leaves the S slabs in ws and writes nothing else: their
    in-order sum from zero is bitwise the EPI_NONE launch's C (the dH GEMM of the step, 8032 x 600 x 6450
    at split 3, scaled down); refused when the effective split is 1."""
    g = torch.Generator().manual_seed(9)
    M, N, K, S = 1000, 600, 2000, 3
    A = ops.to_bf16(torch.randn(M, K, generator=g).to(dev))
    Bm = ops.to_bf16(torch.randn(N, K, generator=g).to(dev))
    Bt = Bm.t().contiguous()  # (K, N): the dH GEMM's W_lin operand is k-major
    nb = _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", M, N, K, S, 1)
    assert nb == S * M * N * 4
    ws = torch.empty(nb, device=dev, dtype=torch.uint8)
    c_ref = torch.empty(M, N, device=dev)
    ops.gemm_bf16_gl(A, Bt, out=c_ref, splitk=S, ws=ws)
    c = torch.full((M, N), 7.0, device=dev)
    ops.gemm_bf16_gl(A, Bt, out=c, splitk=S, ws=ws, epilogue=ops.EPI_SPLIT_SLABS)
    torch.cuda.synchronize()
    assert bool((c == 7.0).all())  # C untouched
    part = ws.view(torch.float32).view(S, M, N)
    acc = torch.zeros(M, N, device=dev)
    for z in range(S):
        acc = acc + part[z]
    assert torch.equal(acc.view(torch.int32), c_ref.view(torch.int32))
    with pytest.raises(RuntimeError):
        ops.gemm_bf16_gl(A[:, :64], Bt[:64], out=c, splitk=S, ws=ws, epilogue=ops.EPI_SPLIT_SLABS)


@pytest.mark.parametrize("cell,L,side", [("lstm", 2, "1"), ("gru", 2, "0")])
def test_step_dh_slabs_bitwise_equals_combine(dev, monkeypatch, cell, L, side):
    """The training step with the dH slabs summed by the top BPTT (the default at B = 32) against the
    combine launch (DL4SS_DH_SLABS=0), from the same state: bitwise equal losses, gradients and updated
    parameters, eager and replayed as a graph."""
    import numpy as np

    from dl4ss_amd import engine, synth

    B, K, N = 32, 2, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=5)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    monkeypatch.setenv("DL4SS_SIDE_DWLIN", side)
    out = {}
    for on in ("1", "0"):
        monkeypatch.setenv("DL4SS_DH_SLABS", on)
        net = engine.SepNet(cell=cell, num_layers=L, adjust=cell == "lstm", device=dev, seed=29)
        tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
        assert (tr.dh_slabs > 1) == (on == "1")
        losses = [tr.step(*batch).clone()]
        losses += [tr.step_graph(*batch).clone() for _ in range(2)]  # capture, then a replay
        tr.check()
        out[on] = (losses, net.grad.detach().clone(), net.flat.detach().clone())
        del tr
    (la, ga, pa), (lb, gb, pb) = out["1"], out["0"]
    assert all(torch.equal(x, y) for x, y in zip(la, lb))
    assert torch.equal(ga, gb) and torch.equal(pa, pb)
