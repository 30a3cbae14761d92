"""GPU parity of the dense / recurrent kernels against torch-CPU (fp64) references."""
import ctypes

import numpy as np
import pytest
import torch

from dl4ss_amd import _lib, ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(257, 130, 129), (64, 600, 301), (1000, 77, 16), (5, 3, 2)])
def test_gemm_f32_matches_fp64(dev, ta, tb, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    ref = (A.double().T if ta else A.double()) @ (B.double().T if tb else B.double()) + bias.double()
    out = ops.gemm(A.to(dev), B.to(dev), transA=ta, transB=tb, bias=bias.to(dev)).cpu().double()
    err = (out - ref).abs().max() / ref.abs().max()
    assert err < 1e-5, err


def test_gemm_tanh_beta_splitk(dev):
    g = torch.Generator().manual_seed(0)
    A, B = torch.randn(300, 650, generator=g), torch.randn(650, 200, generator=g)
    C0 = torch.randn(300, 200, generator=g)
    ref = torch.tanh(A.double() @ B.double() * 0.05)
    out = ops.gemm((A * 0.05).to(dev), B.to(dev), epilogue=ops.EPI_TANH).cpu().double()
    assert (out - ref).abs().max() < 1e-5
    acc = C0.clone().to(dev)
    ops.gemm(A.to(dev), B.to(dev), out=acc, beta=1.0, splitk=4)
    ref2 = C0.double() + A.double() @ B.double()
    assert ((acc.cpu().double() - ref2).abs().max() / ref2.abs().max()) < 1e-5
    # strided (column-slice) operands
    big = torch.randn(400, 90, generator=g)
    outs = ops.gemm(big[:, 30:60].to(dev) if False else big.to(dev)[:, 30:60], B[:30].to(dev))
    assert ((outs.cpu().double() - big[:, 30:60].double() @ B[:30].double()).abs().max()) < 1e-3


def test_gemm_bf16_tolerance(dev):
    g = torch.Generator().manual_seed(1)
    A, B = torch.randn(513, 600, generator=g), torch.randn(2400, 600, generator=g)
    ref = A.double() @ B.double().T
    out = ops.gemm(A.to(dev), B.to(dev), transB=True, precision="bf16").cpu().double()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


def _birnn_ref(cell, B, T, D, H, seed):
    torch.manual_seed(seed)
    rnn = (torch.nn.LSTM if cell == "lstm" else torch.nn.GRU)(D, H, 1, batch_first=True, bidirectional=True).double()
    x = torch.randn(B, T, D, dtype=torch.float64)
    return rnn, x


def _run_birnn_fwd(dev, cell, rnn, x, H):
    B, T, D = x.shape
    NGH = (4 if cell == "lstm" else 3) * H
    wih = torch.cat([rnn.weight_ih_l0, rnn.weight_ih_l0_reverse]).float().to(dev)
    bih = torch.cat([rnn.bias_ih_l0, rnn.bias_ih_l0_reverse]).float().to(dev)
    whh = torch.cat([rnn.weight_hh_l0, rnn.weight_hh_l0_reverse]).float().contiguous().to(dev)
    bhh = torch.cat([rnn.bias_hh_l0, rnn.bias_hh_l0_reverse]).float().to(dev)
    xd = x.float().to(dev).reshape(B * T, D)
    G = ops.gemm(xd, wih.detach(), transB=True, bias=bih.detach())
    out = torch.empty(B, T, 2 * H, device=dev)
    hprev = torch.empty_like(out)
    act = torch.empty(B, T, 2, 4 * H, device=dev)
    cs = torch.empty(B, T, 2, H, device=dev)
    cellid = 0 if cell == "lstm" else 1
    ws = _lib.query("dl4ss_birnn_workspace_bytes", cellid, B, H)
    wsb = torch.empty((ws + 7) // 8, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_fwd", cellid, 0, B, T, H, _lib.ptr(G), _lib.ptr(whh.detach()), _lib.ptr(bhh.detach()),
              _lib.ptr(out), _lib.ptr(hprev), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(status),
              _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    return dict(G=G, out=out, hprev=hprev, act=act, cs=cs, whh=whh, ws=wsb, wsn=ws, status=status, xd=xd, NGH=NGH)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B,T,H", [(3, 17, 300), (32, 9, 300), (1, 40, 300), (5, 11, 40), (2, 1, 300), (4, 2, 40)])
def test_birnn_fwd_matches_torch(dev, cell, B, T, H):
    rnn, x = _birnn_ref(cell, B, T, 23, H, B * 100 + T)
    ref, _ = rnn(x)
    r = _run_birnn_fwd(dev, cell, rnn, x, H)
    err = (r["out"].cpu().double() - ref).abs().max().item()
    assert err < 2e-5, err
    # hprev is the shifted output (zero at each direction's start)
    hp = r["hprev"].cpu().double()
    assert torch.allclose(hp[:, 1:, :H], r["out"].cpu().double()[:, :-1, :H])
    assert torch.allclose(hp[:, :-1, H:], r["out"].cpu().double()[:, 1:, H:])
    assert hp[:, 0, :H].abs().max() == 0 and hp[:, -1, H:].abs().max() == 0


@pytest.mark.parametrize("use_bc", [False, True])
@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B,T,H", [(3, 17, 300), (32, 6, 300), (2, 9, 40), (2, 1, 300), (3, 2, 40)])
def test_birnn_bwd_matches_autograd(dev, cell, B, T, H, use_bc):
    rnn, x = _birnn_ref(cell, B, T, 23, H, 7 + B + T)
    x.requires_grad_(True)
    ref, _ = rnn(x)
    gout = torch.randn(ref.shape, dtype=torch.float64)  # contiguous (batch_first LSTM output is a view)
    bc = torch.randn(B, 2 * H, dtype=torch.float64) * float(use_bc)
    (ref * gout).sum().backward(retain_graph=True)
    # extra broadcast term: d/dh of sum_t bc . h_t
    (ref * bc[:, None, :]).sum().backward()
    r = _run_birnn_fwd(dev, cell, rnn, x.detach(), H)
    NGH = r["NGH"]
    dG = torch.empty(B * T, 2 * NGH, device=dev)
    dGh = torch.empty_like(dG) if cell == "gru" else None
    cellid = 0 if cell == "lstm" else 1
    gout_d, bc_d = gout.float().to(dev), bc.float().to(dev)  # keep alive across the async launch
    _lib.call("dl4ss_birnn_bwd", cellid, 0, B, T, H, _lib.ptr(gout_d), _lib.ptr(bc_d),
              _lib.ptr(r["whh"]), _lib.ptr(r["act"]), _lib.ptr(r["cs"]), _lib.ptr(r["hprev"]), _lib.ptr(dG),
              _lib.ptr(dGh), _lib.ptr(r["ws"]), r["wsn"], _lib.ptr(r["status"]), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(r["status"].item()) == 0
    dGh = dG if dGh is None else dGh
    # weight gradients from dG / dGh via our GEMMs
    wih = torch.cat([rnn.weight_ih_l0, rnn.weight_ih_l0_reverse])
    dwih = ops.gemm(dG, r["xd"], transA=True).cpu().double()
    ref_dwih = torch.cat([rnn.weight_ih_l0.grad, rnn.weight_ih_l0_reverse.grad])
    assert (dwih - ref_dwih).abs().max() / ref_dwih.abs().max() < 1e-4
    hp = r["hprev"].view(B * T, 2 * H)
    for d, name in enumerate(["weight_hh_l0", "weight_hh_l0_reverse"]):
        dwhh = ops.gemm(dGh[:, d * NGH:(d + 1) * NGH], hp[:, d * H:(d + 1) * H], transA=True).cpu().double()
        refw = getattr(rnn, name).grad
        # T = 1: h_{-1} = 0, so dW_hh is exactly zero on both sides
        assert (dwhh - refw).abs().max() / max(float(refw.abs().max()), 1e-12) < 1e-4, name
    dbih = torch.zeros(2 * NGH, device=dev)
    ops.colsum(dG, dbih)
    ref_db = torch.cat([rnn.bias_ih_l0.grad, rnn.bias_ih_l0_reverse.grad])
    assert (dbih.cpu().double() - ref_db).abs().max() / ref_db.abs().max() < 1e-4
    dbhh = torch.zeros(2 * NGH, device=dev)
    ops.colsum(dGh, dbhh)
    ref_dbh = torch.cat([rnn.bias_hh_l0.grad, rnn.bias_hh_l0_reverse.grad])
    assert (dbhh.cpu().double() - ref_dbh).abs().max() / ref_dbh.abs().max() < 1e-4
    dx = ops.gemm(dG, wih.float().to(dev)).cpu().double().view(B, T, -1)
    assert (dx - x.grad).abs().max() / x.grad.abs().max() < 1e-4


def _bf16(x):
    return x.to(torch.bfloat16).to(x.dtype)


class _Bf16MatVec(torch.autograd.Function):
    """gh = bf16(h) bf16(W)^T with fp64 accumulate; backward dh = bf16(dgh) bf16(W):
    the operand rounding of the kernels' bf16 MFMA recurrence (precision 1)."""

    @staticmethod
    def forward(ctx, h, w):
        wb = _bf16(w)
        ctx.save_for_backward(wb)
        return _bf16(h) @ wb.T

    @staticmethod
    def backward(ctx, g):
        (wb,) = ctx.saved_tensors
        return _bf16(g) @ wb, None


def _manual_birnn(cell, G, whh, bhh, H, bf16=False):
    """Explicit bidirectional recurrence on precomputed input projections G (B,T,2,NGH) (fp64, autograd).
    bf16=True rounds the recurrent matvec operands (forward h and W, backward dgh) to bf16."""
    B, T = G.shape[:2]
    outs = [[None] * T, [None] * T]
    for d in range(2):
        h = torch.zeros(B, H, dtype=G.dtype)
        c = torch.zeros(B, H, dtype=G.dtype)
        order = range(T) if d == 0 else range(T - 1, -1, -1)
        for t in order:
            gh = (_Bf16MatVec.apply(h, whh[d]) if bf16 else h @ whh[d].T) + bhh[d]
            gx = G[:, t, d]
            if cell == "lstm":
                i, f, g, o = (gx + gh).chunk(4, 1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
                h = torch.sigmoid(o) * torch.tanh(c)
            else:
                xr, xz, xn = gx.chunk(3, 1)
                hr, hz, hn = gh.chunk(3, 1)
                r, z = torch.sigmoid(xr + hr), torch.sigmoid(xz + hz)
                n = torch.tanh(xn + r * hn)
                h = (1 - z) * n + z * h
            outs[d][t] = h
    return torch.cat([torch.stack(outs[0], 1), torch.stack(outs[1], 1)], dim=2)


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("cell", ["lstm", "gru"])
# (32, T <= 3, 300): the packed BPTT at batch chunks of 4 with one, two, three steps -- the even / odd step
# loaders of its two-step prefetch (BWD_PF2) at their edges
@pytest.mark.parametrize("B,T,H", [(1, 5, 300), (3, 8, 300), (2, 6, 40), (32, 12, 300), (32, 1, 300), (32, 2, 300),
                                   (32, 3, 300)])
def test_birnn_bwd_dG_per_step(dev, cell, B, T, H, prec):
    """prec 0: exact fp32 recurrence vs fp64 (1e-5 abs on h, 1e-4 rel on dG).
    prec 1: bf16-operand MFMA recurrence vs an fp64 recurrence with the same operand
    rounding (_Bf16MatVec); tolerance 3e-3 abs on h, 2e-3 rel on dG (fp32 vs fp64
    accumulation can flip an operand's bf16 rounding: one flip moves that h value by
    2^-9 |h| <= 2e-3, which then propagates through the recurrence)."""
    ng = 4 if cell == "lstm" else 3
    NGH = ng * H
    g = torch.Generator().manual_seed(B * 31 + T)
    G = torch.randn(B, T, 2, NGH, generator=g, dtype=torch.float64) * 0.5
    whh = torch.randn(2, NGH, H, generator=g, dtype=torch.float64) / H ** 0.5
    bhh = torch.randn(2, NGH, generator=g, dtype=torch.float64) * 0.1
    Gl = G.clone().requires_grad_(True)
    bl = bhh.clone().requires_grad_(True)
    out = _manual_birnn(cell, Gl, whh, bl, H, bf16=prec == 1)
    gout = torch.randn(out.shape, generator=g, dtype=torch.float64)
    tol_h, tol_g = (1e-5, 1e-4) if prec == 0 else (3e-3, 2e-3)
    (out * gout).sum().backward()
    cellid = 0 if cell == "lstm" else 1
    Gd = G.float().to(dev).contiguous()
    whd = whh.float().to(dev).contiguous()
    bhd = bhh.float().to(dev).contiguous()
    o = torch.empty(B, T, 2 * H, device=dev)
    hp = torch.empty_like(o)
    act = torch.empty(B, T, 2, 4 * H, device=dev)
    cs = torch.empty(B, T, 2, H, device=dev)
    ws = _lib.query("dl4ss_birnn_workspace_bytes", cellid, B, H)
    wsb = torch.empty((ws + 7) // 8, dtype=torch.int64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_fwd", cellid, prec, B, T, H, _lib.ptr(Gd), _lib.ptr(whd), _lib.ptr(bhd), _lib.ptr(o),
              _lib.ptr(hp), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert (o.cpu().double() - out.detach()).abs().max() < tol_h
    gd = gout.float().to(dev).contiguous()
    dG = torch.zeros(B * T, 2 * NGH, device=dev)
    dGh = torch.zeros_like(dG)
    _lib.call("dl4ss_birnn_bwd", cellid, prec, B, T, H, _lib.ptr(gd), None, _lib.ptr(whd), _lib.ptr(act), _lib.ptr(cs),
              _lib.ptr(hp), _lib.ptr(dG), _lib.ptr(dGh), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    ours = dG.cpu().double().view(B, T, 2, NGH)
    ref = Gl.grad
    errs = [[(ours[:, t, d] - ref[:, t, d]).abs().max().item() for t in range(T)] for d in range(2)]
    scale = ref.abs().max().item()
    assert max(max(e) for e in errs) < tol_g * scale, (errs, scale)
    # b_hh gradient (sum over b,t of dGh)
    dgh = (dGh if cell == "gru" else dG).cpu().double().view(B, T, 2, NGH).sum((0, 1))
    assert (dgh - bl.grad).abs().max() < tol_g * bl.grad.abs().max()


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B,T", [(1, 13), (4, 9), (32, 7)])
def test_birnn_fwd_large_hidden(dev, cell, B, T, prec):
    """Forward-only large-H plan (H = 600: the speaker classifier BiLSTM-3L of
    EvalVer.py:305-326 / GRID.py:178-199; rnn_fwd_kernel<..., HMAX_L>).  prec 0: exact
    fp32 recurrence vs fp64 (2e-5 abs); prec 1: bf16 MFMA matvec vs the fp64
    recurrence with the same operand rounding (3e-3 abs).  BPTT at H > 320 is refused.  The fp32
    plan at H = 600 needs 50 workgroups per group and fits B <= 16 on a full part: at B = 32 the
    library runs it as two B = 16 launches (split_batch)."""
    H = 600
    ng = 4 if cell == "lstm" else 3
    NGH = ng * H
    g = torch.Generator().manual_seed(B * 13 + T + prec)
    G = torch.randn(B, T, 2, NGH, generator=g, dtype=torch.float64) * 0.5
    whh = torch.randn(2, NGH, H, generator=g, dtype=torch.float64) / H ** 0.5
    bhh = torch.randn(2, NGH, generator=g, dtype=torch.float64) * 0.1
    ref = _manual_birnn(cell, G, whh, bhh, H, bf16=prec == 1)
    cellid = 0 if cell == "lstm" else 1
    Gd, whd, bhd = (t.float().to(dev).contiguous() for t in (G, whh, bhh))
    o = torch.empty(B, T, 2 * H, device=dev)
    hp = torch.empty_like(o)
    act = torch.empty(B, T, 2, 4 * H, device=dev)
    cs = torch.empty(B, T, 2, H, device=dev)
    ws = _lib.query("dl4ss_birnn_workspace_bytes", cellid, B, H)
    assert ws > 0
    wsb = torch.empty((ws + 7) // 8, dtype=torch.int64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_fwd", cellid, prec, B, T, H, _lib.ptr(Gd), _lib.ptr(whd), _lib.ptr(bhd), _lib.ptr(o),
              _lib.ptr(hp), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    err = (o.cpu().double() - ref).abs().max().item()
    assert err < (2e-5 if prec == 0 else 3e-3), err
    if B == 1 and prec == 1:
        dG = torch.zeros(B * T, 2 * NGH, device=dev)
        with pytest.raises(RuntimeError):
            _lib.call("dl4ss_birnn_bwd", cellid, prec, B, T, H, _lib.ptr(o), None, _lib.ptr(whd), _lib.ptr(act),
                      _lib.ptr(cs), _lib.ptr(hp), _lib.ptr(dG), _lib.ptr(dG), _lib.ptr(wsb), ws, _lib.ptr(st),
                      _lib.stream_ptr())


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B,T", [(32, 12), (29, 7)])
def test_birnn_batch_chunk_8(dev, cell, B, T):
    """The plan a B >= 33 batch gets on a full MI355X (or B = 32 under a smaller co-residency
    budget, or a CPX partition): batch chunks of BC = 8, 160 cells per group -- 80 per BPTT
    prefetch wave, more than its 64 lanes (the step factors are formed in passes of 64 lanes,
    round-5 fix).  Forced here with a 120-workgroup budget; bf16 and fp32 recurrences against
    the fp64 references of test_birnn_bwd_dG_per_step."""
    lib = _lib.lib()
    info = (ctypes.c_int * 5)()
    lib.dl4ss_debug_set_rnn_max_wg(120)
    try:
        _lib.call("dl4ss_birnn_plan_info", 0 if cell == "lstm" else 1, B, 300, 1, 0, info)
        assert info[0] == 8 and info[4] <= 120, list(info)
        for prec in (1, 0):
            test_birnn_bwd_dG_per_step(dev, cell, B, T, 300, prec)
    finally:
        lib.dl4ss_debug_set_rnn_max_wg(0)
