"""The fused mask-attention + loss kernels on bf16 V (dl4ss_mask_attn_loss_bf16v: attn_q4_kernel, a quad
of lanes per (b, t, f) row) against an fp64 torch restatement of the same arithmetic
(TDAA_beta/main_run_sstune_EvalVer.py:216-226 attention 'dot' + sigmoid, :641,659-666 MSE +
0.5 sum-to-one, PIT over the K targets): masks, loss, dq and the bf16 dPre, for K = 1..3, ragged
tiles (T*F not a multiple of the 256-row tile), a V buffer whose size is not a multiple of 16 B (the
tail chunk), and a dPre row pitch whose rows do not start 16-B aligned (the head / tail words of
the 16-B dPre stores).  Tolerances: fp32 accumulation of bf16 products (masks / loss 1e-5
relative, dq 1e-4 of its max); dPre is bf16 (one rounding: 2^-8 relative)."""
import ctypes

import pytest
import torch

from dl4ss_amd import _lib

pytestmark = pytest.mark.gpu
E = 50


def _ref(Vf, q, X, Y, perm, s1, s2):
    """fp64: masks, loss, dPre, dq of the magnitude path for a given permutation."""
    V, q, X, Y = (t.double().cpu() for t in (Vf, q, X, Y))
    B, R, _ = V.shape
    K = q.shape[1]
    lg = torch.einsum("bre,bke->bkr", V, q)
    m = torch.sigmoid(lg)
    yp = torch.stack([Y[b, perm[b]] for b in range(B)])  # (B, K, R): target of channel k
    d = m * X[:, None, :] - yp
    ds = m.sum(1) - 1.0
    loss = s1 * (d * d).sum() + s2 * (ds * ds).sum()
    dm = 2 * s1 * d * X[:, None, :] + 2 * s2 * ds[:, None, :]
    dl = dm * m * (1 - m)
    dV = torch.einsum("bkr,bke->bre", dl, q)
    dpre = dV * (1 - V * V)
    dq = torch.einsum("bkr,bre->bke", dl, V)
    return m, loss, dpre, dq


@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("B,T,F,ld_pad", [(3, 7, 129, 6), (2, 33, 129, 2), (1, 5, 37, 0)])
def test_attn_bf16v_matches_fp64(dev, K, B, T, F, ld_pad):
    g = torch.Generator(device="cpu").manual_seed(7 * K + T)
    R = T * F
    Vf = torch.tanh(torch.randn(B, R, E, generator=g)).to(torch.bfloat16).to(dev)
    q = (0.3 * torch.randn(B, K, E, generator=g)).to(dev)
    X = torch.rand(B, R, generator=g).to(dev)
    Y = torch.rand(B, K, R, generator=g).to(dev)
    perm = torch.stack([torch.randperm(K, generator=g) for _ in range(B)]).to(torch.int32).to(dev)
    s1, s2 = 1.0 / (B * K * R), 0.5 / (B * R)
    nblk = _lib.query("dl4ss_attn_nblk", T, F)
    part_loss = torch.empty(B, nblk, K * K + 1, device=dev)
    part_dq = torch.empty(B, nblk, K, E, device=dev)
    ldpb = F * E + ld_pad  # even; rows 16-B aligned only when ldpb % 8 == 0
    dpreb = torch.full((B * T, ldpb), float("nan"), device=dev).to(torch.bfloat16)
    mask = torch.empty(B, K, R, device=dev)
    st = _lib.stream_ptr()
    P = ctypes.c_void_p
    for pass_ in (0, 1):
        _lib.call("dl4ss_mask_attn_loss_bf16v", pass_, 0, B, K, T, F, E, _lib.ptr(Vf), _lib.ptr(q), _lib.ptr(X), R,
                  _lib.ptr(Y), K * R, R, _lib.ptr(perm), s1, s2, None, _lib.ptr(dpreb) if pass_ else None,
                  ldpb if pass_ else 0, _lib.ptr(part_loss), _lib.ptr(part_dq) if pass_ else None,
                  _lib.ptr(mask) if pass_ == 0 else None, None, st)
    loss = torch.empty(3, device=dev)
    dq = torch.empty(B, K, E, device=dev)
    _lib.call("dl4ss_loss_finalize", _lib.ptr(part_loss), B, K, nblk, _lib.ptr(perm), s1, s2, _lib.ptr(loss),
              _lib.ptr(part_dq), E, _lib.ptr(dq), st)
    torch.cuda.synchronize()
    m_ref, loss_ref, dpre_ref, dq_ref = _ref(Vf.float(), q, X, Y, perm.long().cpu(), s1, s2)
    assert torch.allclose(mask.double().cpu(), m_ref, rtol=1e-5, atol=1e-6)
    assert abs(float(loss[0]) - float(loss_ref)) <= 1e-5 * abs(float(loss_ref))
    assert float((dq.double().cpu() - dq_ref).abs().max()) <= 1e-4 * float(dq_ref.abs().max())
    got = dpreb[:, :F * E].float().double().cpu().view(B, T, F, E).reshape(B, R, E)
    assert not torch.isnan(got).any()
    assert float((got - dpre_ref).abs().max()) <= 2 ** -8 * float(dpre_ref.abs().max()) + 1e-12
    # the row padding beyond F * E is never written
    if ld_pad:
        assert torch.isnan(dpreb[:, F * E:].float()).all()


def test_attn_bf16v_bitwise_reproducible(dev):
    g = torch.Generator(device="cpu").manual_seed(3)
    B, K, T, F = 4, 2, 40, 129
    R = T * F
    Vf = torch.tanh(torch.randn(B, R, E, generator=g)).to(torch.bfloat16).to(dev)
    q = torch.randn(B, K, E, generator=g).to(dev)
    X = torch.rand(B, R, generator=g).to(dev)
    Y = torch.rand(B, K, R, generator=g).to(dev)
    perm = torch.tensor([[1, 0]] * B, dtype=torch.int32, device=dev)
    nblk = _lib.query("dl4ss_attn_nblk", T, F)
    outs = []
    for _ in range(2):
        pl = torch.empty(B, nblk, K * K + 1, device=dev)
        pd = torch.empty(B, nblk, K, E, device=dev)
        dpreb = torch.empty(B * T, F * E + 6, device=dev, dtype=torch.bfloat16)
        _lib.call("dl4ss_mask_attn_loss_bf16v", 1, 0, B, K, T, F, E, _lib.ptr(Vf), _lib.ptr(q), _lib.ptr(X), R,
                  _lib.ptr(Y), K * R, R, _lib.ptr(perm), 1e-3, 1e-3, None, _lib.ptr(dpreb), F * E + 6, _lib.ptr(pl),
                  _lib.ptr(pd), None, None, _lib.stream_ptr())
        torch.cuda.synchronize()
        outs.append((pl.clone(), pd.clone(), dpreb[:, :F * E].clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _ref_crm(Vf, q, X, Y, perm, s1):
    """fp64: cRM masks (re, im), loss, dPre, dq (cRM_EvalVer.py:259-271, 688, 720-743 arithmetic)."""
    V, q, X, Y = (t.double().cpu() for t in (Vf, q, X, Y))
    B, R, _ = V.shape
    K = q.shape[1]
    lg = torch.stack([torch.einsum("bre,bke->bkr", V, q[:, :, c * E:(c + 1) * E]) for c in range(2)], -1)
    mc = 10 * torch.tanh(lg)
    M = -10 * torch.log((10 - mc) / (10 + mc))  # (B, K, R, 2)
    xr, xi = X[..., 0][:, None], X[..., 1][:, None]
    P = torch.stack([M[..., 0] * xr - M[..., 1] * xi, M[..., 0] * xi + M[..., 1] * xr], -1)
    yp = torch.stack([Y[b, perm[b]] for b in range(B)])
    d = P - yp
    loss = s1 * (d * d).sum()
    g = 2 * s1 * d
    dMr = g[..., 0] * xr + g[..., 1] * xi
    dMi = -g[..., 0] * xi + g[..., 1] * xr
    dmdl = 10 * (1 / (10 - mc) + 1 / (10 + mc)) * 10 * (1 - (mc / 10) ** 2)
    dl = torch.stack([dMr, dMi], -1) * dmdl
    dV = sum(torch.einsum("bkr,bke->bre", dl[..., c], q[:, :, c * E:(c + 1) * E]) for c in range(2))
    dpre = dV * (1 - V * V)
    dq = torch.cat([torch.einsum("bkr,bre->bke", dl[..., c], V) for c in range(2)], -1)
    return M, loss, dpre, dq


@pytest.mark.parametrize("vtype", ["fp32", "bf16"])
@pytest.mark.parametrize("crm,K", [(0, 2), (0, 3), (1, 1), (1, 2)])
@pytest.mark.parametrize("B,T,F,ld_pad", [(3, 7, 129, 6), (1, 5, 37, 0)])
def test_attn_quad_fp32v_and_crm_match_fp64(dev, vtype, crm, K, B, T, F, ld_pad):
    """The quad-per-row kernel's round-5 forms: fp32 V (the split-precision steps) and the cRM path
    (C3), selected by a bf16 dPre output given to BOTH passes, against fp64: masks, loss, dq, dPre."""
    g = torch.Generator(device="cpu").manual_seed(11 * K + T + 3 * crm)
    R = T * F
    QW = 2 * E if crm else E
    Vf = torch.tanh(torch.randn(B, R, E, generator=g))
    Vf = Vf.to(torch.bfloat16).float() if vtype == "bf16" else Vf
    q = ((0.05 if crm else 0.3) * torch.randn(B, K, QW, generator=g)).to(dev)
    X = torch.rand(B, R, 2, generator=g) if crm else torch.rand(B, R, generator=g)
    Y = torch.rand(B, K, R, 2, generator=g) if crm else torch.rand(B, K, R, generator=g)
    X, Y = X.to(dev), Y.to(dev)
    perm = torch.stack([torch.randperm(K, generator=g) for _ in range(B)]).to(torch.int32).to(dev)
    s1, s2 = 1.0 / (B * K * R), (0.0 if crm else 0.5 / (B * R))
    nblk = _lib.query("dl4ss_attn_nblk", T, F)
    part_loss = torch.empty(B, nblk, K * K + 1, device=dev)
    part_dq = torch.empty(B, nblk, K, QW, device=dev)
    ldpb = F * E + ld_pad
    dpreb = torch.full((B * T, ldpb), float("nan"), device=dev).to(torch.bfloat16)
    mask = torch.empty(B, K, R, 2, device=dev) if crm else torch.empty(B, K, R, device=dev)
    Vd = Vf.to(torch.bfloat16).to(dev) if vtype == "bf16" else Vf.to(dev)
    fn = "dl4ss_mask_attn_loss_bf16v" if vtype == "bf16" else "dl4ss_mask_attn_loss_ex"
    st = _lib.stream_ptr()
    for pass_ in (0, 1):
        _lib.call(fn, pass_, crm, B, K, T, F, E, _lib.ptr(Vd), _lib.ptr(q), _lib.ptr(X), R, _lib.ptr(Y), K * R, R,
                  _lib.ptr(perm), s1, s2, None, _lib.ptr(dpreb), ldpb, _lib.ptr(part_loss),
                  _lib.ptr(part_dq) if pass_ else None, _lib.ptr(mask) if pass_ == 0 else None, None, st)
    loss = torch.empty(3, device=dev)
    dq = torch.empty(B, K, QW, device=dev)
    _lib.call("dl4ss_loss_finalize", _lib.ptr(part_loss), B, K, nblk, _lib.ptr(perm), s1, s2, _lib.ptr(loss),
              _lib.ptr(part_dq), QW, _lib.ptr(dq), st)
    torch.cuda.synchronize()
    if crm:
        m_ref, loss_ref, dpre_ref, dq_ref = _ref_crm(Vf, q, X, Y, perm.long().cpu(), s1)
    else:
        m_ref, loss_ref, dpre_ref, dq_ref = _ref(Vf, q, X, Y, perm.long().cpu(), s1, s2)
    assert torch.allclose(mask.double().cpu(), m_ref, rtol=1e-4, atol=1e-5)
    assert abs(float(loss[0]) - float(loss_ref)) <= 1e-4 * abs(float(loss_ref))
    assert float((dq.double().cpu() - dq_ref).abs().max()) <= 1e-4 * float(dq_ref.abs().max())
    got = dpreb[:, :F * E].float().double().cpu().view(B, T, F, E).reshape(B, R, E)
    assert not torch.isnan(got).any()
    assert float((got - dpre_ref).abs().max()) <= 2 ** -8 * float(dpre_ref.abs().max()) + 1e-12
    if ld_pad:
        assert torch.isnan(dpreb[:, F * E:].float()).all()
