"""The fused input projection (dl4ss_birnn_fwd_xw): every workgroup of the packed bf16 forward
recurrence forms x_t W_ih^T + b_ih of its own gate rows with MFMAs instead of reading G from a
separate gemm_gl launch.  Its arithmetic is the GEMM's (one k-ordered MFMA chain, then + b_ih),
so the layer outputs, saved activations and the bf16 copies must equal the GEMM + recurrence
path BIT FOR BIT, for both cells, both layer-input widths of the nets (129 features, 2H = 600)
and ragged batches; the full training step likewise."""
import numpy as np
import pytest
import torch

from dl4ss_amd import _lib, engine, ops, synth

pytestmark = pytest.mark.gpu

CELLS = {"lstm": 0, "gru": 1}


def _layer(dev, cell, B, T, H, K, seed, xw):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ngh = (4 if cell == "lstm" else 3) * H
    p8 = lambda n: (n + 7) // 8 * 8
    x = torch.zeros(B * T, p8(K), dtype=torch.bfloat16)
    x[:, :K] = torch.randn(B * T, K, generator=g).to(torch.bfloat16)
    # row padding is zero, as the engine's bf16 conversions write it (gemm_gl reads whole 16-B
    # chunks up to the first k >= K; the fused kernel masks k >= Kin itself)
    x = x.to(dev)
    wih = torch.zeros(2 * ngh, p8(K), dtype=torch.bfloat16)
    wih[:, :K] = (torch.randn(2 * ngh, K, generator=g) * 0.1).to(torch.bfloat16)
    wih = wih.to(dev)
    bih = (torch.randn(2, ngh, generator=g) * 0.1).to(dev)
    whh = (torch.randn(2, ngh, H, generator=g) * 0.1).to(dev)
    bhh = (torch.randn(2, ngh, generator=g) * 0.1).to(dev)
    f32 = dict(device=dev, dtype=torch.float32)
    out = torch.empty(B, T, 2 * H, **f32)
    hprev = torch.empty(B, T, 2 * H, **f32)
    act = torch.empty(B, T, 2, 4 * H, **f32)
    cs = torch.empty(B, T, 2, H, **f32) if cell == "lstm" else None
    outb = torch.zeros(B * T, p8(2 * H), device=dev, dtype=torch.bfloat16)
    hprevb = torch.zeros(B * T, 2 * p8(H), device=dev, dtype=torch.bfloat16)
    ws_bytes = _lib.query("dl4ss_birnn_workspace_bytes", CELLS[cell], B, H)
    ws = torch.zeros(ws_bytes, device=dev, dtype=torch.uint8)
    status = torch.zeros(1, device=dev, dtype=torch.int32)
    st = _lib.stream_ptr()
    common = (_lib.ptr(whh), _lib.ptr(bhh), _lib.ptr(out), _lib.ptr(hprev), _lib.ptr(act),
              _lib.ptr(cs) if cs is not None else None, _lib.ptr(outb), _lib.ptr(hprevb), _lib.ptr(ws), ws_bytes,
              _lib.ptr(status), st)
    if xw:
        assert _lib.query("dl4ss_birnn_fwd_xw_supported", CELLS[cell], B, T, H, K) == 1
        _lib.call("dl4ss_birnn_fwd_xw", CELLS[cell], B, T, H, _lib.ptr(x), K, x.stride(0), _lib.ptr(wih),
                  wih.stride(0), _lib.ptr(bih), *common, 0)
    else:
        G = torch.empty(B * T, 2 * ngh, **f32)
        ops.gemm_bf16_gl(x[:, :K], wih[:, :K], transB=True, bias=bih.view(-1), out=G)
        _lib.call("dl4ss_birnn_fwd_ex", CELLS[cell], 1, B, T, H, _lib.ptr(G), *common[:10], _lib.ptr(status), st)
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    res = {"out": out, "act": act, "outb": outb[:, :2 * H], "hprevb": hprevb}
    if cs is not None:
        res["cs"] = cs
    if cell == "gru":
        res["hprev"] = hprev
    return res


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B,T,K", [(32, 251, 600), (32, 251, 129), (5, 40, 600), (3, 17, 129), (1, 2, 600)])
def test_fused_projection_bitwise_equals_gemm_path(dev, cell, B, T, K):
    H = 300
    a = _layer(dev, cell, B, T, H, K, seed=B * 1000 + T + K, xw=False)
    b = _layer(dev, cell, B, T, H, K, seed=B * 1000 + T + K, xw=True)
    for name in a:
        if not torch.equal(a[name], b[name]):
            d = (a[name].float() - b[name].float()).abs().max().item()
            pytest.fail(f"{name} differs (max abs {d})")


def test_fused_projection_support_query():
    # host-only: the packed plan exists for the nets' H = 300 at any batch; Kin is capped at 2 HMAX
    assert _lib.query("dl4ss_birnn_fwd_xw_supported", 0, 32, 251, 300, 600) == 1
    assert _lib.query("dl4ss_birnn_fwd_xw_supported", 0, 32, 251, 300, 641) == 0
    assert _lib.query("dl4ss_birnn_fwd_xw_supported", 0, 32, 251, 600, 600) == 0  # the H = 600 classifier


@pytest.mark.parametrize("mode", ["pit", "label"])
def test_step_with_fused_projection_bitwise_equals_gemm_path(dev, mode):
    """One full bf16 training step (mixing .. Adam) with the fused forward projections vs the
    GEMM path from the same state: loss, every gradient and every updated parameter equal."""
    B, K, N = 8, 2, 8000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=5)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    net = engine.SepNet(cell="lstm", num_layers=4, device=dev, seed=7)
    tr = engine.SepTrainer(net, B, K, N, mode=mode, precision="bf16")
    state = (net.flat.detach().clone(), tr.m.clone(), tr.v.clone(), tr.step_count)
    out = []
    for xw in (False, True):
        tr.xw, tr.xw_kmax = xw, 640  # every layer fused
        net.flat.copy_(state[0]); tr.m.copy_(state[1]); tr.v.copy_(state[2]); tr.step_count = state[3]
        loss = tr.step(*batch).clone()
        tr.check()
        out.append((loss, net.grad.detach().clone(), net.flat.detach().clone()))
    (l0, g0, p0), (l1, g1, p1) = out
    assert torch.equal(l0, l1), (l0, l1)
    diff = [n for n in net.named_parameters() if not torch.equal(net.view(n, g0), net.view(n, g1))]
    assert not diff, diff
    assert torch.equal(p0, p1)
