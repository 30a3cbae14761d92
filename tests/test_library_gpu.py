"""dl4ss::* custom ops on the GPU: each op returns what the wrapper / autograd.Function it
registers returns (same kernels: bitwise for the forward ops; the fp32 weight-gradient GEMMs
accumulate split-K partials with float atomics, so gradients are compared at 1e-5), the
backwards registered with torch.library.register_autograd match the autograd.Function ones,
and torch.library.opcheck accepts the schemas, fake kernels and autograd registrations."""
import pytest
import torch

from dl4ss_amd import autograd as ag, library as L, ops  # noqa: F401  (library registers the ops)

pytestmark = pytest.mark.gpu


def _close(a, b, tol=1e-5):
    assert a.shape == b.shape
    den = b.abs().max().clamp_min(1e-30)
    assert float((a - b).abs().max() / den) <= tol


def test_stft_istft_ops_bitwise(dev):
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(3, 8000, generator=g).to(dev)
    c, m = ops.stft(x)
    assert torch.equal(torch.ops.dl4ss.stft_mag(x, False), m)
    assert torch.equal(torch.ops.dl4ss.stft_complex(x, False), c)
    _, lm = ops.stft(x, complex_out=False, log=True)
    assert torch.equal(torch.ops.dl4ss.stft_mag(x, True), lm)
    assert torch.equal(torch.ops.dl4ss.istft(c, False), ops.istft(c))
    # mask apply + iSTFT: a magnitude mask of ones rebuilds the mixture's own iSTFT
    y = torch.ops.dl4ss.istft_apply(c, m, 1, False, False)
    _close(y, ops.istft(c), 1e-5)


def test_mix_sources_op_bitwise(dev):
    g = torch.Generator(device="cpu").manual_seed(2)
    raw = torch.randn(2, 3, 4000, generator=g).to(dev)
    gains = torch.rand(2, 3, generator=g).to(dev) + 0.5
    s0, m0 = ops.mix_sources(raw, gains)
    s1, m1 = torch.ops.dl4ss.mix_sources(raw, gains)
    assert torch.equal(s0, s1) and torch.equal(m0, m1)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_birnn_layer_op_matches_function(dev, cell):
    g = torch.Generator(device="cpu").manual_seed(3)
    B, T, D, H = 2, 17, 129, 300
    ng = (4 if cell == "lstm" else 3) * H

    def mk(*s):
        return (torch.randn(*s, generator=g) * 0.1).to(dev)
    x, wih, bih, whh, bhh = mk(B, T, D), mk(2 * ng, D), mk(2 * ng), mk(2 * ng, H), mk(2 * ng)
    dout = mk(B, T, 2 * H)
    res = []
    for path in ("fn", "op"):
        leaves = [t.clone().requires_grad_(True) for t in (x, wih, bih, whh, bhh)]
        if path == "fn":
            out = ag.BiRNNLayerFn.apply(*leaves, cell, H, "fp32")
        else:
            out = L.birnn(*leaves, cell=cell, H=H, precision="fp32")
        (out * dout).sum().backward()
        res.append((out.detach(), [t.grad for t in leaves]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[1][1], res[0][1]):
        _close(a, b)


def test_linear_tanh_op_matches_function(dev):
    g = torch.Generator(device="cpu").manual_seed(4)
    x = torch.randn(34, 600, generator=g).to(dev)
    w = (torch.randn(645, 600, generator=g) * 0.05).to(dev)
    b = torch.randn(645, generator=g).to(dev)
    dv = torch.randn(34, 645, generator=g).to(dev)
    res = []
    for path in ("fn", "op"):
        leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
        v = ag.LinearTanhFn.apply(*leaves, "fp32") if path == "fn" else torch.ops.dl4ss.linear_tanh(*leaves, "fp32")
        (v * dv).sum().backward()
        res.append((v.detach(), [t.grad for t in leaves]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b_ in zip(res[1][1], res[0][1]):
        _close(a, b_)


@pytest.mark.parametrize("crm", [False, True])
def test_attention_dot_op_matches_function(dev, crm):
    g = torch.Generator(device="cpu").manual_seed(5)
    Bq, R, E = 4, 129 * 9, 50
    V = torch.randn(Bq, R, E, generator=g).to(dev)
    q = (torch.randn(Bq, 2 * E if crm else E, generator=g) * 0.2).to(dev)
    dm = torch.randn(Bq, R, 2, generator=g).to(dev) if crm else torch.randn(Bq, R, generator=g).to(dev)
    res = []
    for path in ("fn", "op"):
        leaves = [t.clone().requires_grad_(True) for t in (V, q)]
        m = ag.AttentionDotFn.apply(*leaves, crm) if path == "fn" else torch.ops.dl4ss.attention_dot(*leaves, crm)
        (m * dm).sum().backward()
        res.append((m.detach(), [t.grad for t in leaves]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[1][1], res[0][1]):
        assert torch.equal(a, b)


def test_top_k_mask_op(dev):
    p = torch.tensor([[0.9, 0.1, 0.7, 0.4], [0.2, 0.3, 0.1, 0.05]], device=dev)
    mask, idx, cnt = torch.ops.dl4ss.top_k_mask(p, 0.5, 2)
    m0, i0, c0 = ag.top_k_mask_device(p, 0.5, 2)
    assert torch.equal(mask, m0) and torch.equal(idx, i0) and torch.equal(cnt, c0)


def test_opcheck(dev):
    g = torch.Generator(device="cpu").manual_seed(6)
    utils = ("test_schema", "test_faketensor", "test_autograd_registration")
    x = torch.randn(2, 4000, generator=g).to(dev)
    torch.library.opcheck(torch.ops.dl4ss.stft_mag.default, (x, False), test_utils=utils)
    w = (torch.randn(64, 32, generator=g) * 0.1).to(dev).requires_grad_(True)
    xx = torch.randn(16, 32, generator=g).to(dev).requires_grad_(True)
    b = torch.randn(64, generator=g).to(dev).requires_grad_(True)
    torch.library.opcheck(torch.ops.dl4ss.linear_tanh.default, (xx, w, b, "fp32"), test_utils=utils)
    V = torch.randn(2, 129, 50, generator=g).to(dev).requires_grad_(True)
    q = torch.randn(2, 50, generator=g).to(dev).requires_grad_(True)
    torch.library.opcheck(torch.ops.dl4ss.attention_dot.default, (V, q, False), test_utils=utils)
