"""bf16-operand GEMM (dl4ss_gemm_bf16, gemm_bb.hip) against dl4ss_gemm in bf16 mode on the
fp32 originals: both round operands to bf16 (RNE) and accumulate the same 32x32x16 MFMA
products in the same k order, so without split-K the results are bit-identical; with
split-K only the fp32 atomic summation order differs (1e-5 relative), and the tanh
epilogue uses v_exp/v_rcp (2e-6 absolute)."""
import pytest
import torch

from dl4ss_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda")


SHAPES = [(300, 200, 129), (8032 // 4, 600, 600), (130, 257, 1000), (64, 70, 8), (1, 1, 1), (515, 129, 77),
          (250, 130, 136)]


@pytest.fixture(params=[0, 1, 2, 3], ids=["auto", "t128x128", "t256x128", "t256x256"])
def tile(request):
    """every tile configuration of gemm_bb.hip (forced through dl4ss_gemm_bf16_set_tile)"""
    ops.gemm_bf16_set_tile(request.param)
    yield request.param
    ops.gemm_bf16_set_tile(0)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_bf16_bit_identical(dev, ta, tb, M, N, K, tile):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(*((K, M) if ta else (M, K)), generator=g).to(dev)
    B = torch.randn(*((N, K) if tb else (K, N)), generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    ref = ops.gemm(A, B, transA=ta, transB=tb, bias=bias, precision="bf16")
    ours = ops.gemm_bf16(ops.to_bf16(A), ops.to_bf16(B), transA=ta, transB=tb, bias=bias)
    torch.cuda.synchronize()
    assert torch.equal(ours, ref)


def test_gemm_bf16_tanh_beta_splitk(dev, tile):
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(700, 300, generator=g).to(dev)
    B = torch.randn(450, 300, generator=g).to(dev)
    Ab, Bb = ops.to_bf16(A), ops.to_bf16(B)
    ref = ops.gemm(A, B, transB=True, epilogue=ops.EPI_TANH, precision="bf16")
    ours = ops.gemm_bf16(Ab, Bb, transB=True, epilogue=ops.EPI_TANH)
    assert (ours - ref).abs().max().item() < 2e-6  # v_exp/v_rcp tanh vs tanhf
    C0 = torch.randn(700, 450, generator=g).to(dev)
    ref = ops.gemm(A, B, transB=True, beta=0.5, out=C0.clone(), precision="bf16")
    ours = ops.gemm_bf16(Ab, Bb, transB=True, beta=0.5, out=C0.clone())
    assert torch.equal(ours, ref)
    # weight-gradient form: long K, split-K atomics
    X = torch.randn(5000, 300, generator=g).to(dev)
    D = torch.randn(5000, 240, generator=g).to(dev)
    ref = ops.gemm(D, X, transA=True, precision="bf16")
    ours = ops.gemm_bf16(ops.to_bf16(D), ops.to_bf16(X), transA=True, out=torch.zeros(240, 300, device=dev),
                         beta=1.0, splitk=4)
    assert ((ours - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_gemm_bf16_padded_rows(dev, tile):
    """operands as column slices of row-padded bf16 buffers (the producers' layout)"""
    g = torch.Generator(device="cpu").manual_seed(9)
    A = torch.randn(333, 136, generator=g).to(dev)[:, :129]
    B = torch.randn(260, 136, generator=g).to(dev)[:, :129]
    ref = ops.gemm(A.contiguous(), B.contiguous(), transB=True, precision="bf16")
    Ab = ops.to_bf16(A.contiguous())
    Ap = torch.zeros(333, 136, device=dev, dtype=torch.bfloat16)
    Ap[:, :129] = Ab
    Bp = torch.zeros(260, 136, device=dev, dtype=torch.bfloat16)
    Bp[:, :129] = ops.to_bf16(B.contiguous())
    ours = ops.gemm_bf16(Ap[:, :129], Bp[:, :129], transB=True)
    assert torch.equal(ours, ref)


def test_to_bf16_matches_torch_rne(dev):
    x = torch.randn(1003, device=dev) * 1e3
    assert torch.equal(ops.to_bf16(x), x.to(torch.bfloat16))


def test_gemm_bf16_batched_matches_members(dev, tile):
    """two column blocks of one matrix in one launch (the per-direction W_hh gradients)"""
    g = torch.Generator(device="cpu").manual_seed(11)
    BT, NGH, H, hp8 = 700, 120, 30, 32
    D = ops.to_bf16(torch.randn(BT, 2 * NGH, generator=g).to(dev))
    Hb = torch.zeros(BT, 2 * hp8, device=dev, dtype=torch.bfloat16)
    Hb[:, :H] = torch.randn(BT, H, generator=g).to(dev).to(torch.bfloat16)
    Hb[:, hp8:hp8 + H] = torch.randn(BT, H, generator=g).to(dev).to(torch.bfloat16)
    out = torch.zeros(2 * NGH, H, device=dev)
    ops.gemm_bf16_batched(D[:, :NGH], Hb[:, :H], out[:NGH], 2, NGH, hp8, NGH * H, NGH, H, BT, transA=True, beta=1.0,
                          splitk=3)
    for d in range(2):
        ref = ops.gemm_bf16(D[:, d * NGH:(d + 1) * NGH], Hb[:, d * hp8:d * hp8 + H], transA=True)
        assert ((out[d * NGH:(d + 1) * NGH] - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("ta,tb", [(True, False), (False, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K", [(2400, 600, 8032), (8032, 600, 2400), (300, 129, 77), (1, 5, 3)])
def test_gemm_bf16_lt_matches_kernel(dev, ta, tb, M, N, K):
    """hipBLASLt path (the plain backward GEMMs) vs the hand-written bf16 kernel on the same
    bf16 operands: same products, different fp32 summation order (1e-5 of the max)."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = ops.to_bf16(torch.randn(*((K, M) if ta else (M, K)), generator=g).to(dev))
    B = ops.to_bf16(torch.randn(*((N, K) if tb else (K, N)), generator=g).to(dev))
    C0 = torch.randn(M, N, generator=g).to(dev)
    ref = ops.gemm_bf16(A, B, transA=ta, transB=tb, out=C0.clone(), beta=0.5)
    ours = ops.gemm_bf16_lt(A, B, C0.clone(), transA=ta, transB=tb, beta=0.5)
    torch.cuda.synchronize()
    assert ((ours - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_gemm_bf16_lt_batched(dev):
    """both W_hh gradient directions in one strided-batch call (the engine's dW_hh)"""
    g = torch.Generator(device="cpu").manual_seed(12)
    BT, NGH, H, hp8 = 700, 120, 30, 32
    D = ops.to_bf16(torch.randn(BT, 2 * NGH, generator=g).to(dev))
    Hb = torch.zeros(BT, 2 * hp8, device=dev, dtype=torch.bfloat16)
    Hb[:, :H] = torch.randn(BT, H, generator=g).to(dev).to(torch.bfloat16)
    Hb[:, hp8:hp8 + H] = torch.randn(BT, H, generator=g).to(dev).to(torch.bfloat16)
    out = torch.zeros(2 * NGH, H, device=dev)
    ops.gemm_bf16_lt(D[:, :NGH], Hb[:, :H], out[:NGH], transA=True, beta=1.0, batch=2, strideA=NGH, strideB=hp8,
                     strideC=NGH * H, M=NGH, N=H, K=BT)
    for d in range(2):
        ref = ops.gemm_bf16(D[:, d * NGH:(d + 1) * NGH], Hb[:, d * hp8:d * hp8 + H], transA=True)
        assert ((out[d * NGH:(d + 1) * NGH] - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_gemm_bf16_tanh_bf16_output(dev):
    """EPI_TANH_BF16 (the Linear's V written as bf16): equals bf16(RNE) of the fp32 tanh epilogue."""
    g = torch.Generator(device="cpu").manual_seed(21)
    A = ops.to_bf16(torch.randn(700, 600, generator=g).to(dev) * 0.1)
    Bw = ops.to_bf16(torch.randn(450, 600, generator=g).to(dev) * 0.1)
    bias = torch.randn(450, generator=g).to(dev)
    ref = ops.gemm_bf16(A, Bw, transB=True, bias=bias, epilogue=ops.EPI_TANH)
    out = torch.empty(700, 450, device=dev, dtype=torch.bfloat16)
    ops.gemm_bf16(A, Bw, transB=True, bias=bias, epilogue=ops.EPI_TANH_BF16, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref.to(torch.bfloat16))


def test_attention_bf16v_matches_fp32_of_bf16(dev):
    """dl4ss_mask_attn_loss_bf16v on bf16 V == dl4ss_mask_attn_loss_ex on the same values in fp32."""
    from dl4ss_amd import _lib
    g = torch.Generator(device="cpu").manual_seed(22)
    B, K, T, F, E = 2, 2, 9, 129, 50
    Vb = (torch.randn(B, T * F, E, generator=g) * 0.3).to(torch.bfloat16).to(dev)
    V = Vb.float()
    q = torch.randn(B, K, E, generator=g).to(dev)
    X = torch.rand(B, T * F, generator=g).to(dev)
    Y = torch.rand(B, K, T * F, generator=g).to(dev)
    nblk = _lib.query("dl4ss_attn_nblk", T, F)
    outs = []
    for fn, v in (("dl4ss_mask_attn_loss_ex", V), ("dl4ss_mask_attn_loss_bf16v", Vb)):
        part = torch.zeros(B, nblk, K * K + 1, device=dev)
        pdq = torch.zeros(B, nblk, K, E, device=dev)
        dpre = torch.zeros(B * T, F * E + 6, device=dev, dtype=torch.bfloat16)
        _lib.call(fn, 1, 0, B, K, T, F, E, _lib.ptr(v), _lib.ptr(q), _lib.ptr(X), T * F, _lib.ptr(Y), K * T * F,
                  T * F, None, 1e-3, 5e-4, None, _lib.ptr(dpre), dpre.stride(0), _lib.ptr(part), _lib.ptr(pdq), None,
                  None, _lib.stream_ptr())
        torch.cuda.synchronize()
        outs.append((part, pdq, dpre))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
