"""LDS-DMA bf16 GEMM (dl4ss_gemm_bf16_gl, gemm_gl.hip) against an fp64 product of the same
bf16-rounded operands: every operand layout (k-contiguous / k-major for A and B), ragged M / N
(tiles past the edge), K tails (zero-line chunks), bias / tanh / tanh -> bf16 epilogues, beta
accumulation, the deterministic split-K (bitwise reproducible; equal to the unsplit product
within fp32 summation order) and the strided batch.  fp32 accumulation of bf16 products: the
tolerance is 2e-6 of sum |a||b| per output (the accumulation-order bound at K <= 8032)."""
import pytest
import torch

from dl4ss_amd import _lib, ops

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1, 2, 3, 4, 5, 6, 7, 8, 9], ids=["auto", "c128x128", "c256x128_3stage", "c128x128_3stage",
                                                     "c256x256_pp8", "c256x256_pp10", "c128x128_deep5x32",
                                                     "c128x128_deep4x32", "c128x128_2x32_4percu", "c64x128"],
                autouse=True)
def gl_config(request):
    """every tile configuration of gemm_gl.hip (forced through dl4ss_gemm_gl_set_config)"""
    _lib.call("dl4ss_gemm_gl_set_config", request.param)
    yield request.param
    _lib.call("dl4ss_gemm_gl_set_config", 0)

SHAPES = [(300, 200, 128), (2008, 600, 600), (130, 257, 1000), (64, 72, 8), (8, 8, 8), (515, 136, 80),
          (250, 130, 136), (129, 1, 64)]


def _ref(Ab, Bb, ta, tb):
    A = Ab.double().cpu()
    B = Bb.double().cpu()
    A = A.t() if ta else A
    B = B.t() if tb else B
    return A @ B, A.abs() @ B.abs()


def _check(ours, ref, mag, tol=2e-6):
    err = (ours.double().cpu() - ref).abs()
    bound = tol * mag + 1e-30
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_gl_layouts(dev, ta, tb, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    # k-major operands need a row stride >= rows rounded up to 8: pad the stored rows
    A = torch.randn(*((K, (M + 7) // 8 * 8) if ta else (M, K)), generator=g).to(dev)
    B = torch.randn(*((N, K) if tb else (K, (N + 7) // 8 * 8)), generator=g).to(dev)
    Ab, Bb = ops.to_bf16(A), ops.to_bf16(B)
    Av = Ab[:, :M] if ta else Ab
    Bv = Bb if tb else Bb[:, :N]
    bias = torch.randn(N, generator=g).to(dev)
    ours = ops.gemm_bf16_gl(Av, Bv, transA=ta, transB=tb, bias=bias)
    torch.cuda.synchronize()
    ref, mag = _ref(Av, Bv, ta, tb)
    _check(ours, ref + bias.double().cpu(), mag)


def test_gemm_gl_epilogues_and_beta(dev):
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(700, 304, generator=g).to(dev)
    B = torch.randn(452, 304, generator=g).to(dev)
    Ab, Bb = ops.to_bf16(A), ops.to_bf16(B)
    bias = torch.randn(452, generator=g).to(dev)
    ref, mag = _ref(Ab, Bb, False, True)
    ref = ref + bias.double().cpu()
    t = ops.gemm_bf16_gl(Ab, Bb, transB=True, bias=bias, epilogue=ops.EPI_TANH)
    assert (t.double().cpu() - torch.tanh(ref)).abs().max().item() < 2e-5
    tb = ops.gemm_bf16_gl(Ab, Bb, transB=True, bias=bias, epilogue=ops.EPI_TANH_BF16)
    assert tb.dtype == torch.bfloat16
    assert (tb.double().cpu() - torch.tanh(ref)).abs().max().item() < 2 ** -8 + 2e-5
    C0 = torch.randn(700, 452, generator=g).to(dev)
    out = ops.gemm_bf16_gl(Ab, Bb, transB=True, beta=0.5, out=C0.clone())
    ref2, _ = _ref(Ab, Bb, False, True)
    _check(out, ref2 + 0.5 * C0.double().cpu(), mag + 0.5 * C0.double().cpu().abs())


@pytest.mark.parametrize("M,N,ld,off", [(8032, 6450, 6450, 0), (8032, 6450, 6450, 2), (700, 452, 458, 4),
                                          (333, 200, 206, 6), (130, 64, 64, 0)],
                         ids=["linear", "linear_off4B", "ld458_off8B", "ld206_off12B", "one_block"])
def test_gemm_gl_bf16_v_epilogue_bitwise(dev, M, N, ld, off):
    """The Linear's tanh -> bf16 V epilogue (rows staged in LDS shifted by their own 16-B misalignment,
    written as aligned 16-B chunks + head / tail words): bitwise the RNE bf16 of the fp32 tanh epilogue
    (same k-loop), for every row misalignment (V rows of 2 ld bytes, V starting off bytes past 16 B),
    the partial last column block and rows past a 128 multiple; nothing outside V is written."""
    g = torch.Generator(device="cpu").manual_seed(M + N + off)
    K = 600
    Ab = ops.to_bf16(torch.randn(M, K, generator=g).to(dev))
    Bb = ops.to_bf16(torch.randn(N, K, generator=g).to(dev))
    bias = torch.randn(N, generator=g).to(dev)
    ref = ops.gemm_bf16_gl(Ab, Bb, transB=True, bias=bias, epilogue=ops.EPI_TANH).to(torch.bfloat16)
    buf = torch.full((M * ld + off + 64,), 7.0, device=dev, dtype=torch.bfloat16)
    V = buf[off:off + M * ld].view(M, ld)[:, :N]
    ops.gemm_bf16_gl(Ab, Bb, transB=True, bias=bias, epilogue=ops.EPI_TANH_BF16, out=V)
    torch.cuda.synchronize()
    assert torch.equal(V.view(torch.int16).cpu(), ref.view(torch.int16).cpu())
    mask = torch.ones(buf.numel(), dtype=torch.bool)
    idx = (off + torch.arange(M)[:, None] * ld + torch.arange(N)[None, :]).reshape(-1)
    mask[idx] = False
    assert bool((buf.cpu()[mask] == 7.0).all())


@pytest.mark.parametrize("ta,tb", [(True, False), (False, False), (True, True)])
def test_gemm_gl_splitk_deterministic(dev, ta, tb):
    """weight-gradient form (long K, small output): split-K slabs summed in fixed order"""
    g = torch.Generator(device="cpu").manual_seed(9)
    M, N, K = 240, 300, 5000
    A = torch.randn(*((K, M) if ta else (M, K)), generator=g).to(dev)
    B = torch.randn(*((N, K) if tb else (K, 304)), generator=g).to(dev)  # 16-B aligned rows
    Ab, Bb = ops.to_bf16(A), ops.to_bf16(B)
    Bb = Bb if tb else Bb[:, :N]
    C0 = torch.randn(M, N, generator=g).to(dev)
    outs = [ops.gemm_bf16_gl(Ab, Bb, transA=ta, transB=tb, beta=1.0, out=C0.clone(), splitk=s) for s in (1, 6, 6)]
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[2])  # bitwise reproducible
    ref, mag = _ref(Ab, Bb, ta, tb)
    for o in outs:
        _check(o, ref + C0.double().cpu(), mag + C0.double().cpu().abs())


@pytest.mark.parametrize("NGH,ldg", [(1200, 1200), (900, 904)], ids=["lstm", "gru_pad8"])
def test_gemm_gl_strided_batch(dev, NGH, ldg):
    """both directions' dW_hh in one launch: member d reads columns d*ldg of dGh and d*pad8(H)
    of h_{t-1} (the engine's batched form), with and without split-K.  GRU: 900 gate rows per
    direction, stored at a 904-column stride (DL4SS_RNN_DGH_PAD8) so member 1 starts 16-B aligned."""
    g = torch.Generator(device="cpu").manual_seed(3)
    BT, H, hp8 = 1004, 300, 304
    dG = ops.to_bf16(torch.randn(BT, 2 * ldg, generator=g).to(dev))
    hp = ops.to_bf16(torch.randn(BT, 2 * hp8, generator=g).to(dev))
    for s in (1, 3, 8):
        out = torch.zeros(2 * NGH, H, device=dev)
        ops.gemm_bf16_gl(dG[:, :NGH], hp[:, :H], transA=True, out=out[:NGH], beta=1.0, splitk=s, batch=2,
                         strideA=ldg, strideB=hp8, strideC=NGH * H, M=NGH, N=H, K=BT)
        torch.cuda.synchronize()
        for d in range(2):
            ref, mag = _ref(dG[:, d * ldg:d * ldg + NGH], hp[:, d * hp8:d * hp8 + H], True, False)
            _check(out[d * NGH:(d + 1) * NGH], ref, mag)


def test_gemm_gl_k_tail_in_zero_padded_rows(dev):
    """K = 6450 (the Linear's F * E): k-contiguous rows padded with zeros to 6456, the k-major
    operand bounded per k-row -- the backward dH = dPre W_lin of the step"""
    g = torch.Generator(device="cpu").manual_seed(4)
    M, N, K = 300, 600, 6450
    A = torch.zeros(M, 6456, device=dev)
    A[:, :K] = torch.randn(M, K, generator=g).to(dev)
    B = torch.randn(K, N, generator=g).to(dev)
    Ab, Bb = ops.to_bf16(A), ops.to_bf16(B)
    out = ops.gemm_bf16_gl(Ab[:, :K], Bb, M=M, N=N, K=K)
    torch.cuda.synchronize()
    ref, mag = _ref(Ab[:, :K], Bb, False, False)
    _check(out, ref, mag)


def test_gemm_gl_rejects_short_rows(dev):
    A = ops.to_bf16(torch.randn(64, 104, device=dev))[:, :100]  # ld 104 >= 104: accepted
    B = ops.to_bf16(torch.randn(64, 100, device=dev))  # ld 100 < 104: rejected
    with pytest.raises(RuntimeError):
        ops.gemm_bf16_gl(A, B, transB=True)
