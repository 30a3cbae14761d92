"""Stream-K bf16 GEMM (dl4ss_gemm_bf16_gl_streamk, gemm_gl.hip) against an fp64 product of the same
bf16-rounded operands: the step's dX (8032 x 600 x 2400) and dH (8032 x 600 x 6450) shapes, ragged
M / N and short K (tiles split across 2-3 workgroups, tiles one workgroup owns, empty ranges when the
grid exceeds the iterations), every operand layout, beta accumulation; bitwise reproducible run to
run.  Tolerance as tests/test_gemm_gl_gpu.py: 2e-6 of sum |a||b| per output."""
import pytest
import torch

from dl4ss_amd import ops

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("M,N,K,ta,tb,grid", [(8032, 600, 2400, False, False, 0), (8032, 600, 6450, False, False, 0),
                                              (300, 200, 128, False, True, 0), (515, 136, 1000, True, False, 0),
                                              (130, 256, 64, True, True, 0), (2008, 600, 600, False, False, 37),
                                              (64, 8, 8, False, False, 0)])
def test_streamk_matches_fp64_and_is_reproducible(dev, M, N, K, ta, tb, grid):
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + 7 * K)
    k8 = (K + 7) // 8 * 8
    A = torch.zeros(*((K, (M + 7) // 8 * 8) if ta else (M, k8)))
    B = torch.zeros(*((N, k8) if tb else (K, (N + 7) // 8 * 8)))
    if ta:
        A[:, :M] = torch.randn(K, M, generator=g)
    else:
        A[:, :K] = torch.randn(M, K, generator=g)
    if tb:
        B[:, :K] = torch.randn(N, K, generator=g)
    else:
        B[:, :N] = torch.randn(K, N, generator=g)
    Ab, Bb = ops.to_bf16(A.to(dev)), ops.to_bf16(B.to(dev))
    Av = Ab[:, :M] if ta else Ab[:, :K]
    Bv = Bb[:, :K] if tb else Bb[:, :N]
    C0 = torch.randn(M, N, generator=g).to(dev)
    outs = []
    for _ in range(2):
        out = C0.clone()
        ops.gemm_bf16_gl_streamk(Av, Bv, out, transA=ta, transB=tb, beta=0.5, grid=grid)
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    ref, mag = _ref(Av, Bv, ta, tb)
    _check(outs[0], ref + 0.5 * C0.double().cpu(), mag + 0.5 * C0.double().abs().cpu())
