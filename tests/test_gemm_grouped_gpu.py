"""Grouped gemm_gl launch (dl4ss_gemm_bf16_gl_grouped, ops.GroupedGemm): the backward's weight
gradients as one launch + one split-K combine.  Every problem of a group must be BITWISE what the
single launch (dl4ss_gemm_bf16_gl) with the same split factor produces -- same tiles, same slabs,
same fixed-order combine -- including beta accumulation onto existing values, unsplit problems
(written directly), ragged edges and N % 4 != 0 (the scalar combine)."""
import pytest
import torch

from dl4ss_amd import ops

pytestmark = pytest.mark.gpu


def _bf(g, dev, *shape):
    return ops.to_bf16(torch.randn(*shape, generator=g).to(dev))


# (M, N, K, splitk): the C2 / C4 weight-gradient shapes (K = B*T) and ragged small ones
PROBS = [(6450, 600, 8032, 2), (2400, 600, 8032, 4), (1200, 300, 8032, 8), (1200, 300, 8032, 8),
         (2400, 129, 8032, 4), (900, 300, 1000, 3), (130, 257, 700, 1), (64, 72, 64, 2), (17, 9, 130, 5)]


@pytest.mark.parametrize("ta,tb", [(True, False), (False, True), (True, True), (False, False)])
def test_grouped_matches_single_launches(dev, ta, tb):
    g = torch.Generator(device="cpu").manual_seed(11 + 2 * ta + tb)
    probs, singles = [], []
    for (M, N, K, sk) in PROBS:
        A = _bf(g, dev, *((K, (M + 7) // 8 * 8) if ta else (M, (K + 7) // 8 * 8)))
        B = _bf(g, dev, *((N, (K + 7) // 8 * 8) if tb else (K, (N + 7) // 8 * 8)))
        if not ta:
            A[:, K:] = 0  # k-contiguous rows: zero padding up to K rounded to 8
        if tb:
            B[:, K:] = 0
        Av = A[:, :M] if ta else A[:, :K]
        Bv = B[:, :K] if tb else B[:, :N]
        C0 = torch.randn(M, N, generator=g).to(dev)
        beta = 1.0 if sk != 3 else 0.0
        out = C0.clone()
        ref = C0.clone()
        probs.append(dict(A=Av, B=Bv, out=out, transA=ta, transB=tb, beta=beta, splitk=sk, M=M, N=N, K=K))
        singles.append(ops.gemm_bf16_gl(Av, Bv, transA=ta, transB=tb, out=ref, beta=beta, splitk=sk, M=M, N=N, K=K))
    grp = ops.GroupedGemm(probs, dev)
    grp.run()
    torch.cuda.synchronize()
    for p, r, shp in zip(probs, singles, PROBS):
        assert torch.equal(p["out"], r), shp
    # a second run accumulates again (beta 1) with the same bits as a second single launch
    grp.run()
    for p, r, (M, N, K, sk) in zip(probs, singles, PROBS):
        ops.gemm_bf16_gl(p["A"], p["B"], transA=ta, transB=tb, out=r, beta=p["beta"], splitk=sk, M=M, N=N, K=K)
    torch.cuda.synchronize()
    for p, r, shp in zip(probs, singles, PROBS):
        assert torch.equal(p["out"], r), shp


def test_grouped_against_fp64(dev):
    g = torch.Generator(device="cpu").manual_seed(5)
    probs, refs = [], []
    for (M, N, K, sk) in [(300, 200, 1000, 4), (129, 1, 64, 1), (515, 136, 2000, 8)]:
        A = _bf(g, dev, K, (M + 7) // 8 * 8)[:, :M]
        B = _bf(g, dev, K, (N + 7) // 8 * 8)[:, :N]
        out = torch.zeros(M, N, device=dev)
        probs.append(dict(A=A, B=B, out=out, transA=True, transB=False, beta=0.0, splitk=sk))
        Ad, Bd = A.double().cpu(), B.double().cpu()
        refs.append((Ad.t() @ Bd, Ad.abs().t() @ Bd.abs()))
    ops.GroupedGemm(probs, dev).run()
    torch.cuda.synchronize()
    for p, (ref, mag) in zip(probs, refs):
        err = (p["out"].double().cpu() - ref).abs()
        assert bool((err <= 2e-6 * mag + 1e-30).all())


def test_grouped_rejects_mixed_layouts(dev):
    A = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    out = torch.zeros(64, 64, device=dev)
    with pytest.raises(RuntimeError):
        ops.GroupedGemm([dict(A=A, B=A, out=out, transA=True, transB=False),
                         dict(A=A, B=A, out=out, transA=False, transB=False)], dev)


def test_grouped_rejects_views_it_would_write_past(dev):
    """out must be (M, N) (or, with explicit M / N / K, hold them), and explicit
    dimensions must stay inside the operand views -- the argument arrays are frozen at build."""
    A = torch.zeros(128, 64, device=dev, dtype=torch.bfloat16)  # transA: K = 128 rows, M = 64
    B = torch.zeros(128, 32, device=dev, dtype=torch.bfloat16)
    ok = dict(A=A, B=B, transA=True, transB=False)
    ops.GroupedGemm([dict(ok, out=torch.zeros(64, 32, device=dev))], dev)
    with pytest.raises(RuntimeError, match="out shape"):
        ops.GroupedGemm([dict(ok, out=torch.zeros(32, 32, device=dev))], dev)
    with pytest.raises(RuntimeError, match="exceed"):
        ops.GroupedGemm([dict(ok, out=torch.zeros(80, 32, device=dev), M=80)], dev)
    with pytest.raises(RuntimeError, match="out view"):
        ops.GroupedGemm([dict(ok, out=torch.zeros(64, 16, device=dev), N=32)], dev)


def test_grouped_empty_problems_are_no_ops(dev):
    """an empty dimension (an empty batch) is a no-op problem, not an error: M or N = 0
    writes nothing, K = 0 leaves C = beta C; the other problems of the group still run."""
    g = torch.Generator().manual_seed(3)
    A = _bf(g, dev, 96, 64)
    B = _bf(g, dev, 96, 32)
    out = torch.zeros(64, 32, device=dev)
    c_k0 = torch.ones(64, 32, device=dev)
    c_k0b = torch.ones(64, 32, device=dev)
    empty_a = torch.zeros(0, 64, device=dev, dtype=torch.bfloat16)
    empty_b = torch.zeros(0, 32, device=dev, dtype=torch.bfloat16)
    probs = [dict(A=A, B=B, out=out, transA=True, transB=False, beta=0.0),
             dict(A=A[:, :0], B=B, out=torch.zeros(0, 32, device=dev), transA=True, transB=False),  # M = 0
             dict(A=empty_a, B=empty_b, out=c_k0, transA=True, transB=False, beta=0.5),  # K = 0
             dict(A=empty_a, B=empty_b, out=c_k0b, transA=True, transB=False, beta=1.0)]
    ops.GroupedGemm(probs, dev).run()
    torch.cuda.synchronize()
    ref = A.double().cpu().t() @ B.double().cpu()
    assert (out.double().cpu() - ref).abs().max() <= 1e-5 * ref.abs().max()
    assert bool((c_k0 == 0.5).all()) and bool((c_k0b == 1.0).all())
    ops.GroupedGemm([probs[1]], dev).run()  # nothing left to launch


@pytest.mark.parametrize("grid,cfg,one", [(16, 1, True), (7, 1, False), (16, 2, False), (16, 6, False), (0, 6, False),
                                          (9, 7, False)])
def test_grouped_persistent_form_matches(dev, grid, cfg, one):
    """dl4ss_gemm_bf16_gl_grouped_ex: `grid` workgroups walk the tiles (the side-stream form beside
    the recurrence).  Each tile's k-loop and epilogue are the one-tile-per-workgroup launch's, so the
    128 x 128 form is bitwise the grouped launch; the 256 x 128 three-stage tiles sum every output in
    the same k order, bitwise too."""
    g = torch.Generator().manual_seed(11)
    probs, probs_p = [], []
    for (M, N, K, sk) in [(900, 300, 1000, 3), (130, 257, 700, 1), (2400, 600, 1024, 1), (17, 9, 130, 5)]:
        A = _bf(g, dev, K, (M + 7) // 8 * 8)[:, :M]
        B = _bf(g, dev, K, (N + 7) // 8 * 8)[:, :N]
        C0 = torch.randn(M, N, generator=g).to(dev)
        probs.append(dict(A=A, B=B, out=C0.clone(), transA=True, transB=False, beta=1.0, splitk=sk))
        probs_p.append(dict(A=A, B=B, out=C0.clone(), transA=True, transB=False, beta=1.0, splitk=sk))
    ops.GroupedGemm(probs, dev).run()
    ops.GroupedGemm(probs_p, dev, grid=grid, cfg=cfg, one_per_cu=one).run()
    torch.cuda.synchronize()
    for p, q in zip(probs, probs_p):
        assert torch.equal(p["out"], q["out"])


@pytest.mark.parametrize("cfg", [2, 1, 6])
def test_grouped_rowsum_is_the_bias_gradient(dev, cfg):
    """The side-stream dW_lin (engine.SepTrainer.side): the persistent grouped launch also forms
    rowsum[m] = beta rowsum[m] + sum_k op(A)(m, k) -- the Linear's bias gradient, the column sums of
    dPre -- from the tiles of column block 0.  Against fp64 (bf16 operands exact, fp32 sums), with
    the weight gradient bitwise the launch without row sums; ragged M, N and K."""
    g = torch.Generator().manual_seed(5)
    M, N, K = 6450 // 5 + 3, 600 // 4 + 6, 8032 // 8 + 5
    A = _bf(g, dev, K, (M + 7) // 8 * 8)[:, :M]  # dPre (K rows of M) -> op(A) = A^T
    B = _bf(g, dev, K, (N + 7) // 8 * 8)[:, :N]
    r0 = torch.randn(M, generator=g).to(dev)
    rs = r0.clone()
    out = torch.zeros(M, N, device=dev)
    out_ref = torch.zeros(M, N, device=dev)
    ops.GroupedGemm([dict(A=A, B=B, out=out, transA=True, transB=False, beta=1.0, splitk=1, rowsum=rs)], dev,
                    grid=16, cfg=cfg).run()
    ops.GroupedGemm([dict(A=A, B=B, out=out_ref, transA=True, transB=False, beta=1.0, splitk=1)], dev,
                    grid=16, cfg=cfg).run()
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    ref = r0.double().cpu() + A.double().cpu().sum(0)
    mag = r0.double().cpu().abs() + A.double().cpu().abs().sum(0)
    assert bool(((rs.double().cpu() - ref).abs() <= 2e-6 * mag).all())
