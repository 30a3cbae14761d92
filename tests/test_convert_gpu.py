"""fp32 -> bf16 conversions of the bf16 step (convert.hip): the multi-segment row-padded form that
writes every layer's W_ih and the Linear weight copy in one launch (dl4ss_f32_to_bf16_2d_multi),
bitwise against torch's round-to-nearest-even bf16 cast, with zero row padding -- on 16-B aligned
segments (8-column chunks) and on segments whose rows are not (the 4-B pair path)."""
import ctypes

import pytest
import torch

from dl4ss_amd import _lib

pytestmark = pytest.mark.gpu


def test_f32_to_bf16_2d_multi_matches_torch(dev):
    g = torch.Generator(device="cpu").manual_seed(2)
    # (rows, cols, ldx, ldy, x element offset): aligned 600 / 129 / 300-wide rows, and rows that
    # start 4 B off a 16-B boundary (x offset 1, odd ldx) or with ldy % 8 != 0
    shapes = [(2400, 600, 600, 600, 0), (2400, 129, 129, 136, 0), (6450, 600, 600, 608, 0), (37, 131, 133, 138, 1),
              (5, 7, 9, 8, 3)]
    xs, ys, keep = [], [], []
    for rows, cols, ldx, ldy, off in shapes:
        base = torch.randn(rows * ldx + off + 4, generator=g).to(dev)
        x = base[off:off + rows * ldx].view(rows, ldx)
        y = torch.full((rows, ldy), -1.0, device=dev).to(torch.bfloat16)
        xs.append(x)
        ys.append(y)
        keep.append(base)
    n = len(shapes)
    P = ctypes.c_void_p
    _lib.call("dl4ss_f32_to_bf16_2d_multi", n, (P * n)(*[x.data_ptr() for x in xs]),
              (ctypes.c_longlong * n)(*[s[2] for s in shapes]), (ctypes.c_int * n)(*[s[0] for s in shapes]),
              (ctypes.c_int * n)(*[s[1] for s in shapes]), (P * n)(*[y.data_ptr() for y in ys]),
              (ctypes.c_longlong * n)(*[s[3] for s in shapes]), _lib.stream_ptr())
    torch.cuda.synchronize()
    for (rows, cols, ldx, ldy, off), x, y in zip(shapes, xs, ys):
        ref = x[:, :cols].to(torch.bfloat16)
        assert torch.equal(y[:, :cols].view(torch.int16), ref.view(torch.int16)), (rows, cols)
        if ldy > cols:
            assert bool((y[:, cols:].float() == 0).all()), (rows, cols)


def test_bf16_conversions_keep_nan_payloads_nan(dev):
    """round-to-nearest-even by integer add carried a NaN with high mantissa bits
    (0x7FFFFFFF, 0xFFFFFFFF) into the sign / exponent (-> -0 / +0 / inf).  Every conversion path
    must keep NaN a NaN, and inf / finite values as torch rounds them."""
    from dl4ss_amd import ops

    bits = torch.tensor([0x7FFFFFFF, -1, 0x7F800001, 0x7FC00000, 0x7F800000, -8388608, 0x3F800000, 0x7F7FFFFF] * 4,
                        dtype=torch.int32)
    x = bits.view(torch.float32).to(dev)
    ref = x.cpu().to(torch.bfloat16)
    for n in (32, 30):  # the flat path: 4-wide, then with a scalar tail
        y = ops.to_bf16(x[:n].contiguous()).cpu()
        r = ref[:n]
        assert torch.equal(torch.isnan(y), torch.isnan(r))
        fin = ~torch.isnan(r)
        assert torch.equal(y[fin].view(torch.int16), r[fin].view(torch.int16))
    # the 2-D multi-segment path (8-column chunks and the 4-B pair path)
    P = ctypes.c_void_p
    x2 = x.view(4, 8).contiguous()
    for ldy in (8, 10):
        y2 = torch.zeros(4, ldy, device=dev, dtype=torch.bfloat16)
        _lib.call("dl4ss_f32_to_bf16_2d_multi", 1, (P * 1)(x2.data_ptr()), (ctypes.c_longlong * 1)(8),
                  (ctypes.c_int * 1)(4), (ctypes.c_int * 1)(8), (P * 1)(y2.data_ptr()), (ctypes.c_longlong * 1)(ldy),
                  _lib.stream_ptr())
        torch.cuda.synchronize()
        y2 = y2[:, :8].cpu().reshape(-1)
        assert torch.equal(torch.isnan(y2), torch.isnan(ref))
        fin = ~torch.isnan(ref)
        assert torch.equal(y2[fin].view(torch.int16), ref[fin].view(torch.int16))


def test_f32_to_bf16_hilo_split_images(dev):
    """dl4ss_f32_to_bf16_hilo (the bf16s step's split operands): hi = bf16(x), lo = bf16(x - hi),
    segments by pattern, zero column padding to segw and to ldy -- bitwise against torch; and the
    K-concatenated product [x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo] within 2e-5 of fp64 (the
    single bf16 product: ~4e-3)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    rows, cols, segw = 37, 129, 136
    x = torch.randn(rows, cols + 3, generator=g).to(dev)[:, :cols]  # ldx 132 > cols
    for pattern, ldy in ((0b010, 3 * segw), (0b100, 3 * segw + 8)):
        y = torch.full((rows, ldy), -3.0, device=dev).to(torch.bfloat16)
        _lib.call("dl4ss_f32_to_bf16_hilo", _lib.ptr(x, True), x.stride(0), rows, cols, _lib.ptr(y), ldy, segw, 3,
                  pattern, _lib.stream_ptr())
        torch.cuda.synchronize()
        hi = x.cpu().to(torch.bfloat16)
        lo = (x.cpu() - hi.float()).to(torch.bfloat16)
        for sg in range(3):
            ref = lo if (pattern >> sg) & 1 else hi
            seg = y[:, sg * segw:sg * segw + cols].cpu()
            assert torch.equal(seg.view(torch.int16), ref.view(torch.int16)), (pattern, sg)
            assert bool((y[:, sg * segw + cols:(sg + 1) * segw].float() == 0).all())
        assert bool((y[:, 3 * segw:].float() == 0).all())
    # the split product
    from dl4ss_amd import ops

    M, N, K = 64, 48, 129
    a = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(N, K, generator=g).to(dev)
    A = torch.empty(M, 3 * segw, device=dev, dtype=torch.bfloat16)
    W = torch.empty(N, 3 * segw, device=dev, dtype=torch.bfloat16)
    for t, img, pat in ((a, A, 0b010), (w, W, 0b100)):
        _lib.call("dl4ss_f32_to_bf16_hilo", _lib.ptr(t), t.stride(0), t.shape[0], K, _lib.ptr(img), img.stride(0), segw,
                  3, pat, _lib.stream_ptr())
    C = ops.gemm_bf16_gl(A, W, transB=True)
    ref = a.double().cpu() @ w.double().cpu().t()
    mag = a.abs().double().cpu() @ w.abs().double().cpu().t()
    assert float(((C.double().cpu() - ref).abs() / mag).max()) < 2e-5
    C1 = ops.gemm_bf16_gl(A[:, :segw], W[:, :segw], transB=True)
    assert float(((C1.double().cpu() - ref).abs() / mag).max()) > 2e-4  # the plain bf16 product, for contrast
