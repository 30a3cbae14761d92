"""Torch-tensor wrappers over the C ABI (device memory / streams are torch's).

Each wrapper validates shapes on the host (so a kernel never sees a shape it
does not assume), allocates outputs with torch and enqueues exactly one C-ABI
call on the current stream.
"""
import torch

from . import _lib

STFT_COMPLEX, STFT_MAG, STFT_LOGMAG, STFT_CONJ = 1, 2, 4, 8
N_FFT, HOP = 256, 128
F_BINS = N_FFT // 2 + 1


def n_frames(n_samples):
    return 1 + n_samples // HOP


def _f32c(t, name):
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        raise RuntimeError(f"{name}: expected a contiguous float32 CUDA tensor")
    return t


def stft(x, complex_out=True, mag_out=True, log=False, conj=False, out_c=None, out_mag=None, out_bf16=None,
         n_bf16=0):
    """x (..., N) fp32 -> (X (..., T, F, 2) fp32 [re,im], mag (..., T, F) fp32).

    librosa stft(n_fft=256, hop=128) restated (periodic Hann, centre/reflect).
    ``log`` writes log(|X| + eps) into the magnitude output instead.  ``out_bf16`` (rows sig * T + t,
    row stride >= F): bf16 copies of the magnitudes of the first ``n_bf16`` signals, written by the
    same launch (dl4ss_stft_fwd_ex; columns >= F untouched).
    """
    _f32c(x, "stft")
    N = x.shape[-1]
    lead = x.shape[:-1]
    n_sig = x.numel() // N
    T = n_frames(N)
    flags = (STFT_COMPLEX if complex_out else 0) | ((STFT_LOGMAG if log else STFT_MAG) if mag_out else 0)
    flags |= STFT_CONJ if conj else 0
    if complex_out and out_c is None:
        out_c = torch.empty(*lead, T, F_BINS, 2, device=x.device, dtype=torch.float32)
    if mag_out and out_mag is None:
        out_mag = torch.empty(*lead, T, F_BINS, device=x.device, dtype=torch.float32)
    if out_bf16 is not None:
        if not mag_out or out_bf16.dtype != torch.bfloat16 or out_bf16.stride(-1) != 1 or \
                out_bf16.shape[0] < n_bf16 * T or out_bf16.stride(0) < F_BINS or n_bf16 > n_sig:
            raise RuntimeError("stft: out_bf16 must be bf16 rows (>= n_bf16 * T, row stride >= 129) of a magnitude")
        _lib.call("dl4ss_stft_fwd_ex", _lib.ptr(x), n_sig, N, N_FFT, HOP, flags,
                  _lib.ptr(out_c) if complex_out else None, _lib.ptr(out_mag), _lib.ptr(out_bf16),
                  out_bf16.stride(0), n_bf16, _lib.stream_ptr())
        return out_c, out_mag
    _lib.call("dl4ss_stft_fwd", _lib.ptr(x), n_sig, N, N_FFT, HOP, flags, _lib.ptr(out_c) if complex_out else None,
              _lib.ptr(out_mag) if mag_out else None, _lib.stream_ptr())
    return out_c, out_mag


def istft(S, conj=False, out=None):
    """S (..., T, F, 2) fp32 -> y (..., 128*(T-1)) fp32 (librosa istft restated)."""
    _f32c(S, "istft")
    if S.shape[-1] != 2 or S.shape[-2] != F_BINS:
        raise RuntimeError("istft: expected (..., T, 129, 2)")
    T = S.shape[-3]
    lead = S.shape[:-3]
    n_sig = S.numel() // (T * F_BINS * 2)
    L = HOP * (T - 1)
    if out is None:
        out = torch.empty(*lead, L, device=S.device, dtype=torch.float32)
    _lib.call("dl4ss_istft", _lib.ptr(S), n_sig, T, N_FFT, HOP, STFT_CONJ if conj else 0, _lib.ptr(out),
              _lib.stream_ptr())
    return out


def mix_sources(raw, gains, out_src=None, out_mix=None, stats_ws=None, lengths=None, shifts=None):
    """raw (B, K, N) fp32 sources, gains (B, K) fp32 -> (scaled sources (B, K, N),
    mixture (B, N)) -- normalise, gain, sum.  lengths (B, K) int32: each
    source's own length (normalised over it, zero beyond; list-file wavs).  shifts (B, K)
    int32: the AUGMENT_DATA rotation np.append(x[s:], x[:s]) over the source's own length,
    after the normalisation (TDAA_beta/predata_fromList_cRM_123.py:198-200)."""
    _f32c(raw, "mix_sources")
    _f32c(gains, "mix_sources(gains)")
    B, K, N = raw.shape
    if tuple(gains.shape) != (B, K):
        raise RuntimeError("mix_sources: gains must be (B, K)")
    if out_src is None:
        out_src = torch.empty(B, K, N, device=raw.device, dtype=torch.float32)
    if out_mix is None:
        out_mix = torch.empty(B, N, device=raw.device, dtype=torch.float32)
    if stats_ws is None:
        stats_ws = torch.empty(B * K * 32, device=raw.device, dtype=torch.float32)
    if lengths is not None and (lengths.dtype != torch.int32 or tuple(lengths.shape) != (B, K)):
        raise RuntimeError("mix_sources: lengths must be (B, K) int32")
    if shifts is not None and (shifts.dtype != torch.int32 or tuple(shifts.shape) != (B, K) or not shifts.is_cuda
                               or not shifts.is_contiguous()):
        raise RuntimeError("mix_sources: shifts must be a contiguous (B, K) int32 CUDA tensor")
    _lib.call("dl4ss_mix_sources_rot", _lib.ptr(raw), _lib.ptr(lengths), _lib.ptr(shifts), _lib.ptr(gains), B, K, N,
              _lib.ptr(stats_ws), _lib.ptr(out_src), _lib.ptr(out_mix), _lib.stream_ptr())
    return out_src, out_mix


# ---------------------------------------------------------------------------
# dense contractions
# ---------------------------------------------------------------------------
PREC = {"fp32": 0, "bf16": 1}
EPI_NONE, EPI_TANH, EPI_TANH_BF16 = 0, 1, 2  # 2: tanh written as bf16 (gemm_bf16_gl only)
# gemm_bf16_gl split-K only: leave the fp32 slabs in ws for their consumer (no combine, out not written;
# DL4SS_EPI_SPLIT_SLABS, include/dl4ss_hip.h)
EPI_SPLIT_SLABS = 3


def _mat(t, name):
    if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1):
        raise RuntimeError(f"{name}: expected a 2-D row-major float32 CUDA matrix (unit inner stride)")
    return t


def auto_splitk(M, N, K, target_wgs=1024, min_k=512):
    """Split-K factor that gives a short-and-wide GEMM ~target_wgs workgroups (128 x 128
    tiles) while keeping >= min_k of K per split."""
    tiles = -(-M // 128) * -(-N // 128)
    s = max(1, min(-(-target_wgs // tiles), K // min_k))
    return int(s)


def gemm(A, B, transA=False, transB=False, bias=None, epilogue=EPI_NONE, beta=0.0, out=None, precision="fp32",
         splitk=1):
    """out = op(A) @ op(B) (+ bias) (tanh) (+ beta*out).  op(A) = A.T if transA.

    A is stored (M, K) or (K, M) if transA; B is stored (K, N) or (N, K) if transB.
    splitk="auto": split K over workgroups (fp32 atomics) when the tile grid is small
    (needs epilogue none; a beta = 0 output is zeroed first).
    """
    _mat(A, "gemm(A)")
    _mat(B, "gemm(B)")
    M, K = (A.shape[1], A.shape[0]) if transA else (A.shape[0], A.shape[1])
    Kb, N = (B.shape[1], B.shape[0]) if transB else (B.shape[0], B.shape[1])
    if K != Kb:
        raise RuntimeError(f"gemm: inner dims differ ({K} vs {Kb})")
    if out is None:
        if beta != 0.0 or splitk > 1:
            raise RuntimeError("gemm: accumulation needs an output tensor")
        out = torch.empty(M, N, device=A.device, dtype=torch.float32)
    _mat(out, "gemm(out)")
    if tuple(out.shape) != (M, N):
        raise RuntimeError(f"gemm: out shape {tuple(out.shape)} != {(M, N)}")
    if bias is not None and (bias.numel() != N or not bias.is_contiguous()):
        raise RuntimeError("gemm: bias must be contiguous with N elements")
    if splitk == "auto":
        splitk = auto_splitk(M, N, K) if epilogue == EPI_NONE else 1
        if splitk > 1 and beta == 0.0:
            out.zero_()
            beta = 1.0
        elif splitk > 1 and beta != 1.0:
            splitk = 1
    _lib.call("dl4ss_gemm", int(transA), int(transB), M, N, K, _lib.ptr(A, True), A.stride(0), _lib.ptr(B, True), B.stride(0),
              _lib.ptr(out, True), out.stride(0), _lib.ptr(bias), epilogue, float(beta), PREC[precision], int(splitk),
              _lib.stream_ptr())
    return out


GEMM_GL_TARGET_WGS = 512  # gemm_gl (2 workgroups per CU): split-K to about two per CU


def _mat_bf16(t, name):
    if not (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1):
        raise RuntimeError(f"{name}: expected a 2-D row-major bfloat16 CUDA matrix (unit inner stride)")
    return t


_gl_ws = {}


def _gl_workspace(dev, nbytes):
    """split-K slab workspace of dl4ss_gemm_bf16_gl, one per device and stream, grown on demand
    (never inside a graph capture: the eager warm-up step sizes it)"""
    key = (dev, torch.cuda.current_stream().cuda_stream)
    ws = _gl_ws.get(key)
    if ws is None or ws.numel() < nbytes:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("gemm_bf16_gl: split-K workspace must be sized before graph capture")
        ws = _gl_ws[key] = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
    return ws


def gemm_bf16_gl(A, B, transA=False, transB=False, bias=None, epilogue=EPI_NONE, beta=0.0, out=None, splitk=1,
                 batch=1, strideA=0, strideB=0, strideC=0, M=None, N=None, K=None, ws=None):
    """out (fp32, or bf16 with EPI_TANH_BF16) = op(A) @ op(B) (+ bias) (epilogue) (+ beta*out)
    with bf16 A and B through the LDS-DMA MFMA kernel (dl4ss_gemm_bf16_gl, gemm_gl.hip).
    Layout conventions as gemm(); split-K is deterministic (fp32 slabs + fixed-order
    reduce); batch > 1 takes raw element strides from the first-member views.  ws: the
    caller's split-K workspace (a uint8 tensor), else a per-device/stream one grown on demand."""
    _mat_bf16(A, "gemm_bf16_gl(A)")
    _mat_bf16(B, "gemm_bf16_gl(B)")
    if M is None:
        M, K = (A.shape[1], A.shape[0]) if transA else (A.shape[0], A.shape[1])
        Kb, N = (B.shape[1], B.shape[0]) if transB else (B.shape[0], B.shape[1])
        if K != Kb:
            raise RuntimeError(f"gemm_bf16_gl: inner dims differ ({K} vs {Kb})")
    if out is None:
        if beta != 0.0:
            raise RuntimeError("gemm_bf16_gl: accumulation needs an output tensor")
        out = torch.empty(M, N, device=A.device,
                          dtype=torch.bfloat16 if epilogue == EPI_TANH_BF16 else torch.float32)
    if epilogue == EPI_TANH_BF16:
        _mat_bf16(out, "gemm_bf16_gl(out, bf16 epilogue)")
    else:
        _mat(out, "gemm_bf16_gl(out)")
    if batch == 1 and tuple(out.shape) != (M, N):
        raise RuntimeError(f"gemm_bf16_gl: out shape {tuple(out.shape)} != {(M, N)}")
    if bias is not None and (bias.numel() != N or not bias.is_contiguous()):
        raise RuntimeError("gemm_bf16_gl: bias must be contiguous with N elements")
    if splitk == "auto":
        splitk = auto_splitk(M, N, K, target_wgs=max(1, GEMM_GL_TARGET_WGS // batch)) if epilogue == EPI_NONE else 1
    nb = _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", M, N, K, int(splitk), int(batch))
    if nb > 0 and ws is not None and ws.numel() < nb:
        raise RuntimeError(f"gemm_bf16_gl: workspace of {ws.numel()} bytes < {nb}")
    ws = (ws if ws is not None else _gl_workspace(A.device, nb)) if nb > 0 else None
    _lib.call("dl4ss_gemm_bf16_gl", int(transA), int(transB), M, N, K, _lib.ptr(A, True), A.stride(0),
              _lib.ptr(B, True), B.stride(0), _lib.ptr(out, True), out.stride(0), _lib.ptr(bias), epilogue,
              float(beta), int(splitk), int(batch), int(strideA), int(strideB), int(strideC), _lib.ptr(ws),
              ws.numel() if ws is not None else 0, _lib.stream_ptr())
    return out


class GroupedGemm:
    """A fixed list of bf16 GEMM problems C_i = op(A_i) @ op(B_i) + beta_i C_i run as ONE grouped
    launch (dl4ss_gemm_bf16_gl_grouped; + one split-K combine launch).  Each problem is a dict
    with A, B (bf16 views, 16-B aligned rows), out (fp32 view), transA, transB, beta, splitk and
    optionally M, N, K (else from the shapes).  The argument arrays are built once: the tensors
    must stay alive (and at the same addresses) for as long as run() is called."""

    def __init__(self, problems, device, grid=0, cfg=1, one_per_cu=False):
        """grid > 0: the persistent form (dl4ss_gemm_bf16_gl_grouped_ex): ``grid`` workgroups walk the
        tiles, in tile configuration ``cfg`` (1: 128 x 128, 2: 256 x 128 one per CU); one_per_cu pads
        cfg 1 to one workgroup per CU."""
        import ctypes
        self.grid, self.cfg, self.one_per_cu = int(grid), int(cfg), int(bool(one_per_cu))
        if not 1 <= len(problems) <= 16:
            raise RuntimeError("GroupedGemm: 1..16 problems")
        ta, tb = int(problems[0]["transA"]), int(problems[0]["transB"])
        dims, self._keep, kept = [], [], []
        self._k0 = []  # K = 0 problems with beta != 1: C = beta C, applied by run()
        for p in problems:
            A, B, out = p["A"], p["B"], p["out"]
            _mat_bf16(A, "GroupedGemm(A)")
            _mat_bf16(B, "GroupedGemm(B)")
            _mat(out, "GroupedGemm(out)")
            if int(p["transA"]) != ta or int(p["transB"]) != tb:
                raise RuntimeError("GroupedGemm: every problem needs the same transA / transB")
            M, K = (A.shape[1], A.shape[0]) if ta else (A.shape[0], A.shape[1])
            Kb, N = (B.shape[1], B.shape[0]) if tb else (B.shape[0], B.shape[1])
            shapeA, shapeB = (M, K), (Kb, N)
            M, N, K = p.get("M", M), p.get("N", N), p.get("K", K)
            if p.get("K") is None and K != Kb:
                raise RuntimeError(f"GroupedGemm: inner dims differ ({K} vs {Kb})")
            if not any(x in p for x in ("M", "N", "K")):
                if tuple(out.shape) != (M, N):
                    raise RuntimeError(f"GroupedGemm: out shape {tuple(out.shape)} != {(M, N)}")
            # explicit M / N / K: the kernel and its combine must stay inside every view
            # (the argument arrays are frozen here, so a wrong view would be written past silently)
            if not (0 <= M <= shapeA[0] and 0 <= K <= shapeA[1] and K <= shapeB[0] and 0 <= N <= shapeB[1]):
                raise RuntimeError(f"GroupedGemm: M, N, K = {(M, N, K)} exceed the operand views")
            if not (out.shape[0] >= M and out.shape[1] >= N and (N == 0 or out.stride(0) >= N)):
                raise RuntimeError(f"GroupedGemm: out view {tuple(out.shape)} (ldc {out.stride(0)}) < {(M, N)}")
            # empty problems (an empty batch: M or N = 0, or K = 0) launch nothing: no output, or
            # C = beta C with an empty sum
            if M == 0 or N == 0:
                continue
            if K == 0:
                if float(p.get("beta", 0.0)) != 1.0:
                    self._k0.append((out[:M, :N], float(p.get("beta", 0.0))))
                continue
            dims.append((M, N, K))
            kept.append(p)
            self._keep += [A, B, out]
        problems = kept
        n = len(problems)
        self.n = n
        if n == 0:
            return
        Iv = lambda xs: (ctypes.c_int * n)(*xs)
        Lv = lambda xs: (ctypes.c_longlong * n)(*xs)
        Pv = lambda xs: (ctypes.c_void_p * n)(*xs)
        self.n, self.ta, self.tb = n, ta, tb
        self.M, self.N, self.K = Iv([d[0] for d in dims]), Iv([d[1] for d in dims]), Iv([d[2] for d in dims])
        self.A = Pv([p["A"].data_ptr() for p in problems])
        self.lda = Lv([p["A"].stride(0) for p in problems])
        self.B = Pv([p["B"].data_ptr() for p in problems])
        self.ldb = Lv([p["B"].stride(0) for p in problems])
        self.C = Pv([p["out"].data_ptr() for p in problems])
        self.ldc = Lv([p["out"].stride(0) for p in problems])
        self.beta = (ctypes.c_float * n)(*[float(p.get("beta", 0.0)) for p in problems])
        self.splitk = Iv([int(p.get("splitk", 1)) for p in problems])
        # optional per-problem row sums of op(A) ("rowsum": an M-float view; persistent form only)
        rs = [p.get("rowsum") for p in problems]
        for r, (M, _, _), p in zip(rs, dims, problems):
            if r is not None:
                _f32c(r, "GroupedGemm(rowsum)")
                if r.numel() < M or int(p.get("splitk", 1)) != 1 or not (p["transA"] and not p["transB"]):
                    raise RuntimeError("GroupedGemm: rowsum needs M floats, an unsplit problem, transA and not transB")
                self._keep.append(r)
        self.rowsum = Pv([r.data_ptr() if r is not None else None for r in rs]) if any(r is not None for r in rs) \
            else None
        nb = _lib.query("dl4ss_gemm_bf16_gl_grouped_ws_bytes", n, self.M, self.N, self.K, self.splitk)
        if nb < 0:
            raise RuntimeError("GroupedGemm: bad problem list")
        self.ws = torch.empty(max(int(nb), 1), device=device, dtype=torch.uint8)

    def run(self):
        for c, beta in self._k0:
            c.zero_() if beta == 0.0 else c.mul_(beta)  # beta 0: C is not read (stale NaN included)
        if self.n == 0:
            return
        if self.grid > 0 or self.cfg != 1 or self.rowsum is not None:
            _lib.call("dl4ss_gemm_bf16_gl_grouped_ex", self.n, self.ta, self.tb, self.M, self.N, self.K, self.A, self.lda,
                      self.B, self.ldb, self.C, self.ldc, self.beta, self.splitk, _lib.ptr(self.ws), self.ws.numel(),
                      self.grid, self.cfg, self.one_per_cu, self.rowsum, _lib.stream_ptr())
            return
        _lib.call("dl4ss_gemm_bf16_gl_grouped", self.n, self.ta, self.tb, self.M, self.N, self.K, self.A, self.lda,
                  self.B, self.ldb, self.C, self.ldc, self.beta, self.splitk, _lib.ptr(self.ws), self.ws.numel(),
                  _lib.stream_ptr())


def to_bf16(x, out=None):
    """bf16 copy (round to nearest even) of a contiguous fp32 CUDA tensor."""
    _f32c(x, "to_bf16")
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    if out.dtype != torch.bfloat16 or not out.is_contiguous() or out.numel() != x.numel():
        raise RuntimeError("to_bf16: out must be a contiguous bfloat16 tensor of the same size")
    _lib.call("dl4ss_f32_to_bf16", _lib.ptr(x), _lib.ptr(out), x.numel(), _lib.stream_ptr())
    return out


def colsum(A, out):
    """out += A.sum(0) for a row-major matrix view A (M, N)."""
    _mat(A, "colsum")
    _lib.call("dl4ss_colsum", _lib.ptr(A, True), A.stride(0), A.shape[0], A.shape[1], _lib.ptr(out), _lib.stream_ptr())
    return out


def adam_(p, g, m, v, step, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, status=None, loss=None, dp_flag=None, gscale=1.0,
          shadow=None):
    """torch Adam step on flat buffers; with ``status`` (the recurrence hand-off status word,
    2 ints: {timed out, refused-update count}) the update is refused on device when a hand-off
    of this step timed out, loss[0] is set to NaN and status[1] counts the refusal
    (dl4ss_adam_guarded_dp's 2-int status form); with ``dp_flag`` (the all-reduced status flag
    behind the flat gradient) also when a data-parallel peer's hand-off timed out.  ``gscale``: the
    update uses g * gscale (1 / world_size on a SUM-reduced gradient; 1 is bitwise the unscaled step).
    ``shadow``: (nseg, seg_off, seg_rows, seg_cols, seg_y, seg_ldy) ctypes arrays -- bf16 copies of the
    updated parameters written by the same launch (dl4ss_adam_guarded_dp_scaled_bf16)."""
    for t in (p, g, m, v):
        _f32c(t, "adam")
    if status is not None and status.numel() < 2:
        raise ValueError("adam_: the status word needs 2 ints (timed out, refused-update count)")
    if shadow is not None:
        _lib.call("dl4ss_adam_guarded_dp_scaled_bf16", _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), p.numel(),
                  float(lr), float(betas[0]), float(betas[1]), float(eps), int(step), _lib.ptr(status),
                  _lib.ptr(dp_flag), float(gscale), _lib.ptr(loss), *shadow, _lib.stream_ptr())
        return
    _lib.call("dl4ss_adam_guarded_dp_scaled", _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), p.numel(),
              float(lr), float(betas[0]), float(betas[1]), float(eps), int(step), _lib.ptr(status), _lib.ptr(dp_flag),
              float(gscale), _lib.ptr(loss), _lib.stream_ptr())


def birnn_plan(cell, B, H, precision="bf16", max_wg=0):
    """The persistent recurrence's plan {BC, NG, J, nchunk, grid} under a co-residency budget
    of max_wg workgroups (0: the current device's); None when no plan fits (host-only for
    max_wg > 0)."""
    import ctypes

    info = (ctypes.c_int * 5)()
    rc = _lib.lib().dl4ss_birnn_plan_info({"lstm": 0, "gru": 1}[cell], int(B), int(H),
                                          1 if precision == "bf16" else 0, int(max_wg), info)
    if rc != 0:
        return None
    return dict(zip(("BC", "NG", "J", "nchunk", "grid"), list(info)))
