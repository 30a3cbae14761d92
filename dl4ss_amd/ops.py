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


def stft(x, complex_out=True, mag_out=True, log=False, conj=False, out_c=None, out_mag=None):
    """x (..., N) fp32 -> (X (..., T, F, 2) fp32 [re,im], mag (..., T, F) fp32).

    librosa stft(n_fft=256, hop=128) restated (periodic Hann, centre/reflect).
    ``log`` writes log(|X| + eps) into the magnitude output instead.
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


def mix_sources(raw, gains, out=None, stats_ws=None):
    """raw (B, K, N) fp32 sources, gains (B, K) fp32 ->
    (B, K+1, N): normalised+scaled sources then their mixture."""
    _f32c(raw, "mix_sources")
    _f32c(gains, "mix_sources(gains)")
    B, K, N = raw.shape
    if gains.shape != (B, K):
        raise RuntimeError("mix_sources: gains must be (B, K)")
    if out is None:
        out = torch.empty(B, K + 1, N, device=raw.device, dtype=torch.float32)
    if stats_ws is None:
        stats_ws = torch.empty(B * K * 2, device=raw.device, dtype=torch.float32)
    _lib.call("dl4ss_mix_sources", _lib.ptr(raw), _lib.ptr(gains), B, K, N, _lib.ptr(stats_ws), _lib.ptr(out),
              _lib.stream_ptr())
    return out
