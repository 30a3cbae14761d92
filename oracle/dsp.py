"""Oracle DSP: framed STFT / iSTFT and source preprocessing (TEST INFRASTRUCTURE ONLY).

Restates the third-party arithmetic the reference calls at its data boundary:

* ``librosa.core.spectrum.stft(y, n_fft=256, hop_length=128)`` as called at
  ``Torch_multi/predata_multiAims_dB.py:180,194,209,214`` and
  ``TDAA_beta/predata_fromList_cRM_123.py:215,217,232,234,250,254,255``
  (librosa is absent and unpinned; restated from its published algorithm:
  periodic Hann window, ``center=True`` reflect padding of n_fft//2, frame t =
  padded[hop*t : hop*t + n_fft], rfft bins 0..n_fft/2, complex64 output;
  librosa <= 0.5.x conjugates the output, >= 0.6 does not).
* ``librosa.core.spectrum.istft(S, hop_length=128)`` as called at
  ``TDAA_beta/main_run_sstune_EvalVer.py:64-65`` and
  ``main_run_sstune_cRM_EvalVer.py:98-99``: per frame irfft * window,
  overlap-add, divide by the summed squared window where it is not tiny, trim
  n_fft//2 from both ends -> hop*(T-1) samples, float32.
* Source preprocessing / mixing:
  ``Torch_multi/predata_multiAims_dB.py:123-197`` (2-spk dB gain on one random
  channel), ``Torch_multi/predata_multiAims_3dB.py:132-145,192-217`` (3-spk
  gains), ``TDAA_beta/predata_fromList_cRM_123.py:174-237`` (list dB gains), and the
  train-split AUGMENT_DATA rotation of the list loaders
  (``TDAA_beta/predata_fromList.py:150-151``, ``predata_fromList_cRM_123.py:198-200``) beside
  the Torch_multi loaders' broadcast form of the same line
  (``Torch_multi/predata_multiAims_dB.py:164-166``, ``predata_multiAims_3dB.py:179-181``).
  Pinned to the reference's own statements by ``tests/golden/ref_r1_augment.npz``.
"""
import math

import numpy as np

N_FFT = 256
HOP = 128


def hann_periodic(n=N_FFT):
    """scipy.signal.get_window('hann', n, fftbins=True) (float64)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def n_frames(n_samples, hop=HOP):
    # centre padding adds n_fft//2 each side -> 1 + floor(N / hop) frames
    return 1 + n_samples // hop


def frame_signal(y, n_fft=N_FFT, hop=HOP):
    """Reflect-pad by n_fft//2 and frame; returns (T, n_fft) float64."""
    y = np.asarray(y, dtype=np.float64)
    pad = n_fft // 2
    yp = np.pad(y, pad, mode="reflect")
    T = 1 + (len(yp) - n_fft) // hop
    idx = hop * np.arange(T)[:, None] + np.arange(n_fft)[None, :]
    return yp[idx]


def stft(y, n_fft=N_FFT, hop=HOP, conj=False):
    """librosa stft restated; returns (F, T) complex64 (librosa orientation)."""
    fr = frame_signal(y, n_fft, hop) * hann_periodic(n_fft)[None, :]
    S = np.fft.rfft(fr, axis=1).T  # (F, T), float64 compute
    if conj:
        S = S.conj()
    return S.astype(np.complex64)


def stft_tf(y, conj=False):
    """np.transpose(stft(y)) as the reference stores it: (T, F) complex64."""
    return np.ascontiguousarray(stft(y, conj=conj).T)


def magnitude(y, conj=False):
    return np.abs(stft_tf(y, conj)).astype(np.float32)


def log_magnitude(y):
    """predata_multiAims.py:194-198 log branch, with the Hann window."""
    return np.log(np.abs(stft_tf(y)) + np.float32(np.spacing(1))).astype(np.float32)


def convert2(S_tf):
    """predata_fromList_cRM_123.py:37-41: (T,F) complex -> (T,F,2) [re, im] float32."""
    o = np.empty(S_tf.shape + (2,), dtype=np.float32)
    o[..., 0] = S_tf.real
    o[..., 1] = S_tf.imag
    return o


def istft(S_ft, hop=HOP, conj=False, dtype=np.float32):
    """librosa istft restated; S_ft is (F, T) complex; returns hop*(T-1) samples."""
    S_ft = np.asarray(S_ft)
    F, T = S_ft.shape
    n_fft = 2 * (F - 1)
    w = hann_periodic(n_fft)
    L = n_fft + hop * (T - 1)
    y = np.zeros(L, dtype=dtype)
    wss = np.zeros(L, dtype=dtype)
    for i in range(T):
        spec = S_ft[:, i]
        if conj:
            spec = spec.conj()
        full = np.concatenate((spec, spec[-2:0:-1].conj()))
        ytmp = w * np.fft.ifft(full).real
        y[i * hop:i * hop + n_fft] += ytmp.astype(dtype)
        wss[i * hop:i * hop + n_fft] += (w * w).astype(dtype)
    nz = wss > np.finfo(dtype).tiny
    y[nz] /= wss[nz]
    return y[n_fft // 2:-(n_fft // 2)]


# ----------------------------------------------------------------------------
# R1: preprocessing and mixing
# ----------------------------------------------------------------------------

def normalise_source(x, max_len, shift=None, broadcast=False):
    """Crop, x -= mean, x /= max|x|, [rotate], zero-pad (predata_multiAims_dB.py:156-175).

    shift: the list loaders' AUGMENT_DATA branch on the train split,
    ``signal = np.append(signal[s:], signal[:s])`` with s drawn from range(len(signal))
    -- a rotation over the source's OWN (cropped) length, before the zero-padding
    (predata_fromList.py:150-151, predata_fromList_cRM_123.py:198-200).  broadcast=True:
    the Torch_multi loaders' form of that line instead (``augment_torch_multi``)."""
    x = np.asarray(x, dtype=np.float64)[:max_len].copy()
    x -= np.mean(x)
    x /= np.max(np.abs(x))
    if shift is not None:
        x = augment_torch_multi(x, shift) if broadcast else np.append(x[shift:], x[:shift])
    if x.shape[0] < max_len:
        x = np.append(x, np.zeros(max_len - x.shape[0]))
    return x


def augment_torch_multi(x, shift):
    """Torch_multi/predata_multiAims_dB.py:164-166 (and _3dB.py:179-181): the same
    augmentation written ``signal[s:] + signal[:s]`` -- a numpy broadcast of two slices of
    lengths len-s and s, which raises ValueError unless one of them has length 1 or both
    are equal (s in {1, len-1, len/2}); then it is an elementwise SUM, not a rotation."""
    x = np.asarray(x, dtype=np.float64)
    return x[shift:] + x[:shift]


def mix_sources_f32(raw, gains, lengths=None, shifts=None):
    """fp32 restatement of the mixing kernel's arithmetic (``mixing.hip``), for bit-exact
    comparison of the index work (crop length, rotation, zero-padding) and of the values:

    mean = fp32(sum_fp64 / len) (the sum correctly rounded here, a fixed tree there -- they
    agree after the fp32 rounding unless the fp64 mean sits within ~1e-12 relative of an fp32
    rounding boundary); peak = max(max x - mean, mean - min x) in fp32 (= max |fl(x - mean)|,
    fp32 subtraction being monotonic); g = fp32(gain * fp32(1 / peak));
    out[i] = fp32(fp32(x[(i + s) mod len] - mean) * g) for i < len, 0 beyond;
    mixture = sum over k in order 0..K-1 in fp32.

    raw (B, K, N) float32, gains (B, K) float32, lengths / shifts (B, K) int or None."""
    raw = np.asarray(raw, np.float32)
    B, K, N = raw.shape
    gains = np.asarray(gains, np.float32)
    src = np.zeros((B, K, N), np.float32)
    for b in range(B):
        for k in range(K):
            ln = N if lengths is None else int(min(max(int(lengths[b][k]), 0), N))
            if ln == 0:
                continue
            x = raw[b, k, :ln]
            mean = np.float32(math.fsum(x.astype(np.float64).tolist()) / ln)
            pk = max(np.float32(x.max() - mean), np.float32(mean - x.min()))
            inv = np.float32(1.0) / pk if pk > 0 else np.float32(0.0)
            g = np.float32(gains[b, k] * inv)
            y = (x - mean).astype(np.float32) * g
            s = 0 if shifts is None else int(shifts[b][k]) % ln
            if s:
                y = np.append(y[s:], y[:s])
            src[b, k, :ln] = y
    mix = np.zeros((B, N), np.float32)
    for k in range(K):
        mix = (mix + src[:, k]).astype(np.float32)
    return src, mix


def mix_sources(sources, gains):
    """Scale each normalised source by its gain and sum (all float64).

    Returns (scaled_sources (K, N), mixture (N,)).
    """
    s = np.stack([np.asarray(x, np.float64) * float(g) for x, g in zip(sources, gains)])
    return s, s.sum(axis=0)


def gains_2spk_db(rng_u, channel_u, db=5.0):
    """predata_multiAims_dB.py:124-130: 10^(dB/20 * U) on one random channel."""
    rate = 10.0 ** (db / 20.0 * rng_u)
    return [rate, 1.0] if channel_u > 0.5 else [1.0, rate]


def gains_3spk_db(u_large, u_small, db=5.0):
    """predata_multiAims_3dB.py:132-137,192-217: draw k=0 gets the 'normal'
    gain 10^(dB/20*0.5), k=1 'large' 10^(dB/20*(0.5+0.5U)), k=2 'small'
    10^(dB/20*0.5U)."""
    normal = 10.0 ** (db / 20.0 * 0.5)
    large = 10.0 ** (db / 20.0 * (0.5 + 0.5 * u_large))
    small = 10.0 ** (db / 20.0 * (0.5 * u_small))
    return [normal, large, small]


def gains_from_list(dbs):
    """predata_fromList_cRM_123.py:206,227: ratio = 10^(dB_i/20)."""
    return [10.0 ** (d / 20.0) for d in dbs]
