"""Seeded synthetic speech-shaped sources -- the stand-in for WSJ0 wavs.

There is no WSJ0 (and no network) in this environment, so every workload uses
synthetic sources with the reference's shapes: 8 kHz, MAX_LEN samples, K speakers
per mixture drawn from ``range(num_labels)``.  Each source is a harmonic stack
(f0 ~ U[85, 255] Hz, 20 partials with 1/k amplitudes, slow f0 drift), a 4 Hz
syllabic AM envelope with random silent gaps, plus -30 dB white noise.  numpy
``PCG64`` seeded with ``seed + 1000 * rank``.
"""
import numpy as np

FRAME_RATE = 8000


def speech_like(rng, n, fs=FRAME_RATE):
    t = np.arange(n, dtype=np.float64) / fs
    f0 = rng.uniform(85.0, 255.0)
    drift = 1.0 + 0.05 * np.sin(2 * np.pi * rng.uniform(0.2, 1.0) * t + rng.uniform(0, 2 * np.pi))
    phase = 2 * np.pi * f0 * np.cumsum(drift) / fs
    x = np.zeros(n)
    for k in range(1, 21):
        if k * f0 >= fs / 2:
            break
        x += np.sin(k * phase + rng.uniform(0, 2 * np.pi)) / k
    env = 0.5 * (1.0 + np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi)))
    # random silent gaps (~15 % of the signal)
    n_gaps = rng.integers(1, 4)
    for _ in range(n_gaps):
        g0 = rng.integers(0, n)
        g1 = min(n, g0 + rng.integers(fs // 20, fs // 4))
        env[g0:g1] = 0.0
    x = x * env
    x /= max(np.max(np.abs(x)), 1e-9)
    x += 10 ** (-30 / 20) * rng.standard_normal(n)
    return x


class SyntheticMixtures:
    """Generates raw (un-normalised) source waveforms and speaker ids.

    ``batch(B)`` returns (sources (B, K, N) float64, spk_idx (B, K) int64 sorted
    ascending, gain uniforms (B, 2) float64).  Sources are returned in ascending
    speaker-index order, which is the reference's channel order
    (EvalVer.py:605, 635-638), so label order == identity assignment.
    """

    def __init__(self, n_samples=32000, k=2, num_labels=101, seed=1, rank=0):
        self.n, self.k, self.num_labels = n_samples, k, num_labels
        self.rng = np.random.Generator(np.random.PCG64(seed + 1000 * rank))

    def batch(self, B):
        src = np.empty((B, self.k, self.n))
        spk = np.empty((B, self.k), dtype=np.int64)
        for b in range(B):
            ids = np.sort(self.rng.choice(self.num_labels, size=self.k, replace=False))
            spk[b] = ids
            for k in range(self.k):
                src[b, k] = speech_like(self.rng, self.n) * self.rng.uniform(0.2, 1.0)
        u = self.rng.uniform(size=(B, 2))
        return src, spk, u


def gains_for(u, k, db=5.0):
    """Per-mixture gains (B, K) from uniforms, matching oracle.dsp's gain rules:
    2-spk: 10^(dB/20*u0) on channel 0 if u1 > 0.5 else channel 1
    (predata_multiAims_dB.py:124-130); 3-spk: normal/large/small
    (predata_multiAims_3dB.py:132-137)."""
    u = np.asarray(u, dtype=np.float64)
    B = u.shape[0]
    g = np.ones((B, k))
    if k == 2:
        rate = 10.0 ** (db / 20.0 * u[:, 0])
        ch0 = u[:, 1] > 0.5
        g[ch0, 0] = rate[ch0]
        g[~ch0, 1] = rate[~ch0]
    elif k == 3:
        g[:, 0] = 10.0 ** (db / 20.0 * 0.5)
        g[:, 1] = 10.0 ** (db / 20.0 * (0.5 + 0.5 * u[:, 0]))
        g[:, 2] = 10.0 ** (db / 20.0 * (0.5 * u[:, 1]))
    return g
