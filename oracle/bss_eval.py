"""BSS-eval (SDR / SIR / SAR + permutation) oracle (TEST INFRASTRUCTURE ONLY).

The reference scores separated speech with ``separation.bss_eval_sources``
(``Torch_multi/bss_test.py:5,55``; called per mixture on the ``batch_output/`` wavs,
``bss_test.py:12-61``).  ``separation`` is NOT vendored by the reference and carries no
version: **parity unpinned** against the reference's own copy.
This file restates the published BSS_EVAL v3 algorithm (Vincent, Gribonval, Fevotte 2006;
the form of ``mir_eval.separation.bss_eval_sources``, which has the same call signature and
return tuple ``(sdr, sir, sar, perm)``), computing the projections EXPLICITLY as that
algorithm does -- the HIP path (``dl4ss_amd/bss.py``) uses the closed form of the same
quantities, so the two are independent restatements:

  for every (estimate e, true source j), with time-invariant 512-tap distortion filters:
    s_true   = P_j(e)          projection of e on the delays 0..511 of source j
    e_interf = P_all(e) - s_true   (P_all: on the delays of every source)
    e_artif  = e - P_all(e)
    SDR = 10 log10(|s_true|^2 / |e_interf + e_artif|^2)
    SIR = 10 log10(|s_true|^2 / |e_interf|^2)
    SAR = 10 log10(|s_true + e_interf|^2 / |e_artif|^2)
  perm = the permutation (itertools order) maximising the mean SIR; the returned rows are
  the criteria of (estimate perm[j], source j).
"""
import itertools

import numpy as np
from scipy.linalg import toeplitz
from scipy.signal import fftconvolve

FLEN = 512


def _project(refs, est, flen=FLEN):
    """Least-squares projection of est on the flen delays of every row of refs (explicit
    Gram matrix via FFT correlations, solve, FIR filtering) -> length nsampl + flen - 1."""
    nsrc, nsampl = refs.shape
    refs = np.hstack((refs, np.zeros((nsrc, flen - 1))))
    est = np.hstack((est, np.zeros(flen - 1)))
    n_fft = int(2 ** np.ceil(np.log2(nsampl + flen - 1.0)))
    sf = np.fft.fft(refs, n=n_fft, axis=1)
    sef = np.fft.fft(est, n=n_fft)
    G = np.zeros((nsrc * flen, nsrc * flen))
    for i in range(nsrc):
        for j in range(nsrc):
            ssf = np.real(np.fft.ifft(sf[i] * np.conj(sf[j])))
            ss = toeplitz(np.hstack((ssf[0], ssf[-1:-flen:-1])), r=ssf[:flen])
            G[i * flen:(i + 1) * flen, j * flen:(j + 1) * flen] = ss
            G[j * flen:(j + 1) * flen, i * flen:(i + 1) * flen] = ss.T
    D = np.zeros(nsrc * flen)
    for i in range(nsrc):
        ssef = np.real(np.fft.ifft(sf[i] * np.conj(sef)))
        D[i * flen:(i + 1) * flen] = np.hstack((ssef[0], ssef[-1:-flen:-1]))
    try:
        C = np.linalg.solve(G, D).reshape(flen, nsrc, order="F")
    except np.linalg.LinAlgError:
        C = np.linalg.lstsq(G, D, rcond=None)[0].reshape(flen, nsrc, order="F")
    sproj = np.zeros(nsampl + flen - 1)
    for i in range(nsrc):
        sproj += fftconvolve(C[:, i], refs[i])[:nsampl + flen - 1]
    return sproj


def _safe_db(num, den):
    if den == 0:
        return np.inf
    return 10 * np.log10(num / den)


def decompose(refs, est, j, flen=FLEN):
    nsampl = refs.shape[1]
    s_true = _project(refs[j][None], est, flen)
    p_all = _project(refs, est, flen)
    e_interf = p_all - s_true
    e_artif = -s_true - e_interf
    e_artif[:nsampl] += est
    return s_true, e_interf, e_artif


def criteria(s_true, e_interf, e_artif):
    sdr = _safe_db(np.sum(s_true ** 2), np.sum((e_interf + e_artif) ** 2))
    sir = _safe_db(np.sum(s_true ** 2), np.sum(e_interf ** 2))
    sar = _safe_db(np.sum((s_true + e_interf) ** 2), np.sum(e_artif ** 2))
    return sdr, sir, sar


def bss_eval_sources(reference_sources, estimated_sources, flen=FLEN):
    """(nsrc, nsampl) x2 float64 -> (sdr, sir, sar, perm), each (nsrc,)."""
    refs = np.atleast_2d(np.asarray(reference_sources, dtype=np.float64))
    ests = np.atleast_2d(np.asarray(estimated_sources, dtype=np.float64))
    nsrc = refs.shape[0]
    sdr = np.empty((nsrc, nsrc))
    sir = np.empty((nsrc, nsrc))
    sar = np.empty((nsrc, nsrc))
    for jest in range(nsrc):
        for jtrue in range(nsrc):
            sdr[jest, jtrue], sir[jest, jtrue], sar[jest, jtrue] = criteria(*decompose(refs, ests[jest], jtrue, flen))
    perms = list(itertools.permutations(range(nsrc)))
    dum = np.arange(nsrc)
    mean_sir = np.array([np.mean(sir[list(p), dum]) for p in perms])
    popt = perms[int(np.argmax(mean_sir))]
    idx = (list(popt), dum)
    return sdr[idx], sir[idx], sar[idx], np.asarray(popt)
