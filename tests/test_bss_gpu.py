"""GPU BSS-eval (replaces separation.bss_eval_sources of Torch_multi/bss_test.py)
vs the explicit BSS_EVAL v3 restatement (oracle/bss_eval.py).  Parity against the reference's
own un-vendored `separation` copy is unpinned.  Bars: permutation identical,
SDR / SIR / SAR within 1e-3 dB (both fp64; the HIP path uses the closed form)."""
import os

import numpy as np
import pytest
import torch

from dl4ss_amd import bss
from oracle import bss_eval as be

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _case(rng, N, swap):
    s = rng.standard_normal((2, N)).astype(np.float32) * np.array([[1.0], [0.5]], dtype=np.float32)
    h = rng.standard_normal(40).astype(np.float32) * 0.2
    h[0] = 1.0
    e0 = np.convolve(s[0], h)[:N] + 0.3 * s[1] + 0.05 * rng.standard_normal(N)
    e1 = 0.9 * s[1] + 0.2 * np.roll(s[0], 700) + 0.1 * rng.standard_normal(N)
    est = np.stack([e1, e0] if swap else [e0, e1]).astype(np.float32)
    return s, est


def test_bss_eval_matches_oracle(dev):
    rng = np.random.default_rng(1)
    N = 6000
    cases = [_case(rng, N, swap) for swap in (False, True, False)]
    refs = torch.from_numpy(np.stack([c[0] for c in cases])).to(dev)
    ests = torch.from_numpy(np.stack([c[1] for c in cases])).to(dev)
    sdr, sir, sar, perm = bss.bss_eval_sources(refs, ests)
    for m, (s, e) in enumerate(cases):
        r = be.bss_eval_sources(s.astype(np.float64), e.astype(np.float64))
        assert perm[m].tolist() == r[3].tolist()
        for ours, ref in zip((sdr[m], sir[m], sar[m]), r[:3]):
            assert np.abs(ours - ref).max() < 1e-3, (m, ours, ref)
    assert perm[1].tolist() == [1, 0]


def test_bss_corr_kernel_direct(dev):
    """R[m][a][b][l] = sum_n x_a[n] x_b[n+l] against numpy (ragged N, L not a multiple of 64)."""
    from dl4ss_amd import _lib
    rng = np.random.default_rng(2)
    M, P, N, L = 2, 3, 2500, 100
    x = rng.standard_normal((M, P, N)).astype(np.float32)
    xd = torch.from_numpy(x).to(dev)
    R = torch.empty(M, P, P, L, dtype=torch.float64, device=dev)
    _lib.call("dl4ss_bss_corr", _lib.ptr(xd), M, P, N, L, _lib.ptr(R), _lib.stream_ptr())
    torch.cuda.synchronize()
    xx = x.astype(np.float64)
    ref = np.zeros((M, P, P, L))
    for m in range(M):
        for a in range(P):
            for b in range(P):
                for l in range(L):
                    ref[m, a, b, l] = np.dot(xx[m, a, :N - l], xx[m, b, l:])
    assert np.abs(R.cpu().numpy() - ref).max() < 1e-9 * np.abs(ref).max()


def test_compat_cal_batch_output(dev, tmp_path):
    """bss_test.cal over a batch_output/ directory written by write_batch_output (PCM16)."""
    from dl4ss_amd.compat import bss_test
    rng = np.random.default_rng(3)
    N = 5000
    s, e = _case(rng, N, False)
    s, e = s / (2 * np.abs(s).max()), e / (2 * np.abs(e).max())
    names = [["spkA", "spkB"]]
    clean = [{"spkA": s[0], "spkB": s[1]}]
    bss_test.write_batch_output(str(tmp_path), e[None], names, mix_wav=(s[0] + s[1])[None], clean=clean)
    got = bss_test.cal(str(tmp_path), 2)
    rd = lambda n: bss_test._read_wav(os.path.join(str(tmp_path), n))  # noqa: E731
    refs = np.stack([rd("0_spkA_realTrue.wav"), rd("0_spkB_realTrue.wav")])
    ests = np.stack([rd("0_spkA_pre.wav"), rd("0_spkB_pre.wav")])
    r = be.bss_eval_sources(refs, ests)
    assert got.shape == (2,)
    assert np.abs(got - r[0]).max() < 1e-3
