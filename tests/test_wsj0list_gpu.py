"""List-file batches through the GPU mixing (per-source lengths) + STFT kernels vs the oracle
restatement of predata_fromList_cRM_123.py:186-255 (normalise over the wav's own length,
zero-pad, gain 10^(dB/20), sum, STFT).  Bars: sources / mixture 1e-6 abs (fp32 vs fp64 of
values in [-1.2, 1.2]), magnitudes 1e-4 relative to the spectrum maximum."""
import numpy as np
import pytest
import torch

from dl4ss_amd import wsj0list as wl
from oracle import dsp

from test_wsj0list_cpu import _dataset

pytestmark = pytest.mark.gpu


def test_list_features_match_oracle(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lst, data, _ = _dataset(tmp_path)
    N = 10000
    (b,) = list(wl.ListBatches(lst, data, "train", batch=2, max_len=N))
    out = wl.features(b, torch.device("cuda", 0))
    torch.cuda.synchronize()
    for r in range(2):
        srcs = [dsp.normalise_source(b["raw"][r, k, :b["lengths"][r, k]].astype(np.float64), N) for k in range(2)]
        s, m = dsp.mix_sources(srcs, b["gains"][r].astype(np.float64))
        assert np.abs(out["src"][r].cpu().numpy() - np.stack(s)).max() < 1e-6
        assert np.abs(out["mix"][r].cpu().numpy() - m).max() < 1e-6
        ref = dsp.magnitude(m)
        assert np.abs(out["mix_mag"][r].cpu().numpy() - ref).max() < 1e-4 * ref.max()
        for k in range(2):
            refk = dsp.magnitude(s[k])
            assert np.abs(out["src_spec"][r, k].cpu().numpy() - refk).max() < 1e-4 * refk.max()
