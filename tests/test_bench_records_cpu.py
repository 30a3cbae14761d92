"""The bench line's roofline fields read committed profile records (no GPU): the PMC traffic of
the STFT launch, the MFMA-busy counter of the in-step Linear GEMM and the measured
streaming ceiling must all resolve, so a renamed kernel (rocprofv3 spells template arguments
out) or a missing profile shows up here instead of as a silent null in BENCH_*.json."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_records_resolve():
    traffic = bench.pmc_traffic("stft_fwd_kernel", [bench.stft_grid_threads(4096, 251)])
    assert traffic is not None and 2.0e9 < traffic < 2.4e9  # algorithmic 2.116 GB per launch
    busy = bench.pmc_mfma_busy(bench.GEMM_GL_LINEAR)
    assert busy is not None and 0.0 < busy < 1.0


def test_stream_ceiling_resolves():
    c = bench.stream_ceiling("r1w3")
    assert c is not None and 3000.0 < c < bench.HBM_PEAK_GBS
