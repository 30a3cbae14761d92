#!/bin/bash
# loss / bias / query small-kernel check: their parity tests, then a kernel trace of the step
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_ref_fixtures_gpu.py tests/test_step_gpu.py tests/test_kernels_gpu.py tests/test_attn_gpu.py tests/test_configs_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/trace.log 2>&1
