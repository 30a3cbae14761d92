#!/bin/bash
# Round-6 change check on the GPU box: the whole GPU suite, an A/B bench of VARIANTS, one kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
VARIANTS="$VARIANTS" ROUNDS=${ROUNDS:-3} bash tools/ab_bench.sh > gpurun_out/$TAG/ab.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/trace.log 2>&1
