#!/bin/bash
# One GPU session: parity tests (gpu marker), smoke(), then a default bench run.
# Each GPU step has its own time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
