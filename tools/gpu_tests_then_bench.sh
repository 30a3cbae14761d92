#!/bin/bash
# GPU session helper: parity tests, then (only if pytest did not crash) a short bench.
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
exit $rc
