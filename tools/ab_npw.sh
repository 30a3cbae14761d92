#!/bin/bash
# A/B: BPTT polling waves (BWD_NPW: shipped library vs the npw1 variant), parity tests first
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_npw
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_npw/tests.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_npw/npw2_$rep.log 2>&1 || exit $?
  DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_npw1.so timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_npw/npw1_$rep.log 2>&1 || exit $?
  echo "rep $rep npw2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_npw/npw2_$rep.log) npw1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_npw/npw1_$rep.log)"
done
