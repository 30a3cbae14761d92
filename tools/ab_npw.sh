#!/bin/bash
# A/B: polling waves of the BiRNN kernels: shipped library (BWD_NPW, FWD_NPW defaults) vs the
# variants named in VARIANTS (tools/variant_lib.py builds), parity tests of the shipped one first
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_npw
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_npw/tests.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_npw/main_$rep.log 2>&1 || exit $?
  line="rep $rep main $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_npw/main_$rep.log)"
  for v in ${VARIANTS:-}; do
    DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_$v.so timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_npw/${v}_$rep.log 2>&1 || exit $?
    line="$line $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_npw/${v}_$rep.log)"
  done
  echo "$line"
done
