#!/bin/bash
# A/B of the shipped library vs variant libraries (VARIANTS): parity tests of the shipped one,
# then per variant a bench line and a rocprofv3 --kernel-trace --stats run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_lib
export TMPDIR=/tmp
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_lib/tests.log 2>&1 || exit $?
for v in main ${VARIANTS:-}; do
  L=$R/dl4ss_amd/libdl4ss_hip.so; [ $v != main ] && L=$R/dl4ss_amd/libdl4ss_hip_$v.so
  DL4SS_LIB=$L timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_lib/$v.log 2>&1 || exit $?
  DL4SS_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_lib/p_$v -o run -- python3 bench.py $BA > gpurun_out/ab_lib/p_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_lib/$v.log)"
done
