#!/bin/bash
# A/B: RNN batch chunk (workgroup count) x weight-gradient side-stream overlap, one bench line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_bc
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
for cfg in "1 0" "8 0" "8 1" "1 1"; do
  set -- $cfg
  DL4SS_RNN_MIN_BC=$1 DL4SS_OVERLAP=$2 timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_bc/bc$1_ov$2.log 2>&1 || exit $?
  echo "bc=$1 ov=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bc/bc$1_ov$2.log)"
done
