#!/bin/bash
# A/B: RNN batch chunk (workgroup count), one bench line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_bc
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
for bc in 1 8; do
  DL4SS_RNN_MIN_BC=$bc timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_bc/bc$bc.log 2>&1 || exit $?
  echo "bc=$bc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bc/bc$bc.log)"
done
