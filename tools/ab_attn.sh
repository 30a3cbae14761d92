#!/bin/bash
# A/B: attention rows per block (DL4SS_ATTN_TILES tiles of 256 rows): bench line + per-kernel stats each
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_attn
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone"
export TMPDIR=/tmp
for t in ${TILES:-4 1 2 3}; do
  DL4SS_ATTN_TILES=$t timeout -k 10 200 python -u bench.py $BA > gpurun_out/ab_attn/t$t.log 2>&1 || exit $?
  DL4SS_ATTN_TILES=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_attn/p$t -o run -- python3 bench.py $BA > gpurun_out/ab_attn/p$t.log 2>&1 || exit $?
  echo "tiles=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_attn/t$t.log)"
done
