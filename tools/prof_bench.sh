#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run; summaries land in gpurun_out/$1
OUT=${1:-prof}
ARGS=${2:---steps 3 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/$OUT.log 2>&1
