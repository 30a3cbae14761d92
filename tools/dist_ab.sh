#!/bin/bash
# The bench's data-parallel path at world size 1 (bench.py --dist: RCCL process group, buckets) against
# two buckets (DL4SS_DP_BUCKETS=2) and the flat all-reduce (=0); alternating, one line per run "<env> <mixtures/s> <ms>".
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for i in $(seq ${ROUNDS:-2}); do
for v in "DL4SS_DP_BUCKETS=3" "DL4SS_DP_BUCKETS=2" "DL4SS_DP_BUCKETS=0"; do
  out=$(env $v timeout -k 10 150 python -u bench.py --dist --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone 2>/dev/null) || exit 1
  echo "$out" | tail -n 1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],1), round(d['ms_per_step'],4))" || exit 1
done; done
