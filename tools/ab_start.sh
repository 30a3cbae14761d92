#!/bin/bash
# same-box A/B of the shipped library against an older build (dl4ss_amd/libdl4ss_hip_$OLD.so, run with $OLD_ENV)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BARGS=${BARGS:---steps 20 --warmup 3}
for i in $(seq ${ROUNDS:-3}); do
  out=$(timeout -k 10 150 python -u bench.py $BARGS --no-cpu-baseline --no-stft-standalone 2>/dev/null) || exit 1
  echo "$out" | tail -n 1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('head', round(d['value'],1), round(d['ms_per_step'],4))" || exit 1
  out=$(env DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$OLD.so $OLD_ENV timeout -k 10 150 python -u bench.py $BARGS --no-cpu-baseline --no-stft-standalone 2>/dev/null) || exit 1
  echo "$out" | tail -n 1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$OLD', round(d['value'],1), round(d['ms_per_step'],4))" || exit 1
done
