#!/bin/bash
# A/B of library variants on the GPU box (run from the repo root via gpurun):
#   VARIANTS="base e1 e2" ROUNDS=2 BARGS="--steps 20 --warmup 3" bash tools/ab_bench.sh
# "base" is the shipped dl4ss_amd/libdl4ss_hip.so, any other tag dl4ss_amd/libdl4ss_hip_<tag>.so
# (tools/variant_lib.py); a tag "env:NAME=VALUE" runs the shipped library with that environment
# variable set (the engine's DL4SS_* tuning knobs; "env:A=1%B=2" sets several).  Alternates the variants ROUNDS times; one line per run:
# "<tag> <mixtures/s> <ms per step>".  Every run has its own time limit; the first failure ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BARGS=${BARGS:---steps 20 --warmup 3}
for i in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    unset DL4SS_LIB
    envset=""
    case "$v" in
      base) ;;
      env:*) envset="${v#env:}"; envset="${envset//%/ }" ;;  # env:A=1%B=2 sets both
      *) export DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$v.so ;;
    esac
    out=$(env $envset timeout -k 10 ${RUN_TIMEOUT:-150} python -u bench.py $BARGS --no-cpu-baseline --no-stft-standalone 2>/dev/null) || exit 1
    echo "$out" | tail -n 1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],1), round(d['ms_per_step'],4))" || exit 1
  done
done
