#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM section) of a short bench
# run for each library variant, from the repo root via gpurun:
#   VARIANTS="base gm8" TAG=r04_pmc bash tools/pmc_traffic.sh
# -> gpurun_out/$TAG_<variant>/pmc_{fetch,write}/run_counter_collection.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}
BARGS=${BARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset DL4SS_LIB; else export DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/${TAG:-pmc}_$v/pmc_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    mkdir -p $(dirname $d)
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py $BARGS > $d.log 2>&1 || exit 1
  done
done
