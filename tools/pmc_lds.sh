#!/bin/bash
# LDS bank-conflict / MFMA-busy pass (one rocprofv3 --pmc run per variant) of a short bench run,
# from the repo root via gpurun:  VARIANTS="base x" TAG=r04_lds bash tools/pmc_lds.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
BARGS=${BARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset DL4SS_LIB; else export DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_$v.so; fi
  d=$R/gpurun_out/${TAG:-lds}_$v
  mkdir -p $d
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $d -o run -- python3 $R/bench.py $BARGS > $d.log 2>&1 || exit 1
done
