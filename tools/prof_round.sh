#!/bin/bash
# One profiling session on the GPU box (run from the repo root via gpurun):
#   1. standalone STFT roofline probe (>= 2048 signals)
#   2. rocprofv3 --kernel-trace --stats of a short bench run  -> gpurun_out/$TAG/trace
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes)  -> gpurun_out/$TAG/pmc_{fetch,write}
#   4. an MFMA / LDS pass (MFMA busy, LDS bank conflicts, GRBM_GUI_ACTIVE)  -> gpurun_out/$TAG/pmc_mfma
#      (per launch, with its grid size: bench.py picks the launches of each measured unit)
# Every GPU step has its own time limit; the chain stops at the first failure.
TAG=${TAG:-prof}
BARGS=${BARGS:---steps 3 --warmup 1 --no-cpu-baseline}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/stft_bench.py > $R/gpurun_out/$TAG/stft_bench.json 2> $R/gpurun_out/$TAG/stft_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/$TAG/bench_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/$TAG/pmc_fetch -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/$TAG/bench_pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/pmc_write -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/$TAG/bench_pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/$TAG/pmc_mfma -o run -- python3 $R/bench.py $BARGS > $R/gpurun_out/$TAG/bench_pmc_mfma.log 2>&1
