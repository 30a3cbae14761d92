# attention GRAD pass: isolated timing + counter breakdown (VALU / LDS / VMEM activity, waits,
# occupancy, L2 fetch) -- each counter pass its own run
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_attn}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn.json 2> gpurun_out/$TAG/attn.err &&
cd /tmp &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $R/gpurun_out/$TAG/pmc1 -o run -- python3 $R/tools/attn_bench.py 5 > $R/gpurun_out/$TAG/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/$TAG/pmc2 -o run -- python3 $R/tools/attn_bench.py 5 > $R/gpurun_out/$TAG/pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/$TAG/pmc3 -o run -- python3 $R/tools/attn_bench.py 5 > $R/gpurun_out/$TAG/pmc3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/pmc4 -o run -- python3 $R/tools/attn_bench.py 5 > $R/gpurun_out/$TAG/pmc4.log 2>&1
