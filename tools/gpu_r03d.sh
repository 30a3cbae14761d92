# round 3: conflict-free LDS layouts of the packed recurrence -- recurrence / step tests, a bench
# line, a kernel trace and the LDS / MFMA counter pass (TAG)
TAG=${TAG:-r03_lds}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_rnn_xw_gpu.py tests/test_step_gpu.py tests/test_robust_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/bench_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/$TAG/pmc_mfma -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/bench_pmc_mfma.log 2>&1
