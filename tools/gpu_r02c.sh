# gemm_gl in the step: parity / reproducibility tests, then bench with gemm_gl and with the
# round-1 GEMM path (DL4SS_GEMM=lt) on the same box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_gemm_gl_gpu.py tests/test_step_gpu.py tests/test_robust_gpu.py tests/test_configs_full_gpu.py tests/test_drivers_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t3.log 2>&1; [ $? -le 1 ] &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_gl.log 2>&1 &&
DL4SS_GEMM=lt timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_lt.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_gl2.log 2>&1
