# gemm_gl: parity tests, then the step-shape timing (beside torch's bf16 matmul)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_gl_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ggl_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/gemm_gl_bench.py $GGL_ARGS > gpurun_out/ggl_bench.log 2>&1
