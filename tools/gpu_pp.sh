# 256x256 ping-pong GEMM: every gemm_gl test (all configs), square calibration, step shapes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_gl_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pp_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/gemm_gl_square.py 1,4,5 > gpurun_out/pp_square.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_gl_bench.py > gpurun_out/pp_shapes.log 2>&1
