# step tests with gemm_gl everywhere, then the profile session r02_prof_b (trace, PMC traffic, MFMA busy)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_robust_gpu.py tests/test_configs_full_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t4.log 2>&1; [ $? -le 1 ] &&
TAG=r02_prof_b bash tools/prof_round.sh
