# attention V prefetch: kernel / step / fixture tests, then the profile session (TAG) and its bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_attn.log 2>&1 &&
TAG=${TAG:-r02_prof_c} bash tools/prof_round.sh
