# custom-op layer + the modular (autograd.Function) paths it shares code with
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest tests/test_library_gpu.py tests/test_compat_gpu.py tests/test_drivers_gpu.py tests/test_kernels_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lib_tests.log 2>&1
