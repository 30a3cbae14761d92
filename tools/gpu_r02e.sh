# BPTT 20-bit partials: recurrence stamps vs the previous build, then the recurrence / step / fixture tests and the bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 120 python -u tools/rnn_stamps.py --bf16 > gpurun_out/stamps.log 2>&1 &&
RNN_TAG=_old timeout -k 10 120 python -u tools/rnn_stamps.py --bf16 > gpurun_out/stamps_old.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_robust_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t5.log 2>&1; [ $? -le 1 ] &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
