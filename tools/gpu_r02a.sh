# round-2 GPU check: recurrence robustness + step parity tests, per-phase stamps, bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest tests/test_robust_gpu.py tests/test_step_gpu.py tests/test_configs_full_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1; [ $? -le 1 ] &&
timeout -k 10 120 python -u tools/rnn_stamps.py --bf16 > gpurun_out/stamps.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
