# fused forward input projection: bitwise tests, step / fixture tests, then bench + per-kernel stats with and without it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/xw && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_rnn_xw_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xw/t_xw.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_kernels_gpu.py tests/test_robust_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xw/t_step.log 2>&1 &&
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-stft-standalone" &&
for v in l0 1 0; do
  DL4SS_RNN_XW=$v timeout -k 10 200 python -u bench.py $BA > gpurun_out/xw/b$v.log 2>&1 || exit $?
  DL4SS_RNN_XW=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/xw/p$v -o run -- python3 bench.py $BA > gpurun_out/xw/p$v.log 2>&1 || exit $?
  echo "xw=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xw/b$v.log)"
done
