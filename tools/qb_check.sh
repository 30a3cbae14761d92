R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qb
cd $R && timeout -k 10 300 python -u -m pytest tests/test_ref_fixtures_gpu.py tests/test_step_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/qb/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/qb/stamps.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qb/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/qb/trace.log 2>&1
