# A/B of the fused input projection on every layer (DL4SS_RNN_XW=1) against the default (first
# layer only): bench lines + a kernel trace of the XW=1 step
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_xw}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_rnn_xw_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_l0.json 2> gpurun_out/$TAG/bench_l0.err &&
DL4SS_RNN_XW=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_all.json 2> gpurun_out/$TAG/bench_all.err &&
cd /tmp &&
DL4SS_RNN_XW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/bench_trace.log 2>&1
