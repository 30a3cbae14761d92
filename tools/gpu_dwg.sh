# grouped weight-gradient launch: bitwise tests, then bench lines per split-factor set
# (DL4SS_DW_SPLITS = dW_lin, dW_ih, dW_hh) and a kernel trace of the default (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_dwg}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_grouped_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
for sp in 2,4,8 2,2,4 2,4,4 1,2,4 2,3,6; do
  DL4SS_DW_SPLITS=$sp timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_$sp.json 2> gpurun_out/$TAG/bench_$sp.err || exit 1
done &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/bench_trace.log 2>&1
