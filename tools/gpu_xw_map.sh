# A/B of the fused-projection tile -> wave map (XW_MAP 0: second tiles on the polling waves; 1: on the
# prefetch waves), every layer fused; kernel traces of both
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_xwmap}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_xwmap1.so timeout -k 10 300 python -u -m pytest tests/test_rnn_xw_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests1.log 2>&1 &&
for v in 0 1; do
  L=$R/dl4ss_amd/libdl4ss_hip.so; [ $v = 1 ] && L=$R/dl4ss_amd/libdl4ss_hip_xwmap1.so
  DL4SS_LIB=$L DL4SS_RNN_XW=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_$v.json 2> gpurun_out/$TAG/bench_$v.err || exit 1
  (cd /tmp && DL4SS_LIB=$L DL4SS_RNN_XW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/trace$v.log 2>&1) || exit 1
done
cd $R && timeout -k 10 300 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps.txt 2>&1
