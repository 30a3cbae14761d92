# round 3: forward matvec tile 4 split over the cell waves (FWD_SPLIT4): recurrence / step / fixture /
# config tests, bench A/B against FWD_SPLIT4=0 (libdl4ss_hip_ns.so), stamps (wave 4 and wave 5) (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_split4}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_rnn_xw_gpu.py tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py tests/test_robust_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
for v in base ns base2; do
  lib=$R/dl4ss_amd/libdl4ss_hip_$v.so; case $v in base*) lib=$R/dl4ss_amd/libdl4ss_hip.so;; esac
  DL4SS_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_$v.json 2> gpurun_out/$TAG/bench_$v.err || exit 1
done &&
for v in "" _w5; do
  RNN_TAG=$v timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps$v.txt 2>&1 || exit 1
done
