# round 3: hand-counted forward polling sweeps (FWD_ASM_POLL) and two memory-queue placements
# (BWD_PF_LATE: BPTT operand loads after B1; FWD_XDMA_EARLY: the forward's projection-row DMA of
# the matvec-less wave before B2): recurrence / step / fixture / config tests, bench A/B against
# variant libraries (libdl4ss_hip_<v>.so), stamps of each (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_pfmap}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_rnn_xw_gpu.py tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py tests/test_robust_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
for v in base cm pe base2; do
  lib=$R/dl4ss_amd/libdl4ss_hip_$v.so; case $v in base*) lib=$R/dl4ss_amd/libdl4ss_hip.so;; esac
  DL4SS_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_$v.json 2> gpurun_out/$TAG/bench_$v.err || exit 1
done &&
for v in "" _cm; do
  RNN_TAG=$v timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps$v.txt 2>&1 || exit 1
done
