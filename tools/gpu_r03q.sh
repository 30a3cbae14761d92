# round 3: BPTT dG stores after B1 (BWD_DG_LATE=1, shipped lib) vs after the publish
# (libdl4ss_hip_dg0.so): recurrence / step / fixture / config tests, bench A/B (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_dglate}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_rnn_xw_gpu.py tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py tests/test_robust_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
for v in base dg0 base2; do
  lib=$R/dl4ss_amd/libdl4ss_hip_$v.so; case $v in base*) lib=$R/dl4ss_amd/libdl4ss_hip.so;; esac
  DL4SS_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_$v.json 2> gpurun_out/$TAG/bench_$v.err || exit 1
done
