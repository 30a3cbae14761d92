# round 3, first GPU pass: the new parity tests (K=3 PIT at full C4, C3 hazard, reference
# checkpoint files through the HIP step), the DP status guard, then bench lines for C2 / C4 / C5
# and the --dist (RCCL world 1) path.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03a && export TMPDIR=/tmp &&
DL4SS_PARITY_OUT=gpurun_out/r03a/r03_parity.json timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider -x \
  tests/test_robust_gpu.py tests/test_checkpoint_gpu.py \
  "tests/test_ref_fixtures_gpu.py::test_hip_pit_equals_reference_label_order_when_identity_is_optimal" \
  "tests/test_step_gpu.py::test_step_c4_pit_3spk_gradients" \
  "tests/test_step_gpu.py::test_step_c4_full_size_pit_3spk_indices" \
  "tests/test_step_gpu.py::test_step_c2_full_size_pit_indices" \
  "tests/test_step_gpu.py::test_graph_step_matches_eager" \
  "tests/test_step_gpu.py::test_step_bitwise_reproducible" \
  "tests/test_configs_full_gpu.py::test_c3_first_non_finite_step_matches_oracle" "tests/test_configs_full_gpu.py::test_c3_finite_window_matches_oracle" > gpurun_out/r03a/tests.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r03a/bench_c2.json 2> gpurun_out/r03a/bench_c2.err &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --dist --no-cpu-baseline --no-stft-standalone > gpurun_out/r03a/bench_c2_dist.json 2> gpurun_out/r03a/bench_c2_dist.err &&
timeout -k 10 240 python -u bench.py --config C4 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03a/bench_c4.json 2> gpurun_out/r03a/bench_c4.err &&
timeout -k 10 240 python -u bench.py --config C5 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03a/bench_c5.json 2> gpurun_out/r03a/bench_c5.err
