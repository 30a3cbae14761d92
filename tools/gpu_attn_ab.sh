# attention: the bf16-V kernel (attn_vb_kernel) vs the round-2 kernel (ATTN_V1 variant library):
# step / fixture / PIT tests, isolated timings, bench lines
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_attn_ab}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py tests/test_library_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn_new.json 2>&1 &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_attnv1.so timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn_old.json 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_new.json 2> gpurun_out/$TAG/bench_new.err &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_attnv1.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_old.json 2> gpurun_out/$TAG/bench_old.err
