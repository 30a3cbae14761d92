# round 3: attention GRAD with 16-B dPre stores -- step / fixture / library / edge / config tests,
# isolated attention timings, a bench line, the other BASELINE configurations (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_attn16}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_convert_gpu.py tests/test_attn_gpu.py tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py tests/test_configs_full_gpu.py tests/test_library_gpu.py tests/test_edge_gpu.py tests/test_drivers_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn.json 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/$TAG/configs.jsonl 2> gpurun_out/$TAG/configs.err
