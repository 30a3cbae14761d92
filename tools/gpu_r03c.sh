# round 3: GRU bitwise reproducibility, then bench lines for C2 --dist / C4 / C5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03c && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -k "bitwise" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c/tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --dist --no-cpu-baseline --no-stft-standalone > gpurun_out/r03c/bench_c2_dist.json 2> gpurun_out/r03c/bench_c2_dist.err &&
timeout -k 10 240 python -u bench.py --config C4 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03c/bench_c4.json 2> gpurun_out/r03c/bench_c4.err &&
timeout -k 10 240 python -u bench.py --config C5 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03c/bench_c5.json 2> gpurun_out/r03c/bench_c5.err
