# round 3: the whole GPU suite (GRU dW_hh on gemm_gl with the padded dGh layout, gemm_bb /
# hipBLASLt removed), then bench lines for C2 / C2 --dist / C4 / C5.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03b && export TMPDIR=/tmp &&
DL4SS_PARITY_OUT=gpurun_out/r03b/r03_parity.json timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b/tests.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r03b/bench_c2.json 2> gpurun_out/r03b/bench_c2.err &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --dist --no-cpu-baseline --no-stft-standalone > gpurun_out/r03b/bench_c2_dist.json 2> gpurun_out/r03b/bench_c2_dist.err &&
timeout -k 10 240 python -u bench.py --config C4 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03b/bench_c4.json 2> gpurun_out/r03b/bench_c4.err &&
timeout -k 10 240 python -u bench.py --config C5 --steps 20 --warmup 3 --no-stft-standalone > gpurun_out/r03b/bench_c5.json 2> gpurun_out/r03b/bench_c5.err
