# round 3: quad-per-row attention (attn_q4_kernel) + grouped weight-gradient GEMM launch --
# their tests and the step tests, attention timings (new vs the ATTN_V1 variant library), a bench
# line and a kernel trace of the step (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_f}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest tests/test_gemm_grouped_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn_new.json 2>&1 &&
DL4SS_ATTN_TILES=2 timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn_new_t2.json 2>&1 &&
DL4SS_ATTN_TILES=4 timeout -k 10 120 python -u tools/attn_bench.py 20 > gpurun_out/$TAG/attn_new_t4.json 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/bench_trace.log 2>&1
