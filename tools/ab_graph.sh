R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/g5
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -k "graph" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g5/test.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stft-standalone > gpurun_out/g5/graph.log 2>&1 &&
timeout -k 10 200 python -u bench.py --eager --no-cpu-baseline --no-stft-standalone > gpurun_out/g5/eager.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stft-standalone > gpurun_out/g5/graph2.log 2>&1
