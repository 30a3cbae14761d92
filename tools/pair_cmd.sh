TAG=pair OLD=start bash tools/trace_pair.sh && mkdir -p gpurun_out/pair && VARIANTS="base nodpp" ROUNDS=3 bash tools/ab_bench.sh > gpurun_out/pair/ab_nodpp.txt 2>&1
