#!/bin/bash
# other configurations (tools/bench_configs.py) with the shipped library and variant $V, alternating
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/cfgab
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_configs.py c1 c3 c4 --precision bf16 > gpurun_out/cfgab/head_$i.jsonl 2> gpurun_out/cfgab/err.log || exit 1
  DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$V.so timeout -k 10 300 python -u tools/bench_configs.py c1 c3 c4 --precision bf16 > gpurun_out/cfgab/${V}_$i.jsonl 2>> gpurun_out/cfgab/err.log || exit 1
done
