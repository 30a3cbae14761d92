#!/bin/bash
# A/B of the standalone STFT (tools/stft_bench.py) between dl4ss_amd/libdl4ss_hip_old.so and
# the in-tree library, alternated twice; run from the repo root on the GPU box
for i in 1 2; do
  DL4SS_LIB=$PWD/dl4ss_amd/libdl4ss_hip_old.so timeout -k 10 100 python -u tools/stft_bench.py > gpurun_out/run/old$i.log 2>&1 &&
  timeout -k 10 100 python -u tools/stft_bench.py > gpurun_out/run/new$i.log 2>&1 || exit 1
done
