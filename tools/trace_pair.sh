#!/bin/bash
# kernel traces of the shipped library and of dl4ss_amd/libdl4ss_hip_$OLD.so ($OLD_ENV) on the same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/head -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/head.log 2>&1 &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_$OLD.so DL4SS_DH_SLABS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/old -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/old.log 2>&1
