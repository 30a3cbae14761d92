#!/bin/bash
# variant library $V: bitwise against the shipped library on C2 training steps, then an A/B bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/$TAG/base.json > gpurun_out/$TAG/bw.log 2>&1 &&
DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$V.so timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/$TAG/var.json >> gpurun_out/$TAG/bw.log 2>&1 &&
python -u tools/lib_bitwise.py --compare gpurun_out/$TAG/base.json gpurun_out/$TAG/var.json >> gpurun_out/$TAG/bw.log 2>&1 &&
for c in ${EXTRA_CFGS:-}; do
  LIB_BW_CFG=$c timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/$TAG/base_$c.json >> gpurun_out/$TAG/bw.log 2>&1 &&
  LIB_BW_CFG=$c DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$V.so timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/$TAG/var_$c.json >> gpurun_out/$TAG/bw.log 2>&1 &&
  python -u tools/lib_bitwise.py --compare gpurun_out/$TAG/base_$c.json gpurun_out/$TAG/var_$c.json >> gpurun_out/$TAG/bw.log 2>&1 || exit 1
done &&
VARIANTS="base $V" ROUNDS=${ROUNDS:-3} bash tools/ab_bench.sh > gpurun_out/$TAG/ab.txt 2>&1
