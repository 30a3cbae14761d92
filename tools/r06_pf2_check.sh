#!/bin/bash
# round 6: the BPTT prefetch two steps ahead (BWD_PF2) -- recurrence tests, bitwise against the one-step
# variant $V on C2 and on smaller-chunk configurations, kernel traces of both on one box
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${V:-pf1}
cd $R && mkdir -p gpurun_out/pf2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/pf2/pytest.log 2>&1 &&
for c in 32,lstm,4 4,gru,2 8,lstm,2 2,lstm,2; do
  LIB_BW_CFG=$c timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/pf2/head_$c.json >> gpurun_out/pf2/bw.log 2>&1 &&
  LIB_BW_CFG=$c DL4SS_LIB=dl4ss_amd/libdl4ss_hip_$V.so timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/pf2/var_$c.json >> gpurun_out/pf2/bw.log 2>&1 &&
  python -u tools/lib_bitwise.py --compare gpurun_out/pf2/head_$c.json gpurun_out/pf2/var_$c.json >> gpurun_out/pf2/bw.log 2>&1 || exit 1
done &&
TAG=pf2 VARS="head $V head_b ${V}_b" bash tools/trace_multi.sh
