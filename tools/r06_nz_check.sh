#!/bin/bash
# round 6: the BPTT's slab count as a kernel template argument -- slab tests, bitwise against the
# session-start library (dH slabs off there), kernel traces of head / head without slabs / the nz1 variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/nz
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bptt_slabs_gpu.py > gpurun_out/nz/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/nz/head.json > gpurun_out/nz/bw.log 2>&1 &&
DL4SS_DH_SLABS=0 timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/nz/head_ns.json >> gpurun_out/nz/bw.log 2>&1 &&
DL4SS_DH_SLABS=0 DL4SS_LIB=dl4ss_amd/libdl4ss_hip_start.so timeout -k 10 200 python -u tools/lib_bitwise.py gpurun_out/nz/start.json >> gpurun_out/nz/bw.log 2>&1 &&
python -u tools/lib_bitwise.py --compare gpurun_out/nz/head.json gpurun_out/nz/head_ns.json >> gpurun_out/nz/bw.log 2>&1 &&
python -u tools/lib_bitwise.py --compare gpurun_out/nz/head.json gpurun_out/nz/start.json >> gpurun_out/nz/bw.log 2>&1 &&
TAG=nz VARS="head head_ns:DL4SS_DH_SLABS=0 nz1:DL4SS_DH_SLABS=0 start:DL4SS_DH_SLABS=0 head_b" bash tools/trace_multi.sh
