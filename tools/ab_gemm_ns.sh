#!/bin/bash
# A/B of the gemm_bb register-ring depth (GBB_NS variants built by tools/variant_lib.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ab_ns
timeout -k 10 120 python -u tools/gemm_bench_bf16.py > gpurun_out/ab_ns/ns3.log 2>&1 || exit $?
for v in ${VARIANTS:-ns4 ns6}; do
  DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_$v.so timeout -k 10 120 python -u tools/gemm_bench_bf16.py > gpurun_out/ab_ns/$v.log 2>&1 || exit $?
done
