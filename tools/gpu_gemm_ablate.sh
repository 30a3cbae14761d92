cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 60 python -u tools/gemm_gl_ablate.py > gpurun_out/abl.log 2>&1 &&
DL4SS_LIB=dl4ss_amd/libdl4ss_hip_no_mfma.so timeout -k 10 60 python -u tools/gemm_gl_ablate.py >> gpurun_out/abl.log 2>&1 &&
DL4SS_LIB=dl4ss_amd/libdl4ss_hip_no_dma.so timeout -k 10 60 python -u tools/gemm_gl_ablate.py >> gpurun_out/abl.log 2>&1
