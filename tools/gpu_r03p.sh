# round 3 final session: whole GPU suite, smoke, bench line (with the CPU baseline), then the
# FWD_SPLIT4=1 variant (libdl4ss_hip_s4.so: forward matvec tile 4 split over the cell waves): its
# recurrence / step tests and an A/B bench line; the rocprofv3 session (kernel trace, FETCH /
# WRITE, MFMA / LDS passes) and the recurrence stamps (shipped; split variant with wave 5) (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_prof_d}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
DL4SS_PARITY_OUT=gpurun_out/$TAG/r03_parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
TAG=$TAG bash tools/prof_round.sh &&
cd $R && timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps.txt 2>&1 &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_s4.so timeout -k 10 600 python -u -m pytest tests/test_rnn_xw_gpu.py tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_ref_fixtures_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests_s4.log 2>&1 &&
DL4SS_LIB=$R/dl4ss_amd/libdl4ss_hip_s4.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_s4.json 2> gpurun_out/$TAG/bench_s4.err &&
RNN_TAG=_w5 timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps_s4_w5.txt 2>&1
