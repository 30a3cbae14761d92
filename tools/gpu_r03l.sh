# round 3 final profile session: whole GPU suite (incl. the 16-phase time-mean kernel), smoke,
# bench line with the CPU baseline, an A/B bench line with the dH GEMM unsplit
# (DL4SS_DH_SPLIT=1), then the rocprofv3 session (kernel trace, FETCH / WRITE, MFMA / LDS) and
# the recurrence stamps (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_prof_c}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
DL4SS_PARITY_OUT=gpurun_out/$TAG/r03_parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
DL4SS_DH_SPLIT=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench_dh1.json 2> gpurun_out/$TAG/bench_dh1.err &&
TAG=$TAG bash tools/prof_round.sh &&
cd $R && timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps.txt 2>&1
