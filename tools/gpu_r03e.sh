# round 3 profile session: whole GPU suite, bench line, HBM probe, then the rocprofv3 session (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_prof_a}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
DL4SS_PARITY_OUT=gpurun_out/$TAG/r03_parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &&
timeout -k 10 120 ./tools/bw_probe > gpurun_out/$TAG/bw_probe.jsonl 2> gpurun_out/$TAG/bw_probe.err &&
TAG=$TAG bash tools/prof_round.sh
