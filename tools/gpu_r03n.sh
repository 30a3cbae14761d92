# round 3: recurrence stamps of the current tree with the second recorded thread on wave 4
# (default), wave 5 (STAMP_T2=320) and wave 6 (STAMP_T2=384); a bench line (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_stw}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
for v in "" _w5 _w6; do
  RNN_TAG=$v timeout -k 10 200 python -u tools/rnn_stamps.py --bf16 > gpurun_out/$TAG/stamps$v.txt 2>&1 || exit 1
done &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stft-standalone > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
