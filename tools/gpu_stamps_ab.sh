# A/B of recurrence variants by per-phase stamps: the shipped form, then each RNN_TAG given
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 120 python -u tools/rnn_stamps.py --bf16 > gpurun_out/stamps.log 2>&1 &&
for t in $TAGS; do RNN_TAG=$t timeout -k 10 120 python -u tools/rnn_stamps.py --bf16 > gpurun_out/stamps$t.log 2>&1 || exit 1; done
