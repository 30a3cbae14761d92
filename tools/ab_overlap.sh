# A/B: weight-gradient GEMMs on a side stream beside the BPTT (DL4SS_OVERLAP), with and without
# the recurrence waves at s_setprio 3 (RNN_PRIO variant library); eager step (the side stream is
# not captured), two rounds each, one bench line per run
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && : > gpurun_out/ab_overlap.log &&
for r in 1 2; do
  for v in base:0 base:1 prio:0 prio:1; do
    lib=dl4ss_amd/libdl4ss_hip.so; [ ${v%%:*} = prio ] && lib=dl4ss_amd/libdl4ss_hip_prio.so
    echo "== $v round $r" >> gpurun_out/ab_overlap.log
    DL4SS_LIB=$lib DL4SS_OVERLAP=${v##*:} timeout -k 10 150 python -u bench.py --eager --no-cpu-baseline --no-stft-standalone --steps 20 --warmup 3 >> gpurun_out/ab_overlap.log 2>&1 || exit 1
  done
done
