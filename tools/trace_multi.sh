#!/bin/bash
# kernel traces on ONE box of the shipped library and of variant libraries: VARS="tag:ENV=.. tag2 ..."
# (tag "head" = the shipped library; other tags dl4ss_amd/libdl4ss_hip_<tag>.so), into gpurun_out/$TAG/<tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  tag=${v%%:*}; envs=""; [ "$tag" != "$v" ] && envs=${v#*:}
  lib=$R/dl4ss_amd/libdl4ss_hip.so; [ "${tag%%_*}" != head ] && lib=$R/dl4ss_amd/libdl4ss_hip_${tag%%_*}.so
  (export DL4SS_LIB=$lib; for e in ${envs//,/ }; do export "$e"; done
   timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/$tag -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/$TAG/$tag.log 2>&1) || exit 1
  tail -n 1 $R/gpurun_out/$TAG/$tag.log
done
