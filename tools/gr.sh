#!/bin/bash
# Local helper: clear gpurun_out/run, then run "$@" on the GPU box via gpurun with
# outputs expected under gpurun_out/run/ (so stale files never look like results).
rm -rf /root/repo/gpurun_out/run && mkdir -p /root/repo/gpurun_out/run
T=${GR_TIMEOUT:-600}
/usr/local/graft/bin/gpurun --timeout $T -- "mkdir -p gpurun_out/run && $*"
rc=$?
python3 -c "
import json;d=json.load(open('/root/repo/gpurun_out/.last_call.json'));print('[gr]', d['status'], 'rc', d['rc'], 'run_s', d.get('run_s'), d['msg'][:200])"
exit $rc
