# Full GPU check: every -m gpu test (no -x: the whole list), smoke(), then the default bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/full.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
