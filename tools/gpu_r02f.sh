# STFT 16-B emit: standalone A/B vs the per-frame-store build, then every -m gpu test, smoke() and the bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/run &&
bash tools/ab_stft.sh &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/full.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
