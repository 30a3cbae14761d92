R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/side
cd /tmp && export TMPDIR=/tmp
for v in "16,2,1,1" "32,7,1,0" "32,6,1,0"; do
  t=$(echo $v | tr ',' '_')
  DL4SS_SIDE_DWLIN=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/side/$t -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stft-standalone > $R/gpurun_out/side/$t.log 2>&1 || exit 1
done
