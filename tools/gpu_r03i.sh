# round 3: the other BASELINE configurations (C1 / C3 / C4 / C5) on the current tree (TAG)
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03_configs}
cd $R && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp &&
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/$TAG/configs.jsonl 2> gpurun_out/$TAG/configs.err
