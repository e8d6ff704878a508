#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -k "rollout_sampled" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for s in 0 2 0 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --slices $s >> $O/bench.json 2>> $O/bench.err || exit 3; done
timeout -k 10 300 python bench.py --no-cpu-baseline --slices 0 --steps 20 --warmup 5 >> $O/bench.json 2>> $O/bench.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --slices 0 > $O/stats_bench.json 2> $O/stats.err || exit 4
