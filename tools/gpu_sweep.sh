#!/bin/bash
# Speed_test's sweep on the GPU box: the sweep parity tests, then one bench row per
# (agents, n_data_msg) at 4000 envs x 50 steps (Speed_test.py:50-71), with the persistent launch
# (--slices 0, the default at 4000 envs) and with 2 env slices.  Usage: tools/gpu_sweep.sh TAG
set -o pipefail
T=${1:-sweep}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -k "sweep" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for AG in 1,1 5,5 10,10; do
  for D in 100 1; do
    N=400000; [ $D = 100 ] && N=1500000
    for G in 0 2; do
      timeout -k 10 300 python bench.py --config default --agents $AG --n-data-msg $D --n-msgs $N --envs 4000 --steps 50 --warmup 5 --no-cpu-baseline --slices $G >> $O/bench.json 2>> $O/bench.err || exit 3
    done
  done
done
