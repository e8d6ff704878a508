#!/bin/bash
# One optimisation iteration on the GPU box: every -m gpu test, per-message-kind costs, bench x2.
# Usage: tools/gpu_iter.sh TAG
set -o pipefail
T=${1:-x}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline >> $O/bench.json 2>> $O/bench.err || exit 3; done
bash tools/msg_cost.sh $T > $O/mc.log 2>&1 || exit 4
