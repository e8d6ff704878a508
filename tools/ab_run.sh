#!/bin/bash
# On the GPU box: per-kind costs + bench for every ab/* variant.  Usage: tools/ab_run.sh TAG
set -o pipefail
T=${1:-x}
cd $GRAFT_REPO_ROOT
for d in ab/*/; do
  n=$(basename $d)
  export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$n/libhftlob.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 64 > gpurun_out/ab_${T}_$n.json 2> gpurun_out/ab_${T}_$n.err || exit 1
  tools/msg_cost.sh ${T}_$n || exit 2
done
