#!/bin/bash
# A/B of library builds: for the in-tree libhftlob.so and each ab/lib_*.so (HFTLOB_LIB), interleaved:
# bench.py (metric, no CPU baseline) and the per-message-kind timing pass of tools/msg_cost.py.
# Usage: tools/ab_libs.sh TAG
set -o pipefail
T=${1:-ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="base $(cd ab && ls lib_*.so | sed 's/\.so$//')"
for r in 1 2; do
  for L in $LIBS; do
    if [ "$L" = base ]; then unset HFTLOB_LIB; else export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2>> $O/bench.err || exit 3
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/mc_${L}_$r -o mc -- python $GRAFT_REPO_ROOT/tools/msg_cost.py > $O/mc_${L}_$r.log 2>&1 ) || exit 4
  done
done
unset HFTLOB_LIB
for L in $LIBS; do
  echo "== $L"; for r in 1 2; do python -c "import json; d=json.load(open('$O/bench_${L}_$r.json')); print(d['value'])"; done
  python tools/msg_cost.py --report $O/mc_${L}_1 | head -8; python tools/msg_cost.py --report $O/mc_${L}_2 | head -8
done > $O/summary.txt 2>&1
