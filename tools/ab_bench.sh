#!/bin/bash
# On the GPU box: bench.py for every ab/* variant, REPS rounds interleaved (noise check).
# Usage: tools/ab_bench.sh TAG [REPS]
set -o pipefail
T=${1:-x}
REPS=${2:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for d in ab/*/; do
    n=$(basename $d)
    HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$n/libhftlob.so timeout -k 10 200 python bench.py --no-cpu-baseline \
      > gpurun_out/abb_${T}_${n}_$r.json 2> gpurun_out/abb_${T}_${n}_$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abb_${T}_${n}_$r.json'));print('$n', $r, d['value'], d['roofline']['kernel_ms'])"
  done
done
