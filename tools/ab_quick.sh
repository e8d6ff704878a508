#!/bin/bash
# Quick A/B of library builds on the GPU box: the in-tree libhftlob.so ("base") and every
# ab/lib_*.so (HFTLOB_LIB), interleaved, 3 rounds, each the metric bench at the profile shape
# (128 steps) and at the driver's shape (--steps 20 --warmup 5).  Usage: tools/ab_quick.sh TAG
set -o pipefail
T=${1:-abq}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="base $(cd ab && ls lib_*.so 2>/dev/null | sed 's/\.so$//')"
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $LIBS; do
    if [ "$L" = base ]; then unset HFTLOB_LIB; else export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline > $O/b128_${L}_$r.json 2>> $O/bench.err || exit 3
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_${L}_$r.json 2>> $O/bench.err || exit 3
  done
done
unset HFTLOB_LIB
for L in $LIBS; do
  python - "$O" "$L" "${ROUNDS:-3}" <<'PY'
import json, sys
O, L, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
v = lambda k, r: json.load(open(f"{O}/{k}_{L}_{r}.json"))["value"] / 1e6
print(f"{L:16s} 128 steps: " + " ".join(f"{v('b128', r):.2f}" for r in range(1, n + 1)) +
      "   20 steps: " + " ".join(f"{v('b20', r):.2f}" for r in range(1, n + 1)))
PY
done > $O/summary.txt 2>&1
