#!/bin/bash
# A/B of library builds at both launch shapes: for the in-tree libhftlob.so and each ab/lib_*.so
# (HFTLOB_LIB), interleaved twice: bench.py --slices 2 (the default) and --slices 0 (persistent).
# Optional: the phase-stamp / in-kernel-clock diagnostic when ab/stamps.so exists.
# Usage: tools/ab_slices.sh TAG
set -o pipefail
T=${1:-abs}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
LIBS="base $(cd ab && ls lib_*.so 2>/dev/null | sed 's/\.so$//')"
for r in 1 2; do
  for L in $LIBS; do
    if [ "$L" = base ]; then unset HFTLOB_LIB; else export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so; fi
    for G in 2 0; do
      timeout -k 10 120 python bench.py --no-cpu-baseline --slices $G > $O/bench_${L}_G${G}_$r.json 2>> $O/bench.err || exit 3
    done
  done
done
unset HFTLOB_LIB
for L in $LIBS; do for G in 2 0; do
  echo "$L slices=$G: $(for r in 1 2; do python -c "import json; print(json.load(open('$O/bench_${L}_G${G}_$r.json'))['value'])"; done | tr '\n' ' ')"
done; done > $O/summary.txt 2>&1
if [ -f ab/stamps.so ]; then
  HFTLOB_STAMPS_LIB=$GRAFT_REPO_ROOT/ab/stamps.so timeout -k 10 300 python tools/diag_stamps.py > $O/stamps.txt 2>&1 || exit 4
fi
