#!/bin/bash
# Parity first, then speed: every -m gpu test on the in-tree library and on each ab/lib_*.so
# (HFTLOB_LIB), then tools/ab_slices.sh (bench A/B at both launch shapes).  Usage: tools/gpu_ab_tests.sh TAG
set -o pipefail
T=${1:-abt}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_base.log 2>&1 || exit 1
for L in $(cd ab && ls lib_*.so 2>/dev/null | sed 's/\.so$//'); do
  HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$L.log 2>&1 || exit 2
done
bash tools/ab_slices.sh $T
