#!/bin/bash
# Run one pytest selection against the in-tree library and each ab/lib_*.so (HFTLOB_LIB).
# Usage: tools/gpu_bisect.sh TAG "pytest -k expr"
set -o pipefail
T=${1:-bisect}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$2" > $O/base.log 2>&1
for L in $(cd ab && ls lib_*.so | sed 's/\.so$//'); do
  HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$2" > $O/$L.log 2>&1
done
for f in $O/*.log; do echo "$(basename $f) $(tail -n 1 $f)"; done > $O/summary.txt
