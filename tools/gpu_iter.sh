#!/bin/bash
# One kernel iteration on the GPU: the engine + env parity tests (one pytest process), then the
# metric bench at both launch shapes (2 slices, persistent), twice each.  Usage: tools/gpu_iter.sh TAG [pytest -k expr] (default: every -m gpu test)
set -o pipefail
T=${1:-it}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do for G in 2 0; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --slices $G > $O/bench_G${G}_$r.json 2>> $O/bench.err || exit 3
done; done
for G in 2 0; do
  echo "slices=$G: $(for r in 1 2; do python -c "import json; print(json.load(open('$O/bench_G${G}_$r.json'))['value'])"; done | tr '\n' ' ')"
done > $O/summary.txt 2>&1
