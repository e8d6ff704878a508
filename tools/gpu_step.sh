#!/bin/bash
# One kernel iteration on the GPU box: every -m gpu test (one pytest process; or -k EXPR), the
# metric bench twice (the default persistent launch, no CPU baseline), and the wave-residency
# diagnostic when ab/wavetime.so exists.  Usage: tools/gpu_step.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-step}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/bench_$r.json 2>> $O/bench.err || exit 3
done
python -c "import json; print([json.load(open('$O/bench_%d.json' % r))['value'] for r in (1, 2)])" > $O/summary.txt
if [ -f ab/wavetime.so ]; then
  timeout -k 10 300 python tools/diag_wavetime.py > $O/wavetime.json 2> $O/wavetime.err || exit 4
fi
