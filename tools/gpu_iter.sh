#!/bin/bash
# One kernel iteration on the GPU box: the -m gpu tests (one pytest process; or -k EXPR, or none
# with NOTEST=1), the driver's bench command twice (20 steps) and the 128-step bench once (no CPU
# baseline), and the rollout phase stamps at 20 and 128 steps when ab/stamps.so exists.
# Usage: tools/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-iter}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest.log 2>&1 || exit 1
fi
for r in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$r.json 2>> $O/bench.err || exit 3
done
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/bench128.json 2>> $O/bench.err || exit 3
python -c "import json; print({n: json.load(open('$O/' + n + '.json'))['value'] for n in ('bench20_1', 'bench20_2', 'bench128')})" > $O/summary.txt
if [ -f ab/stamps.so ]; then
  ST_STEPS=20 timeout -k 10 300 python tools/diag_stamps_rollout.py > $O/stamps20.txt 2> $O/stamps.err || exit 4
  ST_STEPS=128 timeout -k 10 300 python tools/diag_stamps_rollout.py > $O/stamps128.txt 2>> $O/stamps.err || exit 4
fi
