#!/bin/bash
# One GPU iteration of round 5: the -m gpu suite (one pytest process; PYTEST_K narrows it), the
# smoke, the driver's bench command, then (AB=1) interleaved A/B benches of ab/lib_*.so against
# the in-tree library (tools/ab_quick.sh).  Usage: [PYTEST_K=expr] [AB=1] [ROUNDS=n] tools/gpu_round.sh TAG
set -o pipefail
T=${1:-r05}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$PYTEST_K" ]; then K=(-k "$PYTEST_K"); else K=(); fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest.log 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 3
if [ -n "$AB" ]; then bash tools/ab_quick.sh $T/ab || exit 4; fi
