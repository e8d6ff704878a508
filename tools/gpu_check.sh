#!/bin/bash
# One GPU iteration: all -m gpu tests (one pytest process) -> smoke -> bench -> rocprofv3 kernel stats.
# Usage: tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-x}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "${K[@]}" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/stats_bench.json 2> $O/stats.err || exit 4
