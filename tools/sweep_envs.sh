#!/bin/bash
# Launch shape vs batch size (MARLEnv.default_slices): bench.py at 512..16384 envs per GPU with
# slices 0 (one persistent launch), 1 and 2.  Usage: tools/sweep_envs.sh TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-envs}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for E in 512 2048 4096 8192 16384; do for G in 0 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs $E --slices $G > $O/e${E}_G$G.json 2>> $O/err.log || exit 4
done; done
for E in 512 2048 4096 8192 16384; do
  echo "envs=$E $(for G in 0 1 2; do python -c "import json; print('G$G', round(json.load(open('$O/e${E}_G$G.json'))['value'] / 1e6, 2))"; done | tr '\n' ' ')"
done > $O/summary.txt
