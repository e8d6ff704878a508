#!/bin/bash
# Round 5 against round 4, whole stack (host package + kernel), interleaved on one box: the
# working tree's bench and round 4's final tree (ab/r04tree: `git archive 158731f` of bench.py, the
# host package and its library built from that commit), 3 rounds of the profile shape (128 steps)
# and the driver's shape (20 steps).  Usage: tools/ab_round4.sh TAG
set -o pipefail
T=${1:-ab_r04}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
for r in 1 2 3; do
  cd $GRAFT_REPO_ROOT
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/b128_r05_$r.json 2>> $O/err.log || exit 1
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_r05_$r.json 2>> $O/err.log || exit 1
  cd $GRAFT_REPO_ROOT/ab/r04tree
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/b128_r04_$r.json 2>> $O/err.log || exit 2
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_r04_$r.json 2>> $O/err.log || exit 2
done
cd $GRAFT_REPO_ROOT
python - "$O" <<'PY' > $O/summary.txt
import json, sys
O = sys.argv[1]
v = lambda k, t, r: json.load(open(f"{O}/{k}_{t}_{r}.json"))["value"] / 1e6
for t in ("r05", "r04"):
    print(f"{t}  128 steps: " + " ".join(f"{v('b128', t, r):.2f}" for r in (1, 2, 3)) +
          "   20 steps: " + " ".join(f"{v('b20', t, r):.2f}" for r in (1, 2, 3)))
PY
