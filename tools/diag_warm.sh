#!/bin/bash
# Does the driver-shape figure (--steps 20 --warmup 5) depend on how long the GPU ran before the
# timed launch?  bench.py with --settle-ms 0 / 25 / 100 (untimed back-to-back steps before the timed
# run), interleaved, 3 rounds; prints value and the HIP-event kernel time.  Usage: tools/diag_warm.sh TAG
set -o pipefail
T=${1:-warm}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for S in 0 25 100; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --settle-ms $S > $O/s${S}_$r.json 2>> $O/bench.err || exit 3
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 128 --warmup 16 --settle-ms $S > $O/l${S}_$r.json 2>> $O/bench.err || exit 3
  done
done
for S in 0 25 100; do
  python - "$O" "$S" <<'PY'
import json, sys
O, S = sys.argv[1], sys.argv[2]
for k, n in (("s", 20), ("l", 128)):
    b = [json.load(open(f"{O}/{k}{S}_{r}.json")) for r in (1, 2, 3)]
    print(f"settle {S:>3} ms, {n:3d} steps: " + "  ".join(f"{x['value'] / 1e6:.2f} M ({x['roofline']['kernel_ms']:.4f} ms/step, "
          f"{x['clock_settle']['steps']} settle steps)" for x in b))
PY
done > $O/summary.txt 2>&1
