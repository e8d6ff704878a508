#!/bin/bash
# SQ instruction counters of the metric kernel (one 20-step k_env_rollout launch, 4096 envs) for the
# in-tree library ("base") and every ab/lib_*.so (HFTLOB_LIB): per wave and env-step, so a timing
# build's extra work reads as an instruction count.  Usage: tools/pmc_ab.sh TAG
set -o pipefail
T=${1:-pmcab}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LIBS="base $(cd $GRAFT_REPO_ROOT/ab && ls lib_*.so 2>/dev/null | sed 's/\.so$//')"
for L in $LIBS; do
  if [ "$L" = base ]; then unset HFTLOB_LIB; else export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 0 --settle-ms 0 > $O/$L.log 2>&1 || exit 3
done
unset HFTLOB_LIB
python3 - "$O" $LIBS <<'PY' > $O/summary.txt 2>&1
import csv, glob, os, sys
O, libs = sys.argv[1], sys.argv[2:]
for L in libs:
    f = glob.glob(os.path.join(O, L, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for r in csv.DictReader(open(f[0])):
        if "k_env_rollout" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    w = sum(vals["SQ_WAVES"]) / len(vals["SQ_WAVES"])
    print(f"{L:14s}", " ".join(f"{k.replace('SQ_', '')} {sum(v) / len(v) / w / 20:8.0f}" for k, v in sorted(vals.items()) if k != "SQ_WAVES"))
PY
