#!/bin/bash
# SQ counter passes of the metric kernel (one 20-step k_env_rollout launch, 4096 envs, --settle-ms 0)
# for the in-tree library ("base") and every ab/lib_*.so (HFTLOB_LIB), one rocprofv3 run per counter
# set: "inst" (instruction mix, wave cycles), "lds" (LDS bank conflicts / activity), "wait" (issue and
# wait cycles).  Per wave and env-step.  Usage: [SETS="inst lds"] tools/pmc_sets.sh TAG
set -o pipefail
T=${1:-pmcsets}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LIBS="base $(cd $GRAFT_REPO_ROOT/ab && ls lib_*.so 2>/dev/null | sed 's/\.so$//')"
declare -A C
C[inst]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
C[lds]="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
C[wait]="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
for S in ${SETS:-inst lds}; do
  for L in $LIBS; do
    if [ "$L" = base ]; then unset HFTLOB_LIB; else export HFTLOB_LIB=$GRAFT_REPO_ROOT/ab/$L.so; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${C[$S]} --output-format csv -d $O/${S}_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 0 --settle-ms 0 > $O/${S}_$L.log 2>&1 || exit 3
  done
done
unset HFTLOB_LIB
python3 - "$O" "${SETS:-inst lds}" $LIBS <<'PY' > $O/summary.txt 2>&1
import csv, glob, os, sys
O, sets, libs = sys.argv[1], sys.argv[2].split(), sys.argv[3:]
for S in sets:
    print(f"== {S} (per wave and env-step, one 20-step launch)")
    for L in libs:
        f = glob.glob(os.path.join(O, f"{S}_{L}", "**", "*counter_collection.csv"), recursive=True)
        vals = {}
        for r in csv.DictReader(open(f[0])):
            if "k_env_rollout" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        w = sum(vals["SQ_WAVES"]) / len(vals["SQ_WAVES"])
        print(f"{L:14s}", " ".join(f"{k.replace('SQ_', '')} {sum(v) / len(v) / w / 20:8.0f}"
                                   for k, v in sorted(vals.items()) if k != "SQ_WAVES"))
PY
