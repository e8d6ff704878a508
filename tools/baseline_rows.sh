#!/bin/bash
# BASELINE.md §3 rows besides the metric line, on the current kernel.  Usage: tools/baseline_rows.sh TAG
#   C1: mm_debug_fixed_quant at 1 env (HIP, and the C restatement as the line's cpu_baseline);
#   C3 variants: mid 28 M (the f32 rounding regime), 640 steps (10 episodes), step mode;
#   launch shapes at 512 / 8192 / 16384 envs (persistent and 2 slices);
#   C5 at 1024 envs; the IPPO learner's update timing (tools/train_timing.py --graph).  Each line goes to its own JSON file under gpurun_out/rows_TAG.
set -o pipefail
T=${1:-rows}
O=$GRAFT_REPO_ROOT/gpurun_out/rows_$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
B="timeout -k 10 300 python bench.py"
$B --config mm_debug_fixed_quant --envs 1 > $O/c1_1env.json 2> $O/err.log || exit 1
$B --no-cpu-baseline --mid 28000000 > $O/c3_mid28m.json 2>> $O/err.log || exit 2
$B --no-cpu-baseline --steps 640 > $O/c3_640steps.json 2>> $O/err.log || exit 3
$B --no-cpu-baseline --mode step > $O/c3_stepmode.json 2>> $O/err.log || exit 4
for E in 512 8192 16384; do
  for G in 0 2; do
    $B --no-cpu-baseline --envs $E --slices $G > $O/e${E}_G$G.json 2>> $O/err.log || exit 5
  done
done
$B --no-cpu-baseline --config 3_player_fq_fqc_dir --envs 1024 > $O/c5_1024.json 2>> $O/err.log || exit 6
timeout -k 10 400 python tools/train_timing.py --graph > $O/train_timing.txt 2>> $O/err.log || exit 7
echo done > $O/ok
