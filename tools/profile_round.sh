#!/bin/bash
# Round-end measurement on the GPU box: bench (with CPU baseline), rocprofv3
# kernel stats of the same bench command, and FETCH_SIZE / WRITE_SIZE and SQ passes
# (separate, per MI355X_MICROARCH.md).  Usage: [SLICES=G] tools/profile_round.sh TAG
#   SLICES unset: the bench's default launch shape (MARLEnv.default_slices);
#   0: the persistent k_env_rollout launch (the stats run uses 128 warm-up + 128 timed steps, so
#      both launches are 128 steps long; the PMC runs one 128-step launch, warm-up 0, the same
#      launch length, and the traffic passes also one 20-step launch: the driver's bench shape);
#   G >= 1: k_env_step over G env slices (PMC runs: 4 warm-up + 32 steps, one step per launch).
set -o pipefail
T=${1:-r01}
O=$GRAFT_REPO_ROOT/gpurun_out/prof_$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
G=${SLICES:-0}  # the metric's default shape (MARLEnv.default_slices: the persistent launch at 4096 envs)
if [ "$G" = 0 ]; then
  KER=k_env_rollout; STATS_ARGS="--warmup 128 --steps 128"; PMC_ARGS="--warmup 0 --steps 128"; SPL=128; SSPL=128
else
  KER=k_env_step; STATS_ARGS=""; PMC_ARGS="--warmup 4 --steps 32"; SPL=1; SSPL=1
fi
echo "{\"kernel\": \"$KER\", \"slices\": $G, \"steps_per_launch\": $SPL, \"stats_steps_per_launch\": $SSPL, \"commit\": \"${PROF_COMMIT:-}\"}" > $O/shape.json
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 9
timeout -k 10 600 python bench.py --slices $G > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
B="python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --slices $G"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B $STATS_ARGS > $O/stats_bench.json 2> $O/stats.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B $PMC_ARGS > $O/fetch.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B $PMC_ARGS > $O/write.log 2>&1 || exit 4
if [ "$G" = 0 ]; then  # the driver's shape (bench.py --steps 20 --warmup 5): 20-step launches
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats20 -o run -- $B --warmup 20 --steps 20 > $O/stats20_bench.json 2> $O/stats20.err || exit 2
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch20 -o run -- $B --warmup 0 --steps 20 > $O/fetch20.log 2>&1 || exit 3
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write20 -o run -- $B --warmup 0 --steps 20 > $O/write20.log 2>&1 || exit 4
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq20 -o run -- $B --warmup 0 --steps 20 > $O/sq20.log 2>&1 || exit 5
fi
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq -o run -- $B $PMC_ARGS > $O/sq.log 2>&1 || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY --output-format csv -d $O/lds -o run -- $B $PMC_ARGS > $O/lds.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --mode step --no-cpu-baseline > $O/bench_stepmode.json 2> $O/bench_stepmode.err || exit 7
# the driver's command itself (20 steps, CPU baseline included) and the other configs' bench lines
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 10
timeout -k 10 300 python bench.py --envs 512 --no-cpu-baseline > $O/bench_c2_512.json 2> $O/bench_c2.err || exit 11
timeout -k 10 300 python bench.py --config 3_player_fq_fqc_dir --envs 1024 --no-cpu-baseline > $O/bench_c5_1024.json 2> $O/bench_c5.err || exit 12
# phase stamps of the rollout kernel at the driver's launch length (needs ab/stamps.so: make -C jaxmarl-hft_amd/csrc stamps)
if [ -f ab/stamps.so ]; then
  ST_STEPS=20 timeout -k 10 300 python tools/diag_stamps_rollout.py > $O/stamps_rollout20.txt 2> $O/stamps.err || exit 13
  ST_STEPS=128 timeout -k 10 300 python tools/diag_stamps_rollout.py > $O/stamps_rollout128.txt 2>> $O/stamps.err || exit 13
fi
timeout -k 10 200 python tools/diag_host.py > $O/diag_host.txt 2> $O/diag_host.err || exit 14
python $GRAFT_REPO_ROOT/tools/summarize_profiles.py $O > $O/summary.txt 2>&1
