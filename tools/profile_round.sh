#!/bin/bash
# Round-end measurement on the GPU box: bench (with CPU baseline), rocprofv3
# kernel stats of the same bench command, and FETCH_SIZE / WRITE_SIZE passes
# (separate, per MI355X_MICROARCH.md).  Usage: tools/profile_round.sh TAG
set -o pipefail
T=${1:-r01}
O=$GRAFT_REPO_ROOT/gpurun_out/prof_$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 9
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/stats_bench.json 2> $O/stats.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/fetch.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/write.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/sq.log 2>&1 || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY --output-format csv -d $O/lds -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/lds.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --mode step --no-cpu-baseline > $O/bench_stepmode.json 2> $O/bench_stepmode.err || exit 7
python $GRAFT_REPO_ROOT/tools/summarize_profiles.py $O > $O/summary.txt 2>&1
