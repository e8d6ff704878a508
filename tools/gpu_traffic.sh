set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/w1
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline >> $O/bench.json 2>> $O/bench.err || exit 3; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/write.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 32 --warmup 4 > $O/fetch.log 2>&1 || exit 5
