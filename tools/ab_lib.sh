# A/B: bench.py with the in-tree libhftlob.so vs ab/lib$1.so (HFTLOB_LIB), slices 0 and 2, twice each.
set -o pipefail
V=$1
mkdir -p gpurun_out/ab
for r in 1 2; do for G in 2 0; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --slices $G > gpurun_out/ab/base_G${G}_$r.json 2> gpurun_out/ab/base.err || exit 4
  HFTLOB_LIB=$PWD/ab/lib$V.so timeout -k 10 120 python bench.py --no-cpu-baseline --slices $G > gpurun_out/ab/${V}_G${G}_$r.json 2> gpurun_out/ab/$V.err || exit 5
done; done
