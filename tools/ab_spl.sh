set -o pipefail
mkdir -p gpurun_out/ab
for T in 1 8 64; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 128 --steps-per-launch $T > gpurun_out/ab/B_T$T.json 2> gpurun_out/ab/B_T$T.err || exit 4
  HFTLOB_LIB=$PWD/ab/libA.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 128 --steps-per-launch $T > gpurun_out/ab/A_T$T.json 2> gpurun_out/ab/A_T$T.err || exit 5
done
