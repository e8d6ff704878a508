# BASELINE.md rows other than the metric: bench.py at other batch sizes / configs (2 slices and unsliced).
set -o pipefail
mkdir -p gpurun_out/cfgs
for G in 2 0; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs 512 --slices $G > gpurun_out/cfgs/e512_G$G.json 2> gpurun_out/cfgs/err.log || exit 4
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs 8192 --slices $G > gpurun_out/cfgs/e8192_G$G.json 2> gpurun_out/cfgs/err.log || exit 4
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs 16384 --slices $G > gpurun_out/cfgs/e16384_G$G.json 2> gpurun_out/cfgs/err.log || exit 4
  timeout -k 10 120 python bench.py --no-cpu-baseline --envs 1024 --config 3_player_fq_fqc_dir --slices $G > gpurun_out/cfgs/c5_G$G.json 2> gpurun_out/cfgs/err.log || exit 4
done
