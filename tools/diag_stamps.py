"""Diagnostic: per-phase shader-clock cycles of k_env_step (needs a GPU).

Builds a -DHFTLOB_STAMPS variant of libhftlob.so into /tmp, steps the metric
workload and prints the median cycles per phase per env-step.  The stamp
build's absolute time is not the product's; read its shares.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get("HFTLOB_STAMPS_LIB") or "/tmp/libhftlob_stamps.so"
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC",
                "-DHFTLOB_STAMPS", "-mllvm", "-structurizecfg-skip-uniform-regions=true", "-shared", "-o", SO, os.path.join(ROOT, "jaxmarl-hft_amd/csrc/hftlob.hip")],
                   check=True)
os.environ["HFTLOB_LIB"] = SO
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.env import MARLEnv, split_keys  # noqa: E402

cfg = builtin_config(sys.argv[1] if len(sys.argv) > 1 else "2_player_fq_fqc")
w = cfg.world_config
day = generate_day(n_msgs=100_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
env = MARLEnv(None, cfg, data=day, return_info=True, persistent_outputs=True)
params = env.default_params
E = 4096
keys = split_keys(torch.tensor([[0, 0]], dtype=torch.int32, device="cuda"), E + 1)[0][1:].contiguous()
_, state = env.reset(keys, params)
kbuf = [torch.tensor([0, 1], dtype=torch.int32, device="cuda"), torch.empty(2, dtype=torch.int32, device="cuda")]
rows = []
for k in range(80):
    env.step_sampled(kbuf[k % 2], kbuf[(k + 1) % 2], state, params)   # the bench's path
    if k >= 8:
        rows.append(env._out["info"][:, :16].cpu().numpy().copy())
r = np.concatenate(rows).astype(np.int64)
names = ["setup+agent msgs+shuffle", "112-msg book loop", "rewards+state+obs", "store+info"]
tot = r[:, :4].sum(1)
print(f"env-steps sampled: {len(r)}; median total cycles/env-step: {np.median(tot):.0f}")
# in-kernel clock (MI355X_MICROARCH.md DVFS item 6): shader cycles / 100 MHz realtime ticks, per wave-step
clk = r[:, :4].sum(1) / np.maximum(r[:, 15], 1) * 100e6
print(f"in-kernel clock: median {np.median(clk) / 1e9:.3f} GHz (p10 {np.percentile(clk, 10) / 1e9:.3f}, "
      f"p90 {np.percentile(clk, 90) / 1e9:.3f}); median wave-step {np.median(r[:, 15]) * 10:.0f} ns")
for i, n in enumerate(names):
    print(f"  {n:28s} median {np.median(r[:, i]):9.0f}  mean {r[:, i].mean():9.0f}  share {r[:, i].sum() / tot.sum():.3f}")
for i, n in zip(range(5, 15), ["  setup: step keys (PRNG)", "  setup: load book sides", "  setup: agent rows",
                              "  setup: ids + shuffle", "    agents: action msgs", "    agents: cancel rows",
                              "    agents: filter", "  rewards: MM reward", "  rewards: EXE reward",
                              "  rewards: state + obs writes"]):
    print(f"  {n:28s} median {np.median(r[:, i]):9.0f}  mean {r[:, i].mean():9.0f}")
