"""Diagnostic: per-phase shader-clock cycles of the persistent k_env_rollout launch (needs a GPU).

The bench's kernel at the bench's shape: 4096 envs of the metric config, one persistent launch of
ST_STEPS steps (default 20, the driver's `bench.py --steps 20`) from the reset state with
Speed_test's keys.  Loads a -DHFTLOB_STAMPS build of libhftlob.so (HFTLOB_STAMPS_LIB, default
ab/stamps.so, built on the CPU host by `make -C jaxmarl-hft_amd/csrc stamps`), whose env_step_dev
writes its phase stamps into words 0..15 of each step's info row and whose rollout loop adds the
step-key batch (word 16, every 4th step) and the issue-priority update (word 17).  Prints the
median / mean cycles and the share of each phase per env-step.  The stamp build's absolute time
is not the product's (the stamps cost a few hundred cycles per step); read its shares.
HFTLOB_STAMPS_LIB=ab/stamps_coarse.so (the same build without the sub-phase probes, which wait for
the wave's outstanding LDS and scalar operations inside the phases they time) gives the top
phases' shares with less perturbation.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HFTLOB_LIB"] = os.environ.get("HFTLOB_STAMPS_LIB") or os.path.join(ROOT, "ab", "stamps.so")
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.env import MARLEnv, split_keys  # noqa: E402

E = int(os.environ.get("ST_ENVS", 4096))
T = int(os.environ.get("ST_STEPS", 20))
cfg = builtin_config(os.environ.get("ST_CONFIG", "2_player_fq_fqc"))
w = cfg.world_config
day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
env = MARLEnv(None, cfg, data=day, return_info=True, persistent_outputs=True)
params = env.default_params
keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
master = keys[0].clone()
_, state = env.reset(keys[1:].contiguous(), params)
kout = torch.empty(2, dtype=torch.int32, device="cuda")
env.rollout_sampled(master.clone(), kout, state.clone(env), params, T, per_step=True, n_slices=0)  # warm-up
torch.cuda.synchronize()
env.rollout_sampled(master.clone(), kout, state, params, T, per_step=True, n_slices=0)
torch.cuda.synchronize()
r = env.last_info_words.reshape(T, E, -1)[:, :, :18].cpu().numpy().astype(np.int64).reshape(T * E, 18)
r[:, 16] &= 0xFFFFFFFF
r[:, 17] &= 0xFFFFFFFF
# env_step_dev's four top phases + the rollout's key batch and priority update = the whole step
top = np.stack([r[:, 16], r[:, 0], r[:, 1], r[:, 2], r[:, 3], r[:, 17]], 1)
tot = top.sum(1)
print(f"k_env_rollout, {E} envs x {T} steps (one persistent launch from the reset state, Speed_test keys)")
print(f"env-steps sampled: {len(r)}; median total cycles/env-step: {np.median(tot):.0f} (mean {tot.mean():.0f})")
clk = r[:, :4].sum(1) / np.maximum(r[:, 15], 1) * 100e6
print(f"in-kernel clock: median {np.median(clk) / 1e9:.3f} GHz; median env_step_dev wave-step {np.median(r[:, 15]) * 10:.0f} ns")
names = ["step-key batch (every 4th step)", "setup+agent msgs+shuffle", "112-msg book loop", "rewards+state+obs",
         "store+info", "issue priority"]
for i, n in enumerate(names):
    print(f"  {n:32s} median {np.median(top[:, i]):9.0f}  mean {top[:, i].mean():9.0f}  share {top[:, i].sum() / tot.sum():.3f}")
print(f"stamp build: {os.path.basename(os.environ['HFTLOB_LIB'])}" + (" (top phases only)" if not r[:, 5:15].any() else ""))
for i, n in zip(range(5, 15) if r[:, 5:15].any() else [], ["  setup: step keys (LDS row)", "  setup: relink / load book", "  setup: agent rows",
                              "  setup: ids + shuffle", "    agents: action msgs", "    agents: cancel rows",
                              "    agents: filter", "  rewards: MM reward", "  rewards: EXE reward",
                              "  rewards: state + obs writes"]):
    print(f"  {n:32s} median {np.median(r[:, i]):9.0f}  mean {r[:, i].mean():9.0f}")
by_step = np.stack([tot.reshape(T, E).mean(1), top[:, 2].reshape(T, E).mean(1)], 1)
print("mean cycles by step (total, book loop): " + " ".join(f"{t}:{a:.0f}/{b:.0f}" for t, (a, b) in enumerate(by_step)))
