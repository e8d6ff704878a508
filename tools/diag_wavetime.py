"""Diagnostic: wave residency of the persistent k_env_rollout launch (needs a GPU).

Loads a -DHFTLOB_WAVETIME build of libhftlob.so (HFTLOB_WAVETIME_LIB, default ab/wavetime.so;
built on the CPU host by `make -C jaxmarl-hft_amd/csrc wavetime`), runs the metric workload
(4096 envs, the persistent launch, per-step outputs) and reads each wave's start time, hardware
slot (XCC, SE, CU, SIMD) and per-step end times (s_memtime, 100 MHz-normalised shader clock).
Prints where the launch's time goes: the dispatch ramp, the mean / spread of wave lifetimes,
per-CU busy time against the launch span, and the per-step cost spread across envs.

s_memtime counts each XCD's own shader clock (not synchronised across XCDs); s_memrealtime is the
100 MHz reference clock.  Lifetimes use the former, cross-XCD spans the latter.  The raw stamps
go to gpurun_out/wavetime_raw.npz for offline analysis.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HFTLOB_LIB"] = os.environ.get("HFTLOB_WAVETIME_LIB") or os.path.join(ROOT, "ab", "wavetime.so")
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.env import MARLEnv, split_keys  # noqa: E402

E = int(os.environ.get("WT_ENVS", 4096))
T = int(os.environ.get("WT_STEPS", 128))
cfg = builtin_config("2_player_fq_fqc")
w = cfg.world_config
day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
env = MARLEnv(None, cfg, data=day, return_info=True, persistent_outputs=True)
params = env.default_params
keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
master = keys[0].clone()
_, state = env.reset(keys[1:].contiguous(), params)
kout = torch.empty(2, dtype=torch.int32, device="cuda")
env.rollout_sampled(master.clone(), kout, state.clone(env), params, 8, per_step=True, n_slices=0)  # warm-up
torch.cuda.synchronize()
env.rollout_sampled(master.clone(), kout, state, params, T, per_step=True, n_slices=0)
torch.cuda.synchronize()
buf = env.last_info_words  # int32 [T * E, info_words]: words 0..5 hold the stamps in this build
a = buf.reshape(T, E, -1)[:, :, :10].cpu().numpy().astype(np.int64)
u64 = lambda lo, hi: (lo & 0xFFFFFFFF) | ((hi & 0xFFFFFFFF) << 32)  # noqa: E731
end = u64(a[:, :, 0], a[:, :, 1])          # [T, E] step end, the XCD's shader clock
rend = u64(a[:, :, 6], a[:, :, 7])         # [T, E] step end, 100 MHz reference clock
start, rstart = u64(a[0, :, 4], a[0, :, 5]), u64(a[0, :, 8], a[0, :, 9])
hwid, xcc = a[0, :, 2] & 0xFFFFFFFF, a[0, :, 3] & 0xF
cu, se, simd = (hwid >> 8) & 0xF, (hwid >> 13) & 0x7, (hwid >> 4) & 0x3
np.savez(os.path.join(ROOT, "gpurun_out", "wavetime_raw.npz"), end=end, rend=rend, start=start, rstart=rstart,
         hwid=hwid, xcc=xcc)
r0 = rstart.min()
rspan = rend[-1].max() - r0                 # the launch, 10 ns ticks
rlife = rend[-1] - rstart
life = end[-1] - start                      # shader-clock ticks (same XCD for start and end)
step_len = np.diff(np.concatenate([start[None, :], end]), axis=0)  # [T, E] shader ticks
clk = life / np.maximum(rlife, 1) * 100e6   # per-wave shader clock, Hz
slot = xcc * 128 + se * 16 + cu
cus = np.unique(slot)
cu_end = np.array([rend[-1][slot == s_].max() - r0 for s_ in cus])
cu_mean_life = np.array([rlife[slot == s_].mean() for s_ in cus])
n_live = np.array([(rend[-1] > r0 + f * rspan).sum() for f in np.linspace(0, 1, 21)])
res = {
    "envs": E, "steps": T, "cus_seen": int(len(cus)), "xccs": int(len(np.unique(xcc))),
    "waves_per_cu": [int(min((slot == s_).sum() for s_ in cus)), int(max((slot == s_).sum() for s_ in cus))],
    "launch_span_us": round(float(rspan) / 100, 1),
    "dispatch_ramp_us": {"p50": round(float(np.median(rstart - r0)) / 100, 2), "max": round(float((rstart - r0).max()) / 100, 2)},
    "wave_life_over_span": {"mean": round(float(rlife.mean() / rspan), 4), "min": round(float(rlife.min() / rspan), 4),
                            "p10": round(float(np.percentile(rlife, 10) / rspan), 4),
                            "p50": round(float(np.median(rlife) / rspan), 4), "max": round(float(rlife.max() / rspan), 4)},
    "cu_last_end_over_span": {"mean": round(float(cu_end.mean() / rspan), 4), "min": round(float(cu_end.min() / rspan), 4),
                              "p10": round(float(np.percentile(cu_end, 10) / rspan), 4)},
    "cu_mean_wave_life_over_span": round(float(cu_mean_life.mean() / rspan), 4),
    "live_waves_at_span_fraction_0_to_1_by_0.05": [int(x) for x in n_live],
    "shader_clock_ghz": {"p10": round(float(np.percentile(clk, 10)) / 1e9, 3), "p50": round(float(np.median(clk)) / 1e9, 3)},
    "step_shader_ticks": {"mean": round(float(step_len.mean()), 1), "p50": float(np.median(step_len)),
                          "p90": float(np.percentile(step_len, 90)), "max": int(step_len.max())},
    "env_life_cv": round(float(rlife.std() / rlife.mean()), 4),
    "per_step_mean_shader_ticks": [round(float(x), 1) for x in step_len.mean(1)],
}
# ticks -> us: s_memtime counts the shader clock; calibrate with the wall time of the same launch
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
_, state2 = env.reset(keys[1:].contiguous(), params)
ev0.record()
env.rollout_sampled(master.clone(), kout, state2, params, T, per_step=True, n_slices=0)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1)
res["launch_ms_events"] = round(ms, 3)
res["events_over_span"] = round(ms * 1e5 / float(rspan), 4)
print(json.dumps(res))
