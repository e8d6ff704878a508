"""Diagnostic: host-side cost of one bench call at the driver's shape (needs a GPU).

bench.py's timed region at --steps 20 is one MARLEnv.rollout_sampled call: its wall time is
host time up to the launch + the kernel + the completion latency.  This prints, per call (median
of 30): the wall time with synchronisation, the HIP-event time around it, the host time of the
Python call itself (no synchronisation) and of its parts (the ctypes call into libhftlob, the
argument marshalling), so the non-kernel part of the bench's 20-step figure can be attributed.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from hftlob.config_io import builtin_config  # noqa: E402
from hftlob.data.synthetic import generate_day  # noqa: E402
from hftlob.env import MARLEnv, split_keys  # noqa: E402

E, T = 4096, int(os.environ.get("DH_STEPS", 20))
cfg = builtin_config("2_player_fq_fqc")
w = cfg.world_config
day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
params = env.default_params
keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
_, state = env.reset(keys[1:].contiguous(), params)
env.prepare_rollout(0)
k0, k1 = keys[0].clone(), torch.empty(2, dtype=torch.int32, device="cuda")
for _ in range(3):
    env.rollout_sampled(k0, k1, state, params, T, n_slices=0)
torch.cuda.synchronize()
wall, ev, host = [], [], []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    env.rollout_sampled(k0, k1, state, params, T, n_slices=0)
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wall.append(t2 - t0)
    host.append(t1 - t0)
    ev.append(e0.elapsed_time(e1) * 1e-3)
# the same launch as one bare ctypes call with its arguments prepared beforehand: the floor of
# the host path (what the Python wrapper adds is the difference to "host call")
import ctypes as C  # noqa: E402
from hftlob import _lib  # noqa: E402
o = env._outputs(E)
L = _lib.lib()
args = (C.byref(env.cfg_c), E, 0, E, T, k0.data_ptr(), k1.data_ptr(), None, None,
        params.loaded_params.message_data.data_ptr(), params.loaded_params.init_states_array.data_ptr(),
        state.buf.data_ptr(), C.byref(o["struct"]), 0, 0, torch.cuda.current_stream().cuda_stream)
bare = []
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.hftlob_env_rollout_sampled(*args)
    bare.append(time.perf_counter() - t0)
torch.cuda.synchronize()
# where the Python wrapper's time goes: to the C call (pre-launch), the C call, after it
orig = env._abi
marks = {}


def timed_abi(fn, *a):
    marks["enter"] = time.perf_counter()
    orig(fn, *a)
    marks["exit"] = time.perf_counter()


env._abi = timed_abi
pre, post, ccall = [], [], []
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    env.rollout_sampled(k0, k1, state, params, T, n_slices=0)
    t1 = time.perf_counter()
    pre.append(marks["enter"] - t0)
    ccall.append(marks["exit"] - marks["enter"])
    post.append(t1 - marks["exit"])
env._abi = orig
torch.cuda.synchronize()
# a synchronised empty round trip (event record + synchronize): the completion latency floor
rt = []
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    torch.cuda.synchronize()
    rt.append(time.perf_counter() - t0)
med = lambda x: float(np.median(x)) * 1e6  # noqa: E731
print(f"steps {T}: wall {med(wall):.1f} us, events {med(ev):.1f} us, host call {med(host):.1f} us, "
      f"empty sync round trip {med(rt):.1f} us, wall - events {med(wall) - med(ev):.1f} us, "
      f"bare ctypes launch call {med(bare):.1f} us; wrapper: before _abi {med(pre):.1f} us, _abi (device / "
      f"stream lookup + C call) {med(ccall):.1f} us, after it (results) {med(post):.1f} us")
