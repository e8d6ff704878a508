"""Device parity of the tick divisions at tick sizes other than the reference configs' 100.

The kernels replace ``jnp.floor_divide(a, tick_size)`` on int32 by a multiply with a per-launch
magic number (``tick_floordiv``) and ``jnp.floor_divide(x, float(tick_size))`` on float32 by a
reciprocal plus one exact correction (``tick_ffloordiv``), with the jnp formula as the fallback
outside its bounds.  ``World_EnvironmentConfig.tick_size`` is a free field
(/root/reference/gymnax_exchange/jaxob/jaxob_config.py:213), used by the market maker's quotes
(mm_env.py:990-991,1049-1051), the execution agent's prices (exec_env.py:838-932) and the rewards'
reference prices.  Each case generates a synthetic day on that tick's price grid and compares the
HIP env step by step with the oracle, whose floor divisions are the jnp formulas
(oracle/oracle.c ifloordiv / ffloordiv).  tick 1 at mid 2 M puts |x| / tick above the 2^19 bound
and mid 28 M puts |x| above 2^24, so both fallback paths of tick_ffloordiv run on the device.
"""
import dataclasses

import numpy as np
import pytest
import torch

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.env import MARLEnv, split_keys
from oracle import pyoracle as O
from test_abi import tick_magic
from test_gpu_env import _compare_state, rollout_parity

pytestmark = pytest.mark.gpu

TICKS = [1, 3, 7, 25, 128, 1000]


@pytest.mark.parametrize("mid", [2_000_000, 28_000_000])
@pytest.mark.parametrize("tick", TICKS)
@pytest.mark.parametrize("name", ["2_player_fq_fqc", "3_player_fq_fqc_dir"])
def test_tick_size_rollout_parity(name, tick, mid):
    cfg = builtin_config(name)
    w = dataclasses.replace(cfg.world_config, tick_size=tick)
    cfg = dataclasses.replace(cfg, world_config=w)
    day = generate_day(n_msgs=30_000, seed=tick, mid=mid, tick=tick,
                       snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day)
    info = env.launch_info()
    assert info["tick_magic"] == tick_magic(tick), "the kernel's multiplier is the host check's"
    assert info["nfix"] == 100, "the metric kernel family (100/100 slots)"
    rollout_parity(cfg, mid=mid, E=32, K=66, day=day)          # k_env_step, step by step
    # the bench's kernel: one persistent k_env_rollout launch of 66 sampled steps
    E, T = 64, 66
    params = env.default_params
    keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
    _, state = env.reset(keys[1:].contiguous(), params)
    s0 = state.buf.cpu().numpy()
    kin, kout = keys[0].clone(), torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, state, params, T, n_slices=0)
    torch.cuda.synchronize()
    o_st, o_key = O.rollout_sampled(env.cfg_c, kin.cpu().numpy().view(np.uint32), day.msgs,
                                    env._init_states.cpu().numpy(), s0, T)
    _compare_state(env, o_st, state.buf.cpu().numpy(), f"tick {tick}: persistent rollout")
    assert (kout.cpu().numpy().view(np.uint32) == o_key).all(), "carried key"
