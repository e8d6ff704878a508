"""Parity at the metric's exact shape and launch path (bench.py):
2_player_fq_fqc.json, NUM_ENVS = 4096, the 400k-message synthetic day (mid 2 M and 28 M: the
GOOG-like regime rounds prices above 2^24 in float32), Speed_test's seeds
(master_key, *reset_keys = split(PRNGKey(0), NUM_ENVS + 1), Speed_test.py:147) and its rollout
(Speed_test.py:186-196) as the bench runs it: MARLEnv.rollout_sampled as one persistent launch or
over 2 env slices on their own streams, 66 steps (the 64-step episode's auto-reset included).  The end state (every integer
word bit-exact, float words within 1e-5) and the carried master key must equal the CPU oracle's
rollout of the same workload.  Also: a rank's shard of a rollout (key_e0 / key_n, bench.py
--gpus N) equals its rows of the whole-batch rollout."""
import dataclasses

import numpy as np
import pytest
import torch

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.env import MARLEnv, split_keys
from oracle import pyoracle as O
from test_gpu_env import _compare_state, _day

pytestmark = pytest.mark.gpu

_METRIC_DAYS = {}


def _metric_day(mid):
    if mid not in _METRIC_DAYS:
        _METRIC_DAYS[mid] = generate_day(n_msgs=400_000, mid=mid, snap_every=6400)
    return _METRIC_DAYS[mid]


@pytest.mark.parametrize("mid,G", [(2_000_000, 2), (28_000_000, 2), (2_000_000, 0), (28_000_000, 0)])
def test_metric_shape_rollout_parity(mid, G):
    """G env slices on their own streams, or G = 0: one persistent k_env_rollout launch whose waves
    keep their book in LDS from step to step (the book is stored to the record by the last step
    and reloaded after an auto-reset)."""
    cfg = builtin_config("2_player_fq_fqc")
    day = _metric_day(mid)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    params = env.default_params
    init = O.init_states(env.cfg_c.lob, env.windows, day.msgs, cfg.world_config, env.layout.init_rec_words)
    assert (init == env._init_states.cpu().numpy()).all()
    E, T = 4096, 66
    all_keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), E + 1)[0]
    o_keys = O.split_keys(np.zeros((1, 2), np.uint32), E + 1)[0]
    assert (all_keys.cpu().numpy().view(np.uint32) == o_keys).all(), "Speed_test key split"
    _, state = env.reset(all_keys[1:].contiguous(), params)
    o_state, _ = O.env_reset(env.cfg_c, o_keys[1:], init)
    _compare_state(env, o_state, state.buf.cpu().numpy(), "reset")
    kin, kout = all_keys[0].clone(), torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, state, params, T, n_slices=G)       # the bench's launch paths
    torch.cuda.synchronize()
    o_end, o_master = O.rollout_sampled(env.cfg_c, o_keys[0], day.msgs, init, o_state, T)
    _compare_state(env, o_end, state.buf.cpu().numpy(), f"after {T} steps")
    assert (kout.cpu().numpy().view(np.uint32) == o_master).all(), "carried master key"
    # the rollout crossed every env's episode end: each record restarted (step counter < T)
    assert (state.world_state.step_counter.cpu().numpy() < T).all()


def test_rollout_shards_equal_whole_batch():
    """bench.py --gpus N: rank r steps envs [r*E, (r+1)*E) with key_e0 = r*E, key_n = N*E; the
    shards together are the whole-batch rollout, bit for bit (state and carried key).  The shards
    run the persistent launch (n_slices 0, the bench's default at 4096 envs per GPU) and 1 / 2
    slices, over 70 steps so every env crosses its episode end."""
    cfg = builtin_config("2_player_fq_fqc")
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000), persistent_outputs=True)
    params = env.default_params
    E, N, T = 48, 3, 70
    keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), N * E + 1)[0]
    _, whole = env.reset(keys[1:].contiguous(), params)
    shards = [env._wrap(whole.buf[r * E:(r + 1) * E].clone()) for r in range(N)]
    kout = torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(keys[0].clone(), kout, whole, params, T, n_slices=2)
    for r, s in enumerate(shards):
        ko = torch.empty(2, dtype=torch.int32, device="cuda")
        env.rollout_sampled(keys[0].clone(), ko, s, params, T, n_slices=r % 3, key_e0=r * E, key_n=N * E)
        assert (ko == kout).all(), f"rank {r}: carried key"
        assert (s.buf == whole.buf[r * E:(r + 1) * E]).all(), f"rank {r}: state"


@pytest.mark.parametrize("name,E,part", [("2_player_fq_fqc", 4096, True), ("2_player_fq_fqc", 4096, False),
                                         ("3_player_fq_fqc_dir", 1024, True), ("3_player_fq_fqc_dir", 1024, False)])
def test_rank_shard_at_real_size(name, E, part):
    """The last rank's shard of the 8-GPU configs at their real sizes and key offsets, on one GPU
    (BASELINE.json configs C4 / C5; ippo_rnn_JAXMARL_pmap.py:292-332, Speed_test.py:142-147):
    C4 = 2_player_fq_fqc, NUM_ENVS = 32768 over 8 ranks, rank 7 steps envs [7*4096, 8*4096);
    C5 = 3_player_fq_fqc_dir (MM + EXE + directional), NUM_ENVS = 8192, rank 7 steps [7*1024, 8*1024).
    Reset keys split(PRNGKey(0), N*E + 1)[1 + 7E : 1 + 8E], step keys split(master, N*E + 1)[1 + 7E + e]
    (key_e0 = 7E, key_n = N*E), 66 steps (every env crosses its episode end) with the launch shape the
    bench picks for E envs per GPU, partitionable and legacy threefry (with the legacy split, key_n
    changes every key).  End state and carried master key against the CPU oracle's rollout."""
    N, r, T = 8, 7, 66
    cfg = builtin_config(name)
    w = cfg.world_config
    day = generate_day(n_msgs=400_000, mid=2_000_000, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day, prng_partitionable=part, return_info=False, persistent_outputs=True)
    params = env.default_params
    init = env._init_states.cpu().numpy()
    assert (init == O.init_states(env.cfg_c.lob, env.windows, day.msgs, w, env.layout.init_rec_words)).all()
    all_keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), N * E + 1, part)[0]
    o_keys = O.split_keys(np.zeros((1, 2), np.uint32), N * E + 1, part)[0]
    assert (all_keys.cpu().numpy().view(np.uint32) == o_keys).all(), "Speed_test key split over N*E envs"
    rows = slice(1 + r * E, 1 + (r + 1) * E)
    _, state = env.reset(all_keys[rows].contiguous(), params)
    o_state, _ = O.env_reset(env.cfg_c, o_keys[rows], init)
    _compare_state(env, o_state, state.buf.cpu().numpy(), "reset")
    G = env.default_slices(E)
    kin, kout = all_keys[0].clone(), torch.empty(2, dtype=torch.int32, device="cuda")
    env.rollout_sampled(kin, kout, state, params, T, n_slices=G, key_e0=r * E, key_n=N * E)
    torch.cuda.synchronize()
    o_end, o_master = O.rollout_sampled(env.cfg_c, o_keys[0], day.msgs, init, o_state, T, key_e0=r * E, key_n=N * E)
    _compare_state(env, o_end, state.buf.cpu().numpy(), f"rank {r} shard after {T} steps (slices {G})")
    assert (kout.cpu().numpy().view(np.uint32) == o_master).all(), "carried master key"
    assert (state.world_state.step_counter.cpu().numpy() < T).all()


def test_c4_shards_compose_at_real_size():
    """BASELINE.json C4 at its real size on one GPU: NUM_ENVS = 32768 of 2_player_fq_fqc sharded over
    8 ranks (ippo_rnn_JAXMARL_pmap.py:292-332).  Each of the 8 shards of 4096 envs runs, one after
    the other, as its rank would (bench.py --gpus 8: reset keys split(PRNGKey(0), 32769)[1 + 4096 r :
    1 + 4096 (r + 1)], one persistent launch, key_e0 = 4096 r, key_n = 32768, partitionable
    threefry), 66 steps across every env's episode end; the 8 end states concatenated, and every
    shard's carried master key, equal the oracle's single 32768-env rollout.  The 8-GPU run then
    only adds timing."""
    N, E, T = 8, 4096, 66
    cfg = builtin_config("2_player_fq_fqc")
    day = _metric_day(2_000_000)
    env = MARLEnv(None, cfg, data=day, return_info=False, persistent_outputs=True)
    params = env.default_params
    init = env._init_states.cpu().numpy()
    all_keys = split_keys(torch.zeros((1, 2), dtype=torch.int32, device="cuda"), N * E + 1)[0]
    o_keys = O.split_keys(np.zeros((1, 2), np.uint32), N * E + 1)[0]
    assert (all_keys.cpu().numpy().view(np.uint32) == o_keys).all()
    assert env.default_slices(E) == 0
    ends, masters, s0 = [], [], []
    for r in range(N):
        _, s = env.reset(all_keys[1 + r * E:1 + (r + 1) * E].contiguous(), params)
        s0.append(s.buf.cpu().numpy())
        ko = torch.empty(2, dtype=torch.int32, device="cuda")
        env.rollout_sampled(all_keys[0].clone(), ko, s, params, T, key_e0=r * E, key_n=N * E)
        torch.cuda.synchronize()
        ends.append(s.buf.cpu().numpy())
        masters.append(ko.cpu().numpy().view(np.uint32).copy())
        del s
    o_end, o_master = O.rollout_sampled(env.cfg_c, o_keys[0], day.msgs, init, np.concatenate(s0), T)
    del s0
    for r in range(N):
        _compare_state(env, o_end[r * E:(r + 1) * E], ends[r], f"rank {r} of 8 after {T} steps")
        assert (masters[r] == o_master).all(), f"rank {r}: carried master key"
        assert (ends[r][:, env.layout.off_loaded + 5] < T).all(), f"rank {r}: every env crossed its episode end"


def test_default_launch_shape():
    """MARLEnv.default_slices: the persistent launch while its waves of workgroups are full (the
    metric: 4096 envs at 16 per CU, and whole multiples of it), 2 env slices when the last wave
    would be partly empty (6000 envs; profiles/r03_launch_shape_sweep.txt, r04_speed_test_sweep.json)."""
    cfg = builtin_config("2_player_fq_fqc")
    env = MARLEnv(None, cfg, data=_day(cfg.world_config, 2_000_000))
    assert env.lds_bytes_per_env() * 16 <= env.LDS_PER_CU
    assert env.default_slices(4096) == 0 and env.default_slices(512) == 0
    assert env.default_slices(8192) == 0 and env.default_slices(16384) == 0
    assert env.default_slices(6000) == 2
    # Speed_test's [5, 5] / [10, 10] agents: 60 / 120 agent rows inside the trade log (lds_map; [10, 10]'s
    # span two message chunks), 16 envs per CU, so 4000 envs are resident: one persistent launch
    for ag in ([5, 5], [10, 10]):
        big = dataclasses.replace(builtin_config("default"), number_of_agents_per_type=ag)
        envb = MARLEnv(None, big, data=_day(big.world_config, 2_000_000))
        assert envb.launch_info()["rows_alias"] == 1
        assert envb.lds_bytes_per_env() * 16 <= envb.LDS_PER_CU
        assert envb.default_slices(4000) == 0
