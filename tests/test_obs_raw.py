"""save_raw_observations (marl_env.py:684-685) on the C oracle: the raw observation record is
get_observation(normalize=False, flatten=False) — a dict of the obs fields in sorted-key order
with their own dtypes (int32 fields stay int32).  Flattening that dict is the un-normalised
observation (the int32 fields cast to float32), so for normalize=False agents the obs row and
the raw record must agree field for field on every agent that is not done.  The field tables
checked here (hftlob.layout.OBS_FIELDS) are the ones MARLEnv uses to build info["agents"][t]["obs_raw"]."""
import dataclasses

import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import obs_fields, pack_env_cfg
from oracle import pyoracle as O
from test_gpu_env import variant

CASES = [dict(mm="basic", exe="engineered"), dict(mm="engineered", exe="basic"),
         dict(mm="engineered", exe="simplest_case"), dict(mm="basic", exe="engineered", ep="fixed_time")]


def _run(cfg, day, E=8, K=10):
    w = cfg.world_config
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 5
    st, _ = O.env_reset(c, keys, init)
    for k in range(K):
        sk = (keys + 17 * k + 1).astype(np.uint32)
        acts = O.sample_actions(c, sk)
        st_n, obs, _, done_all, dones, _, raw, msgs = O.env_step(c, sk, acts, day.msgs, init, st, extras=True)
        yield c, L, obs, done_all.astype(bool), dones.astype(bool), raw, msgs
        st = st_n


@pytest.mark.parametrize("case", CASES, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_raw_obs_is_the_unnormalised_obs(case, tmp_path_factory):
    cfg = builtin_config("2_player_fq_fqc")
    if case.get("ep") == "fixed_time":
        from test_gpu_env import _loaded
        day = _loaded("fixed_time", str(tmp_path_factory.mktemp("lob")))
        w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300)
        cfg = dataclasses.replace(cfg, world_config=w)
    else:
        w = cfg.world_config
        day = generate_day(n_msgs=20_000, seed=3, snap_every=w.n_data_msg_per_step * w.start_resolution)
    cfg = variant(cfg, "MarketMaking", observation_space=case["mm"], normalize=False)
    cfg = variant(cfg, "Execution", observation_space=case["exe"], normalize=False)
    types = list(cfg.dict_of_agents_configs.values())
    checked = 0
    for c, L, obs, done_all, dones, raw, msgs in _run(cfg, day):
        for a, t in enumerate(L.agent_types):
            fields = obs_fields(types[t], cfg.world_config)
            assert len(fields) == L.obs_dims[t]
            assert [f for f, _ in fields] == sorted(f for f, _ in fields), "flatten order is sorted keys"
            live = ~done_all & ~dones[:, a]
            for k, (name, dt) in enumerate(fields):
                col = raw[:, a, k]
                want = col.astype(np.float32) if dt == "i" else col.view(np.float32)
                got = obs[:, a, k]
                assert np.array_equal(got[live], want[live]), (case, name)
            checked += int(live.sum())
    assert checked > 0


def test_messages_obs_space_rows():
    """The MM "messages" space: the obs row is empty (the messages are the msgs output), the raw
    record holds no words, and the combined messages carry D data rows at the end."""
    cfg = variant(builtin_config("2_player_fq_fqc"), "MarketMaking", observation_space="messages")
    w = cfg.world_config
    day = generate_day(n_msgs=20_000, seed=3, snap_every=w.n_data_msg_per_step * w.start_resolution)
    for c, L, obs, done_all, dones, raw, msgs in _run(cfg, day, K=3):
        assert L.obs_dims[0] == 0 and obs_fields(cfg.dict_of_agents_configs["MarketMaking"], w) is None
        assert (obs[:, 0] == 0).all() and (raw[:, 0] == 0).all()
        assert msgs.shape == (obs.shape[0], L.n_msgs, 8)
        data = msgs[:, L.n_msgs - w.n_data_msg_per_step:]
        assert ((data[:, :, 0] >= 1) & (data[:, :, 0] <= 4)).all()
