"""EXE action spaces (fixed_quants_complex :838-933, simplest_case :935-999,
fixed_quants_1msg :732-836, twap :1126-1227) and observation spaces (basic :1879-1911,
simplest_case :1841-1877) of exec_env.py: the C oracle vs a numpy restatement, on env
states reached by oracle rollouts of the 2-player config.
"""
import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import pack_env_cfg
from oracle import pyoracle as O
from test_gpu_env import variant

F = np.float32


def _gather(a, n):
    i = a + n if a < 0 else a
    return min(max(i, 0), n - 1)


def _levels(w, n_ticks, lba, lbb, sell):
    tick = w.tick_size
    ba, bb = (lba // tick) * tick, (lbb // tick) * tick
    if sell:
        m = int(np.ceil(F(F(bb + ba) / F(2)) // F(tick)) * F(tick))
        return [bb, m, ba, ba + tick * n_ticks]
    return [ba, (bb + ba) // 2 // tick * tick, bb, bb - tick * n_ticks]


def expected_rows(t, w, rec, L, a_off, action):
    M = L.n_msgs
    lba, lbb = int(rec[L.off_best_asks + (M - 1) * 2]), int(rec[L.off_best_bids + (M - 1) * 2])
    st = rec[a_off:a_off + 13]
    task, qe, sell = int(st[1]), int(st[2]), int(st[3])
    left = task - qe
    fq = t.fixed_quant_value
    pl = _levels(w, t.n_ticks_in_book, lba, lbb, sell)
    if t.action_space == "fixed_quants_complex":
        qa = np.array([[0, 0, 0, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1], [2, 0, 0, 0],
                       [0, 2, 0, 0], [0, 0, 2, 0], [0, 0, 0, 2], [5, 0, 0, 0], [0, 5, 0, 0], [0, 0, 5, 0],
                       [0, 0, 0, 5]])
        q = qa[_gather(action, 13)] * fq
        if not q.sum() <= left:
            q = np.floor(F(qa[1] * left)).astype(np.int32)
        return list(zip(q.tolist(), pl))
    if t.action_space == "fixed_quants_1msg":
        i = _gather(action, 5)
        p = [0] + pl
        qq = [0, fq, fq, fq, fq][i]
        return [(qq if qq <= left else 0, p[i])]
    ft, nt = pl[0], pl[2]
    if t.action_space == "simplest_case":
        qa = np.array([[0, 0], [fq, 0], [0, fq]])
        q = qa[_gather(action, 3)]
        if not q.sum() <= left:
            q = np.floor(F(qa[1] * left)).astype(np.int32)
        return list(zip(q.tolist(), [ft, nt]))
    steps_left = int(rec[L.off_loaded + 3]) - int(rec[L.off_loaded + 5]) - 1
    qts = int(np.ceil(F(F(max(left, 0)) / F(steps_left))))
    q = np.array([[1, 0], [0, 1]])[_gather(action, 2)] * qts
    return list(zip(q.tolist(), [ft, nt]))


CASES = [dict(), dict(task_size=35), dict(action_space="simplest_case"), dict(action_space="simplest_case", task_size=25),
         dict(action_space="fixed_quants_1msg"), dict(action_space="fixed_quants_1msg", task_size=40),
         dict(action_space="twap"), dict(action_space="twap", task_size=7, task="buy")]

_DAY = {}


def _setup(changes):
    cfg = variant(builtin_config("2_player_fq_fqc"), "Execution", **changes)
    w = cfg.world_config
    if "day" not in _DAY:
        _DAY["day"] = generate_day(n_msgs=20_000, seed=6, snap_every=w.n_data_msg_per_step * w.start_resolution)
    day = _DAY["day"]
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    return cfg, w, day, c, L, init


@pytest.mark.parametrize("changes", CASES, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()) or "complex")
def test_exe_action_messages_vs_numpy(changes):
    cfg, w, day, c, L, init = _setup(changes)
    t = cfg.dict_of_agents_configs["Execution"]
    E = 12
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2)
    st, _ = O.env_reset(c, keys, init)
    tid = w.trader_id_range_start - 1
    a_off = L.agent_offsets[1]
    for k in range(8):
        for e in range(E):
            for act in range(-1, t.n_actions + 1):
                rows, _ = O.mm_action_msgs(c, 1, 0, st[e], act)
                want = expected_rows(t, w, st[e], L, a_off, act)
                got = [(int(r[2]), int(r[3])) for r in rows]
                assert got == want, f"step {k} env {e} action {act}: oracle {got} numpy {want}"
                side = 1 - 2 * int(st[e, a_off + 3])
                assert all(r[0] == 1 and r[1] == side and r[5] == tid for r in rows)
        acts = O.sample_actions(c, keys + 5 * k)
        st = O.env_step(c, keys + 5 * k, acts, day.msgs, init, st)[0]


@pytest.mark.parametrize("obs,norm", [("basic", True), ("basic", False), ("simplest_case", True),
                                      ("simplest_case", False)])
def test_exe_obs_vs_numpy(obs, norm):
    cfg, w, day, c, L, init = _setup(dict(observation_space=obs, normalize=norm))
    t = cfg.dict_of_agents_configs["Execution"]
    E = 8
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2)
    st, o = O.env_reset(c, keys, init)
    a_off, M = L.agent_offsets[1], L.n_msgs
    for k in range(6):
        for e in range(E):
            rec = st[e]
            task, qe = int(rec[a_off + 1]), int(rec[a_off + 2])
            if obs == "basic":
                ba, bb = int(rec[L.off_best_asks + (M - 1) * 2]), int(rec[L.off_best_bids + (M - 1) * 2])
                want = ([F(ba - 1550000) / F(1e3), F(bb - 1550000) / F(1e3), F(task - qe) / F(t.task_size)] if norm
                        else [F(ba), F(bb), F(task - qe)])
            else:
                tu0 = int(rec[L.off_world]) - int(rec[L.off_loaded])
                tu1 = int(rec[L.off_world + 1]) - int(rec[L.off_loaded + 1])
                ep = F(w.episode_time)
                ptr = F(F(ep - F(F(tu0) + F(tu1) / F(1e9))) / ep)
                prq = F(F(task - qe) / F(task))
                mid = rec[L.off_world + 3:L.off_world + 4].view(np.float32)[0]
                want = ([F(F(mid - F(7560000)) / F(1e3)), F(prq - F(0.5)), F(ptr - F(0.5))] if norm
                        else [mid, prq, ptr])
            got = o[e, 1, :3].tolist()
            assert np.array_equal(np.array(got, np.float32), np.array(want, np.float32)), (k, e, got, want)
        acts = O.sample_actions(c, keys + 3 * k)
        st, o = O.env_step(c, keys + 3 * k, acts, day.msgs, init, st)[:2]


# ------------------------------------------------ fixed_prices (MultiDiscrete quantities)
def _mean_last10(x):
    """best_asks[-10:].mean(axis=0)[0] with f32 accumulation in row order."""
    x = [int(v) for v in x[-10:]]
    s = F(0)
    for v in x:
        s = F(s + F(v))
    return F(s / F(len(x)))


def expected_fixed_price_rows(t, w, rec, L, a_off, action):
    """exec_env.py:1001-1123 restated in numpy."""
    M, tick, n = L.n_msgs, w.tick_size, t.n_actions
    st = rec[a_off:a_off + 13]
    left, sell = int(st[1]) - int(st[2]), int(st[3])
    a = np.atleast_1d(np.asarray(action, np.int32))
    if int(a.sum()) > left:
        a = (a.astype(F) / F(a.sum()) * F(left)).astype(np.int32)
    asks = rec[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2)[:, 0]
    bids = rec[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2)[:, 0]
    ba = int(F(_mean_last10(asks) // F(tick)) * F(tick))
    bb = int(F(_mean_last10(bids) // F(tick)) * F(tick))
    if sell:
        lv = dict(FT=bb // tick * tick, M=int(np.ceil(F(F(bb + ba) / F(2)) // F(tick)) * F(tick)), NT=ba,
                  PP=ba + tick * t.n_ticks_in_book)
    else:
        lv = dict(FT=ba // tick * tick, M=(bb + ba) // 2 // tick * tick, NT=bb, PP=bb - tick * t.n_ticks_in_book)
    names = {4: ("FT", "M", "NT", "PP"), 3: ("FT", "NT", "PP"), 2: ("FT", "NT"), 1: ("FT",)}[n]
    prices = [lv[k] for k in names]
    q = [int(v) for v in a]
    if n == 4 and prices[1] == prices[2]:
        q[2], q[1], prices[1] = q[2] + q[1], 0, -1
    return list(zip(q, prices))


FP_CASES = [dict(n_actions=4), dict(n_actions=4, task_size=30), dict(n_actions=3, task="sell"),
            dict(n_actions=2, task="buy", task_size=12), dict(n_actions=1), dict(n_actions=1, task_size=5)]


@pytest.mark.parametrize("changes", FP_CASES, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_exe_fixed_price_messages_vs_numpy(changes):
    cfg, w, day, c, L, init = _setup(dict(action_space="fixed_prices", fixed_quant_value=11, **changes))
    t = cfg.dict_of_agents_configs["Execution"]
    n = t.n_actions
    assert c.types[1].action_width == n and c.action_words == 1 + n
    E = 10
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 7
    st, _ = O.env_reset(c, keys, init)
    a_off = L.agent_offsets[1]
    rng = np.random.default_rng(3)
    cand = [np.zeros(n, np.int32), np.full(n, 10, np.int32), np.arange(n, dtype=np.int32) * 3,
            np.full(n, -4, np.int32)] + [rng.integers(0, 11, n).astype(np.int32) for _ in range(6)]
    merged = rescaled = 0
    for k in range(8):
        for e in range(E):
            for act in cand:
                rows, _ = O.mm_action_msgs(c, 1, 0, st[e], act)
                want = expected_fixed_price_rows(t, w, st[e], L, a_off, act)
                got = [(int(r[2]), int(r[3])) for r in rows]
                assert got == want, f"step {k} env {e} action {act}: oracle {got} numpy {want}"
                merged += n == 4 and want[1][1] == -1
                left = int(st[e, a_off + 1]) - int(st[e, a_off + 2])
                rescaled += int(act.sum()) > left
        acts = O.sample_actions(c, keys + 5 * k)
        assert acts.shape == (E, 1 + n) and ((acts[:, 1:] >= 0) & (acts[:, 1:] < 11)).all()
        st = O.env_step(c, keys + 5 * k, acts, day.msgs, init, st)[0]
    assert ("task_size" not in changes or rescaled > 0) and (n != 4 or merged > 0)   # both branches ran


def test_mean_last10_order_free_at_tick_prices():
    """The f32 mean of 10 tick-multiple prices below 2**26 is exact in any summation order (the
    reference's XLA reduction order is unspecified; the restatements sum in row order)."""
    rng = np.random.default_rng(0)
    for _ in range(200):
        x = rng.integers(1_000_000 // 100, 6_000_000 // 100, 10) * 100
        assert _mean_last10(x) == F(np.sum(x.astype(F)) / F(10)) == F(np.float64(x.sum()) / 10)


@pytest.mark.parametrize("part", [True, False])
def test_multidiscrete_sampling_vs_numpy(part):
    """Speed_test.py:166-177 with MultiDiscrete.sample (spaces.py:57-65): randint of shape (n,)."""
    from oracle import ref_py as R
    cfg = variant(builtin_config("2_player_fq_fqc"), "Execution", action_space="fixed_prices", n_actions=3,
                  fixed_quant_value=7)
    c, _ = pack_env_cfg(cfg, 4, 10_000, part)
    keys = np.arange(16, dtype=np.uint32).reshape(8, 2) * 977
    acts = O.sample_actions(c, keys)
    for e in range(8):
        sub = R.split(tuple(int(v) for v in keys[e]), 2, part)
        mm = R.randint(R.split(sub[0], 1, part)[0], 0, c.types[0].n_actions, part)
        exe = R.randint_vec(R.split(sub[1], 1, part)[0], 3, 0, 7, part)
        assert acts[e].tolist() == [mm] + exe


# ------------------------------------------------- EXE engineered observation
def exe_engineered_numpy(t, w, rec, L, a_off):
    """_get_obs (exec_env.py:1913-2079) + normalize_obs (:2152-2162), sorted keys, from the record."""
    M = L.n_msgs
    ba = int(rec[L.off_best_asks + 2 * (M - 1)])
    bb = int(rec[L.off_best_bids + 2 * (M - 1)])
    asks = rec[L.off_asks:L.off_asks + 6 * w.nOrders].reshape(-1, 6)
    bids = rec[L.off_bids:L.off_bids + 6 * w.nOrders].reshape(-1, 6)
    va = int(np.where(asks[:, 0] != -1, asks[:, 1], 0).sum())
    vb = int(np.where(bids[:, 0] != -1, bids[:, 1], 0).sum())
    st = rec[a_off:a_off + 13]
    init = rec[a_off:a_off + 1].view(np.float32)[0]
    task, qe, sell = int(st[1]), int(st[2]), int(st[3])
    pa, pp = (bb, ba) if sell else (ba, bb)
    qa, qp = (vb, va) if sell else (va, vb)
    wr, lr = rec[L.off_world:L.off_world + 5], rec[L.off_loaded:L.off_loaded + 6]
    sc, ms = int(lr[5]), int(lr[3])
    rr = F(0) if ms == 0 else F(F(1) - F(F(sc) / F(ms)))
    obs = {"is_sell_task": (sell, 0, 1), "p_aggr": (pa, init, 1e5), "p_pass": (pp, init, 1e5),
           "spread": (abs(pa - pp), 0, 1e4), "q_aggr": (qa, 0, 1000), "q_pass": (qp, 0, 1000),
           "init_price": (init, 0, 1e7), "task_size": (task, 0, t.task_size), "executed_quant": (qe, 0, t.task_size),
           "remaining_quant": (task - qe, 0, t.task_size), "step_counter": (sc, 0, 30), "remaining_ratio": (rr, 0, 1)}
    if w.ep_type == "fixed_time":
        time = F(F(wr[0]) + F(wr[1]) / F(1e9))
        elapsed = F(time - F(F(lr[0]) + F(lr[1]) / F(1e9)))
        obs.update(time=(time, 0, 1e5), delta_time=(wr[4:5].view(np.float32)[0], 0, 10),
                   time_remaining=(F(F(w.episode_time) - elapsed), 0, w.episode_time))
    out = []
    for k in sorted(obs):
        x, m, s = obs[k]
        x = F(F(x) - F(m)) if isinstance(m, np.floating) else F(x)   # int - 0 stays exact
        out.append(F(x / F(s)) if t.normalize else F(obs[k][0]))
    return out


@pytest.mark.parametrize("norm,ep,task", [(True, "fixed_steps", "random"), (False, "fixed_steps", "random"),
                                          (True, "fixed_steps", "buy"), (True, "fixed_time", "random"),
                                          (False, "fixed_time", "sell")])
def test_exe_engineered_obs_vs_numpy(norm, ep, task, tmp_path):
    import dataclasses
    cfg = variant(builtin_config("2_player_fq_fqc"), "Execution", normalize=norm, task=task)
    if ep == "fixed_time":
        from hftlob.data import lobster as Lb
        from hftlob.data.raw_synthetic import write_raw_lobster_day
        w = dataclasses.replace(cfg.world_config, ep_type="fixed_time", episode_time=300, start_resolution=300)
        cfg = dataclasses.replace(cfg, world_config=w)
        write_raw_lobster_day(str(tmp_path), n_events=12_000, seed=3, mid=2_000_000)
        ld = Lb.LoadLOBSTER_resample(str(tmp_path), str(tmp_path), 10, "fixed_time", window_length=300,
                                     window_resolution=300, n_data_msg_per_step=100, stock="SYN",
                                     time_period="2026_Oct")
        day = Lb.LoadedDay.from_arrays(*ld.run_loading("cpu_ft"))
    else:
        w = cfg.world_config
        day = generate_day(n_msgs=20_000, seed=6, snap_every=w.n_data_msg_per_step * w.start_resolution)
    w = cfg.world_config
    t = cfg.dict_of_agents_configs["Execution"]
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 8
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 11
    st, o = O.env_reset(c, keys, init)
    d = L.obs_dims[1]
    assert d == (12 if ep == "fixed_steps" else 15)
    dn = np.zeros((E, 2), np.int32)
    da = np.zeros(E, np.int32)
    for k in range(14):
        for e in range(E):
            if dn[e, 1] and not da[e]:          # done agent, episode running: obs zeroed (marl_env.py:690-699)
                assert not o[e, 1, :d].any()
                continue
            want = exe_engineered_numpy(t, w, st[e], L, L.agent_offsets[1])
            assert np.array_equal(o[e, 1, :d], np.array(want, np.float32)), (k, e, o[e, 1, :d], want)
        acts = O.sample_actions(c, keys + 3 * k)
        st, o, _, da, dn, _ = O.env_step(c, keys + 3 * k, acts, day.msgs, init, st)
