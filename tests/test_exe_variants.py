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
