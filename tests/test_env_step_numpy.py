"""MARLEnv.step's message assembly and book update, restated in numpy from the reference
lines and compared with the C oracle on rollouts of the metric config:

  getCancelMsgs (JaxOrderBookArrays.py:827-853) per agent (mm_env.py:1869-1913,
  exec_env.py:1229-1273); _filter_messages (exec_env.py:413-475 == mm_env.py:520-582);
  order ids, jax.random.permutation of the action rows and [cancels; actions; data]
  (marl_env.py:254-315); the data window (base_env.py:339-369); the scan
  (oracle/ref_py.py, the numpy engine); abort and _ffill_best_prices (marl_env.py:360-364,
  723-749); the world update (marl_env.py:488-515); the combined message array, which is
  also the MM "messages" observation (mm_env.py:2820-2821).

The agents' action rows come from the numpy restatements of tests/test_mm_actions.py and
tests/test_exe_variants.py.  Book, trades, best arrays and world words must match bit for bit.
Steps that end an episode are skipped (the auto-reset replaces the stepped record)."""
import numpy as np
import pytest

from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import pack_env_cfg, trader_ids
from oracle import pyoracle as O
from oracle import ref_py as R
from test_exe_variants import expected_rows as exe_rows
from test_gpu_env import variant
from test_mm_actions import fixed_quant_rows

I32 = np.int32


def cancel_msgs(side_rows, tid, size, side, t, tns):
    """getCancelMsgs: the first `size` rows of the agent (an appended zero row fills the rest)."""
    book = np.concatenate([side_rows, np.zeros((1, 6), I32)])
    idx = list(np.nonzero(book[:, 3] == tid)[0][:size]) + [-1] * size
    return np.array([[2, side, book[i, 1], book[i, 0], book[i, 2], book[i, 3], t, tns] for i in idx[:size]], I32)


def filter_messages(act, cnl):
    """_filter_messages, line by line (jnp.argsort is stable)."""
    act, cnl = act.copy(), cnl.copy()
    pa, pc = act[:, 3], cnl[:, 3]
    res = (pc[None, :] == pa[:, None]) & (pa[:, None] != 0)
    a_mask, c_mask = res.any(1), res.any(0)
    n = len(a_mask)

    def idx(mask):
        i = list(np.nonzero(mask)[0]) + [-1] * len(mask)
        return np.array(i[:len(mask)])

    a_i, c_i = idx(a_mask), idx(c_mask)
    a = np.where(a_i == -1, 0, act[a_i, 2])
    c = np.where(c_i == -1, 0, cnl[c_i, 2])
    rel = (c >= a) * a

    def rank_rev(arr):
        asr = (len(arr) - 1 - np.argsort(arr[::-1], kind="stable"))[::-1]
        return np.argsort(asr, kind="stable")

    act[:, 2] = act[:, 2] - rel[rank_rev(a_mask)]
    act[act[:, 2] == 0] = 0
    cnl[:, 2] = cnl[:, 2] - rel[rank_rev(c_mask)]
    assert n == len(c_mask)
    return act, cnl


def ffill_best(pq, last_valid):
    pq = pq.copy()
    if pq[0, 0] == -1:
        pq[0, 0:2] = [last_valid, 0]
    pq[pq[:, 0] == -1, 1] = 0
    prev = -1
    for m in range(len(pq)):
        prev = pq[m, 0] if pq[m, 0] != -1 else prev
        pq[m, 0] = prev
    return pq


def numpy_step(cfg, L, prev, key, acts, msg_data):
    w = cfg.world_config
    tm, te = cfg.dict_of_agents_configs["MarketMaking"], cfg.dict_of_agents_configs["Execution"]
    (tid_mm,), (tid_exe,) = trader_ids(cfg)
    nO, nT, M, D = w.nOrders, w.nTrades, L.n_msgs, w.n_data_msg_per_step
    asks = prev[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6)
    bids = prev[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6)
    world = prev[L.off_world:L.off_world + 5]
    loaded = prev[L.off_loaded:L.off_loaded + 6]
    t0, t1 = int(world[0]), int(world[1])
    k1, _ = R.split(key, 2)                                          # MARLEnv.step: key, key_reset
    # MM
    r = fixed_quant_rows(tm, w, prev, L, tid_mm, int(acts[0]))
    mm_act = np.array([[ty, sd, q, p, w.placeholder_order_id, tid_mm, t0 + tm.time_delay_obs_act,
                        t1 + tm.time_delay_obs_act] for ty, sd, q, p in r], I32)
    mm_cnl = np.concatenate([cancel_msgs(bids, tid_mm, tm.num_messages_by_agent // 4, 1, t0, t1),
                             cancel_msgs(asks, tid_mm, tm.num_messages_by_agent // 4, -1, t0, t1)])
    mm_act, mm_cnl = filter_messages(mm_act, mm_cnl)
    # EXE
    a_off = L.agent_offsets[1]
    sell = int(prev[a_off + 3])
    side = 1 - 2 * sell
    ex_act = np.array([[1, side, q, p, w.placeholder_order_id, tid_exe, t0 + te.time_delay_obs_act,
                        t1 + te.time_delay_obs_act] for q, p in exe_rows(te, w, prev, L, a_off, int(acts[1]))], I32)
    ex_cnl = cancel_msgs(asks if sell else bids, tid_exe, te.num_messages_by_agent // 2, side, t0, t1)
    ex_act, ex_cnl = filter_messages(ex_act, ex_cnl)
    # assembly
    act = np.concatenate([mm_act, ex_act])
    cnl = np.concatenate([mm_cnl, ex_cnl])
    A = len(act)
    counter = int(world[2])
    act[:, 4] = counter - np.arange(A)
    scan_key = k1
    if w.shuffle_action_messages:
        scan_key, shuffle_key = R.split(k1, 2)
        _, sub = R.split(shuffle_key, 2)                             # _shuffle: one round for A rows
        bits = np.array(R.random_bits(sub, A), np.uint64)
        act = act[np.argsort(bits, kind="stable")]
    start = int(loaded[4]) + D * int(loaded[5])
    start = min(max(start, 0), msg_data.shape[0] - D)
    comb = np.concatenate([cnl, act, msg_data[start:start + D]]).astype(I32)
    ecfg = R.default_cfg(maxint=w.maxint, init_id=w.init_id, book_depth=w.book_depth, cancel_mode=w.cancel_mode,
                         type_4_interpretation=w.type_4_interpretation, check_book_fill=w.check_book_fill,
                         nOrders=nO, nTrades=nT)
    (na, nb, ntr), ba, bb = R.scan_save_bidask(ecfg, comb, asks, bids, np.full((nT, 8), -1, I32), scan_key)
    abort = bool((ba[:, 0] == -1).any() or (bb[:, 0] == -1).any())
    ba = ffill_best(ba, int(prev[L.off_best_asks + 2 * (M - 1)]))
    bb = ffill_best(bb, int(prev[L.off_best_bids + 2 * (M - 1)]))
    f0, f1 = int(comb[-1, 6]), int(comb[-1, 7])
    f32 = np.float32
    mid = f32(f32(int(bb[-1, 0]) + int(ba[-1, 0])) / f32(2))
    dt = f32(f32(f32(f32(f0) + f32(f32(f1) / f32(1e9))) - f32(t0)) - f32(f32(t1) / f32(1e9)))
    return dict(asks=na, bids=nb, trades=ntr, best_asks=ba, best_bids=bb, time=(f0, f1), counter=counter - A,
                mid=mid, dt=dt, step=int(loaded[5]) + 1, abort=abort, comb=comb)


@pytest.mark.parametrize("changes", [dict(), dict(shuffle=False), dict(exe=dict(task="buy")),
                                     dict(mm=dict(auto_liquidate_threshold=2)), dict(nT=12)],
                         ids=lambda d: ",".join(f"{k}:{v}" for k, v in d.items()) or "metric")
def test_env_step_vs_numpy(changes):
    import dataclasses
    cfg = builtin_config("2_player_fq_fqc")
    if "mm" in changes:
        cfg = variant(cfg, "MarketMaking", **changes["mm"])
    if "exe" in changes:
        cfg = variant(cfg, "Execution", **changes["exe"])
    if changes.get("shuffle") is False:
        cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, shuffle_action_messages=False))
    if "nT" in changes:
        cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, nTrades=changes["nT"]))
    w = cfg.world_config
    day = generate_day(n_msgs=20_000, seed=12, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 6
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 21
    st, _ = O.env_reset(c, keys, init)
    checked = 0
    for k in range(12):
        sk = (keys + 13 * k).astype(np.uint32)
        acts = O.sample_actions(c, sk)
        post, _, _, done_all, _, info, _, msgs = O.env_step(c, sk, acts, day.msgs, init, st, extras=True)
        for e in range(E):
            if done_all[e]:
                continue
            want = numpy_step(cfg, L, st[e], tuple(int(v) for v in sk[e]), acts[e], day.msgs)
            p = post[e]
            nO, nT, M = w.nOrders, w.nTrades, L.n_msgs
            assert np.array_equal(p[L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6), want["asks"]), (k, e, "asks")
            assert np.array_equal(p[L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6), want["bids"]), (k, e, "bids")
            assert np.array_equal(p[L.off_trades:L.off_trades + 8 * nT].reshape(nT, 8), want["trades"]), (k, e)
            assert np.array_equal(p[L.off_best_asks:L.off_best_asks + 2 * M].reshape(M, 2), want["best_asks"])
            assert np.array_equal(p[L.off_best_bids:L.off_best_bids + 2 * M].reshape(M, 2), want["best_bids"])
            wr = p[L.off_world:L.off_world + 5]
            assert (int(wr[0]), int(wr[1])) == want["time"] and int(wr[2]) == want["counter"]
            assert wr[3:4].view(np.float32)[0] == want["mid"] and wr[4:5].view(np.float32)[0] == want["dt"]
            assert int(p[L.off_loaded + 5]) == want["step"]
            assert bool(info[e, 12]) == want["abort"]
            # the MM "messages" observation / save_raw_observations messages (mm_env.py:2820-2821)
            assert np.array_equal(msgs[e], want["comb"]), (k, e, "combined messages")
            checked += 1
        st = post
    assert checked >= 50
