"""World debug_mode (marl_env.py:645-656): with world_config.debug_mode the step's info["world"]
also carries "trades" (the step's trade log), "total_msgs" (the combined message array) and
"lob_state" = get_L2_state(asks, bids, 10) of the stepped books (JaxOrderBookArrays.py:1231-1264).

get_L2_state is pinned by a hand-derived golden and a numpy restatement (jnp.unique with size /
fill_value is np.unique truncated and padded), both checked against the C oracle; the oracle's
env step then carries it, and (GPU) the HIP env's debug words equal the oracle's every step of a
rollout that crosses the auto-reset."""
import dataclasses

import numpy as np
import pytest

from hftlob.config import JAXLOB_Configuration
from hftlob.config_io import builtin_config
from hftlob.data.synthetic import generate_day
from hftlob.data.windows import make_windows
from hftlob.layout import L2_LEVELS, debug_words, pack_env_cfg, pack_lob_cfg
from oracle import pyoracle as O
from streams import init_book_messages, random_streams

I32 = np.int32
MAXINT = 2**31 - 1


def l2_numpy(asks, bids, maxint=MAXINT, n=L2_LEVELS):
    """get_L2_state, line by line (int32 wrap-around as jnp)."""
    def unique(x, fill):
        u = np.unique(x)[:n]
        return np.concatenate([u, np.full(n - len(u), fill, I32)]).astype(I32)

    bp = (I32(-1) * unique(I32(-1) * bids[:, 0], 1)).astype(I32)
    ap = unique(np.where(asks[:, 0] == -1, I32(maxint), asks[:, 0]).astype(I32), -1)
    ap = np.where(ap == -1, I32(maxint), ap)
    bp = np.where(bp == -1, I32(-maxint), bp)

    def vol(side, p):
        v = np.array([np.where(side[:, 0] == x, side[:, 1], 0).astype(np.int64).sum() for x in p])
        v = ((v + 2**31) % 2**32 - 2**31).astype(I32)     # int32 sum
        return np.where(v < 0, 0, v)

    return np.stack([ap, vol(asks, ap), bp, vol(bids, bp)], 1).astype(I32).ravel()


def _side(rows, n=100):
    s = np.full((n, 6), -1, I32)
    for i, r in rows.items():
        s[i] = r
    return s


# Hand-derived: asks at 1000300 (q 5 and q 7, slots 0 and 4) and 1000100 (q 3, slot 2), the other
# 97 slots empty.  Ask keys: where(p == -1, maxint, p) -> unique = [1000100, 1000300, maxint] then
# the fill -1 -> maxint: levels [1000100, 1000300, maxint x 8]; volumes 3, 12, and at maxint 0
# (no row is priced maxint).  Bids at 1000000 (q 4) and 999900 (q 6), a stray bid priced -5 (q 2):
# keys -p = [-1000000, -999900, 5, 1 (the 97 empty rows)] -> unique [-1000000, -999900, 1, 5]
# then the fill 1; negated [1000000, 999900, -1, -5, -1 x 6]; -1 -> -maxint: levels
# [1000000, 999900, -maxint, -5, -maxint x 6]; volumes 4, 6, 0, 2, 0...
GOLDEN_ASKS = {0: [1000300, 5, 11, 1, 10, 0], 2: [1000100, 3, 12, 1, 10, 0], 4: [1000300, 7, 13, 1, 11, 0]}
GOLDEN_BIDS = {1: [1000000, 4, 21, 1, 10, 0], 3: [999900, 6, 22, 1, 10, 0], 5: [-5, 2, 23, 1, 10, 0]}
GOLDEN_L2 = ([1000100, 3, 1000000, 4], [1000300, 12, 999900, 6], [MAXINT, 0, -MAXINT, 0], [MAXINT, 0, -5, 2]) + \
    tuple([MAXINT, 0, -MAXINT, 0] for _ in range(6))


def test_l2_state_golden():
    a, b = _side(GOLDEN_ASKS), _side(GOLDEN_BIDS)
    want = np.array(GOLDEN_L2, I32).ravel()
    assert np.array_equal(l2_numpy(a, b), want)
    assert np.array_equal(O.l2_state(pack_lob_cfg(JAXLOB_Configuration()), a, b), want)


def test_l2_state_oracle_vs_numpy():
    """random books from the engine (more and fewer than 10 levels, empty and full sides) and
    raw arrays with negative quantities / prices"""
    cfg = JAXLOB_Configuration()
    lc = pack_lob_cfg(cfg)
    E = 32
    init = init_book_messages(E, seed=3)
    ea = np.full((E, 100, 6), -1, I32)
    et = np.full((E, 100, 8), -1, I32)
    a0, b0, _, _, _ = O.book_process(lc, init, ea, ea, et, save_best=False)
    a1, b1, _, _, _ = O.book_process(lc, random_streams(E, 400, seed=9), a0, b0, et, save_best=False)
    rng = np.random.default_rng(4)
    raw = rng.integers(-3, 40, (8, 2, 100, 6)).astype(I32)
    raw[..., 0] = np.where(rng.random((8, 2, 100)) < 0.5, -1, 995 + raw[..., 0] % 12)
    books = [(a0[e], b0[e]) for e in range(E)] + [(a1[e], b1[e]) for e in range(E)] + [(r[0], r[1]) for r in raw]
    books += [(ea[0], ea[0]), (np.tile([[7, 1, 1, 1, 1, 1]], (100, 1)).astype(I32), ea[0])]
    for a, b in books:
        assert np.array_equal(O.l2_state(lc, a, b), l2_numpy(a, b))


def test_l2_state_refuses_oversized_tables():
    """oracle_l2_state's stack tables hold HFTLOB_MAX_SLOTS (256) rows / levels: a larger
    n_levels or n_orders is refused with HFTLOB_ESHAPE instead of overflowing them."""
    lc = pack_lob_cfg(JAXLOB_Configuration())
    a = b = np.full((100, 6), -1, I32)
    with pytest.raises(RuntimeError, match="-3"):
        O.l2_state(lc, a, b, n_levels=257)
    big = np.full((300, 6), -1, I32)
    lc.n_orders = 300
    with pytest.raises(RuntimeError, match="-3"):
        O.l2_state(lc, big, big)
    lc.n_orders = 100
    with pytest.raises(ValueError):
        O.l2_state(lc, a[:50], b)
    assert O.l2_state(lc, a, b, n_levels=256).shape == (1024,)


def _debug_cfg(name="2_player_fq_fqc"):
    cfg = builtin_config(name)
    return dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, debug_mode=True))


def test_oracle_env_step_debug_words():
    """the oracle's debug words of a step are the stepped record's trades and L2 view (steps that
    do not reset; a reset's record is the new episode's)"""
    cfg = _debug_cfg()
    w = cfg.world_config
    day = generate_day(n_msgs=20_000, seed=5, snap_every=w.n_data_msg_per_step * w.start_resolution)
    win = make_windows(day, w)
    c, L = pack_env_cfg(cfg, len(win.starts), day.msgs.shape[0], True)
    init = O.init_states(c.lob, win, day.msgs, w, L.init_rec_words)
    E = 8
    keys = np.arange(2 * E, dtype=np.uint32).reshape(E, 2) + 1
    st, _ = O.env_reset(c, keys, init)
    nO, nT, n4 = w.nOrders, w.nTrades, 4 * L2_LEVELS
    seen = 0
    for k in range(70):
        acts = O.sample_actions(c, keys + 3 * k)
        post, _, _, da, _, _, _, msgs, dbg = O.env_step(c, keys + 3 * k, acts, day.msgs, init, st, extras=True,
                                                        debug=True)
        assert dbg.shape == (E, debug_words(nT))
        for e in range(E):
            if da[e]:
                continue
            a = post[e, L.off_asks:L.off_asks + 6 * nO].reshape(nO, 6)
            b = post[e, L.off_bids:L.off_bids + 6 * nO].reshape(nO, 6)
            assert np.array_equal(dbg[e, :n4], l2_numpy(a, b)), f"step {k} env {e}: lob_state"
            assert np.array_equal(dbg[e, n4:], post[e, L.off_trades:L.off_trades + 8 * nT]), "trades"
            seen += 1
        st = post
    assert seen > 400


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["2_player_fq_fqc", "3_player_fq_fqc_dir"])
def test_hip_debug_mode_info(name):
    """MARLEnv with world debug_mode: info["world"] trades / total_msgs / lob_state == the oracle's
    every step over 70 steps (the auto-reset included: they are the stepped state's), then the
    per-step sampled rollout's debug words == step-by-step replays."""
    import torch
    from hftlob.env import MARLEnv, split_keys
    cfg = _debug_cfg(name)
    w = cfg.world_config
    day = generate_day(n_msgs=30_000, seed=11, snap_every=w.n_data_msg_per_step * w.start_resolution)
    env = MARLEnv(None, cfg, data=day)
    params = env.default_params
    init = env._init_states.cpu().numpy()
    E = 24
    keys = torch.from_numpy(np.arange(2 * E, dtype=np.uint32).reshape(E, 2).view(np.int32)).cuda()
    _, state = env.reset(keys, params)
    nT, n4 = w.nTrades, 4 * L2_LEVELS
    for k in range(70):
        sk = split_keys(keys + k, 2)[:, 1].contiguous()
        acts = env.sample_actions(sk)
        prev = state.buf.cpu().numpy().copy()
        _, state, _, dones, info = env.step(sk, state, acts, params)
        o = O.env_step(env.cfg_c, sk.cpu().numpy().view(np.uint32), acts.cpu().numpy(), day.msgs, init, prev,
                       extras=True, debug=True)
        omsgs, odbg = o[7], o[8]
        wi = info["world"]
        assert np.array_equal(wi["lob_state"].cpu().numpy(), odbg[:, :n4]), f"step {k}: lob_state"
        assert np.array_equal(wi["trades"].cpu().numpy(), odbg[:, n4:].reshape(E, nT, 8)), f"step {k}: trades"
        assert np.array_equal(wi["total_msgs"].cpu().numpy(), omsgs), f"step {k}: total_msgs"
        assert np.array_equal(state.buf.cpu().numpy(), o[0]), f"step {k}: state"
    # rollout_sampled, per step, one persistent launch and 2 slices
    for G in (0, 2):
        _, s1 = env.reset(keys, params)
        s0 = s1.buf.cpu().numpy().copy()
        kin = torch.tensor([0, 9], dtype=torch.int32, device="cuda")
        kout = torch.empty_like(kin)
        T = 6
        _, _, _, _, info = env.rollout_sampled(kin, kout, s1, params, T, per_step=True, n_slices=G)
        lob = info["world"]["lob_state"].reshape(T, E, n4).cpu().numpy()
        trd = info["world"]["trades"].reshape(T, E, nT, 8).cpu().numpy()
        rng, st = np.array([0, 9], np.uint32), s0
        for t in range(T):
            ks = O.split_keys(rng[None], E + 1)[0]
            rng, sk = ks[0].copy(), ks[1:].copy()
            o = O.env_step(env.cfg_c, sk, O.sample_actions(env.cfg_c, sk), day.msgs, init, st, extras=True,
                           debug=True)
            st = o[0]
            assert np.array_equal(lob[t], o[8][:, :n4]) and np.array_equal(trd[t], o[8][:, n4:].reshape(E, nT, 8)), \
                f"slices {G} step {t}: debug words"
