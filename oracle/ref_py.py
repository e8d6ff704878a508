"""ORACLE — TEST INFRASTRUCTURE ONLY.  Second, independent restatement of the
reference order-book engine, in numpy, written array-op for array-op after
gymnax_exchange/jaxob/JaxOrderBookArrays.py (pure Python loops: small cases
only).  It cross-checks oracle/oracle.c, which in turn checks the HIP path.

jnp semantics restated here: ``jnp.where(cond, size=1, fill_value=-1)[0]``
-> first True in row-major order or -1; negative indices wrap; int32 wraps.
"""
from __future__ import annotations

import numpy as np

I32 = np.int32


def _first(mask) -> int:
    """jnp.where(mask, size=1, fill_value=-1)[0][0] on a 1-D or 2-D mask (row index)."""
    idx = np.argwhere(mask)
    return int(idx[0][0]) if len(idx) else -1


def remove_zero_neg(side):                      # :85-90
    side = side.copy()
    side[side[:, 1] <= 0] = -1
    return side


def add_order(side, msg):                       # :62-83
    i = _first(side == -1)
    side = side.copy()
    side[i] = [msg["price"], max(0, msg["quantity"]), msg["orderid"], msg["traderid"], msg["time"], msg["time_ns"]]
    return remove_zero_neg(side)


def get_init_id_match(cfg, side, msg):          # :120-139
    m = ((side[:, 0] == msg["price"]) & (side[:, 2] <= cfg["init_id"])
         & (side[:, 2] >= cfg["init_id"] - cfg["book_depth"] * 2) & (side[:, 1] >= msg["quantity"]))
    return _first(m)


def _uniform_f32(key, partitionable):
    """jax.random.uniform(key, (), float32): (bits >> 9 | 1.0f) - 1."""
    y0, y1 = threefry2x32(key[0], key[1], 0, 0)
    bits = (y0 ^ y1) if partitionable else y0
    return np.array([(bits >> 9) | 0x3F800000], np.uint32).view(np.float32)[0] - np.float32(1.0)


def _choice_p(key, a, p, partitionable):
    """jax.random.choice(key, a, p=p) for shape=(), replace=True (jax/_src/random.py)."""
    p_cuml = np.cumsum(np.asarray(p, np.float32), dtype=np.float32)
    r = np.float32(p_cuml[-1] * (np.float32(1.0) - _uniform_f32(key, partitionable)))
    ind = int(np.searchsorted(p_cuml, r, side="left"))
    return a[ind]


def get_random_id_match(cfg, key, side, msg, large=False):   # :141-164
    part = cfg.get("partitionable", True)
    key = split(key, 2, part)[0]
    pm = side[:, 0] == msg["price"]
    if not large:
        pm = pm & (side[:, 1] >= msg["quantity"])
    ids = np.where(pm, side[:, 2], 0).astype(I32)
    chosen = _choice_p(key, ids, np.abs(np.sign(ids)), part)
    idx = _first(side[:, 2] == chosen)
    if idx == -1 and not large and cfg["cancel_mode"] == 3:
        idx = get_random_id_match(cfg, key, side, msg, large=True)
    return idx


def cancel_order(cfg, side, msg, key=None):     # :93-117
    idx = _first(side[:, 2] == msg["orderid"])
    if idx == -1:
        idx = get_init_id_match(cfg, side, msg)
        if idx == -1 and cfg["cancel_mode"] in (2, 3):
            idx = get_random_id_match(cfg, key, side, msg)
    side = side.copy()
    side[idx, 1] = np.int32(side[idx, 1] - msg["quantity"])
    return remove_zero_neg(side)


def _top(cfg, side, bid):                       # :241-268
    maxint = cfg["maxint"]
    if bid:
        mp = side[:, 0].max()
    else:
        mp = np.where(side[:, 0] == -1, maxint, side[:, 0]).min()
    times = np.where(side[:, 0] == mp, side[:, 4], maxint)
    mts = times.min()
    tns = np.where(times == mts, side[:, 5], maxint)
    return _first(tns == tns.min())


def match_order(side, top, qtm, trades, msg):   # :172-220
    side, trades = side.copy(), trades.copy()
    newq = max(0, int(side[top, 1]) - qtm)
    rem = qtm - int(side[top, 1])
    e = _first(trades[:, 4] == -1)
    trades[e] = [side[top, 0], -msg["side"] * (int(side[top, 1]) - newq), side[top, 2], msg["orderid"],
                 msg["time"], msg["time_ns"], side[top, 3], msg["traderid"]]
    side[top, 1] = newq
    return remove_zero_neg(side), rem, trades


def match_against(cfg, side, bid, msg, trades):  # :284-331
    qtm, price = int(msg["quantity"]), int(msg["price"])
    top = _top(cfg, side, bid)
    while True:
        tp = int(side[top, 0])
        ok = (tp >= price) if bid else (tp <= price)
        if not (ok and qtm > 0 and tp != -1):
            return side, qtm, trades
        side, qtm, trades = match_order(side, top, qtm, trades, msg)
        top = _top(cfg, side, bid)


def _lim(cfg, msg, own, opp, trades, own_is_bid):
    msg = dict(msg)
    if cfg["type_4_interpretation"] == 2 and not own_is_bid:
        msg["price"] = 0
    opp, rem, trades = match_against(cfg, opp, not own_is_bid, msg, trades)
    if cfg["type_4_interpretation"] == 2 and own_is_bid:
        msg["price"] = cfg["maxint"]
    msg["quantity"] = rem
    if cfg["check_book_fill"]:
        if (own[:, 0] >= 0).all():
            worst = own[:, 0].min() if own_is_bid else own[:, 0].max()
            own = np.where((own[:, 0] == worst)[:, None], -1, own).astype(I32)
    added = add_order(own, msg)
    if cfg["type_4_interpretation"] in (0, 2) and msg["type"] == 4:
        added = own
    return added, opp, trades


def process_msg(cfg, book, data, key=None):     # cond_type_side_save_bidask :687-732
    asks, bids, trades = book
    msg = {"side": -int(data[1]) if data[0] == 4 else int(data[1]), "type": int(data[0]), "price": int(data[3]),
           "quantity": int(data[2]), "orderid": int(data[4]), "traderid": int(data[5]), "time": int(data[6]),
           "time_ns": int(data[7])}
    s, t = msg["side"], msg["type"]
    index = ((s == 1 and t in (1, 4)) * 1 + (s == -1 and t in (2, 3)) * 2 + (s == 1 and t in (2, 3)) * 3
             + (s == 0 and t == 0) * 4)
    if index == 0:
        asks, bids, trades = _lim(cfg, msg, asks, bids, trades, False)
    elif index == 1:
        bids, asks, trades = _lim(cfg, msg, bids, asks, trades, True)
    elif index == 2:
        asks = cancel_order(cfg, asks, msg, key)
    elif index == 3:
        bids = cancel_order(cfg, bids, msg, key)
    return asks, bids, trades


def best_quotes(cfg, asks, bids):               # :932-984
    mn = np.where(asks[:, 0] == -1, cfg["maxint"], asks[:, 0]).min()
    ba = -1 if mn == cfg["maxint"] else int(mn)
    bb = int(bids[:, 0].max())
    return ([ba, int(asks[asks[:, 0] == ba, 1].astype(np.int64).sum())],
            [bb, int(bids[bids[:, 0] == bb, 1].astype(np.int64).sum())])


def scan_save_bidask(cfg, msgs, asks, bids, trades, key=(0, 0)):   # :791-823
    book = (np.array(asks, I32), np.array(bids, I32), np.array(trades, I32))
    ba, bb = [], []
    msgs = np.asarray(msgs, I32)
    keys = split(key, len(msgs), cfg.get("partitionable", True)) if cfg["cancel_mode"] >= 2 else [None] * len(msgs)
    for m, k in zip(msgs, keys):
        book = process_msg(cfg, book, m, k)
        a, b = best_quotes(cfg, book[0], book[1])
        ba.append(a)
        bb.append(b)
    return book, np.array(ba, I32), np.array(bb, I32)


def default_cfg(**kw):
    c = dict(maxint=2147483647, init_id=-2, book_depth=10, cancel_mode=1, type_4_interpretation=0,
             check_book_fill=True, nOrders=100, nTrades=100)
    c.update(kw)
    return c


# ------------------------------------------------------------- JAX PRNG restated
def threefry2x32(k0, k1, x0, x1):
    M = 0xFFFFFFFF

    def rotl(v, r):
        return ((v << r) | (v >> (32 - r))) & M

    ks = [k0, k1, k0 ^ k1 ^ 0x1BD11BDA]
    x0, x1 = (x0 + ks[0]) & M, (x1 + ks[1]) & M
    rots = [(13, 15, 26, 6), (17, 29, 16, 24)]
    for i in range(1, 6):
        for r in rots[(i - 1) % 2]:
            x0 = (x0 + x1) & M
            x1 = rotl(x1, r) ^ x0
        x0 = (x0 + ks[i % 3]) & M
        x1 = (x1 + ks[(i + 1) % 3] + i) & M
    return x0, x1


def split(key, n, partitionable=True):
    if partitionable:
        return [threefry2x32(key[0], key[1], 0, j) for j in range(n)]
    y0, y1 = zip(*[threefry2x32(key[0], key[1], i, n + i) for i in range(n)])
    flat = list(y0) + list(y1)
    return [(flat[2 * j], flat[2 * j + 1]) for j in range(n)]


def randint(key, lo, hi, partitionable=True):
    k1, k2 = split(key, 2, partitionable)

    def bits(k):
        y0, y1 = threefry2x32(k[0], k[1], 0, 0)
        return (y0 ^ y1) if partitionable else y0

    hb, lb = bits(k1), bits(k2)
    span = 1 if hi <= lo else (hi - lo) & 0xFFFFFFFF
    mult = (65536 % span) ** 2 % span
    return lo + (((hb % span) * mult + (lb % span)) & 0xFFFFFFFF) % span


def random_bits(key, n, partitionable=True):
    """jax random_bits(key, 32, (n,)): partitionable counters (0, i) -> y0 ^ y1; legacy: the iota
    split into halves (zero-padded to even length), outputs concatenated [y0..., y1...][:n]."""
    if partitionable:
        return [a ^ b for a, b in (threefry2x32(key[0], key[1], 0, i) for i in range(n))]
    half = (n + 1) // 2
    ctr = list(range(n)) + [0] * (2 * half - n)
    y0, y1 = zip(*[threefry2x32(key[0], key[1], ctr[i], ctr[half + i]) for i in range(half)])
    return (list(y0) + list(y1))[:n]


def randint_vec(key, n, lo, hi, partitionable=True):
    """jax.random.randint(key, (n,), lo, hi) (jax/_src/random.py _randint) for int32."""
    k1, k2 = split(key, 2, partitionable)
    hb, lb = random_bits(k1, n, partitionable), random_bits(k2, n, partitionable)
    span = 1 if hi <= lo else (hi - lo) & 0xFFFFFFFF
    mult = (65536 % span) ** 2 % span
    return [lo + (((h % span) * mult + (l % span)) & 0xFFFFFFFF) % span for h, l in zip(hb, lb)]
