"""Seeded random message streams that exercise the engine's quirks (test helper)."""
import numpy as np


def random_streams(n_env, n_msg, seed, price0=1000, tick=1, spread=12, init_frac=0.1, garbage=0.02, nO=100):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.zeros((n_env, n_msg, 8), dtype=np.int32)
    for e in range(n_env):
        live = []                       # (oid, side, price)
        next_oid = 1000
        t, tn = 34200, 0
        for k in range(n_msg):
            if rng.random() < 0.8:
                tn += int(rng.integers(1, 1000))
            if rng.random() < 0.05:
                t += 1
            u = rng.random()
            side = int(rng.choice([-1, 1]))
            price = price0 + side * int(rng.integers(-3, spread)) * tick
            qty = int(rng.integers(1, 60))
            if rng.random() < 0.01:
                qty = int(rng.integers(-3, 1))
            tid = int(rng.integers(1, 6))
            if u < 0.45:
                typ, oid = 1, next_oid
                next_oid += 1
                live.append((oid, side, price))
            elif u < 0.72:
                typ = int(rng.choice([2, 3]))
                if live and rng.random() < 0.75:
                    oid, side, price = live[int(rng.integers(0, len(live)))]
                elif rng.random() < init_frac * 5:
                    oid = -2 - int(rng.integers(0, 3))      # init-id fallback path
                else:
                    oid = int(rng.integers(1, 5000))
            elif u < 0.95:
                typ = 4
                oid = live[int(rng.integers(0, len(live)))][0] if live else 7
            elif u < 1.0 - garbage:
                typ, side, qty, price, oid = 0, 0, 0, 0, 0
            else:
                typ = int(rng.choice([0, 5, 6, 7])); side = int(rng.choice([-1, 0, 1])); oid = 9
            out[e, k] = (typ, side, qty, price, oid, tid, t, tn)
    return out


def init_book_messages(n_env, seed, price0=1000, tick=1, depth=10):
    rng = np.random.Generator(np.random.PCG64(seed))
    m = np.zeros((n_env, 2 * depth, 8), dtype=np.int32)
    for e in range(n_env):
        for k in range(2 * depth):
            lvl = k // 2 + 1
            side = -1 if k % 2 == 0 else 1
            q = int(rng.integers(0, 200)) if rng.random() > 0.1 else 0
            m[e, k] = (1, side, q, price0 - side * lvl * tick + (5 if side == -1 else -5), -2, -2 - k, 34199, 0)
    return m


def top_streams(n_env, n_msg, seed, price0=1000, maxint=2**31 - 1):
    """Streams for the top-of-book slot (_get_top_*_order_idx) and time priority: a narrow
    price band so most orders join or cross the best level, times drawn from a small set (ties on
    (ts, tns) and orders EARLIER than the standing top are common, so the slot tie-break and the
    time-priority replacement both run), partial and full fills, cancels at the best price, and a
    few maxint times."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.zeros((n_env, n_msg, 8), dtype=np.int32)
    for e in range(n_env):
        live = []
        next_oid = 5000
        for k in range(n_msg):
            t = 34200 + int(rng.integers(0, 3))
            tn = int(rng.integers(0, 4)) * 100
            if rng.random() < 0.01:
                t = maxint
            if rng.random() < 0.01:
                tn = maxint
            side = int(rng.choice([-1, 1]))
            price = price0 + side * int(rng.integers(-2, 3))
            qty = int(rng.integers(1, 40))
            tid = int(rng.integers(1, 4))
            u = rng.random()
            if u < 0.5:
                typ, oid = 1, next_oid
                next_oid += 1
                live.append((oid, side, price))
            elif u < 0.7 and live:
                typ = int(rng.choice([2, 3]))
                oid, side, price = live[int(rng.integers(0, len(live)))]
            elif u < 0.9:
                typ = 4
                oid = live[int(rng.integers(0, len(live)))][0] if live else 7
            else:                                   # marketable limit: crosses deep
                typ, oid = 1, next_oid
                next_oid += 1
                price = price0 - side * 5
            out[e, k] = (typ, side, qty, price, oid, tid, t, tn)
    return out


def neg1_trade_streams(n_env, n_msg, seed, price0=1000):
    """top_streams whose crossing messages (type 4 and the deep marketable limits) often carry
    oid == -1 or time == -1.  match_order (JaxOrderBookArrays.py:205) writes a trade into the
    first row whose col 4 (the message TIME, TradesFeat.SEC) is -1, so a trade made by a
    time == -1 message leaves its row free for the next trade, while an oid == -1 one does not."""
    out = top_streams(n_env, n_msg, seed, price0)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    crossing = (out[..., 0] == 4) | ((out[..., 0] == 1) & (np.abs(out[..., 3] - price0) == 5))
    u = rng.random(out.shape[:2])
    out[..., 4] = np.where(crossing & (u < 0.3), -1, out[..., 4])
    out[..., 6] = np.where(crossing & (u >= 0.3) & (u < 0.6), -1, out[..., 6])
    out[..., 7] = np.where(crossing & (u >= 0.5) & (u < 0.6), -1, out[..., 7])
    return out


def full_book_messages(n_env, seed, nO=100, lo=0.85, hi=1.0, price0=1000):
    """Init messages that leave each side holding between lo * nO and hi * nO orders (per env and
    side), at distinct prices behind the touch, a third of them with the init id (-2, the
    get_init_id_match candidates): books whose last slot is occupied or not, and a few free rows,
    for the no-op skip's room test."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = []
    for e in range(n_env):
        r = []
        for side in (-1, 1):
            n = int(rng.integers(int(lo * nO), int(hi * nO) + 1))
            for k in range(n):
                price = price0 - side * (3 + k) + (0 if side == 1 else 0)
                oid = -2 if rng.random() < 0.33 else 100000 + 1000 * (side + 1) + k
                r.append((1, side, int(rng.integers(1, 50)), price, oid, -2 - k, 34199, k))
        rows.append(r)
    m = max(len(r) for r in rows)
    out = np.zeros((n_env, m, 8), dtype=np.int32)  # doNothing padding
    for e, r in enumerate(rows):
        out[e, :len(r)] = r
    return out


def noop_streams(n_env, n_msg, seed, price0=1000, nO=100):
    """Streams for the chunk pre-pass that skips messages which leave the book unchanged
    (hftlob.hip chunk_noops): mostly cancels of ids no row holds (the replayed day's common
    cancel: its -1 index wraps to the last slot), at prices that do and do not hold init-id rows,
    with quantities 1..50, 0, -1 (skippable) and below -1 (which end the skipping); doNothing rows;
    cancels of live ids and of id -1; non-crossing adds that fill the last free rows of a side
    (the room test's boundary), adds of no quantity (into sides with and without a free row),
    adds carrying an init id or a -1 field (which end the skipping), and executions."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.zeros((n_env, n_msg, 8), dtype=np.int32)
    for e in range(n_env):
        live = []
        next_oid = 20000
        t, tn = 34200, 0
        for k in range(n_msg):
            tn += int(rng.integers(1, 500))
            side = int(rng.choice([-1, 1]))
            lvl = int(rng.integers(1, 12))
            price = price0 - side * lvl
            qty = int(rng.integers(1, 50))
            tid = int(rng.integers(1, 6))
            u = rng.random()
            if u < 0.25:                      # non-crossing add (a fifth of no quantity: a full side evicts for them)
                typ, oid = 1, next_oid
                next_oid += 1
                if rng.random() < 0.2:
                    qty = int(rng.choice([0, 0, -1, -4]))
                else:
                    live.append((oid, side, price))
            elif u < 0.62:                    # cancel of an id no row holds
                typ = int(rng.choice([2, 3]))
                oid = int(rng.integers(1, 10**6))
                v = rng.random()
                qty = 0 if v < 0.08 else (-1 if v < 0.14 else qty)
            elif u < 0.70 and live:           # cancel of a live id
                typ = int(rng.choice([2, 3]))
                oid, side, price = live[int(rng.integers(0, len(live)))]
            elif u < 0.75:                    # zero-quantity cancel
                typ, oid, qty = 3, int(rng.integers(1, 10**6)), 0
            elif u < 0.80:                    # doNothing row
                typ, side, qty, price, oid, tid = 0, 0, 0, 0, 0, 0
            elif u < 0.82:                    # cancel of id -1
                typ, oid = int(rng.choice([2, 3])), -1
                qty = int(rng.choice([1, 0, -1]))
            elif u < 0.85:                    # init-id cancel (get_init_id_match candidates)
                typ, oid = 2, -2 - int(rng.integers(0, 25))
            elif u < 0.87:                    # add carrying an init id (ends the skipping)
                typ, oid = 1, -2 - int(rng.integers(0, 21))
            elif u < 0.89:                    # add with a -1 field (ends the FAST variant)
                typ, oid, tid = 1, next_oid, -1
                next_oid += 1
            elif u < 0.90:                    # cancel of a negative quantity (ends the skipping)
                typ, oid, qty = int(rng.choice([2, 3])), int(rng.integers(1, 10**6)), -int(rng.integers(2, 6))
            elif u < 0.95:                    # execution
                typ = 4
                oid = live[int(rng.integers(0, len(live)))][0] if live else 7
            else:                             # marketable limit (sometimes of no quantity: it matches nothing)
                typ, oid = 1, next_oid
                next_oid += 1
                price = price0 + side * 4
                if rng.random() < 0.2:
                    qty = 0
            out[e, k] = (typ, side, qty, price, oid, tid, t, tn)
    return out


def odd_add_streams(n_env, n_msg, seed, price0=1000, maxint=2**31 - 1):
    """random_streams whose adds include the kernel's RARE decode cases (hftlob.hip decode_msgs):
    limit and type-4 messages priced at or below 0 (-1, -2, -7: a negative ask crosses every bid,
    a negative bid rests behind them all), priced maxint, and add-kind messages whose side is not
    -1 / 1 (type 1 with side 0 or 2 is an ask_lim with that side, as cond_type_side sends it;
    type 4 with side 0 / 2 flips to 0 / -2).  The common add handlers assume 0 <= price, qty > 0
    and side -1 / 1; these must take the general path and leave the book exactly as the oracle's."""
    out = random_streams(n_env, n_msg, seed, price0=price0)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    add = (out[..., 0] == 1) | (out[..., 0] == 4)
    u = rng.random(out.shape[:2])
    neg = add & (u < 0.06)
    out[..., 3] = np.where(neg, rng.choice([-1, -2, -7, 0], size=out.shape[:2]), out[..., 3])
    top = add & (u >= 0.06) & (u < 0.08)
    out[..., 3] = np.where(top, maxint, out[..., 3])
    odd = add & (u >= 0.08) & (u < 0.13)
    out[..., 1] = np.where(odd, rng.choice([0, 2, -2], size=out.shape[:2]), out[..., 1])
    return out
