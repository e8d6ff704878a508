"""Seeded synthetic day in the RAW LOBSTER file format (test / demo input for
``hftlob.data.lobster``; no LOBSTER data ships with the reference or the image).

Writes ``<root>/rawLOBSTER/<stock>/<period>/<stock>_<date>_34200000_57600000_{message,orderbook}_<L>.csv``
the way LOBSTER publishes a day:

* message rows ``time(s after midnight, 9 decimals), type, order_id, size, price, direction``;
  type 1 submit, 2 partial cancel, 3 delete, 4 visible execution (direction =
  the RESTING order's side), 5 hidden execution (book unchanged), 7 trading
  halt marker;
* a marketable submission appears as the executions it causes, all at its
  timestamp (one type-4 row per resting order hit), then the type-1 row of
  the residual — the pattern ``merge_market_orders`` collapses;
* orderbook row k is the L-level book AFTER message k:
  ``ask_p1, ask_s1, bid_p1, bid_s1, ...``; empty levels 9999999999 / -9999999999, size 0;
* a few rows fall before ``day_start`` / after ``day_end`` (the loader drops them).
"""
from __future__ import annotations

import os

import numpy as np
from sortedcontainers import SortedDict

EMPTY_ASK_P, EMPTY_BID_P = 9999999999, -9999999999


def write_raw_lobster_day(root: str, stock: str = "SYN", period: str = "2026_Oct", date: str = "2026-10-16",
                          n_events: int = 20_000, seed: int = 7, mid: int = 2_000_000, tick: int = 100,
                          levels: int = 10, day_start: int = 34200, day_end: int = 57600,
                          outside: float = 0.002):
    """Simulate ``n_events`` order events; returns (message_path, orderbook_path)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    asks, bids = SortedDict(), SortedDict()
    where = {}
    state = {"oid": 1_000_000}
    rows, books = [], []

    def snap():
        a, b = list(asks.items())[:levels], list(reversed(bids.items()))[:levels]
        r = []
        for k in range(levels):
            r += ([a[k][0], sum(q for _, q in a[k][1])] if k < len(a) else [EMPTY_ASK_P, 0])
            r += ([b[k][0], sum(q for _, q in b[k][1])] if k < len(b) else [EMPTY_BID_P, 0])
        return r

    def emit(t_ns, typ, oid, qty, price, direction):
        rows.append((t_ns, typ, oid, qty, price, direction))
        books.append(snap())

    def add(side, price, qty):
        oid = state["oid"]
        state["oid"] += 1
        (bids if side == 1 else asks).setdefault(price, []).append([oid, qty])
        where[oid] = (side, price)
        return oid

    def take(oid, qty):
        side, price = where[oid]
        book = bids if side == 1 else asks
        lvl = book[price]
        for k, (o, q) in enumerate(lvl):
            if o == oid:
                if q <= qty:
                    lvl.pop(k)
                    del where[oid]
                else:
                    lvl[k][1] = q - qty
                break
        if not lvl:
            del book[price]

    for k in range(1, 16):                      # opening book (not logged, as LOBSTER's start-of-day state)
        for _ in range(int(rng.integers(1, 4))):
            add(-1, mid + k * tick, int(rng.integers(1, 300)))
            add(1, mid - k * tick, int(rng.integers(1, 300)))

    lo, hi = (day_start - 60) * 10**9, (day_end + 60) * 10**9
    span = hi - lo
    t = np.sort(rng.integers(0, span, n_events)) + lo
    n_out = int(outside * n_events)
    t[:n_out] = np.sort(rng.integers((day_start - 60) * 10**9, day_start * 10**9, n_out))
    t[n_events - n_out:] = np.sort(rng.integers((day_end + 1) * 10**9, (day_end + 60) * 10**9, n_out))
    t = np.maximum.accumulate(t)
    for i in range(n_events):
        ti = int(t[i])
        u = rng.random()
        if len(asks) < 4 or len(bids) < 4 or len(where) < 40:
            u = 0.0
        best_a, best_b = asks.keys()[0], bids.keys()[-1]
        if u < 0.45:                                         # submission, sometimes marketable
            side = int(rng.choice([-1, 1]))
            g = int(rng.geometric(0.35)) - 1
            qty = int(max(1, round(rng.lognormal(4.0, 1.0))))
            if rng.random() < 0.08:
                price = best_a + g * tick if side == 1 else best_b - g * tick
            else:
                price = best_a - tick * (1 + g) if side == 1 else best_b + tick * (1 + g)
            rest, opp = qty, (asks if side == 1 else bids)
            while rest > 0 and len(opp) and (opp.keys()[0] <= price if side == 1 else opp.keys()[-1] >= price):
                lp = opp.keys()[0] if side == 1 else opp.keys()[-1]
                o, q = opp[lp][0]
                x = min(q, rest)
                take(o, x)
                emit(ti, 4, o, x, lp, -side)                 # direction of the resting order
                rest -= x
            if rest > 0:
                oid = add(side, price, rest)
                emit(ti, 1, oid, rest, price, side)
        elif u < 0.60 or u < 0.85:                           # partial cancel / delete
            oid = list(where.keys())[int(rng.integers(0, len(where)))]
            side, price = where[oid]
            q = next(q for o, q in (bids if side == 1 else asks)[price] if o == oid)
            if u < 0.60 and q > 1:
                c = int(rng.integers(1, q))
                take(oid, c)
                emit(ti, 2, oid, c, price, side)
            else:
                take(oid, q)
                emit(ti, 3, oid, q, price, side)
        elif u < 0.97:                                       # visible execution at the touch
            side = int(rng.choice([-1, 1]))
            book = bids if side == 1 else asks
            lp = book.keys()[-1] if side == 1 else book.keys()[0]
            o, q = book[lp][0]
            x = int(rng.integers(1, q + 1))
            take(o, x)
            emit(ti, 4, o, x, lp, side)
        elif u < 0.995:                                      # hidden execution
            emit(ti, 5, 0, int(rng.integers(1, 100)), best_a if rng.random() < 0.5 else best_b,
                 int(rng.choice([-1, 1])))
        else:                                                # halt marker
            emit(ti, 7, 0, 0, -1, -1)

    d = os.path.join(root, "rawLOBSTER", stock, period)
    os.makedirs(d, exist_ok=True)
    base = f"{stock}_{date}_{day_start}000_{day_end}000"
    mp = os.path.join(d, f"{base}_message_{levels}.csv")
    bp = os.path.join(d, f"{base}_orderbook_{levels}.csv")
    with open(mp, "w") as f:
        for (tn, typ, oid, q, p, di) in rows:
            s, ns = divmod(tn, 10**9)
            f.write(f"{s}.{ns:09d},{typ},{oid},{q},{p},{di}\n")
    np.savetxt(bp, np.asarray(books, dtype=np.int64), fmt="%d", delimiter=",")
    return mp, bp
