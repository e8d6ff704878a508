"""Hand-derived golden vectors for the order-book engine (fixtures, data only).

The reference ships no tests or golden outputs and cannot run here (no jax),
so these expectations were derived BY HAND from the cited reference lines of
gymnax_exchange/jaxob/JaxOrderBookArrays.py, message by message (the
derivation is written next to each message).  They pin the oracles
(oracle/oracle.c, oracle/ref_py.py) before the oracles are trusted to check
the HIP path.  E = all -1 row.

Format: cfg overrides for JAXLOB_Configuration, initial asks/bids (rows),
messages [type, side, q, p, oid, tid, s, ns], expected final asks/bids,
expected non-empty trade rows {index: row}, expected (price, qty) best quotes
after each message.
"""
E6 = [-1] * 6

SCENARIOS = {
    # add / first-free slot / price-time priority (ts then ns) / trade-log overwrite
    # (:172-220, :241-268, :62-83, :205 index -1 -> last row)
    "priority_and_trade_overwrite": dict(
        cfg=dict(nOrders=4, nTrades=3),
        asks=[E6] * 4, bids=[E6] * 4,
        msgs=[
            [1, 1, 10, 100, 11, 1, 5, 0],    # bid 10@100 -> bids[0]
            [1, 1, 5, 101, 12, 2, 5, 1],     # bid 5@101  -> bids[1]
            [1, 1, 7, 101, 13, 3, 5, 0],     # bid 7@101 (earlier ns) -> bids[2]
            [1, -1, 9, 100, 14, 4, 6, 0],    # sell 9@100: hits bids[2] (ns 0 first) 7, then bids[1] 2; rem<0 -> no add
            [2, 1, 4, 100, 11, 1, 7, 0],     # cancel 4 of oid 11 -> q 6
            [3, 1, 50, 555, 999, 0, 7, 1],   # unknown oid, no init match -> slot -1 (last, empty) -> no change
            [4, 1, 20, 99, 15, 5, 8, 0],     # exec on bid side = IOC sell 20@99: bids[1] 3, bids[0] 6 (trade row -1 overwritten)
        ],
        exp_asks=[E6] * 4,
        exp_bids=[E6] * 4,
        exp_trades={0: [101, 7, 13, 14, 6, 0, 3, 4], 1: [101, 2, 12, 14, 6, 0, 2, 4],
                    2: [100, 6, 11, 15, 8, 0, 1, 5]},
        exp_best_asks=[[-1, -4]] * 7,          # empty side: price -1, volume = sum of the -1 qtys
        exp_best_bids=[[100, 10], [101, 5], [101, 12], [101, 3], [101, 3], [101, 3], [-1, -4]],
    ),
    # book-full eviction of ALL worst-price rows, persisting under IOC discard (:395-418, :484-506),
    # init-id cancel fallback (:120-139), failed cancel shrinking the LAST slot (:111-116)
    "eviction_and_cancel_quirks": dict(
        cfg=dict(nOrders=3, nTrades=2),
        asks=[[105, 5, -2, -2, 1, 0], [103, 4, -2, -3, 1, 0], [104, 6, 50, 9, 2, 0]],
        bids=[[100, 3, -2, -4, 1, 0], E6, E6],
        msgs=[
            [1, -1, 2, 106, 60, 7, 3, 0],    # no cross; asks full -> evict worst (105) -> add at slot 0
            [4, 1, 1, 99, 61, 8, 3, 1],      # IOC sell 1@99 hits bid 100; asks full -> evict 106; add discarded
            [2, -1, 4, 103, 777, 0, 4, 0],   # oid miss -> init match (p 103, oid -2, q>=4) -> removed
            [2, -1, 1, 104, 888, 0, 4, 1],   # oid miss, no init match -> last slot (104, oid 50) loses 1
            [1, 1, 10, 104, 62, 3, 5, 0],    # buy 10@104: takes 5 at 104, rest 5 rests at bids[1]
        ],
        exp_asks=[E6, E6, E6],
        exp_bids=[[100, 2, -2, -4, 1, 0], [104, 5, 62, 3, 5, 0], E6],
        exp_trades={0: [100, 1, -2, 61, 3, 1, -4, 8], 1: [104, -5, 50, 62, 5, 0, 9, 3]},
        exp_best_asks=[[103, 4], [103, 4], [104, 6], [104, 5], [-1, -3]],
        exp_best_bids=[[100, 3], [100, 2], [100, 2], [100, 2], [104, 5]],
    ),
    # type_4_interpretation = MKT: sells match at price 0 (set before matching), a buy's
    # remainder is added at maxint (price set AFTER matching) (:391-393, :471-472)
    "mkt_interpretation": dict(
        cfg=dict(nOrders=3, nTrades=2, type_4_interpretation=2),
        asks=[[110, 5, 1, 1, 1, 0], E6, E6], bids=[[90, 5, 2, 2, 1, 0], E6, E6],
        msgs=[
            [1, 1, 3, 100, 10, 5, 2, 0],
            [1, -1, 4, 200, 11, 6, 2, 1],
        ],
        exp_asks=[[110, 5, 1, 1, 1, 0], E6, E6],
        exp_bids=[[90, 4, 2, 2, 1, 0], E6, E6],
        exp_trades={0: [2147483647, 3, 10, 11, 2, 1, 5, 6], 1: [90, 1, 2, 11, 2, 1, 2, 6]},
        exp_best_asks=[[110, 5], [110, 5]],
        exp_best_bids=[[2147483647, 3], [90, 4]],
    ),
    # LIM: a type-4 remainder rests; [0,0,..] is doNothing; an unknown type falls to
    # switch index 0 (ask_lim) with its own side (:720-724)
    "lim_and_dispatch": dict(
        cfg=dict(nOrders=3, nTrades=2, type_4_interpretation=1),
        asks=[E6, E6, E6], bids=[[50, 2, 3, 3, 1, 0], E6, E6],
        msgs=[
            [4, 1, 5, 50, 20, 7, 2, 0],
            [0, 0, 0, 0, 0, 0, 0, 0],
            [5, 1, 2, 49, 21, 8, 3, 0],
            [1, 1, 4, 60, 22, 9, 4, 0],
        ],
        exp_asks=[[50, 1, 20, 7, 2, 0], E6, E6],
        exp_bids=[E6, E6, E6],
        exp_trades={0: [50, 2, 3, 20, 2, 0, 3, 7], 1: [50, -2, 20, 22, 4, 0, 7, 9]},
        exp_best_asks=[[50, 3], [50, 3], [49, 2], [50, 1]],
        exp_best_bids=[[-1, -3]] * 4,
    ),
    # stray q<=0 row in the input book: removed by the first _removeZeroNegQuant on that
    # side (:85-90); equal ts -> min ns -> first slot (:261-268)
    "unclean_input_and_ties": dict(
        cfg=dict(nOrders=4, nTrades=2),
        asks=[[200, 1, 30, 1, 5, 9], [200, 2, 31, 1, 5, 3], [200, 3, 32, 1, 5, 3], [201, 0, 33, 1, 4, 0]],
        bids=[E6] * 4,
        msgs=[[1, 1, 4, 200, 40, 2, 6, 0]],
        exp_asks=[[200, 1, 30, 1, 5, 9], E6, [200, 1, 32, 1, 5, 3], E6],
        exp_bids=[E6] * 4,
        exp_trades={0: [200, -2, 31, 40, 6, 0, 1, 2], 1: [200, -2, 32, 40, 6, 0, 1, 2]},
        exp_best_asks=[[200, 2]],
        exp_best_bids=[[-1, -4]],
    ),
    # negative-quantity cancel on an empty side revives a price -1 row (q = -1 - (-5) = 4);
    # add_order's "first row holding ANY -1" then still finds slot 0
    "negative_cancel_quirk": dict(
        cfg=dict(nOrders=3, nTrades=2),
        asks=[E6] * 3, bids=[E6] * 3,
        msgs=[
            [2, 1, -5, 10, 1, 1, 1, 0],
            [1, 1, 3, 12, 2, 2, 2, 0],
            [1, -1, 1, 5, 3, 3, 3, 0],
        ],
        exp_asks=[E6] * 3,
        exp_bids=[[12, 2, 2, 2, 2, 0], E6, [-1, 4, -1, -1, -1, -1]],
        exp_trades={0: [12, 1, 2, 3, 3, 0, 2, 3]},
        exp_best_asks=[[-1, -3]] * 3,
        exp_best_bids=[[-1, 2], [12, 3], [12, 2]],
    ),
}

# jaxob/jorderbook.py:288-318 (__main__) inputs: l2 init via init_msgs_from_l2
# (:999-1028: oid = init_id - k, tid = init_id, time [0, 0] from OrderBook.reset),
# then the two array messages.  Expected values derived by hand.
JORDERBOOK_L2 = [354200, 452, 350100, 89, 361200, 100, 344000, 400, 362900, 100, 343100, 100, 364000, 400,
                 338700, 100, 371900, 1100, 337100, 1000, 372200, 100, 336400, 1000, 372300, 200, 336000, 300,
                 372800, 1000, 333600, 1000, 374600, 1000, 332500, 100, 376700, 100, 331600, 100]
JORDERBOOK_MSGS = [[1, 1, 99, 346000, 8888, 8888, 3400, 5000000],
                   [1, -1, 2, 346000, 8777, 8777, 3401, 5060000]]
JORDERBOOK_EXPECT = dict(
    bids_rows={0: [350100, 87, -3, -2, 0, 0], 1: [344000, 400, -5, -2, 0, 0],
               10: [346000, 99, 8888, 8888, 3400, 5000000], 11: [-1] * 6},
    asks_rows={0: [354200, 452, -2, -2, 0, 0], 9: [376700, 100, -20, -2, 0, 0], 10: [-1] * 6},
    trades_rows={0: [350100, 2, -3, 8777, 3401, 5060000, -2, 8777], 1: [-1] * 8},
    best_asks=[[354200, 452], [354200, 452]],
    best_bids=[[350100, 89], [350100, 87]],
)


def jorderbook_init_msgs(init_id=-2):
    """init_msgs_from_l2 (:999-1028) for JORDERBOOK_L2 — note oid/tid swapped vs base_env."""
    rows = []
    for k in range(20):
        p, q = JORDERBOOK_L2[2 * k], JORDERBOOK_L2[2 * k + 1]
        rows.append([1, -1 if k % 2 == 0 else 1, q, p, init_id - k, init_id, 0, 0])
    return rows
