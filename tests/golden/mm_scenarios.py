"""Hand-derived golden vectors for one MARLEnv.step of the METRIC config's market maker
(fixtures, data only).

Like env_scenarios.py, every expected value was reasoned BY HAND from the cited reference
lines (no jax here, and the reference ships no env-level outputs); the derivation sits next
to the values.  They pin the market-maker half of 2_player_fq_fqc.json:

  * _getActionMsgs_fixedQuant (mm_env.py:970-1118): the best quotes with the agent's own
    orders masked out (:979-985), the empty_book fallback to world.best_*[-1] (:988-995),
    half = max((ba - bb) / 2, tick / 2) (f32) and hs = (half // tick + 1) * tick (:1028-1029),
    bid = max(bb - off * hs, 0) // tick * tick, ask = max(bid + tick, ba + off * hs) // tick *
    tick (:1043-1052), the tenth action's two type-4 rows [ba + 10 hs, bb - 10 hs] with
    quantities max(-inv, 0), max(inv, 0) (:1073-1081);
  * getCancelMsgs with size num_messages_by_agent // 4 = 1 per side (mm_env.py:1883-1900,
    JaxOrderBookArrays.py:827-853) and _filter_messages (mm_env.py:520-582);
  * get_reward spooner_asym_damped2 (mm_env.py:2247-2430, / reward_scaling_quo :2642):
    passive / aggressive buy and sell attribution (_extract_agent_trade_stats :2214-2243),
    the rebate on passive fills (rebate_bps / 10000, :2363-2369), InventoryPnL on the OLD
    inventory (:2414), and on an episode's last step the fictional unwind trade at the mid
    (unwind_price "mid", penalty 0) placed by add_trade at the first trade row holding any
    -1 (:2285-2317, JaxOrderBookArrays.py:885-893);
  * the MM basic observation, sorted keys [inventory / 10, spread / 1e4] (mm_env.py:2963-3000,
    normalize_obs :3157-3167), from the post-step world (marl_env.py:676-700);
  * update_state_and_get_done_and_info (mm_env.py:2677-2736): posted distances, inventory,
    total_PnL, cash.

Config (mm_golden_config in tests/test_mm_goldens.py): 2_player_fq_fqc.json with only the
world's n_data_msg_per_step D = 2, shuffle_action_messages False and window_selector 0
changed, and the EXE task fixed to "sell"; the agents' own settings are the metric's (MM
fixed_quants / basic / spooner_asym_damped2, fixed_quant_value 1, tick 100, gamma 0.1,
eta 0.6, rebate 0.4 bps, reward_scaling_quo 10; EXE fixed_quants_complex).  MM trader id -100,
EXE -101.  M = D + 4 + 8 = 14 rows: [MM bid cancel, MM ask cancel, 4 EXE cancels, MM bid /
ask actions, 4 EXE actions, 2 data rows] (marl_env.py:260-315).  The EXE agent always plays
action 0 (no quantity: four all-zero rows that still get order ids) and holds no orders, so
its cancels are getCancelMsgs fill rows on its task side (sell: asks).

Pre-step record (unless a scenario says otherwise): world time (100, 5000), order-id counter
-1000, step_counter 3, max_steps 50, start 0, init time (50, 0), window 0; best quote arrays
tiled with `best_ask` / `best_bid`; mid = f32((bb + ba) / 2); EXE state init_price 1000150.0,
task 600, executed 0, sell 1.  Book rows are [price, qty, oid, tid, s, ns]; trade rows
[price, qty (<0: buy aggressor), passive oid, aggressor oid, s, ns, passive tid, aggressor tid].

Float expectations are given as their exact terms; tests/test_mm_goldens.py evaluates the
reference expression in float32 in the reference's operation order.
"""
T = -100                        # the MM's trader id
TE = -101                       # the EXE's trader id
TIME, CNT = (100, 5000), -1000
PAD_BID = [2, 1, 0, 0, 0, 0, 100, 5000]          # getCancelMsgs fill row (bookside[-1] = the appended zero row)
PAD_ASK = [2, -1, 0, 0, 0, 0, 100, 5000]
EXE_PADS = [PAD_ASK] * 4                          # the sell-task EXE's 4 cancel rows, on the ask side
ASK0 = [1000300, 50, 501, 77, 10, 0]
BID0 = [1000000, 40, 601, 77, 10, 0]


def zero_rows(*oids):
    """all-zero action rows (quantity 0 after _filter_messages) that received order ids (marl_env.py:285-290)"""
    return [[0, 0, 0, 0, i, 0, 0, 0] for i in oids]


SCENARIOS = {
    # ---- action 4 on a 300-wide spread: (ba - bb) / 2 = 150, not a tick multiple.
    # masked best ask 1000300, bid 1000000 (no own orders).  half = max(150.0, 50.0) = 150.0;
    # hs = (150 // 100 + 1) * 100 = 200.0.  Offsets (bid, ask) = (4, 4), quantities 1 * 1.
    # bid = max(1000000 - 4 * 200, 0) // 100 * 100 = 999200; ask = max(999200 + 100, 1000300 + 800)
    # = 1001100.  No own orders: both cancels are fill rows, whose price 0 pairs with nothing.
    # Book: the new bid goes to bids slot 1, the new ask to asks slot 1; data bid 999900 (slot 2)
    # and ask 1000200 (slot 2) do not cross; the data ask becomes the best ask at the last row.
    # Reward: no trades; InventoryPnL = 3 * (1000100.0 - 1000150.0) / 100 = -1.5 (old inventory, new
    # mid (1000000 + 1000200) / 2); r = 0 + 0 + 0 + 0.1 * (-1.5 - max(0, 0.6 * -1.5)) = -0.15.
    # Obs (post world): [3 / 10, |1000200 - 1000000| / 1e4].
    "mm_action4_half_spread_150": dict(
        asks=[ASK0], bids=[BID0], best_ask=[1000300, 50], best_bid=[1000000, 40], action=4,
        mm=dict(inv=3, total=0.0, cash=12.5),
        data=[[1, 1, 5, 999900, 701, 88, 100, 9000], [1, -1, 7, 1000200, 702, 88, 101, 0]],
        exp_mm_rows=[(1, 1, 1, 999200), (1, -1, 1, 1001100)],
        exp_msgs=[PAD_BID, PAD_ASK] + EXE_PADS
        + [[1, 1, 1, 999200, -1000, T, 100, 5000], [1, -1, 1, 1001100, -1001, T, 100, 5000]]
        + zero_rows(-1002, -1003, -1004, -1005)
        + [[1, 1, 5, 999900, 701, 88, 100, 9000], [1, -1, 7, 1000200, 702, 88, 101, 0]],
        exp_best_asks=[[1000300, 50]] * 13 + [[1000200, 7]], exp_best_bids=[[1000000, 40]] * 14, exp_abort=0,
        exp_asks={0: ASK0, 1: [1001100, 1, -1001, T, 100, 5000], 2: [1000200, 7, 702, 88, 101, 0]},
        exp_bids={0: BID0, 1: [999200, 1, -1000, T, 100, 5000], 2: [999900, 5, 701, 88, 100, 9000]},
        exp_trades={},
        exp_time=(101, 0), exp_counter=-1006, exp_step=4, exp_mid=1000100.0, exp_done=False,
        exp_reward=dict(buy=0.0, sell=0.0, rebate_value=0.0, inv=3, mid_end=1000100.0, mid_old=1000150.0),
        exp_mm_state=dict(bid_dist=800, ask_dist=800, inv=3, pnl=0.0),
        exp_info=dict(posted_bid_price=999200, posted_ask_price=1001100, bid_distance_from_best=800,
                      ask_distance_from_best=800, bid_quant=1, ask_quant=1, inventory=3, forced_unwind=0),
        exp_obs=[(3, 10), (200, 1e4)],
    ),
    # ---- action 0 with empty_book: the only ask is the agent's own (oid -500).  Masked best ask
    # = -1 -> empty_book: ba, bb = world.best_asks[-1, 0] = 1000500, world.best_bids[-1, 0] = 1000000
    # (not floored), quantities 0 (:1038-1039).  half = max(250.0, 50.0) -> hs = (2 + 1) * 100 = 300.
    # Offsets (0, 0): bid 1000000, ask max(1000100, 1000500) = 1000500; distances 0 / 0.
    # Cancels: bid fill row; ask [2, -1, 1, 1000500, -500, T].  _filter_messages: the ask action
    # (1000500) matches the ask cancel: a = [0, 0], c = [1, 0], rel = (c >= a) * a = [0, 0] -> the
    # cancel keeps q 1, both action rows have q 0 -> all-zero rows.  The cancel empties the ask side:
    # best ask [-1, -100] (get_volume_at_price(-1) sums the 100 empty rows' q = -1) from row 1 to
    # row 12, abort = 1; ffill: row 0 keeps [1000500, 1], -1 prices take the last valid one with q 0;
    # the data ask 1000400 is the last row's best.  Reward: InventoryPnL = -2 * (1000200.0 -
    # 1000250.0) / 100 = 1.0; r = 0.1 * (1.0 - max(0, 0.6 * 1.0)).  Obs [-2 / 10, 400 / 1e4].
    "mm_action0_empty_book": dict(
        asks=[[1000500, 1, -500, T, 90, 0]], bids=[BID0], best_ask=[1000500, 1], best_bid=[1000000, 40],
        action=0, mm=dict(inv=-2, total=1.0, cash=-7.0),
        data=[[1, 1, 5, 999900, 701, 88, 100, 9000], [1, -1, 7, 1000400, 702, 88, 101, 0]],
        exp_mm_rows=[(1, 1, 0, 1000000), (1, -1, 0, 1000500)],
        exp_msgs=[PAD_BID, [2, -1, 1, 1000500, -500, T, 100, 5000]] + EXE_PADS
        + zero_rows(-1000, -1001, -1002, -1003, -1004, -1005)
        + [[1, 1, 5, 999900, 701, 88, 100, 9000], [1, -1, 7, 1000400, 702, 88, 101, 0]],
        exp_best_asks=[[1000500, 1]] + [[1000500, 0]] * 12 + [[1000400, 7]],
        exp_best_bids=[[1000000, 40]] * 14, exp_abort=1,
        exp_asks={0: [1000400, 7, 702, 88, 101, 0]},
        exp_bids={0: BID0, 1: [999900, 5, 701, 88, 100, 9000]}, exp_trades={},
        exp_time=(101, 0), exp_counter=-1006, exp_step=4, exp_mid=1000200.0, exp_done=False,
        exp_reward=dict(buy=0.0, sell=0.0, rebate_value=0.0, inv=-2, mid_end=1000200.0, mid_old=1000250.0),
        exp_mm_state=dict(bid_dist=0, ask_dist=0, inv=-2, pnl=0.0),
        exp_info=dict(posted_bid_price=1000000, posted_ask_price=1000500, bid_distance_from_best=0,
                      ask_distance_from_best=0, bid_quant=0, ask_quant=0, inventory=-2, forced_unwind=0),
        exp_obs=[(-2, 10), (400, 1e4)],
    ),
    # ---- action 9 (tenth_action MarketOrder) with inventory 2, spread 300 -> hs = 200.
    # Rows [4, -1, max(-2, 0) = 0, 1000300 + 2000] and [4, 1, max(2, 0) = 2, 1000000 - 2000 = 998000];
    # the first has q 0 -> all-zero row (id -1000), the second gets id -1001.  Posted prices (the
    # table's offsets 0 at index 9): bid 1000000, ask max(1000100, 1000300) = 1000300; quants 0.
    # Engine: type 4 flips side 1 -> -1: an IOC sell of 2 at 998000 hits bid 1000000 (q 1, slot 0)
    # then bid 999900 (q 40 -> 39): trades [p, -side * filled = +1, passive oid, -1001, 100, 5000,
    # 77, T].  The data bid 999800 takes the freed slot 0; the data ask 1000400 is behind 1000300.
    # Reward: both trades have q >= 0 and the agent as aggressor -> sells (not passive: no rebate).
    # sellPnL = (1000000 - 1000100) / 100 + (999900 - 1000100) / 100 = -3; buyPnL 0; InventoryPnL =
    # 2 * (1000100.0 - 1000150.0) / 100 = -1.0; r = -3 + 0.1 * (-1 - max(0, -0.6)) = -3.1.
    # income 10000 + 9999 = 19999 -> cash -19990 + 19999 = 9.0, total_PnL 0.5 + 19999.
    "mm_action9_market_sell": dict(
        asks=[ASK0], bids=[[1000000, 1, 601, 77, 10, 0], [999900, 40, 602, 77, 11, 0]],
        best_ask=[1000300, 50], best_bid=[1000000, 1], action=9, mm=dict(inv=2, total=0.5, cash=-19990.0),
        data=[[1, 1, 5, 999800, 701, 88, 100, 9000], [1, -1, 7, 1000400, 702, 88, 101, 0]],
        exp_mm_rows=[(4, -1, 0, 1002300), (4, 1, 2, 998000)],
        exp_msgs=[PAD_BID, PAD_ASK] + EXE_PADS + zero_rows(-1000) + [[4, 1, 2, 998000, -1001, T, 100, 5000]]
        + zero_rows(-1002, -1003, -1004, -1005)
        + [[1, 1, 5, 999800, 701, 88, 100, 9000], [1, -1, 7, 1000400, 702, 88, 101, 0]],
        exp_best_asks=[[1000300, 50]] * 14, exp_best_bids=[[1000000, 1]] * 7 + [[999900, 39]] * 7, exp_abort=0,
        exp_asks={0: ASK0, 1: [1000400, 7, 702, 88, 101, 0]},
        exp_bids={0: [999800, 5, 701, 88, 100, 9000], 1: [999900, 39, 602, 77, 11, 0]},
        exp_trades={0: [1000000, 1, 601, -1001, 100, 5000, 77, T], 1: [999900, 1, 602, -1001, 100, 5000, 77, T]},
        exp_time=(101, 0), exp_counter=-1006, exp_step=4, exp_mid=1000100.0, exp_done=False,
        exp_reward=dict(buy=0.0, sell=-3.0, rebate_value=0.0, inv=2, mid_end=1000100.0, mid_old=1000150.0),
        exp_mm_state=dict(bid_dist=0, ask_dist=0, inv=0, pnl=19999.0),
        exp_info=dict(posted_bid_price=1000000, posted_ask_price=1000300, bid_distance_from_best=0,
                      ask_distance_from_best=0, bid_quant=0, ask_quant=0, inventory=0, forced_unwind=0),
        exp_obs=[(0, 10), (400, 1e4)],
    ),
    # ---- step 48 of max 50: ep_done_time = (50 - 48 - 1) <= 1 (marl_env.py:717-718).  The agent
    # (inventory 5) holds two bids; getCancelMsgs (size 1) cancels only the first (slot 1,
    # 999800, oid -400), the one at 999700 (oid -401) stays.  Action 9: masked best bid 1000000
    # (own rows masked), ask 1000300 -> hs 200; rows [4, -1, 0, 1002300] -> zero row (id -1000),
    # [4, 1, 5, 998000] (id -1001).  Engine: the cancel clears slot 1; the IOC sell of 5 fills
    # bid 1000000 (q 2, tid 77) then 999900 (q 3, tid 78) -- the agent's own 999700 is behind them;
    # the data sell of 2 at 999700 then hits the agent's resting bid: a PASSIVE BUY (q = +2 >= 0,
    # passive tid = T), which leaves it q 1.  Trades:
    #   0 [1000000, 2, 601, -1001, 100, 5000, 77, T]   aggressive sell 2
    #   1 [999900, 3, 602, -1001, 100, 5000, 78, T]    aggressive sell 3
    #   2 [999700, 2, -401, 703, 101, 0, T, 88]        passive buy 2
    # Before the unwind: buys 2, sells 5 -> inventory 5 + 2 - 5 = 2 != 0, so the fictional trade
    # [mid 1000000 - 0, sign(2) * 2 = 2, -199, -198, 0, 0, -199, T] goes to row 3 (the first row
    # holding any -1); last mid = (999700 + 1000300) / 2 = 1000000.0.  It is a sell (q >= 0, agent
    # aggressor): sells 7, new inventory 0, forced_unwind 2.  With ref = mid 1000000:
    #   buyPnL  = (1000000 - 999700) / 100 * 2 = 6
    #   sellPnL = 0 * 2 + (999900 - 1000000) / 100 * 3 + 0 * 2 = -3
    #   rebate  = (999700 / 100 * 2) * 0.4e-4       (the passive buy only)
    #   InventoryPnL = 5 * (1000000.0 - 1000150.0) / 100 = -7.5 (old inventory)
    #   r = 6 - 3 + rebate + 0.1 * (-7.5 - max(0, 0.6 * -7.5))
    # income 20000 + 29997 + 20000, outgoing 19994.  The env then auto-resets: record and obs are
    # the reset's (window 0: asks [ASK0], bids [BID0], MM obs [0 / 10, 300 / 1e4]); reward and info
    # are the stepped ones (marl_env.py:787-803).
    "mm_passive_buy_aggressive_sell_unwind": dict(
        asks=[ASK0], bids=[[1000000, 2, 601, 77, 10, 0], [999800, 1, -400, T, 90, 0], [999700, 3, -401, T, 91, 0],
                           [999900, 3, 602, 78, 11, 0]],
        best_ask=[1000300, 50], best_bid=[1000000, 2], action=9, step=48, mm=dict(inv=5, total=2.0, cash=-49990.0),
        data=[[1, -1, 2, 999700, 703, 88, 101, 0], [1, -1, 7, 1000400, 702, 88, 101, 500]],
        exp_mm_rows=[(4, -1, 0, 1002300), (4, 1, 5, 998000)],
        exp_msgs=[[2, 1, 1, 999800, -400, T, 100, 5000], PAD_ASK] + EXE_PADS + zero_rows(-1000)
        + [[4, 1, 5, 998000, -1001, T, 100, 5000]] + zero_rows(-1002, -1003, -1004, -1005)
        + [[1, -1, 2, 999700, 703, 88, 101, 0], [1, -1, 7, 1000400, 702, 88, 101, 500]],
        exp_best_asks=[[1000300, 50]] * 14,
        exp_best_bids=[[1000000, 2]] * 7 + [[999700, 3]] * 5 + [[999700, 1]] * 2, exp_abort=0,
        exp_trades={0: [1000000, 2, 601, -1001, 100, 5000, 77, T], 1: [999900, 3, 602, -1001, 100, 5000, 78, T],
                    2: [999700, 2, -401, 703, 101, 0, T, 88]},
        exp_done=True,
        exp_reward=dict(buy=6.0, sell=-3.0, rebate_value=19994.0, inv=5, mid_end=1000000.0, mid_old=1000150.0),
        exp_unwind=[1000000, 2, -199, -198, 0, 0, -199, T], exp_unwind_row=3,
        exp_info=dict(inventory=0, forced_unwind=2, posted_bid_price=1000000, posted_ask_price=1000300,
                      bid_quant=0, ask_quant=0),
        exp_pnl_terms=dict(income=69997.0, outgoing=19994.0),
        exp_obs=[(0, 10), (300, 1e4)],             # the reset's
        exp_info_step=49,
    ),
}

# the init_states row of window 0 (LoadedEnvState): books, trades all -1, init time (50, 0),
# window 0, max_steps 50, start 0, step 0
INIT = dict(asks=[ASK0], bids=[BID0], loaded=(50, 0, 0, 50, 0, 0))
