"""Hand-derived golden vectors for one MARLEnv.step (fixtures, data only).

Like book_scenarios.py, every expected value here was reasoned BY HAND from the cited
reference lines (no jax here, and the reference ships no env-level outputs); the
derivation is written next to the values.  They pin the env layer above the engine:

  * _filter_messages pairing with two same-price cancels (exec_env.py:413-475, identical
    to mm_env.py:520-582): the k-th matching action row is netted against the k-th
    matching cancel row, whatever their order;
  * zero-quantity action rows become all-zero doNothing rows (mm_env.py:568-572) that
    still receive order ids (marl_env.py:285-290), then [cancels; actions; data]
    (marl_env.py:315);
  * _ffill_best_prices with row 0 empty and a side empty for the whole step
    (marl_env.py:723-749), and the abort flag taken before the fill (:360);
  * the auto-reset leafwise select (marl_env.py:798-803): state and obs from the reset,
    the info / obs_raw from the stepped state;
  * the EXE engineered observation's sorted-key order (exec_env.py:1946-1964,
    ravel_pytree sorts dict keys).

Config (golden_config in tests/test_env_goldens.py): exec_debug_fixed_quants_complex with
n_data_msg_per_step D = 2, shuffle_action_messages False, window_selector 0, EXE task
"sell", normalize False, cancel_mode 1 (no random cancel), time_delay_obs_act 0,
fixed_quant_value 10, n_ticks_in_book 1, tick 100, nOrders = nTrades = 100.  One EXE
agent with trader id -100; M = D + 8 = 10 messages per step.  Nothing here depends on the
step key: no shuffle, no random cancel, fixed task and window.

Pre-step record (unless a scenario says otherwise): world time (100, 5000), order-id
counter -1000, step_counter 3, max_steps 50, start_index 0, init time (50, 0), window 0;
EXE state init_price 1000050.0, task 600, executed 0, is_sell 1, p_vwap 10000.5, the
other floats 0.  The data rows of a step sit at start + D * step_counter (base_env.py:350).
Book rows are [price, qty, oid, tid, s, ns]; E = all -1.  Trade rows are
[price, qty (<0: buy aggressor), passive oid, aggressor oid, s, ns, passive tid, aggressor tid].

EXE engineered obs fields, sorted keys (fixed_steps): executed_quant, init_price,
is_sell_task, p_aggr, p_pass, q_aggr, q_pass, remaining_quant, remaining_ratio, spread,
step_counter, task_size.  q_aggr / q_pass are whole-side volumes (job.get_volume,
JaxOrderBookArrays.py:920-930); remaining_ratio = 1 - step / max_steps in float32.
"""
T = -100                        # the EXE agent's trader id
TIME, CNT = (100, 5000), -1000
DATA = [[1, 1, 5, 999900, 701, 88, 100, 9000],    # bid 5 @ 999900: never crosses
        [1, -1, 7, 1000300, 702, 88, 101, 0]]     # ask 7 @ 1000300: never crosses
PAD_ASK = [2, -1, 0, 0, 0, 0, 100, 5000]          # getCancelMsgs fill row (bookside[-1] = the appended zero row)
PAD_BID = [2, 1, 0, 0, 0, 0, 100, 5000]
ASK0 = [1000100, 30, 501, 77, 10, 0]
BID0 = [1000000, 40, 601, 77, 10, 0]


def act(side, q, p):
    """one raw action row of the agent (type 1, placeholder order id -198, time = world time + 0)"""
    return [1, side, q, p, -198, T, 100, 5000]


def ids(*zero_rows):
    """all-zero action rows that received order ids"""
    return [[0, 0, 0, 0, i, 0, 0, 0] for i in zero_rows]


SCENARIOS = {
    # Sell task, action 4 (PP): prices FT = best bid 1000000, M = ceil(((1000000+1000100)/2) // 100) * 100
    # = 1000000, NT = best ask 1000100, PP = 1000100 + 100 = 1000200 (exec_env.py:646-652);
    # quants [0, 0, 0, 10].  Cancels: the agent's two asks at 1000200 (oids -300, -301), then 2 fill rows.
    # Filter: a_mask = [F,F,F,T], c_mask = [T,T,F,F]; a = [10,0,0,0], c = [10,10,0,0], rel = [10,0,0,0];
    # rank_rev(a_mask) = [1,2,3,0] -> action q [0,0,0,10-10]; rank_rev(c_mask) = [0,1,2,3] ->
    # cancel q [10-10, 10, 0, 0].  Every action row has q 0 -> all-zero rows; ids -1000..-1003.
    # Book: c0 (q 0) leaves -300; c1 removes -301 (row 2 empties); fill rows cancel nothing
    # (oid 0 and price 0 match nothing -> slot -1 loses 0); zero rows: doNothing (type 0, side 0);
    # data bid -> bids row 1; data ask -> asks row 2 (first row holding a -1).  Best quotes never move.
    "filter_two_same_price_cancels": dict(
        asks=[ASK0, [1000200, 10, -300, T, 11, 0], [1000200, 10, -301, T, 12, 0]], bids=[BID0],
        best_ask=[1000100, 30], best_bid=[1000000, 40], action=4,
        raw_actions=[act(-1, 0, 1000000), act(-1, 0, 1000000), act(-1, 0, 1000100), act(-1, 10, 1000200)],
        raw_cancels=[[2, -1, 10, 1000200, -300, T, 100, 5000], [2, -1, 10, 1000200, -301, T, 100, 5000],
                     PAD_ASK, PAD_ASK],
        exp_msgs=[[2, -1, 0, 1000200, -300, T, 100, 5000], [2, -1, 10, 1000200, -301, T, 100, 5000],
                  PAD_ASK, PAD_ASK] + ids(-1000, -1001, -1002, -1003) + DATA,
        exp_best_asks=[[1000100, 30]] * 10, exp_best_bids=[[1000000, 40]] * 10, exp_abort=0,
        exp_asks={0: ASK0, 1: [1000200, 10, -300, T, 11, 0], 2: [1000300, 7, 702, 88, 101, 0]},
        exp_bids={0: BID0, 1: [999900, 5, 701, 88, 100, 9000]}, exp_trades={},
        exp_time=(101, 0), exp_counter=-1004, exp_step=4, exp_mid=1000050.0, exp_done=False,
        # executed, init_price, sell, p_aggr (bid), p_pass (ask), q_aggr 40+5, q_pass 30+10+7, remaining,
        # ratio 1-4/50, spread, step, task
        exp_obs_raw=[0, 1000050.0, 1, 1000000, 1000100, 45, 47, 600, ("ratio", 4, 50), 100, 4, 600],
    ),
    # Sell task, action 0 (no trade): prices [1000000, 1000100, 1000200, 1000300], all q 0.  The
    # agent's only ask (1000200) pairs with the NT row, but a = 0 -> rel = 0: cancel keeps q 10.
    # c0 empties the ask side: best ask [-1, sum of the 100 empty rows' q = -100] for messages 1-9;
    # the data ask (message 10) restores [1000300, 7].  abort = 1 (a -1 before the fill).  Fill:
    # row 0 -1 -> [last valid 1000200, 0]; q of -1 rows -> 0; prices forward-filled.
    "ffill_empty_ask_side": dict(
        asks=[[1000200, 10, -300, T, 11, 0]], bids=[BID0],
        best_ask=[1000200, 10], best_bid=[1000000, 40], action=0,
        raw_actions=[act(-1, 0, 1000000), act(-1, 0, 1000100), act(-1, 0, 1000200), act(-1, 0, 1000300)],
        raw_cancels=[[2, -1, 10, 1000200, -300, T, 100, 5000], PAD_ASK, PAD_ASK, PAD_ASK],
        exp_msgs=[[2, -1, 10, 1000200, -300, T, 100, 5000], PAD_ASK, PAD_ASK, PAD_ASK]
        + ids(-1000, -1001, -1002, -1003) + DATA,
        exp_best_asks=[[1000200, 0]] * 9 + [[1000300, 7]], exp_best_bids=[[1000000, 40]] * 10, exp_abort=1,
        exp_asks={0: [1000300, 7, 702, 88, 101, 0]},
        exp_bids={0: BID0, 1: [999900, 5, 701, 88, 100, 9000]}, exp_trades={},
        exp_time=(101, 0), exp_counter=-1004, exp_step=4, exp_mid=1000150.0, exp_done=False,
        exp_obs_raw=[0, 1000050.0, 1, 1000000, 1000300, 45, 7, 600, ("ratio", 4, 50), 300, 4, 600],
    ),
    # Buy task (is_sell 0 in the record), bid side empty all step, previous best bid 999000.
    # Action 1 (FT): buy prices FT = best ask 1000100, M = ((999000+1000100)//2//100)*100 = 999500,
    # NT = 999000, PP = 998900 (exec_env.py:639-645); quants [10,0,0,0].  Cancels: 4 bid fill rows
    # (side 1) -> price 0 never pairs (p_in_cnl needs p != 0 and equal prices).  Rows 2-4: zero rows.
    # a0 (id -1000) buys 10 of the 30 at 1000100: trade [1000100, -10, 501, -1000, 100, 5000, 77, -100],
    # nothing rests.  Data asks -> asks rows 1, 2.  Best bid [-1, -100] everywhere -> abort 1 and the fill
    # gives [999000, 0] for every row.  EXE executed 10 (|sum of agent trade q|, exec_env.py:1525-1526).
    "buy_cross_empty_bid_side": dict(
        asks=[ASK0], bids=[], best_ask=[1000100, 30], best_bid=[999000, 5], action=1, is_sell=0,
        data=[[1, -1, 5, 1000400, 701, 88, 100, 9000], [1, -1, 7, 1000300, 702, 88, 101, 0]],
        raw_actions=[act(1, 10, 1000100), act(1, 0, 999500), act(1, 0, 999000), act(1, 0, 998900)],
        raw_cancels=[PAD_BID] * 4,
        exp_msgs=[PAD_BID] * 4 + [[1, 1, 10, 1000100, -1000, T, 100, 5000]] + ids(-1001, -1002, -1003)
        + [[1, -1, 5, 1000400, 701, 88, 100, 9000], [1, -1, 7, 1000300, 702, 88, 101, 0]],
        exp_best_asks=[[1000100, 30]] * 4 + [[1000100, 20]] * 6, exp_best_bids=[[999000, 0]] * 10, exp_abort=1,
        exp_asks={0: [1000100, 20, 501, 77, 10, 0], 1: [1000400, 5, 701, 88, 100, 9000],
                  2: [1000300, 7, 702, 88, 101, 0]},
        exp_bids={}, exp_trades={0: [1000100, -10, 501, -1000, 100, 5000, 77, T]},
        exp_time=(101, 0), exp_counter=-1004, exp_step=4, exp_mid=999550.0, exp_done=False,
        # buy: p_aggr = best ask, p_pass = best bid, q_aggr = ask volume 20+5+7, q_pass = bid volume 0
        exp_obs_raw=[10, 1000050.0, 0, 1000100, 999000, 32, 0, 590, ("ratio", 4, 50), 1100, 4, 600],
    ),
    # step_counter 48 of 50: ep_done_time = (50 - 48 - 1) <= 1 (marl_env.py:753-754) -> __all__ done.
    # The stepped EXE state books the remaining 600 as a fictional doom trade (exec_env.py:1581-1586,
    # 1605-1606): executed 600, remaining 0, done.  MARLEnv.step then selects the RESET record and
    # obs (marl_env.py:798-803); info / obs_raw keep the stepped values (:684-685).  Reset of window 0
    # (the init row below; marl_env.py:129-175, exec_env.py:210-266): the init books, best quotes
    # [1000100, 30] / [1000000, 40] tiled over M rows, time = init time (50, 0), counter -200
    # (order_id_counter_start_when_resetting), mid 1000050.0, dt 0; EXE init_price = mid, task 600,
    # executed 0, is_sell 1 (task "sell"), p_vwap = mid / 100 = 10000.5.
    "auto_reset_select": dict(
        asks=[ASK0], bids=[BID0], best_ask=[1000100, 30], best_bid=[1000000, 40], action=0, step=48,
        exp_msgs=[PAD_ASK] * 4 + ids(-1000, -1001, -1002, -1003) + DATA,
        exp_done=True,
        # stepped obs_raw: q_aggr 40+5, q_pass 30+7; executed 600 / remaining 0 after the doom trade
        exp_obs_raw=[600, 1000050.0, 1, 1000000, 1000100, 45, 37, 0, ("ratio", 49, 50), 100, 49, 600],
        exp_obs=[0, 1000050.0, 1, 1000000, 1000100, 40, 30, 600, 1.0, 100, 0, 600],
        exp_reset=dict(asks={0: ASK0}, bids={0: BID0}, best_ask=[1000100, 30], best_bid=[1000000, 40],
                       time=(50, 0), counter=-200, mid=1000050.0, dt=0.0, step=0,
                       exe=dict(init_price=1000050.0, task=600, executed=0, is_sell=1, p_vwap=10000.5)),
        exp_info_step=49,
    ),
}

# the init_states row of window 0 (LoadedEnvState): books, trades all -1, init time (50, 0),
# window 0, max_steps 50, start 0, step 0
INIT = dict(asks=[ASK0], bids=[BID0], loaded=(50, 0, 0, 50, 0, 0))
