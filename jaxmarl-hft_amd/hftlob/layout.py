"""Host mirror of ``include/hftlob.h``: ctypes structs, the per-env state
record layout, and packing of the configuration dataclasses into the C config.

The per-env record is one contiguous int32 row (floats bit-cast) so a single
wavefront loads / stores an environment with a handful of coalesced vector
accesses; named torch views over it reproduce the reference state pytrees
(``StatesandParams.py:14-74``: ``WorldState``, ``MMEnvState``,
``ExecEnvState``).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

from .config import (Execution_EnvironmentConfig, MarketMaking_EnvironmentConfig,
                     MultiAgentConfig)

MAX_TYPES = 4
MAX_AGENTS = 32
MAX_SLOTS = 256
MAX_MSGS = 256
MAX_OBS = 16
INFO_WORLD_WORDS = 14
INFO_AGENT_WORDS = 24

AGENT_MM, AGENT_EXE = 0, 1


class LobCfg(C.Structure):
    _fields_ = [("maxint", C.c_int32), ("init_id", C.c_int32), ("book_depth", C.c_int32),
                ("cancel_mode", C.c_int32), ("type_4_interpretation", C.c_int32),
                ("check_book_fill", C.c_int32), ("n_orders", C.c_int32), ("n_trades", C.c_int32),
                ("prng_partitionable", C.c_int32)]


class AgentTypeCfg(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "kind", "n_agents", "trader_id0", "n_actions", "n_msgs", "n_action_msgs", "obs_dim",
        "action_space", "observation_space", "reward_function", "normalize", "time_delay_obs_act",
        "fixed_quant_value", "tenth_action_market", "sell_buy_all_option", "fixed_action_setting",
        "fixed_action", "auto_liquidate_threshold", "unwind_price_penalty", "inv_penalty",
        "reference_price", "unwind_price", "clip_reward", "exclude_extreme_spreads",
        "volume_traded_bonus")] + [(n, C.c_float) for n in (
        "auto_liquidate_alpha", "inv_penalty_lambda", "inv_penalty_quadratic_factor",
        "inv_penalty_threshold", "reward_scaling_quo", "inventoryPnL_eta", "inventoryPnL_gamma",
        "rebate_bps", "unrealizedPnL_lambda")] + [
        ("task", C.c_int32), ("task_size", C.c_int32), ("n_ticks_in_book", C.c_int32),
        ("doom_price_penalty", C.c_int32), ("reward_lambda", C.c_float),
        ("rebate_factor", C.c_float), ("one_minus_eta", C.c_float),
        ("bob_v0", C.c_int32), ("n_ticks_offset", C.c_int32), ("simple_nothing_action", C.c_int32),
        ("multiplier_type", C.c_int32), ("spread_multiplier", C.c_float), ("skew_multiplier", C.c_float),
        ("avst_var", C.c_float), ("avst_k", C.c_float), ("avst_log_term", C.c_float * 8),
        ("doom_penalty_is_float", C.c_int32), ("doom_penalty_f32", C.c_float), ("action_width", C.c_int32)]


class EnvCfg(C.Structure):
    _fields_ = [("lob", LobCfg)] + [(n, C.c_int32) for n in (
        "n_data_msg", "n_msgs", "n_action_msgs", "n_cancel_msgs", "tick_size", "ep_type",
        "episode_time", "window_selector", "n_windows", "n_data_rows", "placeholder_order_id",
        "artificial_trader_id", "artificial_order_id", "order_id_counter_start",
        "shuffle_action_messages", "prng_partitionable", "n_types", "n_agents", "obs_stride",
        "rec_words", "init_rec_words", "off_asks", "off_bids", "off_trades", "off_loaded",
        "off_best_bids", "off_best_asks", "off_world", "off_agents", "info_words")] + [
        ("action_words", C.c_int32), ("tick_magic", C.c_uint32), ("types", AgentTypeCfg * MAX_TYPES)]


class StepOut(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("rewards", C.c_void_p), ("done_all", C.c_void_p),
                ("dones", C.c_void_p), ("info", C.c_void_p), ("obs_raw", C.c_void_p), ("msgs", C.c_void_p),
                ("debug", C.c_void_p)]


L2_LEVELS = 10                       # get_L2_state levels of world debug_mode (marl_env.py:646-651)


def debug_words(n_trades: int) -> int:
    """int32 words per env of the debug output: lob_state [10][4], then the trade log [nT][8]."""
    return 4 * L2_LEVELS + 8 * n_trades


# ----------------------------------------------------------- enum mappings
MM_ACTION = {"fixed_quants": 0, "directional_trading": 1, "bobRL": 2, "bobStrategy": 3, "AvSt": 4,
             "spread_skew": 5, "simple": 6}
AVST_GAMMA = (0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 20.0)       # mm_env.py:1283
MM_OBS = {"basic": 0, "engineered": 1, "messages": 2}
MM_REWARD = {"portfolio_value": 0, "buy_sell_pnl": 1, "complex": 2, "zero_inv": 3, "spooner": 4,
             "spooner_damped": 5, "spooner_asym_damped": 6, "spooner_asym_damped2": 7,
             "spooner_scaled": 8, "delta_portfolio_value": 9}
PRICE = {"mid": 0, "mid_avg": 1, "far_touch": 2, "near_touch": 3}
INV_PEN = {"none": 0, "linear": 1, "quadratic": 2, "threshold": 3, "exp4": 4}
EXE_ACTION = {"fixed_quants_complex": 0, "simplest_case": 1, "fixed_quants_1msg": 2, "twap": 3, "fixed_prices": 4}
EXE_OBS = {"engineered": 0, "basic": 1, "simplest_case": 2}
EXE_REWARD = {"normal": 0, "finish_fast": 1, "simplest_case": 2}
TASK = {"random": 0, "buy": 1, "sell": 2}

MM_WORDS = ("posted_distance_bid", "posted_distance_ask", "inventory", "total_PnL", "cash_balance")
MM_FLOAT = {"total_PnL", "cash_balance"}
EXE_WORDS = ("init_price", "task_to_execute", "quant_executed", "is_sell_task", "p_vwap",
             "total_revenue", "drift_return", "advantage_return", "slippage_rm", "price_adv_rm",
             "price_drift_rm", "vwap_rm", "trade_duration")
EXE_FLOAT = set(EXE_WORDS) - {"task_to_execute", "quant_executed", "is_sell_task"}

# info buffer field maps (name, is_float)
INFO_WORLD = (("window_index", 0), ("end_mid_price", 1), ("step_counter", 0), ("time_s", 0),
              ("time_ns", 0), ("order_id_counter", 0), ("best_asks", 0), ("best_bids", 0),
              ("average_best_ask", 1), ("average_best_bid", 1), ("delta_time", 1),
              ("ep_done_time", 0), ("abort_episode", 0), ("spread", 0))
INFO_MM = (("reward", 1), ("reward_portfolio_value", 1), ("reward_spooner", 1), ("end_of_ep_pv", 1),
           ("reward_spooner_damped", 1), ("reward_spooner_asym_damped", 1),
           ("reward_spooner_asym_damped2", 1), ("reward_delta_pv", 1), ("total_PnL", 1), ("done", 0),
           ("inventory", 0), ("delta_mid_price", 1), ("market_share", 1), ("buyPnL", 1),
           ("forced_unwind", 0), ("invPnL", 1), ("posted_bid_price", 0), ("posted_ask_price", 0),
           ("bid_distance_from_best", 0), ("ask_distance_from_best", 0), ("ask_quant", 0),
           ("bid_quant", 0), ("sellPnL", 1), ("inventoryValue", 1))
INFO_EXE = (("quant_left", 0), ("done", 0), ("revenue_direction_normalised", 1), ("vwap_rm", 1),
            ("drift", 1), ("advantage", 1), ("doom_quant", 0), ("is_sell_task", 0), ("reward", 1))


def _r4(x: int) -> int:
    return (x + 3) // 4 * 4


EP_TYPE = {"fixed_steps": 0, "fixed_time": 1}


def obs_dim(agent_cfg, world) -> int:
    """observation_space() widths: mm_env.py:3195-3200 (basic 2; engineered 8 fixed_steps, 10 fixed_time);
    exec_env.py:2185-2200 (engineered: 12 fixed_steps, 15 fixed_time).  The MM "messages" space
    (mm_env.py:2820-2821) is the step's int32 [M, 8] message array, not a float row: 0 here
    (its values come from the kernel's msgs output)."""
    if world.ep_type not in EP_TYPE:
        raise ValueError(f"ep_type {world.ep_type!r}: use 'fixed_steps' or 'fixed_time'")
    if isinstance(agent_cfg, MarketMaking_EnvironmentConfig):
        return {"basic": 2, "engineered": 8 if world.ep_type == "fixed_steps" else 10,
                "messages": 0}[agent_cfg.observation_space]
    return {"engineered": 12 if world.ep_type == "fixed_steps" else 15, "basic": 3,
            "simplest_case": 3}[agent_cfg.observation_space]


# get_observation(normalize=False, flatten=False) field names and dtypes ("i" int32, "f" float32), in
# the sorted-key order of the flattened obs: the save_raw_observations info (marl_env.py:684-685)
OBS_FIELDS = {
    ("MM", "basic"): (("inventory", "i"), ("spread", "i")),                     # mm_env.py:2963-3000
    ("MM", "engineered", "fixed_steps"): (("inventory", "i"), ("mid_price", "f"), ("p_ask", "i"), ("p_bid", "i"),
                                          ("q_ask", "i"), ("q_bid", "i"), ("spread", "i"), ("step_counter", "i")),
    ("MM", "engineered", "fixed_time"): (("delta_time", "f"), ("inventory", "i"), ("mid_price", "f"), ("p_ask", "i"),
                                         ("p_bid", "i"), ("q_ask", "i"), ("q_bid", "i"), ("spread", "i"),
                                         ("step_counter", "i"), ("time_remaining", "f")),   # mm_env.py:3004-3154
    ("EXE", "basic"): (("best_ask_price", "i"), ("best_bid_price", "i"), ("remaining_quant", "i")),
    ("EXE", "simplest_case"): (("mid_price", "f"), ("percent_remaining_quant", "f"), ("percent_time_remaining", "f")),
    ("EXE", "engineered", "fixed_steps"): (("executed_quant", "i"), ("init_price", "f"), ("is_sell_task", "i"),
                                           ("p_aggr", "i"), ("p_pass", "i"), ("q_aggr", "i"), ("q_pass", "i"),
                                           ("remaining_quant", "i"), ("remaining_ratio", "f"), ("spread", "i"),
                                           ("step_counter", "i"), ("task_size", "i")),
    ("EXE", "engineered", "fixed_time"): (("delta_time", "f"), ("executed_quant", "i"), ("init_price", "f"),
                                          ("is_sell_task", "i"), ("p_aggr", "i"), ("p_pass", "i"), ("q_aggr", "i"),
                                          ("q_pass", "i"), ("remaining_quant", "i"), ("remaining_ratio", "f"),
                                          ("spread", "i"), ("step_counter", "i"), ("task_size", "i"), ("time", "f"),
                                          ("time_remaining", "f")),              # exec_env.py:1913-2079
}


def obs_fields(agent_cfg, world):
    """(name, dtype) of the raw observation dict of one agent type (sorted keys), or None for "messages"."""
    kind = "MM" if isinstance(agent_cfg, MarketMaking_EnvironmentConfig) else "EXE"
    space = agent_cfg.observation_space
    if space == "messages":
        return None
    return OBS_FIELDS.get((kind, space)) or OBS_FIELDS[(kind, space, world.ep_type)]


@dataclass
class EnvLayout:
    """Record offsets (int32 words) + derived message counts for one config."""
    n_orders: int
    n_trades: int
    n_msgs: int
    n_data_msg: int
    n_action_msgs: int
    n_cancel_msgs: int
    agent_kinds: List[int]          # per agent
    agent_types: List[int]          # type index per agent
    obs_dims: List[int]             # per type
    obs_stride: int
    off_asks: int = 0
    off_bids: int = 0
    off_trades: int = 0
    off_loaded: int = 0
    init_rec_words: int = 0
    off_best_bids: int = 0
    off_best_asks: int = 0
    off_world: int = 0
    off_agents: int = 0
    rec_words: int = 0
    agent_offsets: List[int] = field(default_factory=list)
    info_words: int = 0

    @staticmethod
    def build(cfg: MultiAgentConfig) -> "EnvLayout":
        w = cfg.world_config
        types = list(cfg.dict_of_agents_configs.values())
        counts = list(cfg.number_of_agents_per_type)
        if len(counts) != len(types):
            raise ValueError("number_of_agents_per_type must list one count per agent type")
        D = w.n_data_msg_per_step
        A = sum(t.num_action_messages_by_agent * n for t, n in zip(types, counts))
        M = D + sum(t.num_messages_by_agent * n for t, n in zip(types, counts))
        kinds, tix = [], []
        for i, (t, n) in enumerate(zip(types, counts)):
            k = AGENT_MM if isinstance(t, MarketMaking_EnvironmentConfig) else AGENT_EXE
            kinds += [k] * n
            tix += [i] * n
        dims = [obs_dim(t, w) for t in types]
        L = EnvLayout(n_orders=w.nOrders, n_trades=w.nTrades, n_msgs=M, n_data_msg=D, n_action_msgs=A,
                      n_cancel_msgs=M - D - A, agent_kinds=kinds, agent_types=tix, obs_dims=dims,
                      obs_stride=max(1, max(dims)))
        nO, nT = w.nOrders, w.nTrades
        L.off_asks, L.off_bids, L.off_trades = 0, 6 * nO, 12 * nO
        L.off_loaded = 12 * nO + 8 * nT
        L.init_rec_words = _r4(L.off_loaded + 6)
        L.off_best_bids = L.init_rec_words
        L.off_best_asks = L.off_best_bids + 2 * M
        L.off_world = L.off_best_asks + 2 * M
        off = _r4(L.off_world + 5)
        L.off_agents = off
        for k in kinds:
            L.agent_offsets.append(off)
            off += 5 if k == AGENT_MM else 13
        L.rec_words = _r4(off)
        L.info_words = INFO_WORLD_WORDS + INFO_AGENT_WORDS * len(kinds)
        return L


def _f(x) -> float:
    """A Python scalar as the weak-typed f32 JAX would use."""
    return float(x)


def action_width(agent_cfg) -> int:
    """int32 words of one agent's action: n_actions for the EXE fixed_prices
    MultiDiscrete space (exec_env.py:2167-2171), 1 for every Discrete space."""
    if isinstance(agent_cfg, Execution_EnvironmentConfig) and agent_cfg.action_space == "fixed_prices":
        return int(agent_cfg.n_actions)
    return 1


def pack_agent_type(t, n_agents: int, trader_id0: int, world) -> AgentTypeCfg:
    a = AgentTypeCfg()
    a.n_agents, a.trader_id0 = n_agents, trader_id0
    a.n_actions, a.n_msgs, a.n_action_msgs = t.n_actions, t.num_messages_by_agent, t.num_action_messages_by_agent
    a.obs_dim = obs_dim(t, world)
    a.normalize, a.time_delay_obs_act, a.fixed_quant_value = int(t.normalize), t.time_delay_obs_act, t.fixed_quant_value
    a.reward_scaling_quo = _f(t.reward_scaling_quo)
    a.action_width = action_width(t)
    if isinstance(t, MarketMaking_EnvironmentConfig):
        a.kind = AGENT_MM
        if t.action_space == "fixed_prices":
            raise NotImplementedError("MM action_space 'fixed_prices': the reference's _getActionMsgs_fixedPrice "
                                      "reads an undefined `state` (mm_env.py:1625, NameError at trace time)")
        if t.action_space not in MM_ACTION:
            raise ValueError("Invalid action_space specified.")
        if t.observation_space not in MM_OBS:
            raise NotImplementedError(f"MM observation_space {t.observation_space!r} not implemented (the "
                                      "'messages_new_tokenizer' space needs the LOB foundation model's tokenizer "
                                      "config, get_config() of the absent lobgen package, mm_env.py:2824-2960)")
        if t.reward_function not in MM_REWARD:
            raise ValueError("Invalid reward_space specified.")
        if t.inv_penalty not in INV_PEN:
            raise NotImplementedError(f"inv_penalty {t.inv_penalty!r} not implemented")
        if t.action_space == "spread_skew" and t.multiplier_type not in ("tick", "spread"):
            raise ValueError(f"multiplier_type {t.multiplier_type!r}")
        if t.unwind_price not in ("mid", "mid_avg", "far_touch"):
            raise ValueError("Invalid unwind price type.")
        a.action_space, a.observation_space = MM_ACTION[t.action_space], MM_OBS[t.observation_space]
        a.reward_function, a.inv_penalty = MM_REWARD[t.reward_function], INV_PEN[t.inv_penalty]
        a.reference_price, a.unwind_price = PRICE[t.reference_price], PRICE[t.unwind_price]
        a.tenth_action_market = int(t.tenth_action == "MarketOrder")
        a.sell_buy_all_option = int(t.sell_buy_all_option)
        a.fixed_action_setting, a.fixed_action = int(t.fixed_action_setting), t.fixed_action
        a.auto_liquidate_threshold, a.unwind_price_penalty = t.auto_liquidate_threshold, t.unwind_price_penalty
        a.clip_reward, a.exclude_extreme_spreads = int(t.clip_reward), int(t.exclude_extreme_spreads)
        a.volume_traded_bonus = int(t.volume_traded_bonus == "market_share")
        a.auto_liquidate_alpha = _f(t.auto_liquidate_alpha)
        a.inv_penalty_lambda = _f(t.inv_penalty_lambda)
        a.inv_penalty_quadratic_factor = _f(t.inv_penalty_quadratic_factor)
        a.inv_penalty_threshold = _f(t.inv_penalty_threshold)
        a.inventoryPnL_eta, a.inventoryPnL_gamma = _f(t.inventoryPnL_eta), _f(t.inventoryPnL_gamma)
        a.rebate_bps, a.unrealizedPnL_lambda = _f(t.rebate_bps), _f(t.unrealizedPnL_lambda)
        a.rebate_factor = _f(t.rebate_bps / 10_000)          # formed in Python double (mm_env.py:2369)
        a.one_minus_eta = _f(1 - t.inventoryPnL_eta)          # mm_env.py:2434
        a.bob_v0, a.n_ticks_offset = t.bob_v0, t.n_ticks_offset
        a.simple_nothing_action = int(t.simple_nothing_action)
        a.multiplier_type = int(t.multiplier_type == "spread")
        a.spread_multiplier, a.skew_multiplier = _f(t.spread_multiplier), _f(t.skew_multiplier)
        a.avst_var, a.avst_k = _f(t.avst_var_parameter), _f(t.avst_k_parameter)
        for i, g in enumerate(AVST_GAMMA):                    # f32 gamma / f32 k, + 1 in f32, log rounded once
            q = np.float32(np.float32(g) / np.float32(t.avst_k_parameter))
            a.avst_log_term[i] = float(np.float32(math.log(float(np.float32(np.float32(1.0) + q)))))
    else:
        a.kind = AGENT_EXE
        if t.action_space == "fixed_quants":
            raise NotImplementedError("EXE action_space 'fixed_quants': the reference's _getActionMsgs_fixedQuant "
                                      "returns a bare array that get_messages unpacks into two values "
                                      "(exec_env.py:727,1239-1244)")
        if t.action_space == "fixed_prices" and t.n_actions not in (1, 2, 3, 4):
            raise ValueError(f"EXE fixed_prices n_actions={t.n_actions}: the price-level functions "
                             "return 1..4 levels (exec_env.py:1042-1076)")
        if t.action_space not in EXE_ACTION:
            raise ValueError("Invalid action_space specified.")
        if t.action_space == "fixed_quants_1msg" and t.larger_far_touch_quant:
            raise NotImplementedError("fixed_quants_1msg with larger_far_touch_quant: Python `and` on a traced "
                                      "action in the reference (exec_env.py:801)")
        if t.action_space == "twap" and world.ep_type != "fixed_steps":
            raise NotImplementedError("TWAP not implemented for fixed time episodes (exec_env.py:1141-1142)")
        if t.observation_space not in EXE_OBS:
            raise NotImplementedError(f"EXE observation_space {t.observation_space!r} not implemented")
        if t.reward_function not in EXE_REWARD:
            raise NotImplementedError(f"EXE reward_function {t.reward_function!r} not implemented")
        if t.reference_price not in ("mid", "far_touch"):
            raise ValueError("Invalid reference price type.")
        a.action_space, a.observation_space = EXE_ACTION[t.action_space], EXE_OBS[t.observation_space]
        a.reward_function, a.reference_price = EXE_REWARD[t.reward_function], PRICE[t.reference_price]
        if t.task not in TASK:
            raise ValueError(f"invalid task {t.task!r}")
        a.task, a.task_size, a.n_ticks_in_book = TASK[t.task], t.task_size, t.n_ticks_in_book
        a.reward_lambda = _f(t.reward_lambda)
        pen = t.doom_price_penalty
        if isinstance(pen, float) and not pen.is_integer():
            a.doom_penalty_is_float, a.doom_penalty_f32 = 1, _f(pen * world.tick_size)
        else:
            a.doom_price_penalty = int(pen)
            a.doom_penalty_f32 = _f(int(pen) * world.tick_size)
    return a


def pack_lob_cfg(w, prng_partitionable: bool = True) -> LobCfg:
    if w.simulator_mode != 0:
        raise NotImplementedError("simulator_mode LOBSTER_INTERPRETER is not implemented (reference: NotImplementedError)")
    if w.cancel_mode not in (0, 1, 2, 3):
        raise ValueError(f"cancel_mode {w.cancel_mode} (jaxob_constants.CancelMode has 0..3)")
    if w.book_depth < 0 or w.init_id - 2 * w.book_depth < -2**31:
        raise ValueError("book_depth must be >= 0 and init_id - 2 * book_depth must fit in int32 "
                         "(the init-order id range of get_init_id_match, JaxOrderBookArrays.py:120-139)")
    c = LobCfg()
    c.maxint, c.init_id, c.book_depth = w.maxint, w.init_id, w.book_depth
    c.cancel_mode, c.type_4_interpretation = w.cancel_mode, w.type_4_interpretation
    c.check_book_fill, c.n_orders, c.n_trades = int(w.check_book_fill), w.nOrders, w.nTrades
    c.prng_partitionable = int(prng_partitionable)
    return c


def pack_env_cfg(cfg: MultiAgentConfig, n_windows: int, n_data_rows: int,
                 prng_partitionable: bool = True) -> Tuple[EnvCfg, EnvLayout]:
    w = cfg.world_config
    L = EnvLayout.build(cfg)
    if len(cfg.dict_of_agents_configs) > MAX_TYPES or len(L.agent_kinds) > MAX_AGENTS:
        raise ValueError("too many agent types / agents")
    c = EnvCfg()
    c.lob = pack_lob_cfg(w, prng_partitionable)
    c.n_data_msg, c.n_msgs, c.n_action_msgs, c.n_cancel_msgs = L.n_data_msg, L.n_msgs, L.n_action_msgs, L.n_cancel_msgs
    c.tick_size, c.ep_type, c.episode_time = w.tick_size, EP_TYPE[w.ep_type], w.episode_time
    c.window_selector, c.n_windows, c.n_data_rows = w.window_selector, n_windows, n_data_rows
    c.placeholder_order_id = w.placeholder_order_id
    c.artificial_trader_id, c.artificial_order_id = w.artificial_trader_id_end_episode, w.artificial_order_id_end_episode
    c.order_id_counter_start = w.order_id_counter_start_when_resetting
    c.shuffle_action_messages, c.prng_partitionable = int(w.shuffle_action_messages), int(prng_partitionable)
    c.n_types, c.n_agents, c.obs_stride = len(cfg.dict_of_agents_configs), len(L.agent_kinds), L.obs_stride
    c.action_words = sum(action_width(t) * n for t, n in zip(cfg.dict_of_agents_configs.values(),
                                                             cfg.number_of_agents_per_type))
    for name in ("rec_words", "init_rec_words", "off_asks", "off_bids", "off_trades", "off_loaded",
                 "off_best_bids", "off_best_asks", "off_world", "off_agents", "info_words"):
        setattr(c, name, getattr(L, name))
    tid = w.trader_id_range_start                    # marl_env.py:103-115, mm_env.py:189-202
    for i, (t, n) in enumerate(zip(cfg.dict_of_agents_configs.values(), cfg.number_of_agents_per_type)):
        c.types[i] = pack_agent_type(t, n, tid, w)
        tid -= n
    return c, L


def trader_ids(cfg: MultiAgentConfig) -> List[List[int]]:
    out, tid = [], cfg.world_config.trader_id_range_start
    for n in cfg.number_of_agents_per_type:
        out.append(list(range(tid, tid - n, -1)))
        tid -= n
    return out
