"""Configuration dataclasses — the drop-in configuration surface.

Same class names, field names, defaults and ``__post_init__`` derivations as
``gymnax_exchange/jaxob/jaxob_config.py`` (``JAXLOB_Configuration`` :12-30,
``MarketMaking_EnvironmentConfig`` :33-141, ``Execution_EnvironmentConfig``
:144-200, ``World_EnvironmentConfig`` :205-223, ``MultiAgentConfig`` :228-250),
so JSON configs written for the reference load unchanged.  The objects are
frozen and hashable; the HIP path packs the fields it needs into a plain C
struct (``hftlob.layout.pack_env_cfg``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List

from . import constants as cst


def _set(obj, name, value):
    object.__setattr__(obj, name, value)


@dataclass(frozen=True)
class JAXLOB_Configuration:
    maxint: int = cst.MaxInt._64_Bit_Signed.value
    init_id: int = cst.INITID
    book_depth: int = 10
    cancel_mode: int = cst.CancelMode.INCLUDE_INITS.value
    type_4_interpretation: int = cst.Type4Interpretation.IOC.value
    seed: int = cst.SEED
    nTrades: int = cst.NTRADE_CAP
    nOrders: int = cst.NORDER_CAP
    simulator_mode: int = cst.SimulatorMode.GENERAL_EXCHANGE.value
    empty_slot_val: int = cst.EMPTY_SLOT
    debug_mode: bool = False
    check_book_fill: bool = True
    start_resolution: int = 6400
    alphatradePath: str = os.path.expanduser("~")
    dataPath: str = os.path.expanduser("~") + "/data"
    stock: str = "AMZN"
    timePeriod: str = "2024_Dec"


# (n_actions, num_messages_by_agent, num_action_messages_by_agent) per MM
# action space — jaxob_config.py:101-141.
_MM_BOB_ACTIONS = {1: 3, 2: 5, 5: 11, 10: 21}


@dataclass(frozen=True)
class MarketMaking_EnvironmentConfig:
    debug_mode: bool = False
    short_name: str = "MM"
    normalize: bool = True
    clip_reward: bool = False
    exclude_extreme_spreads: bool = False
    fixed_action_setting: bool = False
    fixed_action: int = 0
    simple_nothing_action: bool = True
    sell_buy_all_option: bool = False
    based_on_mid_price_of_action: bool = True
    tenth_action: str = "MarketOrder"
    bob_v0: int = 1
    action_space: str = "bobRL"
    observation_space: str = "engineered"
    reward_function: str = "spooner_asym_damped2"
    spread_multiplier: float = 3.0
    skew_multiplier: float = 5.0
    n_ticks_offset: int = 1
    fixed_quant_value: int = 10
    auto_liquidate_threshold: int = 10000
    auto_liquidate_alpha: float = 1.0
    unwind_price_penalty: int = 5
    inv_penalty: str = "none"
    volume_traded_bonus: str = "none"
    reference_price: str = "mid"
    unwind_price: str = "mid"
    inv_penalty_lambda: float = 1.0
    inv_penalty_quadratic_factor: float = 50.0
    inv_penalty_threshold: float = 10.0
    multiplier_type: str = "tick"
    reward_scaling_quo: float = 1.0
    inventoryPnL_eta: float = 0.6
    inventoryPnL_gamma: float = 0.5
    rebate_bps: float = 10.0
    unrealizedPnL_lambda: float = 0.1
    avst_k_parameter: float = 0.4
    avst_var_parameter: float = 1e-8
    time_delay_obs_act: int = 0
    n_actions: int = 10
    num_messages_by_agent: int = 4
    num_action_messages_by_agent: int = 2

    def __post_init__(self):
        a = self.action_space
        if a == "fixed_quants":
            if self.tenth_action == "NA":
                _set(self, "n_actions", 9)
            elif self.tenth_action == "MarketOrder":
                _set(self, "n_actions", 10)
            else:
                raise ValueError(f"Invalid tenth_action {self.tenth_action} for fixed_quants action space")
            _set(self, "num_messages_by_agent", 4)
            _set(self, "num_action_messages_by_agent", 2)
        elif a in ("spread_skew", "bobStrategy", "directional_trading", "AvSt"):
            _set(self, "n_actions", {"spread_skew": 6, "bobStrategy": 5,
                                     "directional_trading": 3, "AvSt": 8}[a])
            _set(self, "num_messages_by_agent", 4)
            _set(self, "num_action_messages_by_agent", 2)
        elif a == "bobRL":
            if self.bob_v0 not in _MM_BOB_ACTIONS:
                raise ValueError(f"Invalid bob_v0 {self.bob_v0} for bobRL action space")
            _set(self, "n_actions", _MM_BOB_ACTIONS[self.bob_v0])
            _set(self, "num_messages_by_agent", 4)
            _set(self, "num_action_messages_by_agent", 2)
        elif a == "fixed_prices":
            _set(self, "num_messages_by_agent", self.n_actions * 2)
            _set(self, "num_action_messages_by_agent", self.n_actions)


# exec action space -> (n_actions, msgs, action msgs); jaxob_config.py:180-200
_EXE_SPACES = {
    "fixed_quants": (5, 8, 4),
    "fixed_quants_complex": (13, 8, 4),
    "simplest_case": (3, 4, 2),
    "fixed_quants_1msg": (5, 2, 1),
    "twap": (1, 4, 2),
}


@dataclass(frozen=True)
class Execution_EnvironmentConfig:
    debug_mode: bool = False
    larger_far_touch_quant: bool = False
    normalize: bool = True
    short_name: str = "EXE"
    action_type: str = "pure"
    task: str = "random"
    action_space: str = "fixed_quants_complex"
    observation_space: str = "engineered"
    reward_function: str = "normal"
    task_size: int = 600
    n_ticks_in_book: int = 1
    fixed_quant_value: int = 10
    reward_lambda: float = 0.0
    reward_scaling_quo: float = 1.0
    doom_price_penalty: int = 5
    reference_price: str = "mid"
    time_delay_obs_act: int = 0
    n_actions: int = 5
    num_messages_by_agent: int = 8
    num_action_messages_by_agent: int = 4

    def __post_init__(self):
        if self.action_space in _EXE_SPACES:
            n, m, am = _EXE_SPACES[self.action_space]
            _set(self, "n_actions", n)
            _set(self, "num_messages_by_agent", m)
            _set(self, "num_action_messages_by_agent", am)
        elif self.action_space == "fixed_prices":
            _set(self, "num_messages_by_agent", self.n_actions * 2)
            _set(self, "num_action_messages_by_agent", self.n_actions)


@dataclass(frozen=True)
class World_EnvironmentConfig(JAXLOB_Configuration):
    n_data_msg_per_step: int = 1
    window_selector: int = -1
    ep_type: str = "fixed_steps"
    episode_time: int = 6400
    day_start: int = 34200
    day_end: int = 57600
    tick_size: int = 100
    trader_id_range_start: int = -100
    placeholder_order_id: int = -198
    artificial_trader_id_end_episode: int = -199
    artificial_order_id_end_episode: int = -199
    any_message_obs_space: bool = False
    order_id_counter_start_when_resetting: int = -200
    shuffle_action_messages: bool = True
    use_pickles_for_init: bool = True
    save_raw_observations: bool = False


@dataclass(frozen=True)
class MultiAgentConfig:
    world_config: World_EnvironmentConfig = field(default_factory=World_EnvironmentConfig)
    dict_of_agents_configs: Dict[str, object] = field(default_factory=lambda: {
        "MarketMaking": MarketMaking_EnvironmentConfig(),
        "Execution": Execution_EnvironmentConfig(),
    })
    number_of_agents_per_type: List[int] = field(default_factory=lambda: [1, 1])

    def __post_init__(self):
        for agent_cfg in self.dict_of_agents_configs.values():
            if "message" in agent_cfg.observation_space:
                _set(self.world_config, "any_message_obs_space", True)

    def __hash__(self):  # dict / list fields: hash the frozen pieces by identity of content
        return hash((self.world_config, tuple(self.dict_of_agents_configs.items()),
                     tuple(self.number_of_agents_per_type)))


CONFIG_OBJECT_DICT = {"MarketMaking": MarketMaking_EnvironmentConfig,
                      "Execution": Execution_EnvironmentConfig}
