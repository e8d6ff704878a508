"""Config dataclasses, JSON/YAML I/O and the state-record layout (host only)."""
import dataclasses
import os

import pytest

from hftlob import config_io
from hftlob.config import Execution_EnvironmentConfig, MarketMaking_EnvironmentConfig, MultiAgentConfig
from hftlob.config_io import builtin_config
from hftlob.layout import EnvLayout, pack_env_cfg

BUILTIN = ["2_player_fq_fqc", "mm_debug_fixed_quant", "3_player_fq_fqc_dir", "exec_debug_fixed_quants_complex"]


@pytest.mark.parametrize("name", BUILTIN)
def test_builtin_configs_load_and_pack(name):
    cfg = builtin_config(name)
    c, L = pack_env_cfg(cfg, 12, 50_000, True)
    assert c.n_agents == sum(cfg.number_of_agents_per_type)
    assert L.n_msgs == cfg.world_config.n_data_msg_per_step + L.n_action_msgs + L.n_cancel_msgs
    assert c.rec_words % 4 == 0 and c.init_rec_words % 4 == 0
    assert L.off_bids == 6 * cfg.world_config.nOrders and L.off_trades == 12 * cfg.world_config.nOrders


def test_metric_config_shapes():
    # M = 100 + 4 + 8 = 112, MM 10 actions / 2 obs, EXE 13 actions / 12 obs
    cfg = builtin_config("2_player_fq_fqc")
    _, L = pack_env_cfg(cfg, 62, 400_000, True)
    assert (L.n_msgs, L.n_action_msgs, L.n_cancel_msgs) == (112, 6, 6)
    mm, ex = cfg.dict_of_agents_configs["MarketMaking"], cfg.dict_of_agents_configs["Execution"]
    assert (mm.n_actions, ex.n_actions) == (10, 13)
    assert L.obs_dims == [2, 12]


def test_three_agent_config():
    cfg = builtin_config("3_player_fq_fqc_dir")
    d = cfg.dict_of_agents_configs["Directional"]
    assert isinstance(d, MarketMaking_EnvironmentConfig)        # auto-detected (config_io.py:144-162)
    assert d.n_actions == 3 and d.action_space == "directional_trading"
    _, L = pack_env_cfg(cfg, 4, 10_000, True)
    assert L.n_msgs == 116


def test_post_init_derivations():
    assert MarketMaking_EnvironmentConfig(action_space="fixed_quants", tenth_action="NA").n_actions == 9
    assert Execution_EnvironmentConfig(action_space="fixed_quants_complex").num_messages_by_agent == 8
    with pytest.raises(ValueError):
        MarketMaking_EnvironmentConfig(action_space="fixed_quants", tenth_action="bogus")


@pytest.mark.parametrize("fmt", ["json", "yaml"])
def test_roundtrip(tmp_path, fmt):
    cfg = builtin_config("2_player_fq_fqc")
    p = str(tmp_path / f"c.{fmt}")
    if fmt == "json":
        config_io.save_config_to_file(cfg, p)
        back = config_io.load_config_from_file(p)
    else:
        config_io.save_config_to_yaml(cfg, p)
        back = config_io.load_config_from_yaml(p)
    assert back == cfg


@pytest.mark.parametrize("agent,changes,err", [
    ("MarketMaking", dict(action_space="fixed_prices"), NotImplementedError),   # reference NameError
    ("MarketMaking", dict(action_space="bogus"), ValueError),
    ("MarketMaking", dict(reward_function="bogus"), ValueError),
    ("MarketMaking", dict(unwind_price="near_touch"), ValueError),
    ("Execution", dict(action_space="fixed_quants"), NotImplementedError),   # reference unpack error
    ("Execution", dict(action_space="fixed_prices", n_actions=5), ValueError),   # 1..4 price levels only
    ("Execution", dict(action_space="fixed_quants_1msg", larger_far_touch_quant=True), NotImplementedError),
    ("Execution", dict(reference_price="near_touch"), ValueError),
])
def test_unsupported_options_fail_loudly(agent, changes, err):
    cfg = builtin_config("2_player_fq_fqc")
    agents = dict(cfg.dict_of_agents_configs)
    agents[agent] = dataclasses.replace(agents[agent], **changes)
    with pytest.raises(err):
        pack_env_cfg(dataclasses.replace(cfg, dict_of_agents_configs=agents), 4, 10_000, True)


def test_cancel_mode_values():
    cfg = builtin_config("2_player_fq_fqc")
    for mode in (0, 1, 2, 3):
        c = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, cancel_mode=mode))
        packed, _ = pack_env_cfg(c, 4, 10_000, False)
        assert packed.lob.cancel_mode == mode and packed.lob.prng_partitionable == 0 == packed.prng_partitionable
    cfg = dataclasses.replace(cfg, world_config=dataclasses.replace(cfg.world_config, cancel_mode=4))
    with pytest.raises(ValueError):
        pack_env_cfg(cfg, 4, 10_000, True)


REF_CFG_DIR = "/root/reference/config/env_configs"


@pytest.mark.skipif(not os.path.isdir(REF_CFG_DIR), reason="reference configs not mounted")
@pytest.mark.parametrize("fname", sorted(os.listdir(REF_CFG_DIR)) if os.path.isdir(REF_CFG_DIR) else [])
def test_reference_env_configs_pack(fname):
    """Every env config the reference ships loads with our loader and packs for the HIP path."""
    from hftlob.config_io import load_config_from_file
    cfg = load_config_from_file(os.path.join(REF_CFG_DIR, fname))
    c, L = pack_env_cfg(cfg, 4, 100_000, True)
    assert c.n_msgs == L.n_msgs and c.n_types == len(cfg.dict_of_agents_configs)
    assert c.action_words == sum(c.types[t].n_agents * c.types[t].action_width for t in range(c.n_types))


@pytest.mark.skipif(not os.path.isdir(REF_CFG_DIR), reason="reference configs not mounted")
def test_reference_env_config_fixture_is_current():
    """tests/golden/reference_env_configs.json (what the GPU run test steps) is the reference's
    config/env_configs as our loader reads them."""
    import json
    from dataclasses import asdict
    from hftlob.config_io import load_config_from_file
    with open(os.path.join(os.path.dirname(__file__), "golden", "reference_env_configs.json")) as f:
        fix = json.load(f)
    names = sorted(n for n in os.listdir(REF_CFG_DIR) if n.endswith(".json"))
    assert sorted(fix) == names
    for n in names:
        assert json.loads(json.dumps(asdict(load_config_from_file(os.path.join(REF_CFG_DIR, n))))) == fix[n], n
