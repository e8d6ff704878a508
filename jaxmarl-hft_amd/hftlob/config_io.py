"""JSON / YAML <-> ``MultiAgentConfig``.

Behaviour follows ``gymnax_exchange/jaxob/config_io.py``: missing fields take
the dataclass default (:84-124), agent types other than "MarketMaking" /
"Execution" are auto-detected by field overlap with ties going to the market
maker (:144-162; this is how a third "Directional" MM-type agent is declared),
and ``number_of_agents_per_type`` defaults to ``[1]`` (:72).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, fields
from typing import Any, Dict

from .config import (Execution_EnvironmentConfig, MarketMaking_EnvironmentConfig,
                     MultiAgentConfig, World_EnvironmentConfig)


def _fill(cls, d: Dict[str, Any]):
    default = cls()
    return cls(**{f.name: d.get(f.name, getattr(default, f.name)) for f in fields(cls)})


def _auto_detect(d: Dict[str, Any]):
    keys = set(d)
    mm = len(keys & {f.name for f in fields(MarketMaking_EnvironmentConfig)})
    ex = len(keys & {f.name for f in fields(Execution_EnvironmentConfig)})
    return _fill(MarketMaking_EnvironmentConfig if mm >= ex else Execution_EnvironmentConfig, d)


def dict_to_multiagent_config(d: Dict[str, Any]) -> MultiAgentConfig:
    world = _fill(World_EnvironmentConfig, d.get("world_config", {}))
    agents = {}
    for name, ad in d.get("dict_of_agents_configs", {}).items():
        if name == "MarketMaking":
            agents[name] = _fill(MarketMaking_EnvironmentConfig, ad)
        elif name == "Execution":
            agents[name] = _fill(Execution_EnvironmentConfig, ad)
        else:
            agents[name] = _auto_detect(ad)
    return MultiAgentConfig(world_config=world, dict_of_agents_configs=agents,
                            number_of_agents_per_type=list(d.get("number_of_agents_per_type", [1])))


def load_config_from_file(path: str) -> MultiAgentConfig:
    with open(path) as f:
        return dict_to_multiagent_config(json.load(f))


def save_config_to_file(config: MultiAgentConfig, path: str) -> None:
    if os.path.dirname(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(asdict(config), f, indent=2)


def load_config_from_yaml(path: str) -> MultiAgentConfig:
    import yaml
    with open(path) as f:
        return dict_to_multiagent_config(yaml.safe_load(f))


def save_config_to_yaml(config: MultiAgentConfig, path: str) -> None:
    import yaml
    if os.path.dirname(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(asdict(config), f, default_flow_style=False, indent=2)


# reference names
_dict_to_multiagent_config = dict_to_multiagent_config
_auto_detect_agent_config = _auto_detect

CONFIG_DIR = os.path.join(os.path.dirname(__file__), "configs")


def builtin_config(name: str) -> MultiAgentConfig:
    """Load one of the env configs shipped under ``hftlob/configs`` by file stem; ``"default"`` is
    ``MultiAgentConfig()`` itself (MM bobRL / engineered + EXE fixed_quants_complex, world defaults):
    the config Speed_test.py:101-113 times (its list_of_agents_configs attribute is not read by
    MARLEnv, which iterates dict_of_agents_configs, marl_env.py:71)."""
    if name == "default":
        return MultiAgentConfig()
    return load_config_from_file(os.path.join(CONFIG_DIR, name + ".json"))
