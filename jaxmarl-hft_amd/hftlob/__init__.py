"""hftlob — MI355X-native limit-order-book engine and multi-agent HFT env step.

Host package (PyTorch-ROCm tensors) over ``libhftlob.so`` (HIP, gfx950).
Drop-in names follow biiiipy/JaxMARL-HFT (``gymnax_exchange.jaxob`` /
``gymnax_exchange.jaxen``): config dataclasses, ``MARLEnv``, and the
engine operators ``scan_through_entire_array[_save_bidask]``.
"""
from .config import (JAXLOB_Configuration, MarketMaking_EnvironmentConfig, Execution_EnvironmentConfig,
                     World_EnvironmentConfig, MultiAgentConfig, CONFIG_OBJECT_DICT)
from .config_io import load_config_from_file, save_config_to_file, builtin_config

__all__ = ["JAXLOB_Configuration", "MarketMaking_EnvironmentConfig", "Execution_EnvironmentConfig",
           "World_EnvironmentConfig", "MultiAgentConfig", "CONFIG_OBJECT_DICT", "load_config_from_file",
           "save_config_to_file", "builtin_config"]
