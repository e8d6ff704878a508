"""Writes tests/golden/reference_env_configs.json: every env config the reference ships
(config/env_configs/*.json), loaded through hftlob.config_io and re-serialised as our own
dataclass dicts (asdict), so the GPU tests can run each of them where /root/reference is absent.
Usage (in the build container): python tests/golden/make_reference_env_configs.py"""
import json
import os
import sys
from dataclasses import asdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "jaxmarl-hft_amd"))
from hftlob.config_io import load_config_from_file  # noqa: E402

SRC = "/root/reference/config/env_configs"
out = {f: asdict(load_config_from_file(os.path.join(SRC, f))) for f in sorted(os.listdir(SRC)) if f.endswith(".json")}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_env_configs.json"), "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)
print(len(out), "configs")
