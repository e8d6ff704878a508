"""The kernels' divisions by the tick (hftlob.hip tick_floordiv: integer floor division by a
host-set multiplier; tick_ffloordiv: float floor division from the reciprocal with one exact
correction) restated in host C and checked bit for bit against the jnp.floor_divide formulas the
oracle uses (tools/magic_check.c, tools/ffloordiv_check.c; their quick samples here, the full
sweeps by hand: 0 mismatches in both)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
@pytest.mark.parametrize("src", ["magic_check.c", "ffloordiv_check.c"])
def test_tick_division_host_check(src, tmp_path):
    exe = tmp_path / src.replace(".c", "")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "tools", src), "-lm"],
                   check=True)
    out = subprocess.run([str(exe), "quick"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 or "mismatches: 0" in out.stdout, out.stdout
    assert "mismatches: 0" in out.stdout, out.stdout
