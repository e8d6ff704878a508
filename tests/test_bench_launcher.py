"""bench.py's multi-GPU entry point on the CPU: `--gpus N` outside torchrun starts N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set before anything touches the GPU);
`--dry-run` stops each rank before the GPU (gloo) and rank 0 prints the layout.  The ranks own
contiguous, disjoint env blocks of ONE Speed_test rollout over N * E envs (the reference's pmap
layout, ippo_rnn_JAXMARL_pmap.py:292-332)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*flags):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *flags], capture_output=True, text=True,
                       env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_n_launches_n_ranks(n):
    E = 4096
    out = _run("--gpus", str(n), "--dry-run")
    assert out["dry_run"] and out["n_gpus"] == n and out["num_envs_total"] == n * E
    ranks = out["ranks"]
    assert [r["rank"] for r in ranks] == list(range(n))
    # contiguous, disjoint, covering [0, n*E); reset keys are rows 1.. of split(PRNGKey(0), n*E + 1)
    assert [r["envs"] for r in ranks] == [[i * E, (i + 1) * E] for i in range(n)]
    assert [r["reset_key_rows"] for r in ranks] == [[1 + i * E, 1 + (i + 1) * E] for i in range(n)]
    assert all(r["key_e0"] == r["envs"][0] and r["key_n"] == n * E for r in ranks)


def test_failing_rank_fails_the_launch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--envs", "x"],
                       capture_output=True, text=True, env=env, timeout=120, cwd=ROOT)
    assert r.returncode != 0


def test_timed_window():
    """config.timed_window: the driver's 20-step window from the reset state never reaches the
    64-step episode's end (marl_env.py:711-718 fires at step counter 62); 128 steps cross two."""
    import bench
    assert "no episode end" in bench.timed_window(20, 64)
    assert "at timed step(s) [62, 125]" in bench.timed_window(128, 64)
    assert "at timed step(s) [62]" in bench.timed_window(63, 64)
    assert "no episode end" in bench.timed_window(62, 64)
