"""bench.py's launcher: ``--gpus N`` outside torchrun starts N ranks itself;
checked on CPU with gloo ranks timing an empty step (no GPU here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                          "--launch-selftest"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3


def test_bench_defaults_are_one_gpu():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse([])
    assert a.gpus == 1 and a.config == "C3" and a.steps >= 100
