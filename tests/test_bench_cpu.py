"""CPU tests of bench.py's launch logic: `--gpus N` without a launcher spawns N worker processes that
rendezvous over gloo (127.0.0.1) and reduce max-over-ranks; rank 0's line is the only stdout output."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.parametrize("world", [2, 3])
def test_bench_spawns_ranks(world):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--launch-check"],
                         capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == world
    assert res["launch_check"] == {"world": world, "max_rank": world - 1, "local_rank": 0}


def test_bench_cli_defaults():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse_args([])
    assert a.gpus == 1 and a.sigma == 4 and a.text_bytes == 1 << 30 and not a.strong
    assert a.strong_bytes == 1 << 32
