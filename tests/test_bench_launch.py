"""bench.py's own rank launcher: `python bench.py --gpus N` with no WORLD_SIZE starts N ranks
itself (torch.distributed.run's environment, MASTER_ADDR 127.0.0.1), so the driver's plain invocation cannot
fail on launch.  CPU: the process group alone over gloo (--launch-check).  GPU: a short multi-rank bench
(ranks sharing cuda:0 over gloo on a 1-GPU box)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ, OMB_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_own_ranks(n):
    rc, lines, err = _run(["--gpus", str(n), "--launch-check", "--log2-cand", "10"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1                                   # one JSON line, from rank 0
    rec = json.loads(lines[0])
    assert rec["world_size"] == n and rec["backend"] == "gloo" and rec["ranks"] == list(range(n))
    assert rec["master_addr"] == "127.0.0.1"


@pytest.mark.gpu
def test_bench_two_ranks_on_device():
    rc, lines, err = _run(["--gpus", "2", "--log2-cand", "12", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                           "--no-kblock"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["distributed"]["world_size"] == 2
    assert rec["distributed"]["backend"] == "gloo"
    assert rec["config"]["global_batch"] == 2 * 4096 and rec["value"] > 0
    assert rec["best"]["index"] >= 0


def test_bench_help_renders():
    """Every option's help text formats (argparse %-expands it: a stray '%' broke `bench.py --help`)."""
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=240, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "--config" in p.stdout and "--timing-stride" in p.stdout
