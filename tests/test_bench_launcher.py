"""bench.py --gpus N without torch.distributed.run's environment starts the ranks itself
(a child `torch.distributed.run` process; no GPU touched before it) and returns the child's
exit status.  CPU only: --launch-probe ranks report their environment and exit."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.slow
def test_gpus_n_self_launches_n_ranks():
    r = _run("--gpus", "3", "--launch-probe")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert all(d["world"] == 3 and d["master"] == "127.0.0.1" for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1, 2]


@pytest.mark.slow
def test_child_failure_propagates_nonzero_status():
    r = _run("--gpus", "2", "--launch-probe", "--config", "no-such-config")
    assert r.returncode != 0


def test_emulate_flags_validated_before_any_gpu_call():
    r = _run("--emulate-world", "8", "--emulate-rank", "9")
    assert r.returncode == 2 and "emulate" in r.stderr
