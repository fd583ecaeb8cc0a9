"""The RCCL exchange on one GPU: a fresh child process with a one-rank "nccl" group runs
ShardedLogLik's all-gather + rank-order fold (blocking and pipelined) and loglik_scan, and
checks them bit-identical to the local partials (tests/rccl_one_rank.py); the bench's
--force-collective run gives the log-likelihood of the plain run."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1")
    return env


def test_one_rank_rccl_exchange(dev):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_one_rank.py")], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "RCCL_ONE_RANK_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_bench_force_collective_same_loglik(dev):
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5", "--cpu-seconds", "0",
            "--n", "200000"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    plain = subprocess.run(base, capture_output=True, text=True, timeout=240, env=env)
    forced = subprocess.run(base + ["--force-collective"], capture_output=True, text=True, timeout=240, env=env)
    assert plain.returncode == 0, plain.stderr[-3000:]
    assert forced.returncode == 0, forced.stderr[-3000:]
    a, b = json.loads(plain.stdout), json.loads(forced.stdout)
    assert a["loglik"] == b["loglik"]
    assert b["collective"].startswith("torch.distributed") and a["collective"].startswith("none")
