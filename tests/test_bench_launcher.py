"""bench.py's launcher (CPU, no GPU work): `--gpus N` starts N ranks itself when
no launcher did, agrees with torch.distributed.run when one did, and refuses to
report an n_gpus that differs from the ranks actually running."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(PCADV_BENCH_BACKEND="gloo", **kw)
    return env


def _json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_spawns_n_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=REPO,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    j = _json(r.stdout)
    assert j["n_gpus"] == 2 and j["world_size"] == 2 and j["launcher"] == "bench.py spawn"


def test_bench_under_torchrun():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), "bench.py", "--gpus", "2", "--launch-check"], cwd=REPO,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    j = _json(r.stdout)
    assert j["n_gpus"] == 2 and j["launcher"] == "torch.distributed.run"


def test_bench_refuses_mismatched_world():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=REPO,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "refusing" in r.stderr
