"""GPU: bench.py's N > 1 path (two ranks, barrier/max timing, per-rank graphs,
post-solve mapping gather) rehearsed on one GPU with gloo collectives
(KS_BENCH_REHEARSAL=1); the real run uses RCCL with one GPU per rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("workload", ["full", "batch"])
def test_two_rank_bench_line(workload):
    env = dict(os.environ, KS_BENCH_REHEARSAL="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--workload", workload, "--steps", "1", "--warmup", "0", "--config", "config2", "--graphs", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                       # rank 0 prints the one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["cpu_baseline"] is None
    g = d["gather"]
    assert g is not None and g["scheduled"] > 0
    if workload == "batch":
        assert g["graphs"] == 4
