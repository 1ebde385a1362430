"""CPU suite, config 5 / multi-GPU path: round-robin sharding of independent
graphs and the post-solve gather of task→PU mappings (ksched_amd/batch.py),
rehearsed with world size 2 over gloo."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from ksched_amd import batch

HERE = os.path.dirname(os.path.abspath(__file__))


def test_assign_is_a_partition():
    for num in (1, 7, 64):
        for world in (1, 2, 4, 8):
            got = sorted(g for r in range(world) for g in batch.assign(num, world, r))
            assert got == list(range(num))
            for g in range(num):
                r, s = batch.owner(g, world)
                assert batch.assign(num, world, r)[s] == g
                assert s < batch.slots_per_rank(num, world)


def test_assign_rejects_bad_rank():
    with pytest.raises(ValueError):
        batch.assign(4, 2, 2)


def test_pack_pads_with_zero():
    b = batch.pack([np.array([5, 0, 7]), np.array([9])], 3, 4)
    assert b.tolist() == [[5, 0, 7, 0], [9, 0, 0, 0], [0, 0, 0, 0]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_gather(tmp_path):
    out = tmp_path / "res.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "gloo_batch_worker.py"), str(out)]
    subprocess.run(cmd, check=True, timeout=240, env=env, capture_output=True)
    res = json.loads(out.read_text())
    assert res["ok"] and res["world"] == 2
    assert res["shape"] == [7, 150] and res["scheduled"] > 0


def test_union_costs_split_per_graph():
    """The disjoint union's optimum is the sum of the parts' optima, and the
    per-part costs recovered from the union's flow records match each part."""
    from ksched_amd import gen
    from oracle import ko
    graphs = [gen.quincy(200, 20, 2, 4, 50 + i) for i in range(4)]
    u, noff, aoff = batch.union(graphs)
    assert (u.n, u.m) == (sum(g.n for g in graphs), sum(g.m for g in graphs))
    st, cost, flow, fl = ko.cost_scaling(u)
    assert st == 0
    parts = [ko.cost_scaling(g)[1] for g in graphs]
    assert cost == sum(parts)
    pos = np.nonzero(fl > 0)[0]
    rec = np.zeros(pos.shape[0], [("src", "<u8"), ("dst", "<u8"), ("flow", "<i8")])
    rec["src"], rec["dst"], rec["flow"] = u.src[pos], u.dst[pos], fl[pos]
    assert batch.split_costs(u, noff, rec).tolist() == parts
