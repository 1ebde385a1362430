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


# --- the C-ABI gather layout (ks_batch.hip: ks_batch_owner / ks_batch_block_len /
# ks_batch_unpack are the exact host functions ks_batch_load / ks_batch_gather use)
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c_abi_row_layout_every_graph_lands_in_order(world):
    """Every rank packs one block [status][rows] for the graphs it owns (as
    ks_batch_gather does); rank 0 receives the blocks in rank order and unpacks
    them: each graph's row must come back at its own index with its own content."""
    from ksched_amd import native
    ngraphs, max_tasks = 64, 5
    block = native.batch_block_len(ngraphs, world, max_tasks)
    slots = -(-ngraphs // world)
    assert block == 1 + slots * (2 + max_tasks)
    gathered = np.zeros(world * block, np.int64)
    owned = {r: [] for r in range(world)}
    for g in range(ngraphs):
        r, sl = native.batch_owner(g, world)
        assert r == g % world and sl == g // world     # round-robin
        owned[r].append(g)
        assert owned[r].index(g) == sl                 # slot = position among the rank's graphs
    for r, gs in owned.items():                        # each rank packs its own block
        for sl, g in enumerate(gs):
            row = r * block + 1 + sl * (2 + max_tasks)
            gathered[row] = 1000 + g                   # cost
            gathered[row + 1] = 2000 + g               # flow
            gathered[row + 2:row + 2 + max_tasks] = 10 * g + np.arange(max_tasks)
    pu, cost, flow = native.batch_unpack(gathered, ngraphs, world, max_tasks)
    assert cost.tolist() == [1000 + g for g in range(ngraphs)]
    assert flow.tolist() == [2000 + g for g in range(ngraphs)]
    for g in range(ngraphs):
        assert pu[g].tolist() == [10 * g + k for k in range(max_tasks)]


def test_c_abi_unpack_reports_a_failed_rank():
    from ksched_amd import native
    ngraphs, world, max_tasks = 8, 4, 3
    block = native.batch_block_len(ngraphs, world, max_tasks)
    gathered = np.zeros(world * block, np.int64)
    gathered[2 * block] = native.KS_E_INVALID          # rank 2's status word
    with pytest.raises(native.KsError) as e:
        native.batch_unpack(gathered, ngraphs, world, max_tasks)
    assert e.value.code == native.KS_E_INVALID


def test_c_abi_layout_matches_python_sharding():
    """The Python helpers (bench / torch.distributed path) and the C-ABI agree."""
    from ksched_amd import native
    for world in (1, 2, 4, 8):
        for g in range(64):
            assert native.batch_owner(g, world) == batch.owner(g, world)
        assert native.load().ks_batch_slots(64, world) == batch.slots_per_rank(64, world)


def test_gather_has_no_early_return_after_the_status_all_reduce():
    """VERDICT r4 item 5 (structure): between the status all-reduce and the end of
    the send/receive group, ks_batch_gather neither returns nor uses KB_HIP (which
    returns): a failing rank must never leave its peers waiting in ncclSend."""
    src = open(os.path.join(os.path.dirname(HERE), "ksched_amd", "csrc", "ks_batch.hip")).read()
    body = src[src.index("int ks_batch_gather("):]
    a = body.index("b->nccl->AllReduce(")
    g = body.index("const ncclResult_t ge = b->nccl->GroupEnd();", body.index("// 3. one group"))
    seg = body[a:g]
    # the only exits in between: the all-reduce's own error (after its GroupEnd) and
    # the agreed error of every rank (the all-reduce's result), both before any send
    exits = [ln.strip() for ln in seg.splitlines()
             if ("return" in ln or "KB_HIP" in ln) and not ln.strip().startswith("//")]
    assert not any("KB_HIP" in e for e in exits), exits
    send = seg.index("// 3. one group")
    assert all(seg.index(e) < send for e in exits), exits
    assert "hipMalloc" not in seg[send:] and "KB_TRY" not in seg[send:]


# --- tests/fake_comm: the world-2 rehearsal library checks the protocol it runs ---
def _fake_comm():
    """The fake communicator's entry points, from the TEST build of the library
    (libksmcmf_fakecomm.so; built here if missing). The shipped library must not
    contain them."""
    import ctypes as C
    from ksched_amd import _build
    lib = C.CDLL(_build.build_fake_comm())
    base = C.CDLL(_build.LIB)
    assert not hasattr(base, "ks_fake_ncclGroupEnd"), "the shipped library carries the fake communicator"

    class F:
        pass
    f = F()
    for name in ("CommInitAll", "GroupStart", "GroupEnd", "AllReduce", "Send", "Recv", "CommDestroy"):
        fn = getattr(lib, "ks_fake_nccl" + name)
        fn.restype = C.c_int
        setattr(f, "nccl" + name, fn)
    return C, f


NCCL_INVALID_USAGE = 5   # rccl.h ncclInvalidUsage
NCCL_INT64, NCCL_MIN = 4, 3


def test_fake_comm_refuses_a_one_sided_all_reduce():
    """A rank that skipped the status all-reduce would hang a real RCCL job; the
    fake communicator (tests/fake_comm, in the test build the world-2 GPU tests
    use) reports it as ncclInvalidUsage at GroupEnd instead — before any device
    call, so it runs here."""
    C, lib = _fake_comm()
    comms = (C.c_void_p * 2)()
    devs = (C.c_int * 2)(0, 0)
    assert lib.ncclCommInitAll(comms, 2, devs) == 0
    buf = C.c_void_p(0x1000)
    assert lib.ncclGroupStart() == 0
    assert lib.ncclAllReduce(buf, buf, 1, NCCL_INT64, NCCL_MIN, C.c_void_p(comms[0]), None) == 0
    assert lib.ncclGroupEnd() == NCCL_INVALID_USAGE
    # outside a group: refused (ks_batch always groups)
    assert lib.ncclAllReduce(buf, buf, 1, NCCL_INT64, NCCL_MIN, C.c_void_p(comms[0]), None) == NCCL_INVALID_USAGE
    for c in comms:
        assert lib.ncclCommDestroy(C.c_void_p(c)) == 0


def test_fake_comm_refuses_an_unmatched_send():
    C, lib = _fake_comm()
    comms = (C.c_void_p * 2)()
    assert lib.ncclCommInitAll(comms, 2, (C.c_int * 2)(0, 0)) == 0
    buf = C.c_void_p(0x1000)
    assert lib.ncclGroupStart() == 0
    assert lib.ncclSend(buf, 8, NCCL_INT64, 0, C.c_void_p(comms[1]), None) == 0   # rank 1 → 0, no receive posted
    assert lib.ncclGroupEnd() == NCCL_INVALID_USAGE
    assert lib.ncclGroupStart() == 0
    assert lib.ncclRecv(buf, 8, NCCL_INT64, 1, C.c_void_p(comms[0]), None) == 0   # a receive nobody sends
    assert lib.ncclGroupEnd() == NCCL_INVALID_USAGE
    for c in comms:
        assert lib.ncclCommDestroy(C.c_void_p(c)) == 0
