"""World 2 through the REAL ks_batch_gather on one GPU.

The driver's round-end node is where RCCL runs at world > 1; until then the
gather's world > 1 path — the status all-reduce, the send/receive group, the
status protocol of fault_inject bits 2 and 3 — would only ever have run at world 1
(where no collective is made). Here the TEST build of the library,
libksmcmf_fakecomm.so (-DKS_FAKE_COMM: tests/fake_comm/fake_nccl.cpp compiled in
place of RCCL; _build.build_fake_comm), runs ks_batch_create(devices=[0, 0]): two
ranks of one process on device 0. The fake communicator checks the protocol as it
runs it:
an all-reduce must be posted by every rank, and every receive must meet a send of
the same size (else ncclInvalidUsage — what would be a hang on RCCL). The RCCL
path itself stays unmeasured on hardware here."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import load_goldens
from ksched_amd import _build, gen, native
from test_gpu_parity import check_mapping

pytestmark = pytest.mark.gpu


FAKE = _build.FAKE_COMM_TAG


@pytest.fixture
def fake_comm():
    if not os.path.exists(_build.variant_path(FAKE)):
        pytest.fail("ksched_amd/libksmcmf_fakecomm.so is not built (__graft_entry__.build())")
    lib = native.load(variant=FAKE)

    def stats():
        out = (C.c_longlong * 4)()
        lib.ks_fake_nccl_stats(out)
        return list(out)        # [all-reduces, sends, receives, groups]
    return stats


def _graphs(k):
    T, M, R, J, _ = gen.CONFIGS["config2"]
    gold = {e["seed"]: e for e in load_goldens() if e["params"] == [T, M, R, J]}
    seeds = list(range(1000, 1000 + k))
    return T, [gen.quincy(T, M, R, J, s) for s in seeds], [gold[s] for s in seeds]


def test_world2_gather_matches_goldens(fake_comm):
    """Eight config-2 cells over two ranks (graph g on rank g mod 2, each rank's four
    cells in one cell-solver launch): rank 1's rows travel by the group's send /
    receive, and every cost, flow and task row on rank 0 equals the golden."""
    T, graphs, gold = _graphs(8)
    s0 = fake_comm()
    b = native.Batch(devices=[0, 0], variant=FAKE)
    try:
        b.load(graphs)
        res = b.solve()
        assert len(res) == 2
        assert all(r.raw["solver"] == 1 and r.raw["cells"] == 4 for r in res)
        pu, cost, flow = b.gather(T)
        assert cost.tolist() == [e["cost"] for e in gold]
        assert flow.tolist() == [e["flow"] for e in gold]
        for i in (0, 1, 6, 7):                     # rows of both ranks: valid task → PU maps
            g = graphs[i]
            tasks = np.nonzero(g.ntype == 1)[0] + 1
            mp = {int(t): int(p) for t, p in zip(tasks, pu[i]) if p}
            assert len(mp) > 0.9 * T
            check_mapping(g, mp)
        s1 = fake_comm()
        # one status all-reduce, one block from rank 1 to rank 0, two groups
        assert [a - b for a, b in zip(s1, s0)] == [1, 1, 1, 2]
        pu2, cost2, _ = b.gather(T)                # a second gather reuses the buffers
        assert cost2.tolist() == cost.tolist() and np.array_equal(pu2, pu)
    finally:
        b.close()


@pytest.mark.parametrize("fault,msg", [(4, "injected pack failure"), (8, "injected root buffer allocation failure")])
def test_world2_gather_failure_reaches_both_ranks(fake_comm, fault, msg):
    """fault_inject bit 2 (rank 0's packing fails) and bit 3 (rank 0's receive
    buffer cannot be allocated) at world 2: both ranks still enter the status
    all-reduce (the fake library would refuse a one-sided one), every rank learns
    the failure from it, and the send/receive group is never entered."""
    T, graphs, _ = _graphs(4)
    s0 = fake_comm()
    b = native.Batch(devices=[0, 0], variant=FAKE, fault_inject=fault)
    try:
        b.load(graphs)
        b.solve()
        with pytest.raises(native.KsError) as e:
            b.gather(T)
        assert e.value.code == native.KS_E_DEVICE
        assert msg in str(e.value)
        s1 = fake_comm()
        assert [a - b for a, b in zip(s1, s0)] == [1, 0, 0, 1]   # the all-reduce ran, no send / receive
    finally:
        b.close()
