"""One rank of the world-size-2 gloo rehearsal of the config-5 batch path
(launched by tests/test_batch_cpu.py through torch.distributed.run).

Each rank takes its round-robin share of small cell graphs, computes their
task→PU vectors with the CPU oracle (test infrastructure standing in for the
GPU solve), packs them and all-gathers over gloo with ksched_amd.batch; rank 0
checks the gathered block against every graph's expected vector."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from graphs import flow_mapping  # noqa: E402
from ksched_amd import batch, gen  # noqa: E402
from oracle import ko  # noqa: E402

NUM, T, M, R, J = 7, 150, 15, 3, 4


def task_vector(g):
    st, cost, flow, fl = ko.cost_scaling(g)
    assert st == 0
    mp = flow_mapping(g, fl)
    tasks = np.nonzero(g.ntype == 1)[0] + 1
    return np.asarray([mp.get(int(t), 0) for t in tasks], np.int64), cost


def main():
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = batch.assign(NUM, world, rank)
    slots = batch.slots_per_rank(NUM, world)
    vecs = [task_vector(gen.quincy(T, M, R, J, 1000 + g))[0] for g in mine]
    block = torch.from_numpy(batch.pack(vecs, slots, T))
    full = batch.gather(block, NUM, dist)
    if rank == 0:
        ok = True
        for g in range(NUM):
            exp = task_vector(gen.quincy(T, M, R, J, 1000 + g))[0]
            ok &= bool(np.array_equal(full[g].numpy(), exp))
        with open(out_path, "w") as f:
            json.dump({"ok": ok, "world": world, "shape": list(full.shape),
                       "scheduled": int((full > 0).sum())}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
