"""GPU: the reference's own solver harness (TestMultiScheduleIteration,
scheduling/flow/flowscheduler/schedule_iteration_test.go:16-91) replayed as the
exact DIMACS stream the reference writes to its solver
(tests/golden/multi_schedule_iteration.json), two ways: through the C-ABI
(ks_load_graph, then ks_apply_deltas per change block) and through the
flow_scheduler-compatible daemon. Every round must give the known answers
(costs 9/15/15/9/5, flows 3/5/3/3/3); the flow value is measured on the device
from the resident flow, not copied from the supplies."""
import subprocess

import pytest

from conftest import load_known_answers
from graphs import graph_from_lists, load_multi_schedule, parse_dimacs
from ksched_amd import _build, native
from test_gpu_parity import check_mapping

pytestmark = pytest.mark.gpu


def test_replay_through_c_abi():
    ka = load_known_answers()["multi_schedule_iteration"]
    rounds = load_multi_schedule()
    with native.Context(0) as ctx:
        got, placed = [], []
        for r in rounds:
            nodes, arcs, d = parse_dimacs(r["dimacs"])
            if r["kind"] == "full":
                g = graph_from_lists(nodes, arcs)
                ctx.load_graph(g)
            else:
                ctx.apply_deltas(d)
            res = ctx.solve()
            got.append((res.cost, res.flow))
            mp = ctx.task_mapping()
            if r["kind"] == "full":
                check_mapping(g, mp)
            placed.append(len(mp))
            # the reference's consumer requires PU destinations (graph_manager.go:259-262);
            # the number of tasks holding a PU equals the fixture's (running + newly placed)
            assert len(mp) == len(r["mapping"]), f"round {r['round']}"
        assert got == list(zip(ka["round_costs"], ka["round_flows"]))


@pytest.mark.parametrize("coalesce", [False, True])
def test_replay_through_daemon(coalesce):
    ka = load_known_answers()["multi_schedule_iteration"]
    daemon = _build.build_daemon()
    text = "".join(r["dimacs"] for r in load_multi_schedule())
    args = [daemon, "--graph_has_node_types=true", "--algorithm=successive_shortest_path",
            "--print_assignments=false", "--debug_output=true"] + (["--coalesce"] if coalesce else [])
    p = subprocess.run(args, input=text, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    costs = [int(l.split()[1]) for l in p.stdout.splitlines() if l.startswith("s ")]
    assert costs == ka["round_costs"]
