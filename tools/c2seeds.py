"""Median solve time of config-2-sized graphs over several seeds, per ks_opts setting
(round-5 alpha study). Usage: python tools/c2seeds.py "alpha=16" "alpha=1024" ..."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ksched_amd import gen, native  # noqa: E402


def parse(spec):
    o = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        o[k] = int(v)
    return o


T, M, R, J, _ = gen.CONFIGS["config2"]
seeds = [2, 7, 11] + list(range(1000, 1009))
graphs = [gen.quincy(T, M, R, J, s) for s in seeds]
_gold = {e["seed"]: e["cost"] for e in __import__("json").load(open(__import__("os").path.join(
    __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))),
    "tests", "golden", "goldens.json")))["graphs"] if e["family"] == "quincy" and e["params"] == [T, M, R, J]}
for spec in sys.argv[1:] or [""]:
    opts = parse(spec)
    cells = opts.pop("cell", 0)
    ms, costs = [], []
    with native.Context(0, cell_nodes=20000 if cells else -1, **opts) as ctx:
        for g in graphs:
            ctx.load_graph(g)
            ctx.solve()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                r = ctx.solve()
                ts.append(1e3 * (time.perf_counter() - t0))
            ms.append(float(np.median(ts)))
            costs.append(r.cost)
            s_ = seeds[len(costs) - 1]
            assert s_ not in _gold or _gold[s_] == r.cost, (s_, r.cost, _gold[s_])
    tag = __import__("os").environ.get("KS_LIB_VARIANT", "")
    print(f"{tag + ':' + (spec or 'default'):>24}: median {np.median(ms):6.2f} ms, mean {np.mean(ms):6.2f}, max {max(ms):6.2f}; "
          f"per seed {' '.join(f'{x:.1f}' for x in ms)}; costs {costs[:3]}", flush=True)
