import os, sys
sys.path.insert(0, "/root/repo")
from ksched_amd import gen, native
opts = {}
for kv in filter(None, sys.argv[1].split(",")) if len(sys.argv) > 1 else []:
    k, v = kv.split("="); opts[k] = int(v)
g = gen.quincy(*gen.CONFIGS["config2"])
ctx = native.Context(0, log_cycles=1, **opts)
ctx.load_graph(g)
ref = None
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
    print(f"=== solve {i}", file=sys.stderr, flush=True)
    try:
        r = ctx.solve()
    except native.KsError as e:
        print(f"FAIL solve {i}: {e}", flush=True)
        sys.exit(1)
    ref = ref or (r.cost, r.flow)
    if (r.cost, r.flow) != ref:
        print(f"MISMATCH solve {i}: {r.cost} {r.flow} vs {ref}", flush=True)
        sys.exit(1)
print("ok", ref, flush=True)
