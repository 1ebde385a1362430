"""CPU suite: the C-ABI library (include/ksmcmf.h) loads, exports every declared
entry point, and its struct layouts match what the bindings assume. No compute
calls are made here (there is no GPU in the build container)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from ksched_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ksmcmf.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ks_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = native.load(build_if_missing=True)
    names = declared_functions()
    assert len(names) >= 11
    for n in names:
        assert hasattr(lib, n), f"{n} declared in ksmcmf.h but not exported"
    assert set(names) == set(native.EXPORTED_SYMBOLS)


def test_abi_version_and_default_opts():
    lib = native.load()
    assert lib.ks_abi_version() == native.ABI_VERSION == 5
    o = native.default_opts()
    assert (o.alpha, o.verify, o.auto_sink) == (0, 1, 1)   # alpha 0: the size-dependent default
    assert o.price_refine == 1 and o.gu_interval > 0 and o.warm_start == 0
    assert o.cell_nodes == 0   # the cell solver on by default for graphs its LDS holds


def test_create_fails_loudly_without_device():
    """The product path never falls back to the CPU: no HIP device → KsError."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(native.KsError):
        native.Context(0)


LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "ksmcmf.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F))
int main(void) {
  printf("ks_opts %zu\nks_node %zu\nks_arc %zu\nks_delta %zu\nks_result %zu\nks_flow %zu\nks_store_stats %zu\n",
         sizeof(ks_opts), sizeof(ks_node), sizeof(ks_arc), sizeof(ks_delta), sizeof(ks_result), sizeof(ks_flow),
         sizeof(ks_store_stats));
  P(ks_node, excess); P(ks_node, type);
  P(ks_arc, dst); P(ks_arc, low); P(ks_arc, cap); P(ks_arc, cost); P(ks_arc, type);
  P(ks_delta, id); P(ks_delta, src); P(ks_delta, dst); P(ks_delta, low); P(ks_delta, cap);
  P(ks_delta, cost); P(ks_delta, old_cost); P(ks_delta, excess);
  P(ks_result, status); P(ks_result, sweeps); P(ks_result, ms_phase); P(ks_result, n_nodes);
  P(ks_result, ms_gu_kernels); P(ks_result, rebuilt); P(ks_result, recoveries); P(ks_result, cell_fallbacks);
  P(ks_result, cycles_cancelled); P(ks_result, fb_resets); P(ks_result, compact); P(ks_result, cycles_rejected); P(ks_result, gu_leaf_scans);
  P(ks_opts, warm_start); P(ks_opts, walk_slack); P(ks_opts, fault_inject); P(ks_opts, walk_passes); P(ks_opts, tail_nodes); P(ks_opts, bf_bound); P(ks_opts, fwd_nodes); P(ks_opts, cell_nodes); P(ks_opts, warm_shift); P(ks_opts, warm_canon); P(ks_opts, compact_pos);
  P(ks_store_stats, superseded); P(ks_store_stats, residual_slots);
  P(ks_flow, flow);
  return 0;
}
"""


def test_struct_layouts_match_bindings(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.splitlines())
    out = {k: int(v) for k, v in out.items()}
    assert out["ks_opts"] == C.sizeof(native.KsOpts)
    assert out["ks_result"] == C.sizeof(native.KsResult)
    assert out["ks_node"] == native.NODE_DT.itemsize
    assert out["ks_arc"] == native.ARC_DT.itemsize
    assert out["ks_delta"] == native.DELTA_DT.itemsize
    assert out["ks_flow"] == native.FLOW_DT.itemsize
    assert out["ks_store_stats"] == C.sizeof(native.KsStoreStats)
    for f in ("superseded", "residual_slots"):
        assert getattr(native.KsStoreStats, f).offset == out[f"ks_store_stats.{f}"], f
    for dt, cname in ((native.NODE_DT, "ks_node"), (native.ARC_DT, "ks_arc"), (native.DELTA_DT, "ks_delta"),
                      (native.FLOW_DT, "ks_flow")):
        for f in dt.names:
            key = f"{cname}.{f}"
            if key in out:
                assert dt.fields[f][1] == out[key], key
    for f in ("status", "sweeps", "ms_phase", "n_nodes", "ms_gu_kernels", "rebuilt", "recoveries", "cell_fallbacks",
              "cycles_cancelled", "fb_resets", "compact", "cycles_rejected", "gu_leaf_scans"):
        assert getattr(native.KsResult, f).offset == out[f"ks_result.{f}"], f
    for f in ("warm_start", "walk_slack", "fault_inject", "walk_passes", "tail_nodes", "bf_bound", "fwd_nodes",
              "cell_nodes", "warm_shift", "warm_canon", "compact_pos"):
        assert getattr(native.KsOpts, f).offset == out[f"ks_opts.{f}"], f


def test_delta_dtype_roundtrip():
    d = np.zeros(2, native.DELTA_DT)
    d[0]["kind"] = native.KS_ADD_ARC
    d[0]["src"], d[0]["dst"], d[0]["cap"], d[0]["cost"] = 5, 7, 1, -3
    raw = d.tobytes()
    assert len(raw) == 2 * native.DELTA_DT.itemsize
    back = np.frombuffer(raw, native.DELTA_DT)
    assert int(back[0]["cost"]) == -3 and int(back[0]["dst"]) == 7
