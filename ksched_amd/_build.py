"""Build libksmcmf.so in-tree for gfx950 (hipcc, no JIT cache)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libksmcmf.so")
SOURCES = [os.path.join(CSRC, f) for f in ("ks_engine.hip", "ks_cell.hip", "ks_store.hip", "ks_sched.hip",
                                           "ks_batch.hip", "ks_host.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("ks_engine.h", "ks_cell.h", "ks_store.h", "ks_sched.h", "ks_ctx.h",
                                                  "ks_pos.h")] + [
    os.path.join(ROOT, "include", "ksmcmf.h")]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm 7.x required)")


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in DEPS)


OBJ_DIR = os.path.join(HERE, "build")
HEADERS = [p for p in DEPS if p.endswith(".h")]


def _flags(arch: str, defines=()) -> list[str]:
    return [f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I" + os.path.join(ROOT, "include"), *[f"-D{d}" for d in defines]]


def _compile_all(arch: str, tag: str, defines=(), force: bool = False, verbose: bool = False,
                 extra=()) -> list[str]:
    """One object per source, compiled in parallel (a source is rebuilt when it or
    any header is newer than its object)."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in HEADERS)
    sources = list(SOURCES) + list(extra)
    jobs = []
    for src in sources:
        obj = os.path.join(OBJ_DIR, f"{tag}_{os.path.basename(src)}.o")
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            jobs.append((src, obj))
    def run(job):
        src, obj = job
        cmd = [hipcc(), *_flags(arch, defines), "-c", src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
    with ThreadPoolExecutor(max(1, min(len(jobs), os.cpu_count() or 1))) as ex:
        list(ex.map(run, jobs))
    return [os.path.join(OBJ_DIR, f"{tag}_{os.path.basename(src)}.o") for src in sources]


def _link(objs: list[str], arch: str, out: str, verbose: bool = False):
    cmd = [hipcc(), f"--offload-arch={arch}", "-shared", "-fPIC", *objs, "-ldl", "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    arch = os.environ.get("KS_OFFLOAD_ARCH", "gfx950")
    _link(_compile_all(arch, "lib", force=force, verbose=verbose), arch, LIB, verbose)
    return LIB


DAEMON = os.path.join(HERE, "ks_flow_scheduler")
DAEMON_SRC = os.path.join(CSRC, "ks_flow_scheduler.cpp")


def build_daemon(force: bool = False) -> str:
    """The flow_scheduler-compatible DIMACS daemon, linked against the in-tree library."""
    if not force and os.path.exists(DAEMON) and os.path.getmtime(DAEMON) >= max(
            os.path.getmtime(DAEMON_SRC), os.path.getmtime(LIB)):
        return DAEMON
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"), DAEMON_SRC,
           "-L" + HERE, "-lksmcmf", "-Wl,-rpath,$ORIGIN", "-o", DAEMON + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(DAEMON + ".tmp", DAEMON)
    return DAEMON


FAKE_COMM_SRC = os.path.join(ROOT, "tests", "fake_comm", "fake_nccl.cpp")
FAKE_COMM_TAG = "fakecomm"


def build_fake_comm(force: bool = False) -> str:
    """TEST INFRASTRUCTURE: libksmcmf_fakecomm.so, the library compiled with
    -DKS_FAKE_COMM and tests/fake_comm/fake_nccl.cpp (RCCL's entry points for the
    ranks of one process) for the world-2 rehearsal of ks_batch_gather on one GPU.
    The shipped libksmcmf.so is built without either."""
    out = variant_path(FAKE_COMM_TAG)
    deps = DEPS + [FAKE_COMM_SRC]
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(p) for p in deps):
        return out
    arch = os.environ.get("KS_OFFLOAD_ARCH", "gfx950")
    _link(_compile_all(arch, "v_" + FAKE_COMM_TAG, ["KS_FAKE_COMM"], force=force, extra=[FAKE_COMM_SRC]), arch, out)
    return out


def variant_path(tag: str) -> str:
    """ksched_amd/libksmcmf_<tag>.so; tags are plain identifiers (no paths)."""
    if not tag.replace("_", "").isalnum():
        raise ValueError(f"library variant tag {tag!r}: letters, digits and _ only")
    return os.path.join(HERE, f"libksmcmf_{tag}.so")


def build_variant(tag: str, defines: list[str]) -> str:
    """An extra copy of the library compiled with -D<defines> (tuning experiments)."""
    out = variant_path(tag)
    _link(_compile_all("gfx950", "v_" + tag, defines, force=True), "gfx950", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_daemon(force=True))
    print(build_fake_comm(force=True))
