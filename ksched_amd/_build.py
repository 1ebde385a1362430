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
SOURCES = [os.path.join(CSRC, f) for f in ("ks_engine.hip", "ks_store.hip", "ks_sched.hip", "ks_batch.hip",
                                           "ks_host.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("ks_engine.h", "ks_store.h", "ks_sched.h", "ks_ctx.h")] + [
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


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    arch = os.environ.get("KS_OFFLOAD_ARCH", "gfx950")
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"),
           *SOURCES, "-ldl", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
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


def variant_path(tag: str) -> str:
    return os.path.join(HERE, f"libksmcmf_{tag}.so")


def build_variant(tag: str, defines: list[str]) -> str:
    """An extra copy of the library compiled with -D<defines> (tuning experiments)."""
    out = variant_path(tag)
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"), *[f"-D{d}" for d in defines],
           *SOURCES, "-ldl", "-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_daemon(force=True))
