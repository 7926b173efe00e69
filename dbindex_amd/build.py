"""Builds the in-tree HIP library ``dbindex_amd/libdbindex_hip.so`` for gfx950.

Plain ``hipcc`` (no torch JIT cache): the .so lives in the repo tree so it
travels to the GPU box with the snapshot.  ``-ffp-contract=off`` keeps the
fp64 mass accumulation a plain sequential sum (bit-identical to Java).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libdbindex_hip.so")
SOURCES = ["dbi_device.hip", "dbi_engine.hip", "dbi_shard.hip", "dbi_stream.hip", "dbi_persist.hip", "dbi_store.cpp", "dbi_fasta.cpp"]
ARCH = os.environ.get("DBI_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
         "-Wno-unused-result", "-Wshadow", f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build dbindex_amd)")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(force: bool = False, verbose: bool = False, lib_out: str = LIB, defines=()) -> str:
    """Compile + link the library (``defines``: extra -D flags for experiment variants)."""
    deps = [os.path.join(CSRC, s) for s in SOURCES]
    deps += [os.path.join(CSRC, "dbi_internal.h"), os.path.join(CSRC, "dbi_lane.h"), os.path.join(CSRC, "dbi_engine.h"), os.path.join(ROOT, "include", "dbindex_hip.h")]
    if not force and _newer(lib_out, deps):
        return lib_out
    objdir = os.path.join(HERE, "build") if lib_out == LIB else \
        os.path.join(HERE, "build", os.path.basename(lib_out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    cc = hipcc()
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(objdir, src.replace(".", "_") + ".o")
        cmd = [cc, *FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include")]
        if src.endswith(".cpp"):
            cmd += ["-x", "hip"]
        cmd += ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode(errors='replace')}")
        if out:  # warnings are never silent
            print(out.decode(errors="replace"), file=sys.stderr)
    tmp = lib_out + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout.decode(errors='replace')}")
    os.replace(tmp, lib_out)
    return lib_out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
