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
# the test-hook variant (options test_fail / test_split_skew): tests only
LIB_HOOKS = os.path.join(HERE, "libdbindex_hip_hooks.so")
HOOK_SOURCES = ("dbi_engine.hip", "dbi_shard.hip")
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


def _compile(cc, jobs, verbose):
    """jobs: (src, obj, defines); compiled in parallel."""
    procs = []
    for src, obj, defines in jobs:
        cmd = [cc, *FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include")]
        if src.endswith(".cpp"):
            cmd += ["-x", "hip"]
        cmd += ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode(errors='replace')}")
        if out:  # warnings are never silent
            print(out.decode(errors="replace"), file=sys.stderr)


def _link(cc, objs, lib_out):
    tmp = lib_out + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout.decode(errors='replace')}")
    os.replace(tmp, lib_out)


def build(force: bool = False, verbose: bool = False, lib_out: str = LIB, defines=()) -> str:
    """Compile + link the library (``defines``: extra -D flags for experiment
    variants).  The in-tree build also links the test-hook variant
    (LIB_HOOKS: dbi_engine / dbi_shard again with -DDBI_TEST_HOOKS, every
    other object shared), which only the failure-injection tests load."""
    deps = [os.path.join(CSRC, s) for s in SOURCES]
    deps += [os.path.join(CSRC, "dbi_internal.h"), os.path.join(CSRC, "dbi_lane.h"), os.path.join(CSRC, "dbi_engine.h"), os.path.join(CSRC, "dbi_fasta.h"), os.path.join(ROOT, "include", "dbindex_hip.h")]
    main = lib_out == LIB
    if not force and _newer(lib_out, deps) and (not main or _newer(LIB_HOOKS, deps)):
        return lib_out
    # experiment variants keep their objects beside their library, out of the package tree
    objdir = os.path.join(HERE, "build") if main else \
        os.path.join(os.path.dirname(os.path.abspath(lib_out)), "build", os.path.basename(lib_out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    cc = hipcc()
    obj = {src: os.path.join(objdir, src.replace(".", "_") + ".o") for src in SOURCES}
    hook_obj = {src: os.path.join(objdir, "hooks_" + src.replace(".", "_") + ".o") for src in HOOK_SOURCES}
    jobs = [(src, obj[src], tuple(defines)) for src in SOURCES]
    if main:
        jobs += [(src, hook_obj[src], tuple(defines) + ("DBI_TEST_HOOKS",)) for src in HOOK_SOURCES]
    _compile(cc, jobs, verbose)
    _link(cc, [obj[src] for src in SOURCES], lib_out)
    if main:
        _link(cc, [hook_obj.get(src, obj[src]) for src in SOURCES], LIB_HOOKS)
    return lib_out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
