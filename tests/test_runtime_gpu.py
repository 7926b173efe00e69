"""GPU: the library inside a PyTorch process (torch.distributed loaded FIRST).

PyTorch-ROCm bundles its own libamdhip64.so.7 and librccl.so.1 with the same
sonames as /opt/rocm's, so whichever is loaded first serves both: with torch
imported first the library binds torch's HIP runtime and RCCL (one copy of
each in the process; _native.check_single_runtime refuses two).  This test
runs that order in a fresh process: torch.distributed's own RCCL process group
(world size 1) does an all-reduce on the GPU, then the library's RCCL
communicator runs the 1-rank sharded build (the single-owner build and the
general path: samples, partition, exchange, owner merge), routed queries and
the replicated index, each checked against the oracle."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import json, os, sys
import torch.distributed as dist          # torch's ROCm runtime and RCCL first
import torch
import numpy as np
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[1], rank=0, world_size=1)
x = torch.arange(1024, dtype=torch.float64, device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
assert float(x.sum()) == 1023 * 1024 / 2

from dbindex_amd import _native, fasta, shard
from dbindex_amd.engine import Engine
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses

info = _native.runtime_info()              # raises on two runtimes / two RCCLs
pp = fasta.config("1k")
cp = DBIndexSearchParams.trypsin(2).to_c()
oix = cref.Index(cp, pp.residues, pp.offsets)
d_res = _native.DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
d_off = _native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
m, t = query_masses(oix, 2000)
of, oc = oix.query_batch(m, t)
comm = shard.ShardComm(shard.ShardComm.unique_id(), 1, 0, 0)
try:
    with Engine(cp, 0) as eng:
        for full_path in ("0", "1"):
            eng.set_option("shard_full_path", int(full_path))
            for rep in ("cold", "warm"):
                st = shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins,
                                         0, pp.n_proteins)
                assert st.g_total == oix.n_total and st.g_unique == oix.n_unique and st.g_keys == oix.n_keys
                dm, dt = _native.DeviceBuffer.from_numpy(m, 0), _native.DeviceBuffer.from_numpy(t, 0)
                df, dc = _native.DeviceBuffer(8 * m.shape[0], 0), _native.DeviceBuffer(8 * m.shape[0], 0)
                shard.query_sharded(eng, comm, dm.ptr, dt.ptr, m.shape[0], df.ptr, dc.ptr)
                f, c = df.download(np.uint64, m.shape[0]), dc.download(np.uint64, m.shape[0])
                assert np.array_equal(c, oc) and np.array_equal(f[oc > 0], of[oc > 0]), (full_path, rep)
                shard.replicate(eng, comm)
                assert_index_equal(eng, oix, f"replica full_path={full_path} [{rep}]")
                assert_queries_equal(eng, oix, m, t, f"replica full_path={full_path} [{rep}]")
finally:
    comm.close()
# torch's process group still works after the library's collectives
y = torch.ones(8, device="cuda:0")
dist.all_reduce(y)
torch.cuda.synchronize()
dist.destroy_process_group()
print("RESULT " + json.dumps(info))
'''


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(400)  # a fresh box's first `import torch` can take minutes
def test_library_after_torch_distributed():
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-c", SCRIPT, str(_free_port())], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=360)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
    info = json.loads(line[len("RESULT "):])
    # one HIP runtime and one RCCL, both torch's (loaded first), serve torch and the library
    assert len(info["mapped"]["libamdhip64"]) == 1 and len(info["mapped"]["librccl"]) == 1, info
    for key in ("libamdhip64", "librccl"):
        assert os.path.realpath(info[key]) == info["mapped"][key][0], info
    print(info)
