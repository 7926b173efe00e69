"""The bench's torch-free host coordination (dbindex_amd/coord.py) across real
processes: rendezvous through the launcher-keyed file, barrier, max / sum
all-reduce, all-gather and broadcast — what bench.py --gpus N uses instead of
torch.distributed (which would map PyTorch's own HIP runtime and RCCL)."""
from __future__ import annotations

import multiprocessing as mp
import os
import sys
import uuid

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank_main(world: int, rank: int, key: str, directory: str, q) -> None:
    sys.path.insert(0, ROOT)
    from dbindex_amd.coord import Coordinator
    c = Coordinator(world, rank, key=key, timeout=60, directory=directory)
    c.barrier()
    mx = c.allreduce([rank, -rank, 1.5], "max")
    sm = c.allreduce([rank, 1], "sum")
    mn = c.allreduce([rank + 10], "min")
    ga = c.allgather({"r": rank, "sq": rank * rank})
    bc = c.broadcast(os.urandom(16).hex() if rank == 0 else None)
    c.barrier()
    c.close()
    q.put((rank, mx, sm, mn, ga, bc))


@pytest.mark.parametrize("world", [2, 3, 5])
def test_coordinator_collectives(world, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = uuid.uuid4().hex
    procs = [ctx.Process(target=_rank_main, args=(world, r, key, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    bcs = {r[5] for r in res}
    assert len(bcs) == 1 and len(bcs.pop()) == 32  # rank 0's value everywhere
    for rank, mx, sm, mn, ga, _ in res:
        assert mx == [world - 1, 0, 1.5]
        assert sm == [world * (world - 1) / 2, world]
        assert mn == [10]
        assert ga == [{"r": r, "sq": r * r} for r in range(world)]
    assert not os.listdir(tmp_path)  # the rendezvous file is gone


def test_coordinator_single_rank_is_local():
    sys.path.insert(0, ROOT)
    from dbindex_amd.coord import Coordinator
    c = Coordinator(1, 0, key="unused")
    c.barrier()
    assert c.allreduce([3.0, 4.0], "max") == [3.0, 4.0]
    assert c.allgather(7) == [7]
    assert c.broadcast("x") == "x"


def test_coordinator_times_out_without_rank0(tmp_path):
    sys.path.insert(0, ROOT)
    from dbindex_amd.coord import Coordinator
    with pytest.raises(TimeoutError):
        Coordinator(2, 1, key="nobody", timeout=0.3, directory=str(tmp_path))


def test_bench_has_no_torch_import():
    """bench.py must not import torch: its HIP runtime and RCCL would be mapped
    beside /opt/rocm's."""
    import ast
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    names = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            names.update(a.name.split(".")[0] for a in node.names)
        elif isinstance(node, ast.ImportFrom) and node.module:
            names.add(node.module.split(".")[0])
    assert "torch" not in names


def test_coordinator_stale_file_is_retried(tmp_path):
    """A rendezvous file a crashed rank 0 left behind names a dead port: the
    connection is refused, and the rank re-reads the file until the new rank 0
    replaces it, instead of failing at once."""
    import socket as _s
    import threading
    import time as _t
    sys.path.insert(0, ROOT)
    from dbindex_amd.coord import Coordinator
    dead = _s.socket()
    dead.bind(("127.0.0.1", 0))
    port = dead.getsockname()[1]
    dead.close()  # nothing listens there any more
    (tmp_path / "dbindex_coord_stale").write_text(str(port))
    out = {}

    def rank1():
        c = Coordinator(2, 1, key="stale", timeout=30, directory=str(tmp_path))
        out["sum"] = c.allreduce([1.0], "sum")
        c.close()

    t = threading.Thread(target=rank1)
    t.start()
    _t.sleep(0.5)  # rank 1 is polling the stale file now
    c0 = Coordinator(2, 0, key="stale", timeout=30, directory=str(tmp_path))
    assert c0.allreduce([2.0], "sum") == [3.0]
    c0.close()
    t.join(timeout=30)
    assert out["sum"] == [3.0]


def test_coordinator_key_changes_with_restart(monkeypatch):
    sys.path.insert(0, ROOT)
    from dbindex_amd.coord import _default_key
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    k0 = _default_key()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert _default_key() != k0
