"""Host-side coordination of the ranks of one node without torch.

`bench.py --gpus N` runs one process per GPU (launched by
``torch.distributed.run``, which only sets RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_PORT in the environment).  The data path of a sharded build runs over
RCCL inside libdbindex_hip.so; what is left for the host is a barrier, the
max / sum over ranks of a few numbers and handing rank 0's RCCL unique id to
the others.  Importing torch for that would map PyTorch's own HIP runtime and
RCCL into the process next to /opt/rocm's (the library's), so this module does
it with plain sockets:

* rendezvous: rank 0 listens on an ephemeral TCP port of 127.0.0.1 and writes
  the port to ``/tmp/dbindex_coord_<key>``, key = the launcher's pid (every
  local rank is a child of the same torchrun agent) + MASTER_PORT; the other
  ranks poll for that file and connect;
* every operation is a gather to rank 0 and a broadcast back, one JSON line
  per message.
"""
from __future__ import annotations

import json
import os
import socket
import time
from typing import Any, List, Optional, Sequence


def _default_key() -> str:
    # a restarted worker group (torchrun --max-restarts) gets a new key: a file a
    # crashed rank 0 left behind is never read by the next attempt's ranks
    return (f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('TORCHELASTIC_RUN_ID', '')}"
            f"_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}")


class _Line:
    """Line-oriented JSON over a socket."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = b""

    def send(self, obj: Any) -> None:
        self.sock.sendall(json.dumps(obj).encode() + b"\n")

    def recv(self) -> Any:
        while b"\n" not in self.buf:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                raise ConnectionError("coordinator peer closed the connection")
            self.buf += chunk
        line, self.buf = self.buf.split(b"\n", 1)
        return json.loads(line)


class Coordinator:
    """Barrier / all-reduce / broadcast of small host values across the ranks of one node."""

    def __init__(self, world: int, rank: int, key: Optional[str] = None, timeout: float = 300.0,
                 directory: str = "/tmp"):
        self.world, self.rank = world, rank
        self.peers: List[_Line] = []
        self.root: Optional[_Line] = None
        self.path = os.path.join(directory, f"dbindex_coord_{key or _default_key()}")
        if world <= 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(world)
            tmp = self.path + ".tmp"
            with open(tmp, "w") as fh:
                fh.write(str(srv.getsockname()[1]))
            os.replace(tmp, self.path)
            srv.settimeout(timeout)
            by_rank = {}
            try:
                while len(by_rank) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(None)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    ln = _Line(conn)
                    by_rank[int(ln.recv()["rank"])] = ln
            finally:
                srv.close()
                try:
                    os.unlink(self.path)
                except OSError:
                    pass
            self.peers = [by_rank[r] for r in range(1, world)]
        else:
            t_end = time.time() + timeout
            sock = None
            while sock is None:
                port = None
                try:
                    with open(self.path) as fh:
                        txt = fh.read().strip()
                    port = int(txt) if txt else None
                except (OSError, ValueError):
                    port = None
                if port is not None:
                    # a stale file (rank 0 gone, or not yet replaced) refuses the
                    # connection: read the file again until the timeout
                    try:
                        sock = socket.create_connection(("127.0.0.1", port),
                                                        timeout=max(1.0, t_end - time.time()))
                    except OSError:
                        sock = None
                if sock is None:
                    if time.time() > t_end:
                        raise TimeoutError(f"rank {rank}: no coordinator at {self.path} after {timeout:.0f} s")
                    time.sleep(0.05)
            # the connect timeout must not carry over to the collectives: a rank
            # that connected near the end of the wait would time out in them
            sock.settimeout(None)
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.root = _Line(sock)
            self.root.send({"rank": rank})

    def _gather_bcast(self, value: Any, combine) -> Any:
        if self.world <= 1:
            return combine([value])
        if self.rank == 0:
            vals = [value] + [p.recv() for p in self.peers]
            out = combine(vals)
            for p in self.peers:
                p.send(out)
            return out
        self.root.send(value)
        return self.root.recv()

    def barrier(self) -> None:
        self._gather_bcast(0, lambda v: 0)

    def allreduce(self, values: Sequence[float], op: str = "sum") -> List[float]:
        """Element-wise sum / max / min over ranks."""
        f = {"sum": sum, "max": max, "min": min}[op]
        return self._gather_bcast([float(x) for x in values], lambda vs: [f(col) for col in zip(*vs)])

    def allgather(self, value: Any) -> List[Any]:
        """Every rank's (JSON-serialisable) value, in rank order."""
        return self._gather_bcast(value, lambda vs: vs)

    def broadcast(self, value: Any = None) -> Any:
        """Rank 0's value on every rank."""
        return self._gather_bcast(value, lambda vs: vs[0])

    def close(self) -> None:
        for ln in self.peers + ([self.root] if self.root else []):
            try:
                ln.sock.close()
            except OSError:
                pass
        self.peers, self.root = [], None
