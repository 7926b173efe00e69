"""A fresh engine's one-off build from host arrays, bracketed for a HIP API
trace: where dbi_open + dbi_build spend their time beyond the cold kernels.

  rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
      -d gpurun_out/TAG/trace -- python3 tools/e2e_trace.py [config] [fasta]
  python3 tools/api_timeline.py gpurun_out/TAG/trace

With "fasta" the builds are dbi_build_fasta of the proteome written as a
FASTA file.  Each phase is preceded by a dbi_runtime_info_get call (hipRuntimeGetVersion), which
tools/api_timeline.py uses as the phase marker.  The process first builds once
on another engine (code objects loaded, as in bench.py's end-to-end leg)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import WORKLOADS  # noqa: E402
from dbindex_amd import fasta  # noqa: E402
from dbindex_amd._native import runtime_info, synchronize  # noqa: E402
from dbindex_amd.engine import Engine  # noqa: E402


def main() -> None:
    config = sys.argv[1] if len(sys.argv) > 1 else "swissprot"
    _, proteome, make_params, _ = WORKLOADS[config]
    pp = fasta.synthetic(with_defs=False, **fasta.CONFIGS[proteome])
    prm = make_params()
    with Engine(prm, device=0) as e:
        e.build(pp)
        synchronize(0)
    out = []
    fused = len(sys.argv) > 2 and sys.argv[2] == "fasta"
    if fused:  # dbi_build_fasta of the proteome written as a FASTA file
        import tempfile
        td = tempfile.mkdtemp()
        path = os.path.join(td, "p.fasta")
        with open(path, "w") as fh:
            fasta.write_fasta(pp, fh)
    for rep in range(3):
        runtime_info()  # marker: open
        t0 = time.perf_counter()
        e3 = Engine(prm, device=0)
        e3.set_timing(False)
        runtime_info()  # marker: build
        t1 = time.perf_counter()
        if fused:
            e3.build_fasta(path)
        else:
            e3.build(pp)
        synchronize(0)
        t2 = time.perf_counter()
        runtime_info()  # marker: close
        e3.close()
        t3 = time.perf_counter()
        out.append(dict(open_ms=1e3 * (t1 - t0), build_ms=1e3 * (t2 - t1), close_ms=1e3 * (t3 - t2)))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
