"""dbindex_amd — MI355X-native peptide-index builder and mass-lookup engine.

The drop-in for proteomicsyates/dbIndex's digestion + index + mass-window
query hot path (DBIndexer.cutSeq -> DBIndexStore -> getSequences(mass, tol)),
implemented as hand-written CDNA4 HIP kernels behind a C-ABI
(include/dbindex_hip.h, libdbindex_hip.so).  See DESIGN.md.
"""
from .params import DBIndexSearchParams, calculate_mass, tolerance_in_dalton  # noqa: F401
from . import fasta  # noqa: F401

__all__ = ["DBIndexSearchParams", "calculate_mass", "tolerance_in_dalton", "fasta",
           "Engine", "DBIndexStoreHip", "DBIndexer", "load"]


def load():
    """Loads the HIP library (raises ImportError if it was not built)."""
    from . import _native
    return _native.lib()


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "DBIndexStoreHip":
        from .store import DBIndexStoreHip
        return DBIndexStoreHip
    if name == "DBIndexer":
        from .indexer import DBIndexer
        return DBIndexer
    raise AttributeError(name)
