"""``DBIndexStoreHip`` — Python face of the dbi_store_* C-ABI, method-for-method
the ``DBIndexStore`` interface of the reference
(``/root/reference/src/main/java/edu/scripps/yates/dbindex/DBIndexStore.java:19-194``)
with the semantics of ``DBIndexStoreSQLiteMult`` (the store ``DBIndexer`` builds).

It is what a JNI ``DBIndexStoreHip implements DBIndexStore`` does on the Java
side: each Java method is one C call; non-zero statuses become
``DBIndexStoreException``.  The value types below mirror the external
``IndexedSequence`` / ``IndexedProtein`` / ``ResidueInfo`` / ``MassRange``
classes of ``edu.scripps.yates.utilities`` (not vendored).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterator, List, Optional, Sequence

import numpy as np

from . import _native
from ._native import DbiSeqList, DBIndexStoreException, check
from .params import DBIndexSearchParams, DbiParams

FilterResult_INCLUDE = _native.FILTER_INCLUDE
FilterResult_SKIP = _native.FILTER_SKIP
FilterResult_SKIP_PROTEIN_START = _native.FILTER_SKIP_PROTEIN_START


@dataclass
class ResidueInfo:
    """``edu.scripps.yates.utilities.fasta.dbindex.ResidueInfo`` (external):
    the 3-residue left/right flanks, padded with '-'."""

    resLeft: str
    resRight: str

    def getResLeft(self) -> str:
        return self.resLeft

    def getResRight(self) -> str:
        return self.resRight


@dataclass
class IndexedSequence:
    """``new IndexedSequence(0, seqMass, peptideSequence, "", "")`` +
    ``setProteinIds`` + ``setResidues`` (IndexMerge.java:459-470)."""

    mass: float
    sequence: str
    proteinIds: List[int]
    residues: ResidueInfo
    sequenceOffset: int
    sequenceLen: int
    uniqueId: int = -1

    def getSequence(self) -> str:
        return self.sequence

    def getMass(self) -> float:
        return self.mass

    def getProteinIds(self) -> List[int]:
        return self.proteinIds

    def getResLeft(self) -> str:
        return self.residues.resLeft

    def getResRight(self) -> str:
        return self.residues.resRight

    def getSequenceOffset(self) -> int:
        return self.sequenceOffset

    def getSequenceLen(self) -> int:
        return self.sequenceLen


@dataclass(frozen=True)
class IndexedProtein:
    accession: str
    id: int

    def getAccession(self) -> str:
        return self.accession

    def getId(self) -> int:
        return self.id


@dataclass
class MassRange:
    precMass: float
    tolerance: float

    def getPrecMass(self) -> float:
        return self.precMass

    def getTolerance(self) -> float:
        return self.tolerance


class ProteinCache:
    """``ProteinCache`` (ProteinCache.java:22-179): definitions and sequences by
    insertion position.  ``DBIndexer.run`` fills it with EVERY FASTA protein
    (DBIndexer.java:605) and hands it to the store (:595), which resolves
    protein ids through it (SQLiteMult.java:297, :457; IndexMerge.java:452-461)."""

    def __init__(self):
        self.defs: List[str] = []
        self.sequences: List[str] = []

    def addProtein(self, definition: str, protein: Optional[str] = None) -> int:
        self.defs.append(definition.replace("\t", " "))  # :87-89
        if protein is not None:
            self.sequences.append(protein)
        return len(self.defs) - 1

    def getNumberProteins(self) -> int:
        return len(self.sequences)

    def isPopulated(self) -> bool:
        return bool(self.sequences)

    def getProteinSequence(self, proteinId: int) -> Optional[str]:
        return self.sequences[proteinId] if len(self.sequences) > proteinId else None  # :60-65

    def getProteinDef(self, proteinId: int) -> str:
        return self.defs[proteinId]

    def getPeptideSequence(self, protId: int, seqOffset: int, seqLen: int) -> Optional[str]:
        """String.substring's bounds; the reference logs the exception and
        returns null (:112-127)."""
        p = self.getProteinSequence(protId)
        if p is None or seqOffset < 0 or seqLen < 0 or seqOffset + seqLen > len(p):
            return None
        return p[seqOffset:seqOffset + seqLen]


def _seq_list(ptr) -> List[IndexedSequence]:
    l = ptr.contents
    n = l.n
    out: List[IndexedSequence] = []
    if n == 0:
        return out
    seq_off = np.ctypeslib.as_array(l.seq_off, shape=(n + 1,))
    chars = ctypes.string_at(l.seq_chars, int(seq_off[n])).decode("ascii")
    left = ctypes.string_at(l.res_left, 3 * n).decode("ascii")
    right = ctypes.string_at(l.res_right, 3 * n).decode("ascii")
    prot_off = np.ctypeslib.as_array(l.prot_off, shape=(n + 1,))
    nprot = int(prot_off[n])
    prot_ids = np.ctypeslib.as_array(l.prot_ids, shape=(max(nprot, 1),))[:nprot]
    mass = np.ctypeslib.as_array(l.mass, shape=(n,))
    off = np.ctypeslib.as_array(l.offset, shape=(n,))
    ln = np.ctypeslib.as_array(l.length, shape=(n,))
    uid = np.ctypeslib.as_array(l.unique_id, shape=(n,))
    for i in range(n):
        out.append(IndexedSequence(
            mass=float(mass[i]), sequence=chars[seq_off[i]:seq_off[i + 1]],
            proteinIds=[int(x) for x in prot_ids[prot_off[i]:prot_off[i + 1]]],
            residues=ResidueInfo(left[3 * i:3 * i + 3], right[3 * i:3 * i + 3]),
            sequenceOffset=int(off[i]), sequenceLen=int(ln[i]), uniqueId=int(uid[i])))
    return out


class DBIndexStoreHip:
    """``implements DBIndexStore`` on the MI355X engine."""

    def __init__(self, sparam, device: int = 0, device_digest: bool = False, persist: bool = False):
        if isinstance(sparam, DBIndexSearchParams):
            self.sparam = sparam
            cp = sparam.to_c()
        else:
            self.sparam = None
            cp = sparam
        assert isinstance(cp, DbiParams)
        self._cp = cp
        self.proteinCache: Optional[ProteinCache] = None
        s = ctypes.c_void_p()
        check(_native.lib().dbi_store_create(ctypes.byref(cp), device, ctypes.byref(s)))
        self.s = s
        if device_digest:
            self.setDeviceDigest(True)
        if persist:  # <databaseID>.dbihip: loaded by init() when it matches, written by stopAddSeq()
            check(_native.lib().dbi_store_set_persist(self.s, 1))

    def close(self) -> None:
        if getattr(self, "s", None):
            _native.lib().dbi_store_close(self.s)
            self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- DBIndexerHip hook ----------------------------------------------------
    def setDeviceDigest(self, on: bool) -> None:
        check(_native.lib().dbi_store_set_device_digest(self.s, 1 if on else 0))

    # --- DBIndexStore ---------------------------------------------------------
    def lastBuffertoDatabase(self) -> None:
        raise NotImplementedError("Not supported yet.")  # DBIndexStoreSQLiteByte.java:720-730

    def init(self, databaseID: Optional[str]) -> None:
        check(_native.lib().dbi_store_init(self.s, (databaseID or "").encode()))

    def startAddSeq(self) -> None:
        check(_native.lib().dbi_store_start_add_seq(self.s))

    def stopAddSeq(self) -> None:
        check(_native.lib().dbi_store_stop_add_seq(self.s))

    def indexExists(self) -> bool:
        v = ctypes.c_int()
        check(_native.lib().dbi_store_index_exists(self.s, ctypes.byref(v)))
        return bool(v.value)

    def filterSequence(self, precMass: float, sequence: str) -> int:
        b = sequence.encode("ascii")
        v = ctypes.c_int()
        check(_native.lib().dbi_store_filter_sequence(self.s, precMass, b, len(b), ctypes.byref(v)))
        return v.value

    def addSequence(self, precMass: float, sequenceOffset: int, sequenceLen: int, sequence=None,
                    resLeft=None, resRight=None, proteinId: int = 0) -> None:
        check(_native.lib().dbi_store_add_sequence(self.s, precMass, sequenceOffset, sequenceLen, proteinId))

    def getSequences(self, precMass, tolerance=None) -> List[IndexedSequence]:
        """``getSequences(double, double)`` or ``getSequences(List<MassRange>)``."""
        L = _native.lib()
        r = ctypes.POINTER(DbiSeqList)()
        if tolerance is None:
            ranges: Sequence[MassRange] = precMass
            m = np.ascontiguousarray([x.getPrecMass() for x in ranges], np.float64)
            t = np.ascontiguousarray([x.getTolerance() for x in ranges], np.float64)
            check(L.dbi_store_get_sequences_ranges(self.s, m.ctypes.data_as(ctypes.c_void_p),
                                                   t.ctypes.data_as(ctypes.c_void_p), m.shape[0],
                                                   ctypes.byref(r)))
        else:
            check(L.dbi_store_get_sequences(self.s, float(precMass), float(tolerance), ctypes.byref(r)))
        try:
            seqs = _seq_list(r)
        finally:
            L.dbi_seq_list_free(r)
        return self._resolve(seqs)

    def getSequencesIterator(self, ranges: Sequence[MassRange]) -> Iterator[IndexedSequence]:
        return iter(self.getSequences(ranges))

    def addProteinDef(self, num: int, accession: str, protSequence: str) -> int:
        b = protSequence.encode("ascii")
        out = ctypes.c_int64()
        check(_native.lib().dbi_store_add_protein_def(self.s, num, accession.encode(), b, len(b),
                                                      ctypes.byref(out)))
        return out.value

    def setProteinCache(self, proteinCache: Optional[ProteinCache]) -> None:
        """The store keeps its own copy of the proteins given to
        ``addProteinDef``; a cache set here is where protein ids are RESOLVED,
        as in every reference store (peptide text and flanks
        IndexMerge.java:452-461, definitions SQLiteMult.java:457, residues
        :297).  The two agree unless ``run()`` discarded decoys that precede a
        target: the cache holds every protein (DBIndexer.java:605) while the
        ids advance only for the non-decoys (:609-616), so the reference's
        answers for later ids come from shifted cache entries -- reproduced."""
        self.proteinCache = proteinCache

    def _resolve(self, seqs: List[IndexedSequence]) -> List[IndexedSequence]:
        pc = getattr(self, "proteinCache", None)
        if pc is None:
            return seqs
        for s in seqs:
            pid, off, ln = s.proteinIds[0], s.sequenceOffset, s.sequenceLen
            prot = pc.getProteinSequence(pid)
            if prot is None or off > len(prot):  # Util.getResidues' substring throws (Util.java:132-138)
                raise DBIndexStoreException(_native.DBI_E_INVALID, f"protein {pid} of the ProteinCache cannot hold "
                                            f"offset {off} (String index out of range)")
            s.sequence = pc.getPeptideSequence(pid, off, ln)
            s.residues = get_residues(off, ln, prot)
        return seqs

    def supportsProteinCache(self) -> bool:
        return True

    def getProteins(self, sequence: IndexedSequence) -> List[IndexedProtein]:
        pc = getattr(self, "proteinCache", None)
        name = pc.getProteinDef if pc is not None else self.getProteinDef
        return [IndexedProtein(name(pid), pid) for pid in sequence.getProteinIds()]

    def getNumberSequences(self) -> int:
        v = ctypes.c_int64()
        check(_native.lib().dbi_store_get_number_sequences(self.s, ctypes.byref(v)))
        return v.value

    def getTotalSeqCount(self) -> int:
        v = ctypes.c_int64()
        check(_native.lib().dbi_store_get_total_seq_count(self.s, ctypes.byref(v)))
        return v.value

    def getResidues(self, peptideSequence: IndexedSequence, protein: IndexedProtein) -> ResidueInfo:
        """SQLiteMult.getResidues (:294-312) -> Util.getResidues (Util.java:130-162)."""
        pc = getattr(self, "proteinCache", None)
        prot = (pc.getProteinSequence if pc is not None else self.getProteinSequence)(protein.getId())
        off = peptideSequence.getSequenceOffset()
        if off is None or off < 0:
            off = prot.find(peptideSequence.getSequence())
        if off == -1:
            raise RuntimeError("Could not get subsequence, unexpected error")
        return get_residues(off, peptideSequence.getSequenceLen(), prot)

    def getEntryKeys(self) -> List[int]:
        L = _native.lib()
        n = ctypes.c_uint64()
        check(L.dbi_store_get_entry_keys(self.s, None, 0, ctypes.byref(n)))
        keys = np.zeros(n.value, np.int32)
        if n.value:
            check(L.dbi_store_get_entry_keys(self.s, keys.ctypes.data_as(ctypes.c_void_p), n.value,
                                             ctypes.byref(n)))
        return [int(k) for k in keys]

    # --- ProteinCache accessors ----------------------------------------------
    def getNumberProteins(self) -> int:
        v = ctypes.c_uint64()
        check(_native.lib().dbi_store_protein_count(self.s, ctypes.byref(v)))
        return v.value

    def getProteinDef(self, pid: int) -> str:
        p = ctypes.c_char_p()
        n = ctypes.c_uint64()
        check(_native.lib().dbi_store_protein_def(self.s, pid, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p, n.value).decode()

    def getProteinSequence(self, pid: int) -> str:
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        check(_native.lib().dbi_store_protein_sequence(self.s, pid, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p, n.value).decode("ascii") if n.value else ""

    def engine_handle(self):
        return _native.lib().dbi_store_engine(self.s)


class MassRangeFilteringIndexHip(DBIndexStoreHip):
    """``MassRangeFilteringIndex`` (the SEARCH_UNINDEXED store,
    MassRangeFilteringIndex.java) on the engine.

    The reference re-cuts every cached protein per search and keeps the
    peptides whose mass lies in a range (``filterSequence`` :90-108,
    ``addSequence`` :111-130).  Here the proteins given to ``addProteinDef``
    are digested once on the device at ``stopAddSeq`` (no buckets, no
    mandatory-residue filter: ``dbi_store_set_unindexed``) and every search is
    a union of windows over the mass-sorted table -- the same set: one entry
    per sequence (its first occurrence), protein ids without repeats, cutSeq's
    own flanks.  Order is ascending mass (the reference's is THashMap order).
    """

    RESIDENT, STREAM = 1, 2  # DBI_UNINDEXED_*

    def __init__(self, sparam, device: int = 0, mode: int = RESIDENT):
        """``mode``: RESIDENT keeps one device index of every peptide (searches
        are windows over it); STREAM keeps only the proteins in HBM and
        re-digests them through each search's ranges (memory for the matches
        only -- for proteomes or enzymes whose full index does not fit)."""
        super().__init__(sparam, device)
        check(_native.lib().dbi_store_set_unindexed(self.s, int(mode)))

    def cutAndSearch(self, massRanges: Sequence[MassRange]) -> List[IndexedSequence]:
        """``DBIndexer.cutAndSearch`` (DBIndexer.java:707-747)."""
        L = _native.lib()
        r = ctypes.POINTER(DbiSeqList)()
        m = np.ascontiguousarray([x.getPrecMass() for x in massRanges], np.float64)
        t = np.ascontiguousarray([x.getTolerance() for x in massRanges], np.float64)
        check(L.dbi_store_cut_and_search(self.s, m.ctypes.data_as(ctypes.c_void_p),
                                         t.ctypes.data_as(ctypes.c_void_p), m.shape[0], ctypes.byref(r)))
        try:
            return _seq_list(r)
        finally:
            L.dbi_seq_list_free(r)

    def getResidues(self, peptideSequence: IndexedSequence, protein: IndexedProtein) -> ResidueInfo:
        # stored in the sequence itself (MassRangeFilteringIndex.java:185-191)
        return ResidueInfo(peptideSequence.getResLeft(), peptideSequence.getResRight())


def get_residues(offset: int, length: int, prot: str) -> ResidueInfo:
    """Util.getResidues (Util.java:130-162), incl. the right-flank quirk
    ``min(3, protLen - end - 1)``."""
    n = len(prot)
    left_i = offset - 3 if offset >= 3 else 0
    left = prot[left_i:left_i + min(3, offset)]
    end = offset + length
    right_len = min(3, n - end - 1)
    right = prot[end:end + right_len] if (end < n and right_len > 0) else ""
    return ResidueInfo("-" * (3 - len(left)) + left, right + "-" * (3 - len(right)))
