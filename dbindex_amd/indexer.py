"""``DBIndexer`` mirror with the ``DBIndexerHip`` digestion hook.

Reference: ``/root/reference/src/main/java/edu/scripps/yates/dbindex/DBIndexer.java``.
The drop-in overrides the protected ``cutSeq(String, String)`` (``:237``) so it
only registers the protein with the store (``addProteinDef(++protNum, ...)``,
``:251``); the whole digestion loop (``:256-397``) then runs on the GPU when
the store finalises (``stopAddSeq``, ``:666``).  The query-side logic that
lives in ``DBIndexer`` (ppm probe loop ``:787-844``, exact-mass protein lookup
``:925-947``, parent masses ``:979-992``) is mirrored here unchanged, on top of
the store's ``getSequences``.
"""
from __future__ import annotations

import os
import re

from typing import Iterable, List, Optional, Set, Tuple, Union

from .fasta import PackedProteins, fasta_accession, iter_fasta, uniprot_accession
from .params import DBIndexSearchParams, calculate_mass, tolerance_in_dalton
from .store import (DBIndexStoreHip, IndexedProtein, IndexedSequence, MassRange, MassRangeFilteringIndexHip,
                    ProteinCache)

PRECISION = 0.000001  # Constants.java:50


class DBIndexerException(Exception):
    pass


class IndexerMode:
    INDEX = "INDEX"
    SEARCH_INDEXED = "SEARCH_INDEXED"
    SEARCH_UNINDEXED = "SEARCH_UNINDEXED"


class DBIndexer:
    """``DBIndexerHip extends DBIndexer``: device digestion behind the same API."""

    def __init__(self, sparam: DBIndexSearchParams, mode: str = IndexerMode.INDEX,
                 indexStore: Optional[DBIndexStoreHip] = None, device: int = 0,
                 database_name: str = "synthetic.fasta"):
        self.sparam = sparam
        self.mode = mode
        if indexStore is None:  # DBIndexer(sparam, mode) (:167-200)
            indexStore = (MassRangeFilteringIndexHip(sparam, device) if mode == IndexerMode.SEARCH_UNINDEXED
                          else DBIndexStoreHip(sparam, device))
        if mode == IndexerMode.SEARCH_UNINDEXED and not isinstance(indexStore, MassRangeFilteringIndexHip):
            raise DBIndexerException("SEARCH_UNINDEXED needs the MassRangeFilteringIndex store")
        self.indexStore = indexStore
        self.indexStore.setDeviceDigest(True)
        self.protNum = -1
        self.decoyDiscarded = 0
        self.inited = False
        self.database_name = database_name
        self._cache_populated = False

    # DBIndexer.init (:412-451)
    def init(self) -> None:
        if self.inited:
            raise RuntimeError("Already inited")
        self.protNum = -1
        self.indexStore.init(self.database_name + "_dbindex_hip")
        if self.mode == IndexerMode.SEARCH_UNINDEXED and os.path.isfile(self.database_name):
            self._set_protein_cache(self.database_name)  # setProteinCache() (:443-444, :463-500)
        elif (self.mode == IndexerMode.SEARCH_INDEXED and os.path.isfile(self.database_name)
              and self.indexStore.indexExists()):
            # a reused index: the cache holds every FASTA protein (:438-442, :483-489)
            protCache = ProteinCache()
            for d, s in _fasta_items(self.database_name):
                protCache.addProtein(d, s)
            self.indexStore.setProteinCache(protCache)
        self.inited = True

    def _set_protein_cache(self, fasta) -> None:
        """SEARCH_UNINDEXED: every FASTA protein into the ProteinCache (no decoy
        filter, :482-488), digested once on the device."""
        if self._cache_populated:
            return
        self.indexStore.startAddSeq()
        try:
            for d, s in _fasta_items(fasta):
                self.cutSeq(d, s)
        finally:
            self.indexStore.stopAddSeq()
        self._cache_populated = True

    # DBIndexerHip.cutSeq: only hand the protein to the store (DBIndexer.java:251)
    def cutSeq(self, protAccession: str, protSeq: str) -> None:
        # inline '[formula]' PTMs (DBIndexer.java:288-303) are digested on the
        # device as the reference does (dbi_build: k_ptm_digest)
        self.protNum += 1
        self.indexStore.addProteinDef(self.protNum, protAccession, protSeq)

    # DBIndexer.run (:508-684), INDEX mode
    def run(self, fasta: Union[PackedProteins, str, Iterable[Tuple[str, str]], None] = None) -> None:
        if not self.inited:
            raise RuntimeError("Not initialized.")
        if self.mode == IndexerMode.SEARCH_UNINDEXED:
            # the reference returns here (:516-518) and cuts the ProteinCache per
            # search; a FASTA given here fills the cache when init() had no file
            if fasta is not None:
                self._set_protein_cache(fasta)
            return
        if self.indexStore.indexExists():
            return  # "Found existing index, skipping indexing." (:522-527)
        items = _fasta_items(fasta)
        if not any(uniprot_accession(d) for d, _ in items):
            raise DBIndexerException("Reading FASTA file was not able to extract any single Uniprot "
                                     "protein accession.")  # :560-565
        decoy = re.compile(self.sparam.discard_decoy_regexp) if self.sparam.discard_decoy_regexp else None
        self.indexStore.startAddSeq()
        try:
            protCache = ProteinCache()  # :594-595
            self.indexStore.setProteinCache(protCache)
            self.decoyDiscarded = 0
            for d, s in items:
                protCache.addProtein(d, s)  # every protein, decoys included (:605)
                if decoy is not None and decoy.search(fasta_accession(d)):  # Matcher.find (:609-615)
                    self.decoyDiscarded += 1
                    continue
                self.cutSeq(d, s)
        finally:
            self.indexStore.stopAddSeq()

    # --- queries (DBIndexer.java:762-871) -------------------------------------
    def getSequencesUsingDaltonTolerance(self, precursorMass: float, massToleranceInDa: float):
        if self.mode == IndexerMode.SEARCH_UNINDEXED:
            return self.indexStore.cutAndSearch([MassRange(precursorMass, massToleranceInDa)])
        return self.indexStore.getSequences(precursorMass, massToleranceInDa)

    def getSequencesUsingPPMTolerance(self, precursorMass: float, massToleranceInPPM: float):
        massTolerance = tolerance_in_dalton(precursorMass, massToleranceInPPM)
        if self.mode == IndexerMode.SEARCH_UNINDEXED:  # no upper-bound probe loop (:797-802)
            return self.indexStore.cutAndSearch([MassRange(precursorMass, massTolerance)])
        sequences = self.indexStore.getSequences(precursorMass, massTolerance)
        seen = {s.getSequence() for s in sequences}
        upperBound = precursorMass + massTolerance
        while True:  # upper-bound probe loop (:808-839)
            massTolerance2 = tolerance_in_dalton(upperBound, massToleranceInPPM)
            lowerBoundOfUpperBoundMass = upperBound - massTolerance2
            if lowerBoundOfUpperBoundMass < precursorMass:
                sequences2 = self.indexStore.getSequences(upperBound, 0.0)
                if not sequences2:
                    break
                for s2 in sequences2:
                    if s2.getSequence() not in seen:
                        sequences.append(s2)
                        seen.add(s2.getSequence())
            else:
                break
            newupperBound = upperBound + PRECISION
            if newupperBound == upperBound:
                break
            upperBound = newupperBound
        return sequences

    def getSequences(self, massRanges: List[MassRange]):
        if self.mode == IndexerMode.SEARCH_UNINDEXED:
            return self.indexStore.cutAndSearch(massRanges)
        return self.indexStore.getSequences(massRanges)

    def getProteins(self, seq: Union[IndexedSequence, str]):
        if isinstance(seq, IndexedSequence):
            return self.indexStore.getProteins(seq)
        # getProteins(String) (:925-947): exact-mass lookup then string equality
        mass = calculate_mass(seq, self.sparam)
        ret: Set[IndexedProtein] = set()
        for s in self.getSequencesUsingDaltonTolerance(mass, 0.0):
            if s.getSequence() == seq:
                ret.update(self.indexStore.getProteins(s))
        return ret

    def getNumParentMasses(self) -> int:
        return self.indexStore.getNumberSequences()

    def getParentMasses(self) -> List[float]:
        return [k * 1.0 / self.sparam.mass_group_factor for k in self.indexStore.getEntryKeys()]


def _fasta_items(fasta) -> List[Tuple[str, str]]:
    if isinstance(fasta, PackedProteins):
        from .fasta import uniprot_header
        return [(fasta.defs[i] if fasta.defs else uniprot_header(i), fasta.sequence(i))
                for i in range(fasta.n_proteins)]
    if isinstance(fasta, str):  # a FASTA file: the library's multi-threaded parser (dbi_fasta_read)
        from .fasta import read_fasta
        pp = read_fasta(fasta)
        return [(pp.defs[i], pp.sequence(i)) for i in range(pp.n_proteins)]
    return list(fasta)
