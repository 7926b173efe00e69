"""Search parameters for the index build — the host-side mirror of the
reference's ``DBIndexSearchParams`` getters that the hot loop reads, plus the
pinned ``AssignMass`` residue table and ``Enzyme`` cleavage sets.

Reference pointers (relative to
``/root/reference/src/main/java/edu/scripps/yates/dbindex/``):

* ``io/DBIndexSearchParamsImpl.java:46-75`` — the programmatic constructor
  (index type, index factor, missed cleavages, min/max precursor, nocut and
  enzyme residues, mono/avg, H2O+H+, mass group factor, mandatory AAs, semi).
* ``/root/reference/src/main/resources/dbindex.properties:6-22`` — defaults
  (index_factor 8, 500..6000 Da, trypsin "KR", empty nocut, factor 10000).
* ``Constants.java:10`` — ``MIN_PEP_LENGTH = 6``.
* ``AssignMass`` (external, ``edu.scripps.yates:utilities:1.6-SNAPSHOT``,
  not vendored): the residue table below is PINNED by this project (standard
  monoisotopic residue masses, Unimod values) and is an *input* of the engine —
  a Java caller passes ``AssignMass.getMass(c)`` for every char instead, so the
  arithmetic is identical to the reference's by construction.

``to_c()`` packs the flat ``dbi_params`` struct of ``include/dbindex_hip.h``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, Optional

# Pinned monoisotopic residue masses (Da).  Letters absent here map to 0.0.
MONO_RESIDUE_MASS: Dict[str, float] = {
    "G": 57.021464, "A": 71.037114, "S": 87.032028, "P": 97.052764,
    "V": 99.068414, "T": 101.047679, "C": 103.009185, "L": 113.084064,
    "I": 113.084064, "N": 114.042927, "D": 115.026943, "Q": 128.058578,
    "K": 128.094963, "E": 129.042593, "M": 131.040485, "H": 137.058912,
    "F": 147.068414, "R": 156.101111, "Y": 163.063329, "W": 186.079313,
    "U": 150.953636, "O": 237.147727,
}
H2O = 18.0105646863
PROTON = 1.00727646688
H2O_PROTON = H2O + PROTON  # AssignMass.H2O_PROTON (pinned)

MAX_PRECURSOR_MASS = 8000.0  # Constants.java:20
MIN_PEP_LENGTH = 6           # Constants.java:10
CANONICAL_AA = "ACDEFGHIKLMNPQRSTVWY"


class DbiParams(ctypes.Structure):
    """ctypes image of ``struct dbi_params`` (include/dbindex_hip.h)."""

    _fields_ = [
        ("min_mh", ctypes.c_double),
        ("max_mh", ctypes.c_double),
        ("h2o_proton", ctypes.c_double),
        ("cterm", ctypes.c_double),
        ("nterm", ctypes.c_double),
        ("mass", ctypes.c_double * 256),
        ("cleave", ctypes.c_uint8 * 256),
        ("nocut", ctypes.c_uint8 * 256),
        ("mandatory", ctypes.c_uint8 * 256),
        ("max_missed", ctypes.c_int32),
        ("semi", ctypes.c_int32),
        ("add_h2o_proton", ctypes.c_int32),
        ("min_len", ctypes.c_int32),
        ("mass_group_factor", ctypes.c_int32),
        ("index_factor", ctypes.c_int32),
        ("mandatory_mode", ctypes.c_int32),
        ("mandatory_count", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 8),
    ]


@dataclass
class DBIndexSearchParams:
    """Mirror of the getters ``DBIndexer.cutSeq`` and the SQLiteMult store read.

    Field names follow the Java getters (``getMaxMissedCleavages`` ->
    ``max_missed_cleavages`` ...).  ``enzyme_residues`` is the Enzyme's cleave
    set (``DBIndexSearchParamsImpl.java:62-65``); ``semi_cleavage`` the
    ``isSemiCleavage()`` flag; ``mandatory_internal_aas`` is ``None`` (the
    reference default) or a string of residues.
    """

    max_missed_cleavages: int = 2
    min_precursor_mass: float = 500.0
    max_precursor_mass: float = 6000.0
    enzyme_residues: str = "KR"
    enzyme_nocut_residues: str = ""
    semi_cleavage: bool = False
    h2o_plus_proton_added: bool = True
    mass_group_factor: int = 10000
    index_factor: int = 8
    mandatory_internal_aas: Optional[str] = None
    discard_decoy_regexp: Optional[str] = None  # getDiscardDecoyRegexp (DBIndexSearchParamsImpl.java:483)
    min_pep_length: int = MIN_PEP_LENGTH
    h2o_proton: float = H2O_PROTON
    cterm: float = 0.0
    nterm: float = 0.0
    residue_mass: Dict[str, float] = field(default_factory=lambda: dict(MONO_RESIDUE_MASS))

    # --- named configurations of BASELINE.json --------------------------------
    @classmethod
    def trypsin(cls, missed: int = 2, **kw) -> "DBIndexSearchParams":
        return cls(max_missed_cleavages=missed, **kw)

    @classmethod
    def semi_tryptic(cls, missed: int = 2, **kw) -> "DBIndexSearchParams":
        return cls(max_missed_cleavages=missed, semi_cleavage=True, **kw)

    @classmethod
    def non_specific(cls, max_len: int = 50, **kw) -> "DBIndexSearchParams":
        """Non-specific digestion, lengths 6..max_len: every canonical residue is
        a cleavage site, so ``mc = len-1`` and ``mc <= max_len-1`` <=> ``len <= max_len``
        (SURVEY.md §8(a) A2)."""
        return cls(enzyme_residues=CANONICAL_AA, max_missed_cleavages=max_len - 1, **kw)

    # --- static modifications (SearchParamReader.java:357-362, 401-583) --------
    STATIC_MOD_ORDER = "GASPVTCLIXNOBDQKZEMHFRYW"  # the reader's add_<X>_<name> order

    def with_static_mods(self, mods: Dict[str, float], n15_enrichment: float = 0.0,
                         cterm: Optional[float] = None, nterm: Optional[float] = None) -> "DBIndexSearchParams":
        """A copy with the params file's static modifications applied to the
        residue table: ``add_<X>_<name> = f`` goes through
        ``AssignMassToStaticParam.addMassAndStaticParam`` (model/AssignMassToStaticParam.java:7-14),
        which ignores ``f <= 0`` and otherwise calls ``AssignMass.addMass(X, f)``
        (external jar; restated as mass[X] += f -- parity unpinned).  With N15
        enrichment e > 0, f becomes ``f * e``, except cysteine:
        ``f + e * (f - 57.02146f)`` (:451-456, float literal).  ``add_C_terminus`` /
        ``add_N_terminus`` SET cTerm / nTerm (``AssignMass.setcTerm``, :401-407)."""
        import dataclasses
        import numpy as np
        unknown = set(mods) - set(self.STATIC_MOD_ORDER)
        if unknown:
            raise ValueError(f"no add_<X> parameter for residue(s) {sorted(unknown)}")
        table = dict(self.residue_mass)
        for ch in self.STATIC_MOD_ORDER:
            f = float(mods.get(ch, 0.0))
            if n15_enrichment > 0:
                if ch == "C":
                    f = f + n15_enrichment * (f - float(np.float32(57.02146)))
                else:
                    f = f * n15_enrichment
            if f <= 0:
                continue
            table[ch] = table.get(ch, 0.0) + f
        out = dataclasses.replace(self, residue_mass=table)
        if cterm is not None:
            out.cterm = float(cterm)
        if nterm is not None:
            out.nterm = float(nterm)
        return out

    # --- helpers ---------------------------------------------------------------
    def mass_table(self):
        t = [0.0] * 256
        for k, v in self.residue_mass.items():
            t[ord(k)] = float(v)
        return t

    def bucket_mass_range(self) -> int:
        return int(MAX_PRECURSOR_MASS) // self.index_factor  # DBIndexStoreSQLiteMult.java:56

    def to_c(self) -> DbiParams:
        p = DbiParams()
        p.min_mh = float(self.min_precursor_mass)
        p.max_mh = float(self.max_precursor_mass)
        p.h2o_proton = float(self.h2o_proton)
        p.cterm = float(self.cterm)
        p.nterm = float(self.nterm)
        for i, v in enumerate(self.mass_table()):
            p.mass[i] = v
        for ch in self.enzyme_residues:
            p.cleave[ord(ch)] = 1
        for ch in self.enzyme_nocut_residues:
            p.nocut[ord(ch)] = 1
        if self.mandatory_internal_aas is not None:
            p.mandatory_mode = 1
            p.mandatory_count = len(self.mandatory_internal_aas)
            for ch in self.mandatory_internal_aas:
                p.mandatory[ord(ch)] = 1
        p.max_missed = int(self.max_missed_cleavages)
        p.semi = 1 if self.semi_cleavage else 0
        p.add_h2o_proton = 1 if self.h2o_plus_proton_added else 0
        p.min_len = int(self.min_pep_length)
        p.mass_group_factor = int(self.mass_group_factor)
        p.index_factor = int(self.index_factor)
        return p


def tolerance_in_dalton(actual_mass: float, ppm: float) -> float:
    """``IndexUtil.getToleranceInDalton`` (util/IndexUtil.java:238-240)."""
    return actual_mass * (1 - 1 / (ppm / 1000000 + 1))


def calculate_mass(seq: str, params: DBIndexSearchParams) -> float:
    """``IndexUtil.calculateMass(seq, h2o)`` (util/IndexUtil.java:197-208):
    H2O+H+, cTerm, nTerm, then residues left to right — the same order as the
    cutSeq accumulation, so the result is bit-identical to the index mass."""
    t = params.residue_mass
    mass = 0.0
    if params.h2o_plus_proton_added:
        mass += params.h2o_proton
    mass += params.cterm
    mass += params.nterm
    for ch in seq:
        mass += t.get(ch, 0.0)
    return mass
