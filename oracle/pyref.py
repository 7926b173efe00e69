"""oracle/pyref.py — TEST INFRASTRUCTURE ONLY.

Pure-Python twin of oracle/cpu_ref.cpp, written independently from the Java
sources (paths relative to /root/reference/src/main/java/edu/scripps/yates/dbindex/):

* ``cut_seq``         — DBIndexer.cutSeq(String,String), DBIndexer.java:237-405
* ``filter_sequence`` — DBIndexStoreSQLiteMult.filterSequence, :245-268
* ``Store``           — SQLiteMult buckets (:215-291) -> SQLiteByte rows keyed by
                        (int)(mass*factor) (DBIndexStoreSQLiteByte.java:185-226) ->
                        IndexMerge.getMergedData (:620-719)
* ``Store.get_sequences`` — SQLiteMult.getSequences(m,tol) :315-350 +
                        IndexMerge.getSequences/parseAddPeptideInfo :146-217,386-481
* ``get_residues``    — Util.getResidues, Util.java:130-162
* ``cut_and_search``  — DBIndexer.cutAndSearch :707-747 over MassRangeFilteringIndex
                        (init :40-67, filterSequence :90-108, addSequence :111-130)

Only for small inputs (pure-Python loops).  Agreement with the C++ oracle is
bit-exact (masses compared as float64 bit patterns).  Ties between different
peptides of identical mass inside one row are ordered by (16-bit tag of the
string -- its length and first / last four residues hashed --, first appearance): the reference's THashMap order is unspecified,
so this project pins it (DESIGN.md semantics A7).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

MAX_PRECURSOR_INT = 8000
INCLUDE, SKIP, SKIP_PROTEIN_START = 0, 1, 2


def java_int(d: float) -> int:
    """Java ``(int) d`` (JLS 5.1.3)."""
    if math.isnan(d):
        return 0
    if d >= 2147483647.0:
        return 2147483647
    if d <= -2147483648.0:
        return -2147483648
    return int(d)  # truncation toward zero


class Enzyme:
    """Pinned ``Enzyme`` rule (external class)."""

    def __init__(self, residues: str, nocut: str, semi: bool):
        self.residues = set(residues)
        self.nocut = set(nocut)
        self.semi = semi

    def is_enzyme(self, c: str) -> bool:
        return c in self.residues

    def check_cleavage(self, seq: str, start: int, end: int) -> bool:
        if start == 0:
            n_ok = True
        else:
            n_ok = seq[start - 1] in self.residues and seq[start] not in self.nocut
        if end == len(seq) - 1:
            c_ok = True
        else:
            c_ok = seq[end] in self.residues and seq[end + 1] not in self.nocut
        return (n_ok or c_ok) if self.semi else (n_ok and c_ok)


def filter_sequence(params, prec_mass: float, sequence: str) -> int:
    mand = params.mandatory_internal_aas
    if mand is not None and len(mand) > 0:
        seen = set()
        for aa in mand:
            if aa in seen:
                continue
            seen.add(aa)
            if aa in sequence[: len(sequence) - 1]:
                return INCLUDE
        return SKIP
    if params.max_precursor_mass < prec_mass or params.min_precursor_mass > prec_mass:
        return SKIP
    return INCLUDE


def cut_seq(params, prot_seq: str, protein_id: int, out: list, filt=None) -> None:
    """Appends (mass, protein_id, offset, length, dropped) per INCLUDE'd peptide;
    ``filt`` replaces the store's filterSequence (default: SQLiteMult's)."""
    filt = filt or filter_sequence
    enz = Enzyme(params.enzyme_residues, params.enzyme_nocut_residues, params.semi_cleavage)
    table = params.residue_mass
    length = len(prot_seq)
    max_mc = params.max_missed_cleavages
    br = MAX_PRECURSOR_INT // params.index_factor
    for start in range(length):
        end = start
        prec = 0.0
        if params.h2o_plus_proton_added:
            prec += params.h2o_proton
        prec += params.cterm
        prec += params.nterm
        pep_size = 0
        mc = -1
        while prec <= params.max_precursor_mass and end < length:
            pep_size += 1
            prec = prec + table.get(prot_seq[end], 0.0)
            pep = prot_seq[start: end + 1]
            if enz.is_enzyme(prot_seq[end]):
                mc += 1
            if enz.check_cleavage(prot_seq, start, end):
                if mc > max_mc:
                    break
                if prec > params.max_precursor_mass:
                    break
                if pep_size >= params.min_pep_length and prec >= params.min_precursor_mass:
                    if params.mandatory_internal_aas is not None:
                        if not any(aa in pep for aa in params.mandatory_internal_aas):
                            break
                    fr = filt(params, prec, pep)
                    if fr == SKIP_PROTEIN_START:
                        break
                    if fr == INCLUDE:
                        bucket = java_int(prec) // br
                        out.append((prec, protein_id, start, end - start + 1,
                                    bucket > params.index_factor - 1))
            end += 1


def digest(params, proteins: Sequence[str]) -> list:
    out: list = []
    for pid, s in enumerate(proteins):
        cut_seq(params, s, pid, out)
    return out


def peptide_tag(s: str) -> int:
    """Pinned tie-break between different peptides of bit-identical mass
    (DESIGN.md A7): a 16-bit hash of the length and the first and last (up
    to) four residues."""
    b = s.encode("ascii")
    n = len(b)
    head = sum(b[k] << (8 * k) for k in range(min(4, n)))
    tail = sum(b[n - 1 - k] << (8 * k) for k in range(min(4, n)))
    M = 0xFFFFFFFF
    x = ((head * 0x9E3779B1) & M) ^ ((tail * 0x85EBCA77) & M) ^ ((n * 0xC2B2AE3D) & M)
    x ^= x >> 15
    x = (x * 0x2C1B3C6D) & M
    x ^= x >> 12
    return (x >> 16) ^ (x & 0xFFFF)


# FormulaCalculator.calculateMass (edu.scripps.yates.utilities, not vendored),
# restated independently of oracle/cpu_ref.cpp and of the product: its own
# element table (monoisotopic masses of the most abundant isotope, IUPAC /
# NIST values), a regular-expression tokenizer, and the count x mass terms
# summed left to right.  An element symbol without a mass, a sign without
# digits or anything that is not "Symbol[-]digits*" is unknown: NaN.
_ELEMENT_MONO = {
    "H": 1.00782503207, "D": 2.0141017778, "B": 11.0093054, "C": 12.0, "N": 14.0030740048,
    "O": 15.99491461956, "F": 18.99840322, "Na": 22.9897692809, "Mg": 23.9850417, "Si": 27.9769265325,
    "P": 30.97376163, "S": 31.97207100, "Cl": 34.96885268, "K": 38.96370668, "Ca": 39.96259098,
    "Li": 7.01600455, "Fe": 55.9349375, "Cu": 62.9295975, "Zn": 63.9291422, "Se": 79.9165213,
    "Br": 78.9183371, "I": 126.904473, "Hg": 201.970643,
}


def formula_mass(formula: str) -> float:
    import re
    pos, mass = 0, 0.0
    for m in re.finditer(r"([A-Z][a-z]*)(-?)([0-9]*)", formula):
        if m.start() != pos:
            return float("nan")
        sym, neg, digits = m.groups()
        if neg and not digits:
            return float("nan")
        if sym not in _ELEMENT_MONO:
            return float("nan")
        count = int(digits) if digits else 1
        mass = mass + float(-count if neg else count) * _ELEMENT_MONO[sym]
        pos = m.end()
    return mass if pos == len(formula) else float("nan")


def get_residues(offset: int, length: int, prot: str) -> Tuple[str, str]:
    """Util.getResidues (Util.java:130-162), including its right-flank quirk."""
    n = len(prot)
    left_i = offset - 3 if offset >= 3 else 0
    left_len = min(3, offset)
    left = prot[left_i: left_i + left_len]
    end = offset + length
    right_len = min(3, n - end - 1)
    right = prot[end: end + right_len] if end < n else ""
    return "-" * (3 - len(left)) + left, right + "-" * (3 - len(right))


class Store:
    """SQLiteMult + SQLiteByteIndexMerge semantics over in-memory rows."""

    def __init__(self, params, proteins: Sequence[str]):
        self.p = params
        self.proteins = list(proteins)
        self.nb = params.index_factor
        self.br = MAX_PRECURSOR_INT // self.nb
        self.buckets: List[Dict[int, list]] = [dict() for _ in range(self.nb)]
        self.total_seq_count = 0
        self.flat: list = []

    def add_sequence(self, mass: float, offset: int, length: int, pid: int) -> None:
        self.total_seq_count += 1
        bucket = java_int(mass) // self.br
        if bucket > self.nb - 1:
            return
        key = java_int(mass * self.p.mass_group_factor)
        self.buckets[bucket].setdefault(key, []).append((mass, offset, length, pid))

    def stop_add_seq(self) -> None:
        for b in range(self.nb):
            for key in list(self.buckets[b].keys()):
                recs = self.buckets[b][key]
                groups: Dict[str, list] = {}  # dict keeps first-appearance order
                for (mass, off, ln, pid) in recs:
                    pep = self.proteins[pid][off: off + ln]
                    if pep not in groups:
                        groups[pep] = [mass, off, ln, [pid]]
                    else:
                        groups[pep][3].append(pid)
                # stable sort by mass; equal masses by (16-bit tag, first appearance)
                merged = [groups[k] for k in sorted(groups, key=lambda k: (groups[k][0], peptide_tag(k)))]
                self.buckets[b][key] = merged
        self.flat = []
        for b in range(self.nb):
            for key in sorted(self.buckets[b].keys()):
                for g in self.buckets[b][key]:
                    g.append(len(self.flat))
                    self.flat.append(g)

    def number_sequences(self) -> int:
        return sum(len(b) for b in self.buckets)

    def entry_keys(self) -> List[int]:
        out = []
        for b in self.buckets:
            out.extend(sorted(b.keys()))
        return out

    def get_sequences(self, prec_mass: float, tol: float) -> List[int]:
        lo = prec_mass - tol
        if lo < 0:
            lo = 0
        hi = prec_mass + tol
        b0, b1 = java_int(lo) // self.br, java_int(hi) // self.br
        if b0 > self.nb - 1 or b1 > self.nb - 1:
            return []
        out = []
        f = self.p.mass_group_factor
        for b in range(b0, b1 + 1):
            lo_f = prec_mass - tol
            if lo_f < 0.0:
                lo_f = 0.0
            hi_f = prec_mass + tol
            kmin = max(0, java_int(lo_f * f))
            kmax = java_int(hi_f * f)
            for key in sorted(self.buckets[b].keys()):
                if key < kmin or key > kmax:
                    continue
                for g in self.buckets[b][key]:
                    if g[0] > hi_f:
                        break
                    if g[0] < lo_f:
                        continue
                    out.append(g[4])
        return out


def build(params, proteins: Sequence[str]) -> Store:
    st = Store(params, proteins)
    for (mass, pid, off, ln, _dropped) in digest(params, proteins):
        st.add_sequence(mass, off, ln, pid)
    st.stop_add_seq()
    return st


def range_filter(min_masses: Sequence[float], max_masses: Sequence[float]):
    """MassRangeFilteringIndex.filterSequence (MassRangeFilteringIndex.java:90-108)."""
    def filt(params, prec_mass: float, sequence: str) -> int:
        skip_start = True
        for lo, hi in zip(min_masses, max_masses):
            if prec_mass <= hi:
                skip_start = False
                if prec_mass >= lo:
                    return INCLUDE
        return SKIP_PROTEIN_START if skip_start else SKIP
    return filt


def cut_flanks(prot: str, offset: int, length: int) -> Tuple[str, str]:
    """The flanks cutSeq builds for addSequence (DBIndexer.java:356-383)."""
    end = offset + length - 1
    left = prot[max(0, offset - 3): offset].rjust(3, "-")
    right = prot[end + 1: end + 1 + max(0, min(3, len(prot) - end - 1))].ljust(3, "-")
    return left, right


def cut_and_search(params, proteins: Sequence[str], ranges: Sequence[Tuple[float, float]]) -> Dict[str, tuple]:
    """DBIndexer.cutAndSearch: every protein of the cache re-cut through the
    range filter; one entry per sequence (the first occurrence's mass, offset,
    length and flanks) with its protein ids without repeats.  Returns
    {sequence: (mass, offset, length, left, right, [protein ids])}."""
    mins = [m - t for m, t in ranges]  # `if (minMass == 0) minMass = 0f` changes nothing
    maxs = [m + t for m, t in ranges]
    filt = range_filter(mins, maxs)
    occ: list = []
    for pid, s in enumerate(proteins):
        cut_seq(params, s, pid, occ, filt)
    out: Dict[str, tuple] = {}
    for mass, pid, off, ln, _ in occ:
        seq = proteins[pid][off: off + ln]
        e = out.get(seq)
        if e is None:
            left, right = cut_flanks(proteins[pid], off, ln)
            out[seq] = (mass, off, ln, left, right, [pid])
        elif pid not in e[5]:
            e[5].append(pid)
    return out
