"""FASTA input for the index build: a packed-protein container, a UniProt-style
FASTA reader/writer, and the seeded synthetic generator of SURVEY.md §8(d).

Protein numbering follows the reference: protein id = 0-based position in FASTA
order (``DBIndexer.java:251,418``; ``ProteinCache.addProtein``
``ProteinCache.java:84-95``; ``DBIndexStoreSQLiteMult.addProteinDef`` returns
``num`` ``:446-450``).  The reference rejects FASTA without UniProt accessions
(``DBIndexer.java:560-565``), so synthetic headers are UniProt style.
"""
from __future__ import annotations

import hashlib
import io
from dataclasses import dataclass, field
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

# SwissProt residue frequencies (percent), SURVEY.md §8(d)
AA_FREQ = {
    "A": 8.25, "R": 5.53, "N": 4.06, "D": 5.45, "C": 1.37, "Q": 3.93, "E": 6.75,
    "G": 7.07, "H": 2.27, "I": 5.96, "L": 9.66, "K": 5.84, "M": 2.42, "F": 3.86,
    "P": 4.70, "S": 6.56, "T": 5.34, "W": 1.08, "Y": 2.92, "V": 6.87,
}
CANONICAL = "".join(AA_FREQ)

# Named synthetic configurations (BASELINE.json configs; seeds per SURVEY.md §8(d))
CONFIGS = {
    "1k": dict(n_proteins=1000, seed=1),
    "human": dict(n_proteins=20000, seed=2),
    "swissprot": dict(n_proteins=560000, seed=3),
}


@dataclass
class PackedProteins:
    """Proteins packed for HBM: ``residues`` (u8, all sequences concatenated in
    FASTA order) + ``offsets`` (u64, P+1 entries) + the FASTA definitions."""

    residues: np.ndarray
    offsets: np.ndarray
    defs: List[str] = field(default_factory=list)

    @property
    def n_proteins(self) -> int:
        return int(self.offsets.shape[0] - 1)

    @property
    def n_residues(self) -> int:
        return int(self.residues.shape[0])

    def sequence(self, i: int) -> str:
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return self.residues[a:b].tobytes().decode("ascii")

    def sequences(self) -> List[str]:
        return [self.sequence(i) for i in range(self.n_proteins)]

    def sha256(self) -> str:
        h = hashlib.sha256()
        h.update(np.ascontiguousarray(self.residues).tobytes())
        h.update(np.ascontiguousarray(self.offsets, dtype=np.uint64).tobytes())
        return h.hexdigest()

    def slice(self, p0: int, p1: int) -> "PackedProteins":
        """Proteins [p0, p1) as a new container (offsets rebased to 0)."""
        a, b = int(self.offsets[p0]), int(self.offsets[p1])
        offs = (self.offsets[p0: p1 + 1] - np.uint64(a)).astype(np.uint64)
        defs = self.defs[p0:p1] if self.defs else []
        return PackedProteins(self.residues[a:b].copy(), offs, defs)

    @staticmethod
    def from_sequences(seqs: Sequence[str], defs: Optional[Sequence[str]] = None) -> "PackedProteins":
        lens = np.array([len(s) for s in seqs], dtype=np.uint64)
        offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        res = np.frombuffer("".join(seqs).encode("ascii"), dtype=np.uint8).copy()
        return PackedProteins(res, offs, list(defs) if defs is not None else [])


def uniprot_header(i: int) -> str:
    return (f"sp|S{i:07d}|SYN{i}_HUMAN Synthetic {i} OS=Homo sapiens OX=9606 "
            f"GN=SYN{i} PE=1 SV=1")


def synthetic(n_proteins: int, seed: int, copy_frac: float = 0.10,
              len_mu: float = float(np.log(300.0)), len_sigma: float = 0.6,
              len_min: int = 30, len_max: int = 35000, with_defs: bool = True) -> PackedProteins:
    """Seeded synthetic proteome: 20 canonical residues i.i.d.
    at SwissProt frequencies, lognormal lengths clipped to [30, 35000], and 10 %
    of proteins overwritten with a random 50-300 aa segment of an earlier
    protein (shared peptides exercise the dedup of IndexMerge.getMergedData)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.clip(np.rint(rng.lognormal(len_mu, len_sigma, n_proteins)), len_min, len_max)
    lens = lens.astype(np.uint64)
    offs = np.zeros(n_proteins + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    letters = np.frombuffer("".join(AA_FREQ.keys()).encode("ascii"), dtype=np.uint8)
    probs = np.array(list(AA_FREQ.values()), dtype=np.float64)
    probs /= probs.sum()
    res = letters[rng.choice(len(letters), size=total, p=probs)]
    # shared segments: protein i copies [s, s+L) of an earlier protein j
    donors = np.nonzero(rng.random(n_proteins) < copy_frac)[0]
    for i in donors:
        if i == 0:
            continue
        j = int(rng.integers(0, i))
        seg = int(rng.integers(50, 301))
        li, lj = int(lens[i]), int(lens[j])
        seg = min(seg, li, lj)
        sj = int(rng.integers(0, lj - seg + 1))
        si = int(rng.integers(0, li - seg + 1))
        a, b = int(offs[i]) + si, int(offs[j]) + sj
        res[a: a + seg] = res[b: b + seg]
    defs = [uniprot_header(i) for i in range(n_proteins)] if with_defs else []
    return PackedProteins(res, offs, defs)


# ----------------------------------------------------------------------------
# Counter-based synthetic proteome (TrEMBL scale, generated on the device by
# dbi_synth_proteome; this is its numpy twin for tests and the CPU baseline)
# ----------------------------------------------------------------------------
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_RES_SALT = np.uint64(0xD1B54A32D192ED03)


def _fmix64(k: np.ndarray) -> np.ndarray:
    k = k.copy()
    k ^= k >> np.uint64(33)
    k *= np.uint64(0xFF51AFD7ED558CCD)
    k ^= k >> np.uint64(33)
    k *= np.uint64(0xC4CEB9FE1A85EC53)
    k ^= k >> np.uint64(33)
    return k


def synth_tables(len_mu: float = float(np.log(300.0)), len_sigma: float = 0.6, len_min: int = 30,
                 len_max: int = 35000):
    """(len_table u16[4096], res_table u8[65536]): lognormal length quantiles
    clipped to [len_min, len_max] (SURVEY.md §8(d) length model) and the
    residue CDF at SwissProt frequencies."""
    from statistics import NormalDist
    nd = NormalDist()
    q = [(k + 0.5) / 4096 for k in range(4096)]
    lens = np.array([np.exp(len_mu + len_sigma * nd.inv_cdf(x)) for x in q])
    len_table = np.clip(np.rint(lens), len_min, len_max).astype(np.uint16)
    letters = np.frombuffer(CANONICAL.encode("ascii"), dtype=np.uint8)
    probs = np.array([AA_FREQ[c] for c in CANONICAL], np.float64)
    cdf = np.cumsum(probs / probs.sum())
    idx = np.searchsorted(cdf, (np.arange(65536) + 0.5) / 65536.0, side="right")
    res_table = letters[np.minimum(idx, len(letters) - 1)]
    return len_table, np.ascontiguousarray(res_table, np.uint8)


def synth_lengths(seed: int, p_begin: int, n: int, len_table: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        k = np.uint64(seed) * _GOLDEN + np.arange(p_begin + 1, p_begin + n + 1, dtype=np.uint64)
        return len_table[(_fmix64(k) >> np.uint64(52)).astype(np.int64)].astype(np.uint64)


def synth_residue_base(seed: int, p_begin: int, len_table: np.ndarray, chunk: int = 1 << 22) -> int:
    """Global index of protein p_begin's first residue (sum of earlier lengths)."""
    tot = 0
    for a in range(0, p_begin, chunk):
        tot += int(synth_lengths(seed, a, min(chunk, p_begin - a), len_table).sum())
    return tot


def synth_proteome(seed: int, p_begin: int, n: int, res_base: int, tables=None) -> PackedProteins:
    len_table, res_table = tables or synth_tables()
    lens = synth_lengths(seed, p_begin, n, len_table)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) ^ _RES_SALT) * _GOLDEN + np.uint64(res_base)
        g = key + np.arange(total, dtype=np.uint64)
        res = res_table[(_fmix64(g) >> np.uint64(48)).astype(np.int64)]
    return PackedProteins(np.ascontiguousarray(res, np.uint8), offs, [])


def config(name: str, **kw) -> PackedProteins:
    c = dict(CONFIGS[name])
    c.update(kw)
    return synthetic(**c)


# ----------------------------------------------------------------------------
# FASTA text I/O
# ----------------------------------------------------------------------------
def write_fasta(pp: PackedProteins, fh: io.TextIOBase, width: int = 60) -> None:
    for i in range(pp.n_proteins):
        d = pp.defs[i] if pp.defs else uniprot_header(i)
        fh.write(">" + d + "\n")
        s = pp.sequence(i)
        for k in range(0, len(s), width):
            fh.write(s[k: k + width] + "\n")


def iter_fasta(lines: Iterable[str]) -> Iterator[Tuple[str, str]]:
    """Yields (definition, sequence) in file order; definition without '>'.
    Sequence lines are concatenated with whitespace stripped."""
    d: Optional[str] = None
    parts: List[str] = []
    for line in lines:
        if line.startswith(">"):
            if d is not None:
                yield d, "".join(parts)
            d = line[1:].rstrip("\r\n")
            parts = []
        elif d is not None:
            parts.append("".join(line.split()))
    if d is not None:
        yield d, "".join(parts)


def read_fasta(path: str, threads: int = 0, with_defs: bool = True) -> PackedProteins:
    """Packs a FASTA file with the library's multi-threaded parser
    (dbi_fasta_read; same semantics as iter_fasta)."""
    return _from_native(lambda out: _native_lib().dbi_fasta_read(path.encode(), threads, out), with_defs)


def parse_fasta(text, threads: int = 0, with_defs: bool = True) -> PackedProteins:
    """Packs FASTA text (str or bytes) with dbi_fasta_parse."""
    import ctypes
    b = text.encode() if isinstance(text, str) else bytes(text)
    buf = ctypes.create_string_buffer(b, len(b))
    return _from_native(lambda out: _native_lib().dbi_fasta_parse(buf, len(b), threads, out), with_defs)


def _native_lib():
    from . import _native
    return _native.lib()


class _NativeFasta:
    """Owns a dbi_fasta result: freed when the last array viewing its residues goes."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        from . import _native
        _native.lib().dbi_fasta_free(self.ptr)


def _from_native(call, with_defs: bool) -> PackedProteins:
    """The parser's packed proteome without copying its residues: the array
    views the library's buffer (2-MiB pages, dbi_fasta_read), which is freed
    with the array; offsets and definitions are copied (small)."""
    import ctypes
    from . import _native
    out = ctypes.POINTER(_native.DbiFasta)()
    _native.check(call(ctypes.byref(out)))
    owner = _NativeFasta(out)
    f = out.contents
    P, R = f.n_proteins, f.n_residues
    if R:
        buf = (ctypes.c_uint8 * R).from_address(f.residues)
        buf._owner = owner  # the memoryview under the array keeps buf, buf keeps the result
        res = np.ctypeslib.as_array(buf)
    else:
        res = np.zeros(0, np.uint8)
    offs = np.ctypeslib.as_array(f.offsets, shape=(P + 1,)).astype(np.uint64)
    defs: List[str] = []
    if with_defs and P:
        doff = np.ctypeslib.as_array(f.def_off, shape=(P + 1,))
        raw = ctypes.string_at(f.defs, int(doff[-1])).decode("latin-1")
        defs = [raw[int(doff[i]):int(doff[i + 1])] for i in range(P)]
    pp = PackedProteins(res, offs, defs)
    pp.n_uniprot = int(f.n_uniprot)
    return pp


def uniprot_accession(definition: str) -> Optional[str]:
    """Accession of a UniProt-style header ``db|ACC|NAME ...`` (the reference's
    FastaReader.getACCsFromFasta requirement, DBIndexer.java:560-565)."""
    head = definition.split(" ", 1)[0]
    parts = head.split("|")
    if len(parts) >= 3 and parts[0] in ("sp", "tr") and parts[1]:
        return parts[1]
    return None


def fasta_accession(definition: str) -> str:
    """What ``DBIndexer.run`` matches the decoy regexp against
    (``fasta.getAccession()``, DBIndexer.java:608): the UniProt accession of a
    ``db|ACC|NAME`` header, else the header's first word (decoy prefixes such as
    ``Reverse_sp|...`` stay in it).  ``Fasta`` lives in the absent
    edu.scripps.yates.utilities jar: parity unpinned."""
    acc = uniprot_accession(definition)
    return acc if acc is not None else definition.split(None, 1)[0] if definition.strip() else ""
