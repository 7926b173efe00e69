// dbi_fasta.h — the FASTA parser's internal interface to the engine.
#pragma once
#include <cstdint>

namespace dbi {

// Is [p, p + n) inside a live dbi_fasta residue buffer (2-MiB pages, which
// dbi_build pins and DMAs directly)?  *ptm_known: the parser looked for '['
// (inline PTMs), *ptm: it found one.
bool fasta_residue_buffer(const void* p, uint64_t n, bool* ptm_known, bool* ptm);

}  // namespace dbi
