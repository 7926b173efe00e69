// dbi_fasta.h — the FASTA parser's internal interface for the fused one-off
// build (dbi_build_fasta, dbi_engine.hip): the parser hands each thread's
// packed residues to a sink as it goes, so they reach HBM while the rest of
// the file is still being parsed.
#pragma once
#include <cstdint>

#include "../../include/dbindex_hip.h"

namespace dbi {

struct FastaSink {
    virtual ~FastaSink() = default;
    // After the count pass (threads = the parse threads): *stream = true to
    // receive the residues through slot / flush, false to have them packed
    // into the host buffer as dbi_fasta_read does.  Non-zero: abort with it.
    virtual int sized(uint64_t n_res, uint64_t n_prot, int threads, bool ptm_known, bool ptm, bool* stream) = 0;
    // thread t's next staging buffer (cap bytes; the previous one was handed over)
    virtual uint8_t* slot(int t, uint64_t* cap) = 0;
    // thread t packed residues [at, at + n) of the proteome into p (its current slot)
    virtual bool flush(int t, uint64_t at, const uint8_t* p, uint64_t n) = 0;
};

// dbi_fasta_parse / dbi_fasta_read with an optional sink (streamed: the
// returned dbi_fasta has residues == NULL)
int fasta_parse_core(const char* buf, uint64_t len, int threads, FastaSink* sink, dbi_fasta** out);
int fasta_read_core(const char* path, int threads, FastaSink* sink, dbi_fasta** out);

// is [p, p + n) inside a live dbi_fasta residue buffer (2-MiB pages)?
// *ptm_known: the parser looked for '[' (inline PTMs), *ptm: found one
bool fasta_residue_buffer(const void* p, uint64_t n, bool* ptm_known, bool* ptm);

}  // namespace dbi
