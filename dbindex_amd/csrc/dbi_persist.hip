// dbi_persist.hip — a built index on disk and back.
//
// The reference persists its index in SQLite files named after the FASTA and
// an md5 of the search parameters (IndexUtil.java:270-324;
// DBIndexStoreSQLiteMult.java:92-149), and DBIndexer.run skips indexing when
// indexExists() finds it (DBIndexer.java:522-527).  Here one little-endian
// binary file holds the proteome the index refers to (residues, offsets and,
// for the DBIndexStore mirror, the ProteinCache definitions) and the index
// itself (unique table + occurrence CSR); its header carries a fingerprint of
// every parameter the build read, so a file is reused only for the same
// parameters — the role of the reference's params md5.
//
//   header  (dbi_index_header below, 128 B)
//   u8  residues[R]            u64 offsets[P+1]
//   u64 def_off[P+1]           char defs[def_bytes]        (empty for engine saves)
//   f64 mass[U]  u32 prot_id[U]  u32 offset[U]  u32 length[U]  u32 occ_off[U+1]  u32 occ_prot[K]
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "dbi_engine.h"

using namespace dbi;

namespace dbi {
namespace {

// format 02: the pinned tie order of equal-mass peptides is the end-bytes tag
// (dbi_internal.h peptide_tag, round 3); a 01 file (FNV-1a tag) orders such
// ties differently from a fresh build, so it is not reused (rebuilt instead)
constexpr char MAGIC[8] = {'D', 'B', 'I', 'H', 'I', 'P', '0', '2'};

struct dbi_index_header {
    char magic[8];
    uint32_t abi, reserved;
    uint64_t params_fp;
    uint64_t n_res, n_prot, n_unique, n_kept, n_total, n_dropped, n_keys, def_bytes;
    uint64_t pad[5];
};
static_assert(sizeof(dbi_index_header) == 128, "128-B header");

// FNV-1a 64 over the parameter fields the build reads (everything before
// `reserved`: no padding there)
uint64_t params_fingerprint(const dbi_params& p) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(&p);
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < offsetof(dbi_params, reserved); ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
};

int io_fail(const std::string& what, const char* path) {
    return set_error(DBI_E_INVALID, what + ": " + path);
}

template <typename T>
bool put(FILE* f, const T* p, uint64_t n) {
    return n == 0 || std::fwrite(p, sizeof(T), n, f) == n;
}
template <typename T>
bool get(FILE* f, T* p, uint64_t n) {
    return n == 0 || std::fread(p, sizeof(T), n, f) == n;
}

int read_header(FILE* f, dbi_index_header* hd, const char* path) {
    if (!get(f, hd, 1) || std::memcmp(hd->magic, MAGIC, 8) != 0) return io_fail("not a dbindex-hip index file", path);
    if (hd->abi != DBI_ABI_VERSION) return io_fail("index file written by another ABI version", path);
    return 0;
}

}  // namespace

// engine index (+ optional ProteinCache definitions) -> file
int index_save(dbi_handle* h, const char* path, const std::string* defs, const std::vector<uint64_t>* def_off) {
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    // the file is the bucketed store's index; unbucketed / window-filtered
    // builds (SEARCH_UNINDEXED) are transient and carry other contents
    if (!h->dp.buckets || h->dp.filter)
        return set_error(DBI_E_STATE, "only a bucketed, unfiltered index can be saved");
    DBI_HIP(hipSetDevice(h->device));
    const uint64_t R = h->n_res, P = h->n_prot, U = h->stats.n_unique, K = h->stats.n_kept;
    std::vector<uint8_t> res(R);
    std::vector<uint32_t> off32(P + 1);
    hipStream_t s = h->stream;
    if (R) DBI_HIP(hipMemcpyAsync(res.data(), h->d_res, R, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipMemcpyAsync(off32.data(), h->d_poff, 4 * (P + 1), hipMemcpyDeviceToHost, s));
    std::vector<double> mass(U);
    std::vector<uint32_t> pid(U), uoff(U), ulen(U), occ_off(U + 1), occ(K);
    if (U) {
        DBI_HIP(hipMemcpyAsync(mass.data(), h->umass.p, 8 * U, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipMemcpyAsync(pid.data(), h->upid.p, 4 * U, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipMemcpyAsync(uoff.data(), h->uoff.p, 4 * U, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipMemcpyAsync(ulen.data(), h->ulen.p, 4 * U, hipMemcpyDeviceToHost, s));
    }
    DBI_HIP(hipMemcpyAsync(occ_off.data(), h->occ_off.p, 4 * (U + 1), hipMemcpyDeviceToHost, s));
    if (K) DBI_HIP(hipMemcpyAsync(occ.data(), h->occ_pid.p, 4 * K, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> off(P + 1);
    for (uint64_t i = 0; i <= P; ++i) off[i] = off32[i];
    std::vector<uint64_t> doff(P + 1, 0);
    if (defs && def_off && def_off->size() == P + 1) doff = *def_off;
    const uint64_t def_bytes = defs ? defs->size() : 0;

    dbi_index_header hd{};
    std::memcpy(hd.magic, MAGIC, 8);
    hd.abi = DBI_ABI_VERSION;
    hd.params_fp = params_fingerprint(h->params);
    hd.n_res = R;
    hd.n_prot = P;
    hd.n_unique = U;
    hd.n_kept = K;
    hd.n_total = h->stats.n_total;
    hd.n_dropped = h->stats.n_dropped;
    hd.n_keys = h->stats.n_keys;
    hd.def_bytes = def_bytes;
    const std::string tmp = std::string(path) + ".tmp";
    {
        File f;
        f.f = std::fopen(tmp.c_str(), "wb");
        if (!f.f) return io_fail("cannot write index file", tmp.c_str());
        const bool ok = put(f.f, &hd, 1) && put(f.f, res.data(), R) && put(f.f, off.data(), P + 1) &&
                        put(f.f, doff.data(), P + 1) && (def_bytes == 0 || put(f.f, defs->data(), def_bytes)) &&
                        put(f.f, mass.data(), U) && put(f.f, pid.data(), U) && put(f.f, uoff.data(), U) &&
                        put(f.f, ulen.data(), U) && put(f.f, occ_off.data(), U + 1) && put(f.f, occ.data(), K);
        if (!ok || std::fflush(f.f) != 0) return io_fail("short write to index file", tmp.c_str());
    }
    if (std::rename(tmp.c_str(), path) != 0) return io_fail("cannot move index file into place", path);
    return 0;
}

// file -> engine index; the proteome (and definitions) to the caller's vectors when given
int index_load(dbi_handle* h, const char* path, std::vector<uint8_t>* res_out, std::vector<uint64_t>* off_out,
               std::string* defs_out, std::vector<uint64_t>* def_off_out) {
    if (!h->dp.buckets || h->dp.filter)
        return set_error(DBI_E_STATE, "a saved index loads into a bucketed, unfiltered engine only");
    File f;
    f.f = std::fopen(path, "rb");
    if (!f.f) return io_fail("cannot open index file", path);
    dbi_index_header hd;
    int rc = read_header(f.f, &hd, path);
    if (rc) return rc;
    if (hd.params_fp != params_fingerprint(h->params))
        return io_fail("index file was built with other search parameters", path);
    const uint64_t R = hd.n_res, P = hd.n_prot, U = hd.n_unique, K = hd.n_kept;
    if (R >= (1ull << 32) - 1 || P >= (1ull << 32) - 1 || K >= (1ull << 32) - 1)
        return io_fail("index file too large for one device", path);
    // the header must describe exactly this file (nothing allocated from an
    // unchecked header: a damaged size would otherwise throw across the C-ABI)
    if (U > K || hd.n_kept + hd.n_dropped != hd.n_total || hd.n_keys > U || hd.def_bytes >= (1ull << 40))
        return io_fail("corrupt index file header", path);
    if (std::fseek(f.f, 0, SEEK_END) != 0) return io_fail("cannot seek index file", path);
    const long long fsize = std::ftell(f.f);
    const unsigned long long want = sizeof(dbi_index_header) + R + 16ull * (P + 1) + hd.def_bytes + 8ull * U +
                                    4ull * (3 * U + (U + 1) + K);
    if (fsize < 0 || (unsigned long long)fsize != want) return io_fail("index file size does not match its header", path);
    if (std::fseek(f.f, (long)sizeof(dbi_index_header), SEEK_SET) != 0) return io_fail("cannot seek index file", path);
    std::vector<uint8_t> res;
    std::vector<uint64_t> off, doff;
    std::string defs;
    std::vector<double> mass;
    std::vector<uint32_t> pid, uoff, ulen, occ_off, occ;
    try {
        res.resize(R);
        off.resize(P + 1);
        doff.resize(P + 1);
        defs.resize(hd.def_bytes);
        mass.resize(U);
        pid.resize(U);
        uoff.resize(U);
        ulen.resize(U);
        occ_off.resize(U + 1);
        occ.resize(K);
    } catch (const std::exception&) {
        return set_error(DBI_E_OOM, std::string("host memory for index file: ") + path);
    }
    const bool ok = get(f.f, res.data(), R) && get(f.f, off.data(), P + 1) && get(f.f, doff.data(), P + 1) &&
                    (hd.def_bytes == 0 || get(f.f, &defs[0], hd.def_bytes)) && get(f.f, mass.data(), U) &&
                    get(f.f, pid.data(), U) && get(f.f, uoff.data(), U) && get(f.f, ulen.data(), U) &&
                    get(f.f, occ_off.data(), U + 1) && get(f.f, occ.data(), K);
    if (!ok) return io_fail("truncated index file", path);
    if (off[0] != 0 || off[P] != R) return io_fail("corrupt offsets in index file", path);
    // contents: the invariants a build guarantees (dbi_build_occurrences checks
    // the same of caller occurrences); a violation would mean out-of-range
    // reads in queries and materialisation
    for (uint64_t i = 0; i < P; ++i)
        if (off[i + 1] < off[i]) return io_fail("corrupt offsets in index file", path);
    // definition offsets: monotone from 0 to def_bytes (all zero without definitions)
    if (doff[0] != 0 || doff[P] != hd.def_bytes) return io_fail("corrupt definitions", path);
    for (uint64_t i = 0; i < P; ++i)
        if (doff[i + 1] < doff[i]) return io_fail("corrupt definitions", path);
    if (occ_off[0] != 0 || occ_off[U] != K) return io_fail("corrupt occurrence offsets in index file", path);
    for (uint64_t u = 0; u < U; ++u) {
        if (occ_off[u + 1] <= occ_off[u]) return io_fail("corrupt occurrence offsets in index file", path);
        if (!(mass[u] >= 1.0 && mass[u] < 65536.0) || (u > 0 && mass[u] < mass[u - 1]))
            return io_fail("corrupt peptide masses in index file (not finite, ascending, in [1, 65536))", path);
        if (pid[u] >= P || ulen[u] == 0 || (uint64_t)uoff[u] + ulen[u] > off[pid[u] + 1] - off[pid[u]])
            return io_fail("corrupt peptide location in index file", path);
    }
    for (uint64_t k = 0; k < K; ++k)
        if (occ[k] >= P) return io_fail("corrupt occurrence protein id in index file", path);

    if ((rc = begin_build(h, R, P))) return rc;
    hipStream_t s = h->stream;
    std::vector<uint32_t> off32(P + 1);
    for (uint64_t i = 0; i <= P; ++i) off32[i] = (uint32_t)off[i];
    if ((rc = h->res.ensure(R + 16)) || (rc = h->poff.ensure(P + 1)) || (rc = h->umass.ensure(U)) ||
        (rc = h->upid.ensure(U)) || (rc = h->uoff.ensure(U)) || (rc = h->ulen.ensure(U)) ||
        (rc = h->occ_off.ensure(U + 1)) || (rc = h->occ_pid.ensure(K)))
        return rc;
    if (R) DBI_HIP(hipMemcpyAsync(h->res.p, res.data(), R, hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->poff.p, off32.data(), 4 * (P + 1), hipMemcpyHostToDevice, s));
    if (U) {
        DBI_HIP(hipMemcpyAsync(h->umass.p, mass.data(), 8 * U, hipMemcpyHostToDevice, s));
        DBI_HIP(hipMemcpyAsync(h->upid.p, pid.data(), 4 * U, hipMemcpyHostToDevice, s));
        DBI_HIP(hipMemcpyAsync(h->uoff.p, uoff.data(), 4 * U, hipMemcpyHostToDevice, s));
        DBI_HIP(hipMemcpyAsync(h->ulen.p, ulen.data(), 4 * U, hipMemcpyHostToDevice, s));
    }
    DBI_HIP(hipMemcpyAsync(h->occ_off.p, occ_off.data(), 4 * (U + 1), hipMemcpyHostToDevice, s));
    if (K) DBI_HIP(hipMemcpyAsync(h->occ_pid.p, occ.data(), 4 * K, hipMemcpyHostToDevice, s));
    DBI_HIP(hipStreamSynchronize(s));  // host vectors go out of scope
    h->d_res = h->res.p;
    h->d_poff = h->poff.p;
    dbi_stats& st = h->stats;
    st.n_residues = R;
    st.n_proteins = P;
    st.n_total = hd.n_total;
    st.n_dropped = hd.n_dropped;
    st.n_kept = K;
    st.n_unique = U;
    st.n_keys = hd.n_keys;
    h->built = true;
    ++h->build_serial;
    if (res_out) res_out->swap(res);
    if (off_out) off_out->swap(off);
    if (defs_out) defs_out->swap(defs);
    if (def_off_out) def_off_out->swap(doff);
    return 0;
}

int index_file_matches(const dbi_params& p, const char* path, bool* out) {
    *out = false;
    File f;
    f.f = std::fopen(path, "rb");
    if (!f.f) return 0;
    dbi_index_header hd;
    if (!get(f.f, &hd, 1) || std::memcmp(hd.magic, MAGIC, 8) != 0 || hd.abi != DBI_ABI_VERSION) return 0;
    *out = hd.params_fp == params_fingerprint(p);
    return 0;
}

}  // namespace dbi

extern "C" {

int dbi_index_save(dbi_handle* h, const char* path) {
    if (!h || !path) return set_error(DBI_E_INVALID, "NULL argument");
    return index_save(h, path, nullptr, nullptr);
}

int dbi_index_load(dbi_handle* h, const char* path) {
    if (!h || !path) return set_error(DBI_E_INVALID, "NULL argument");
    return index_load(h, path, nullptr, nullptr, nullptr, nullptr);
}

int dbi_index_file_matches(const dbi_params* params, const char* path, int* out) {
    if (!params || !path || !out) return set_error(DBI_E_INVALID, "NULL argument");
    bool m = false;
    const int rc = index_file_matches(*params, path, &m);
    *out = m ? 1 : 0;
    return rc;
}

}  // extern "C"
