// dbi_fasta.cpp — multi-threaded FASTA parser + packer.
//
// The reference reads the FASTA through FastaReader one protein at a time
// (DBIndexer.run, DBIndexer.java:546-616; IndexUtil.getFastaReader :326-345)
// and numbers proteins in file order (ProteinCache.addProtein :84-95).  Once
// the device build takes milliseconds, parsing dominates end to end, so the
// host side packs the whole file in parallel straight into the layout the
// device build reads: residues (sequences concatenated, whitespace dropped)
// and offsets[P+1], plus the definition lines for the ProteinCache.
//
// Semantics (= dbindex_amd/fasta.py iter_fasta): a record starts at a '>' at
// the start of a line; its definition is the rest of that line with trailing
// CR/LF removed; its sequence is every following line up to the next record
// with all ASCII whitespace removed; lines before the first record are
// ignored.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/dbindex_hip.h"

namespace dbi {
int set_error(int code, const std::string& msg);
}

namespace {

struct WsTable {
    bool t[256] = {};
    WsTable() { t[(unsigned char)' '] = t[(unsigned char)'\t'] = t[(unsigned char)'\n'] = t[(unsigned char)'\r'] =
                    t[(unsigned char)'\v'] = t[(unsigned char)'\f'] = true; }
};
const WsTable g_ws;
inline bool is_ws(unsigned char c) { return g_ws.t[c]; }

// first record start (a '>' at a line start) at or after position p
uint64_t next_record(const char* b, uint64_t n, uint64_t p) {
    if (p == 0 && n > 0 && b[0] == '>') return 0;
    while (p < n) {
        const void* q = std::memchr(b + p, '\n', n - p);
        if (!q) return n;
        p = (uint64_t)((const char*)q - b) + 1;
        if (p < n && b[p] == '>') return p;
    }
    return n;
}

struct Part {
    uint64_t lo = 0, hi = 0;          // byte range: records starting in [lo, hi)
    uint64_t n_rec = 0, n_res = 0, n_def = 0, n_uni = 0;
};

// definition of the record at p ('>' at b[p]): [p+1, e) with trailing CR/LF removed; returns the line end
uint64_t def_range(const char* b, uint64_t n, uint64_t p, uint64_t* e) {
    const void* q = std::memchr(b + p, '\n', n - p);
    const uint64_t le = q ? (uint64_t)((const char*)q - b) : n;
    uint64_t d = le;
    while (d > p + 1 && (b[d - 1] == '\r' || b[d - 1] == '\n')) --d;
    *e = d;
    return le;
}

bool uniprot(const char* d, uint64_t len) {
    // "db|ACC|..." with db in {sp, tr} and a non-empty accession (fasta.py uniprot_accession)
    uint64_t sp = 0;
    while (sp < len && d[sp] != ' ') ++sp;
    if (sp < 4 || !((d[0] == 's' && d[1] == 'p') || (d[0] == 't' && d[1] == 'r')) || d[2] != '|') return false;
    uint64_t k = 3;
    while (k < sp && d[k] != '|') ++k;
    return k < sp && k > 3;
}

// pass over the records starting in [lo, hi); write = false: count only
template <bool WRITE>
void scan_part(const char* b, uint64_t n, Part& pt, uint8_t* res, uint64_t* off, char* defs, uint64_t* doff,
               uint64_t res0, uint64_t rec0, uint64_t def0) {
    uint64_t p = pt.lo;
    uint64_t nr = 0, nres = 0, ndef = 0, nuni = 0;
    while (p < pt.hi) {
        uint64_t de;
        const uint64_t le = def_range(b, n, p, &de);
        const uint64_t dl = de - (p + 1);
        if (WRITE) {
            off[rec0 + nr] = res0 + nres;
            doff[rec0 + nr] = def0 + ndef;
            std::memcpy(defs + def0 + ndef, b + p + 1, dl);
        } else {
            nuni += uniprot(b + p + 1, dl);
        }
        ndef += dl;
        // sequence: up to the next record start
        const uint64_t s0 = le < n ? le + 1 : n;
        const uint64_t s1 = next_record(b, n, le < n ? le : n);
        // line by line: a line's bytes up to its first whitespace byte are
        // copied as one block (the common case: the whole line minus its end)
        uint64_t i = s0;
        while (i < s1) {
            uint64_t j = i;
            while (j < s1 && !is_ws((unsigned char)b[j])) ++j;
            if (WRITE && j > i) std::memcpy(res + res0 + nres, b + i, j - i);
            nres += j - i;
            i = j;
            while (i < s1 && is_ws((unsigned char)b[i])) ++i;
        }
        ++nr;
        p = s1;
    }
    if (!WRITE) {
        pt.n_rec = nr;
        pt.n_res = nres;
        pt.n_def = ndef;
        pt.n_uni = nuni;
    }
}

}  // namespace

extern "C" {

int dbi_fasta_parse(const char* buf, uint64_t len, int threads, dbi_fasta** out) {
    if (!out || (!buf && len)) return dbi::set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)T, len / (1u << 20) + 1));  // >= 1 MiB per thread
    std::vector<Part> parts(T);
    const uint64_t first = next_record(buf, len, 0);
    for (int t = 0; t < T; ++t) {
        const uint64_t a = first + (len - first) * (uint64_t)t / (uint64_t)T;
        parts[t].lo = t == 0 ? first : next_record(buf, len, a > 0 ? a - 1 : 0);
    }
    for (int t = 0; t < T; ++t) parts[t].hi = t + 1 < T ? parts[t + 1].lo : len;
    for (int t = 0; t < T; ++t) parts[t].lo = std::min(parts[t].lo, parts[t].hi);
    auto run = [&](auto fn) {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(fn, t);
        fn(0);
        for (auto& x : th) x.join();
    };
    run([&](int t) { scan_part<false>(buf, len, parts[t], nullptr, nullptr, nullptr, nullptr, 0, 0, 0); });
    uint64_t R = 0, P = 0, D = 0, U = 0;
    std::vector<uint64_t> r0(T), p0(T), d0(T);
    for (int t = 0; t < T; ++t) {
        r0[t] = R;
        p0[t] = P;
        d0[t] = D;
        R += parts[t].n_res;
        P += parts[t].n_rec;
        D += parts[t].n_def;
        U += parts[t].n_uni;
    }
    dbi_fasta* f = (dbi_fasta*)std::calloc(1, sizeof(dbi_fasta));
    if (!f) return dbi::set_error(DBI_E_OOM, "calloc");
    f->n_proteins = P;
    f->n_residues = R;
    f->n_uniprot = U;
    f->residues = (uint8_t*)std::malloc(std::max<uint64_t>(R, 1) + 16);
    f->offsets = (uint64_t*)std::malloc(8 * (P + 1));
    f->defs = (char*)std::malloc(std::max<uint64_t>(D, 1));
    f->def_off = (uint64_t*)std::malloc(8 * (P + 1));
    if (!f->residues || !f->offsets || !f->defs || !f->def_off) {
        dbi_fasta_free(f);
        return dbi::set_error(DBI_E_OOM, "malloc");
    }
    run([&](int t) {
        scan_part<true>(buf, len, parts[t], f->residues, f->offsets, f->defs, f->def_off, r0[t], p0[t], d0[t]);
    });
    f->offsets[P] = R;
    f->def_off[P] = D;
    std::memset(f->residues + R, 0, 16);
    *out = f;
    return 0;
}

int dbi_fasta_read(const char* path, int threads, dbi_fasta** out) {
    if (!path || !out) return dbi::set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return dbi::set_error(DBI_E_INVALID, std::string("cannot open FASTA file ") + path);
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        ::close(fd);
        return dbi::set_error(DBI_E_INVALID, std::string("cannot stat FASTA file ") + path);
    }
    const uint64_t len = (uint64_t)st.st_size;
    int rc;
    if (len == 0) {
        rc = dbi_fasta_parse("", 0, threads, out);
    } else {
        void* m = ::mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            ::close(fd);
            return dbi::set_error(DBI_E_OOM, "mmap of the FASTA file failed");
        }
        ::madvise(m, len, MADV_SEQUENTIAL);
        rc = dbi_fasta_parse((const char*)m, len, threads, out);
        ::munmap(m, len);
    }
    ::close(fd);
    return rc;
}

void dbi_fasta_free(dbi_fasta* f) {
    if (!f) return;
    std::free(f->residues);
    std::free(f->offsets);
    std::free(f->defs);
    std::free(f->def_off);
    std::free(f);
}

}  // extern "C"
