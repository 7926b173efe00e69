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
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)
#include <emmintrin.h>
#endif
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#define DBI_FASTA_AVX512 1
#endif

#include "../../include/dbindex_hip.h"
#include "dbi_fasta.h"

namespace dbi {
int set_error(int code, const std::string& msg);
}

namespace {

// ASCII whitespace (' ', \t \n \v \f \r), branch-free
inline bool is_ws(unsigned char c) { return c == ' ' || (unsigned char)(c - 9u) < 5u; }

#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)
// 16 bytes -> 0xFF where whitespace, else 0
inline __m128i ws_bytes16(const char* p) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const __m128i x = _mm_sub_epi8(v, _mm_set1_epi8(9));  // \t..\r -> 0..4
    const __m128i ctl = _mm_cmpeq_epi8(_mm_min_epu8(x, _mm_set1_epi8(4)), x);
    return _mm_or_si128(ctl, _mm_cmpeq_epi8(v, _mm_set1_epi8(' ')));
}
#endif

#ifdef DBI_FASTA_AVX512
// AVX-512 (VBMI2: byte compress) variants, picked at run time: 64 bytes a
// step, whitespace as a 64-bit mask, the kept bytes compressed in a register
// and written by a byte-masked store (never past the bytes it packs); the
// last partial block by a masked load.  The SSE2 pack's line-end cases
// (a temporary and a store-forwarded reload per 16 bytes) made packing ~3x
// slower than counting.
__attribute__((target("avx512f,avx512bw"))) inline uint64_t ws_mask64(__m512i v) {
    const __mmask64 sp = _mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8(' '));
    const __mmask64 ctl = _mm512_cmple_epu8_mask(_mm512_sub_epi8(v, _mm512_set1_epi8(9)), _mm512_set1_epi8(4));
    return (uint64_t)(sp | ctl);
}

__attribute__((target("avx512f,avx512bw,popcnt"))) uint64_t count_residues_512(const char* b, uint64_t len) {
    uint64_t n = 0, i = 0;
    for (; i + 64 <= len; i += 64) n += 64 - (uint64_t)__builtin_popcountll(ws_mask64(_mm512_loadu_si512(b + i)));
    if (i < len) {
        const __mmask64 valid = (__mmask64)(~0ull >> (64 - (len - i)));
        n += (uint64_t)__builtin_popcountll(~ws_mask64(_mm512_maskz_loadu_epi8(valid, b + i)) & valid);
    }
    return n;
}

__attribute__((target("avx512f,avx512bw,avx512vbmi2,popcnt")))
uint64_t pack_residues_512(uint8_t* out, const char* b, uint64_t len) {
    uint64_t n = 0, i = 0;
    for (; i < len; i += 64) {
        const __mmask64 valid = len - i >= 64 ? (__mmask64)~0ull : (__mmask64)(~0ull >> (64 - (len - i)));
        const __m512i v = _mm512_maskz_loadu_epi8(valid, b + i);
        const __mmask64 keep = (__mmask64)(~ws_mask64(v)) & valid;
        const uint32_t k = (uint32_t)__builtin_popcountll((uint64_t)keep);
        if (keep == valid && k == 64) {
            _mm512_storeu_si512(out + n, v);
        } else {
            const __m512i c = _mm512_maskz_compress_epi8(keep, v);
            _mm512_mask_storeu_epi8(out + n, (__mmask64)(k == 64 ? ~0ull : (1ull << k) - 1ull), c);
        }
        n += k;
    }
    return n;
}

// One record's sequence in one pass: from b[s] up to the next record start
// (a '>' right after a newline) or n, counting (WRITE: packing into out) the
// non-whitespace bytes; *end = that record start.  (The SSE2 path finds the
// record start by memchr first, then counts or packs: two passes.)
template <bool WRITE>
__attribute__((target("avx512f,avx512bw,avx512vbmi2,popcnt,bmi")))
uint64_t seq_scan_512(uint8_t* out, const char* b, uint64_t n, uint64_t s, uint64_t* end, uint64_t* brackets) {
    uint64_t cnt = 0, br = 0;
    uint64_t prev_nl = s > 0 && b[s - 1] == '\n';
    for (uint64_t i = s; i < n; i += 64) {
        const __mmask64 valid = n - i >= 64 ? (__mmask64)~0ull : (__mmask64)(~0ull >> (64 - (n - i)));
        const __m512i v = _mm512_maskz_loadu_epi8(valid, b + i);
        const uint64_t nl = (uint64_t)_mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8('\n'));
        const uint64_t gt = (uint64_t)_mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8('>'));
        const uint64_t start = gt & ((nl << 1) | prev_nl) & (uint64_t)valid;
        uint64_t lim = (uint64_t)valid;
        uint32_t j = 64;
        if (start) {
            j = (uint32_t)__builtin_ctzll(start);
            lim &= j ? ~0ull >> (64 - j) : 0ull;
        }
        const uint64_t keep = ~ws_mask64(v) & lim;
        const uint32_t k = (uint32_t)__builtin_popcountll(keep);
        if (!WRITE) br |= (uint64_t)_mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8('[')) & keep;  // inline PTMs
        if (WRITE) {
            if (k == 64) {
                _mm512_storeu_si512(out + cnt, v);
            } else if (k) {
                const __m512i c = _mm512_maskz_compress_epi8((__mmask64)keep, v);
                _mm512_mask_storeu_epi8(out + cnt, (__mmask64)((1ull << k) - 1ull), c);
            }
        }
        cnt += k;
        if (start) {
            *end = i + j;
            if (!WRITE) *brackets |= br;
            return cnt;
        }
        prev_nl = nl >> 63;
    }
    *end = n;
    if (!WRITE) *brackets |= br;
    return cnt;
}

bool detect_avx512() {
    __builtin_cpu_init();  // (a static initializer may run before the runtime's own CPU detection)
    return __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vbmi2");
}
const bool g_avx512 = detect_avx512();
#endif

// non-whitespace bytes of b[0, len)
uint64_t count_residues(const char* b, uint64_t len) {
#ifdef DBI_FASTA_AVX512
    if (g_avx512) return count_residues_512(b, len);
#endif
    uint64_t n = 0, i = 0;
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)
    // whitespace bytes counted per byte lane (a mask byte is -1), folded by
    // psadbw every 255 blocks
    while (i + 16 <= len) {
        const uint64_t nb = std::min<uint64_t>((len - i) / 16, 255);
        __m128i acc = _mm_setzero_si128();
        for (uint64_t k = 0; k < nb; ++k, i += 16) acc = _mm_sub_epi8(acc, ws_bytes16(b + i));
        const __m128i s2 = _mm_sad_epu8(acc, _mm_setzero_si128());
        n += 16 * nb - (uint64_t)(_mm_cvtsi128_si64(s2) + _mm_cvtsi128_si64(_mm_unpackhi_epi64(s2, s2)));
    }
#endif
    for (; i < len; ++i) n += !is_ws((unsigned char)b[i]);
    return n;
}

// the non-whitespace bytes of b[0, len) packed into out; returns their count.
// Never writes past the bytes it packs (the threads' output ranges abut).
uint64_t pack_residues(uint8_t* out, const char* b, uint64_t len) {
#ifdef DBI_FASTA_AVX512
    if (g_avx512) return pack_residues_512(out, b, len);
#endif
    uint64_t n = 0, i = 0;
#if defined(__SSE2__) && !defined(__HIP_DEVICE_COMPILE__)
    for (; i + 16 <= len; i += 16) {
        const uint32_t m = (uint32_t)_mm_movemask_epi8(ws_bytes16(b + i));
        if (m == 0) {  // a run of residues (most of a sequence line)
            std::memcpy(out + n, b + i, 16);
            n += 16;
        } else if ((m & (m - 1)) == 0 && i + 32 <= len) {  // one line end inside: the 15 bytes around it
            const uint32_t k = (uint32_t)__builtin_ctz(m);
            uint8_t tmp[32];
            std::memcpy(tmp, b + i, 16);
            std::memcpy(tmp + k, b + i + k + 1, 16);
            std::memcpy(out + n, tmp, 15);
            n += 15;
        } else {
            uint8_t tmp[16];
            uint32_t k = 0;
            for (uint32_t j = 0; j < 16; ++j) {
                tmp[k] = (uint8_t)b[i + j];
                k += ((m >> j) & 1u) ^ 1u;
            }
            std::memcpy(out + n, tmp, k);
            n += k;
        }
    }
#endif
    for (; i < len; ++i)
        if (!is_ws((unsigned char)b[i])) out[n++] = (uint8_t)b[i];
    return n;
}

// first record start r > p (a '>' after a newline), or 0 when p == 0 and the
// text starts with '>'; n if none.  Records are found by their '>' (memchr over
// whole sequences, which hold none), then checked for a line start.
uint64_t next_record(const char* b, uint64_t n, uint64_t p) {
    if (p == 0 && n > 0 && b[0] == '>') return 0;
    for (uint64_t q = p + 1; q < n;) {
        const void* f = std::memchr(b + q, '>', n - q);
        if (!f) return n;
        const uint64_t r = (uint64_t)((const char*)f - b);
        if (b[r - 1] == '\n') return r;
        q = r + 1;
    }
    return n;
}

struct Part {
    uint64_t lo = 0, hi = 0;          // byte range: records starting in [lo, hi)
    uint64_t n_rec = 0, n_res = 0, n_def = 0, n_uni = 0;
    bool ptm_known = false, ptm = false;  // (the AVX-512 count pass sees '[' on the way)
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
    uint64_t nr = 0, nres = 0, ndef = 0, nuni = 0, brackets = 0;
    while (p < pt.hi) {
        uint64_t de;
        const uint64_t le = def_range(b, n, p, &de);
        const uint64_t dl = de - (p + 1);
        if (WRITE) {
            off[rec0 + nr] = res0 + nres;
            doff[rec0 + nr] = def0 + ndef;
            if (defs) std::memcpy(defs + def0 + ndef, b + p + 1, dl);
        } else {
            nuni += uniprot(b + p + 1, dl);
        }
        ndef += dl;
        // sequence: every non-whitespace byte up to the next record start
        const uint64_t s0 = le < n ? le + 1 : n;
        uint64_t s1;
#ifdef DBI_FASTA_AVX512
        if (g_avx512) {
            nres += seq_scan_512<WRITE>(WRITE ? res + res0 + nres : nullptr, b, n, s0, &s1, &brackets);
        } else
#endif
        {
            s1 = next_record(b, n, le < n ? le : n);
            nres += WRITE ? pack_residues(res + res0 + nres, b + s0, s1 - s0) : count_residues(b + s0, s1 - s0);
        }
        ++nr;
        p = s1;
    }
    if (!WRITE) {
        pt.n_rec = nr;
        pt.n_res = nres;
        pt.n_def = ndef;
        pt.n_uni = nuni;
#ifdef DBI_FASTA_AVX512
        pt.ptm_known = g_avx512;
#endif
        pt.ptm = brackets != 0;
    }
}

// A large host buffer on 2-MiB pages where the kernel allows them
// (transparent huge pages in "madvise" mode): a 200-MB proteome then
// faults in ~100 times instead of ~50 000 (4-KiB pages, each zeroed on its
// first write) -- the page faults, not the parse, bounded the reader.
// std::free releases it.
void* alloc_big(uint64_t bytes) {
    constexpr uint64_t HUGE = 2ull << 20;
    if (bytes < HUGE) return std::malloc(bytes);
    void* p = nullptr;
    if (posix_memalign(&p, HUGE, bytes) != 0) return nullptr;
    ::madvise(p, (bytes + HUGE - 1) & ~(HUGE - 1), MADV_HUGEPAGE);
    return p;
}

int parse_threads(int threads) {
    return threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// The live dbi_fasta residue buffers on 2-MiB pages: dbi_build registers
// such a buffer for DMA directly (~0.6 ms for 201 MB on 2-MiB pages; ~10 ms
// on 4-KiB pages, which go through the engine's pinned ring instead).
struct ResidueBuf {
    uintptr_t p;
    uint64_t n;
    bool ptm_known, ptm;
};
std::mutex g_bufs_mu;
std::vector<ResidueBuf> g_bufs;

}  // namespace

namespace dbi {
bool fasta_residue_buffer(const void* p, uint64_t n, bool* ptm_known, bool* ptm) {
    std::lock_guard<std::mutex> lk(g_bufs_mu);
    const uintptr_t a = (uintptr_t)p;
    for (const ResidueBuf& r : g_bufs)
        if (a >= r.p && a + n <= r.p + r.n) {
            *ptm_known = r.ptm_known;
            *ptm = r.ptm;
            return true;
        }
    return false;
}
}  // namespace dbi

extern "C" {

int dbi_fasta_parse(const char* buf, uint64_t len, int threads, dbi_fasta** out) {
    if (!out || (!buf && len)) return dbi::set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    int T = parse_threads(threads);
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
    bool ptm_known = true, ptm = false;
    std::vector<uint64_t> r0(T), p0(T), d0(T);
    for (int t = 0; t < T; ++t) {
        r0[t] = R;
        p0[t] = P;
        d0[t] = D;
        R += parts[t].n_res;
        P += parts[t].n_rec;
        D += parts[t].n_def;
        U += parts[t].n_uni;
        ptm_known &= parts[t].ptm_known;
        ptm |= parts[t].ptm;
    }
    dbi_fasta* f = (dbi_fasta*)std::calloc(1, sizeof(dbi_fasta));
    if (!f) return dbi::set_error(DBI_E_OOM, "calloc");
    f->n_proteins = P;
    f->n_residues = R;
    f->n_uniprot = U;
    f->residues = (uint8_t*)alloc_big(std::max<uint64_t>(R, 1) + 16);
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
    std::memset(f->residues + R, 0, 16);
    if (R + 16 >= (2u << 20)) {  // (alloc_big's 2-MiB pages)
        std::lock_guard<std::mutex> lk(g_bufs_mu);
        g_bufs.push_back({(uintptr_t)f->residues, R + 16, ptm_known, ptm});
    }
    f->offsets[P] = R;
    f->def_off[P] = D;
    *out = f;
    return 0;
}

// The file is mapped read-only and parsed in place: the parse threads' first
// touches map the page-cache pages (fault-around, in parallel), with no copy
// and no fresh pages to zero.  (A parallel pread into a huge-page buffer,
// the previous way, paid a 257-MB copy and the buffer's page faults: 52-66
// vs 35-43 ms for the SwissProt-scale file on 8 threads.)  Files that cannot
// be mapped are read with pread.
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
    if (len > 0) {
        void* m = ::mmap(nullptr, (size_t)len, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m != MAP_FAILED) {
            ::close(fd);
            (void)::madvise(m, (size_t)len, MADV_SEQUENTIAL);
            const int rc = dbi_fasta_parse((const char*)m, len, threads, out);
            ::munmap(m, (size_t)len);
            return rc;
        }
    }
    char* buf = (char*)alloc_big(std::max<uint64_t>(len, 1));
    if (!buf) {
        ::close(fd);
        return dbi::set_error(DBI_E_OOM, "FASTA read buffer");
    }
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)parse_threads(threads), len / (4u << 20) + 1));
    std::vector<int> bad(T, 0);
    auto rd = [&](int t) {
        uint64_t a = len * (uint64_t)t / (uint64_t)T;
        const uint64_t e = len * (uint64_t)(t + 1) / (uint64_t)T;
        while (a < e) {
            const ssize_t k = ::pread(fd, buf + a, (size_t)std::min<uint64_t>(e - a, 1ull << 30), (off_t)a);
            if (k <= 0) {
                bad[t] = 1;
                return;
            }
            a += (uint64_t)k;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(rd, t);
    rd(0);
    for (auto& x : th) x.join();
    ::close(fd);
    int rc;
    if (std::count(bad.begin(), bad.end(), 1)) rc = dbi::set_error(DBI_E_INVALID, std::string("cannot read FASTA file ") + path);
    else rc = dbi_fasta_parse(buf, len, threads, out);
    std::free(buf);
    return rc;
}

void dbi_fasta_free(dbi_fasta* f) {
    if (!f) return;
    {
        std::lock_guard<std::mutex> lk(g_bufs_mu);
        for (size_t i = 0; i < g_bufs.size(); ++i)
            if (g_bufs[i].p == (uintptr_t)f->residues) {
                g_bufs.erase(g_bufs.begin() + (long)i);
                break;
            }
    }
    std::free(f->residues);
    std::free(f->offsets);
    std::free(f->defs);
    std::free(f->def_off);
    std::free(f);
}

}  // extern "C"
