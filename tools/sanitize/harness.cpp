// tools/sanitize/harness.cpp — host-code sanitizer driver:
// built with -fsanitize=address,undefined together with the oracle's
// restatement (oracle/cpu_ref.cpp) and the host FASTA parser
// (dbindex_amd/csrc/dbi_fasta.cpp), both compiled from their own sources, and
// run by tests/test_sanitizers.py.  It exercises their C entry points on
// seeded inputs, edge cases included, and checks basic invariants; any
// out-of-bounds access, leak or undefined behaviour aborts the run.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <random>
#include <string>
#include <vector>

#include "dbindex_hip.h"

namespace dbi {
// the library's error plumbing (dbi_engine.hip) is not part of this build
static thread_local std::string g_err;
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace dbi

extern "C" {
const char* dbi_last_error(void) { return dbi::g_err.c_str(); }
void dbi_params_default(dbi_params* p, int32_t max_missed, int32_t semi) {
    std::memset(p, 0, sizeof(*p));
    const char* aa = "GASPVTCLINDQKEMHFRYW";
    const double m[] = {57.021464, 71.037114, 87.032028, 97.052764, 99.068414, 101.047679, 103.009185,
                        113.084064, 113.084064, 114.042927, 115.026943, 128.058578, 128.094963, 129.042593,
                        131.040485, 137.058912, 147.068414, 156.101111, 163.063329, 186.079313};
    for (int i = 0; aa[i]; ++i) p->mass[(unsigned char)aa[i]] = m[i];
    p->min_mh = 500.0;
    p->max_mh = 6000.0;
    p->h2o_proton = 18.0105646863 + 1.00727646688;
    p->cleave[(unsigned char)'K'] = p->cleave[(unsigned char)'R'] = 1;
    p->max_missed = max_missed;
    p->semi = semi;
    p->add_h2o_proton = 1;
    p->min_len = 6;
    p->mass_group_factor = 10000;
    p->index_factor = 8;
}
// oracle/cpu_ref.cpp
struct oref_index;
void oref_set_threads(int n);
int oref_build(const dbi_params*, const uint8_t*, const uint64_t*, uint64_t, oref_index**);
int oref_digest(const dbi_params*, const uint8_t*, const uint64_t*, uint64_t, double*, uint32_t*, uint32_t*,
                uint32_t*, uint8_t*, uint64_t, uint64_t*);
int oref_count(const dbi_params*, const uint8_t*, const uint64_t*, uint64_t, uint64_t*, uint64_t*);
void oref_free(oref_index*);
uint64_t oref_n_unique(const oref_index*);
uint64_t oref_n_kept(const oref_index*);
uint64_t oref_n_keys(const oref_index*);
int oref_unique(const oref_index*, double*, uint32_t*, uint32_t*, uint32_t*, uint64_t*, uint32_t*);
int oref_entry_keys(const oref_index*, int32_t*);
int oref_query(const oref_index*, double, double, uint64_t*, uint64_t, uint64_t*);
int oref_query_batch(const oref_index*, const double*, const double*, uint64_t, uint64_t*, uint64_t*);
int oref_query_ranges(const oref_index*, const double*, const double*, uint64_t, uint64_t*, uint64_t, uint64_t*);
}

#define CHECK(x)                                                        \
    do {                                                                \
        if (!(x)) {                                                     \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #x, __LINE__); \
            std::exit(2);                                               \
        }                                                               \
    } while (0)

static void fasta_cases() {
    const char* cases[] = {
        "", ">", ">a\n", "junk\n>sp|A|B x\nMKR\nTT\n>tr|C|D\r\nAA AA\r\n", ">x\nAC", "\n\n>p\n\n\nK\n",
        ">only header no newline",
    };
    for (const char* c : cases)
        for (int th : {1, 2, 7}) {
            dbi_fasta* f = nullptr;
            CHECK(dbi_fasta_parse(c, std::strlen(c), th, &f) == 0);
            CHECK(f->offsets[0] == 0 && f->offsets[f->n_proteins] == f->n_residues);
            dbi_fasta_free(f);
        }
    // a large random file, parsed with many threads (split points inside records)
    std::mt19937_64 rng(5);
    std::string big;
    for (int i = 0; i < 3000; ++i) {
        big += ">sp|P" + std::to_string(i) + "|X desc\n";
        const int len = 1 + (int)(rng() % 700);
        for (int k = 0; k < len; ++k) {
            big += "ACDEFGHIKLMNPQRSTVWY"[rng() % 20];
            if (k % 60 == 59) big += (rng() & 1) ? "\n" : "\r\n";
        }
        big += "\n";
    }
    dbi_fasta* a = nullptr;
    dbi_fasta* b = nullptr;
    CHECK(dbi_fasta_parse(big.data(), big.size(), 1, &a) == 0);
    CHECK(dbi_fasta_parse(big.data(), big.size(), 16, &b) == 0);
    CHECK(a->n_proteins == 3000 && b->n_proteins == 3000 && a->n_residues == b->n_residues);
    CHECK(std::memcmp(a->offsets, b->offsets, 8 * (a->n_proteins + 1)) == 0);
    // the same text read from a file (mapped: the scans' last blocks end at the mapping's end)
    char path[] = "/tmp/dbi_sanitize_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0);
    CHECK(write(fd, big.data(), big.size()) == (ssize_t)big.size());
    close(fd);
    for (int th : {1, 5, 16}) {
        dbi_fasta* r = nullptr;
        CHECK(dbi_fasta_read(path, th, &r) == 0);
        CHECK(r->n_proteins == a->n_proteins && r->n_residues == a->n_residues);
        CHECK(std::memcmp(r->offsets, a->offsets, 8 * (a->n_proteins + 1)) == 0);
        CHECK(std::memcmp(r->residues, a->residues, a->n_residues) == 0);
        dbi_fasta_free(r);
    }
    unlink(path);
    dbi_fasta_free(a);
    dbi_fasta_free(b);
    CHECK(dbi_fasta_read("/nonexistent/file.fasta", 2, &a) != 0);
}

static void oracle_cases() {
    std::mt19937_64 rng(3);
    std::vector<uint8_t> res;
    std::vector<uint64_t> off{0};
    for (int p = 0; p < 400; ++p) {
        const int len = (p % 37 == 0) ? 0 : 30 + (int)(rng() % 900);
        for (int k = 0; k < len; ++k) res.push_back((uint8_t) "ACDEFGHIKLMNPQRSTVWY"[rng() % 20]);
        off.push_back(res.size());
    }
    for (int semi : {0, 1})
        for (int th : {1, 4}) {
            dbi_params p;
            dbi_params_default(&p, 2, semi);
            oref_set_threads(th);
            oref_index* ix = nullptr;
            CHECK(oref_build(&p, res.data(), off.data(), off.size() - 1, &ix) == 0);
            const uint64_t U = oref_n_unique(ix), K = oref_n_kept(ix);
            std::vector<double> mass(U);
            std::vector<uint32_t> pid(U), o(U), l(U), occ(K);
            std::vector<uint64_t> oo(U + 1);
            std::vector<int32_t> keys(oref_n_keys(ix));
            CHECK(oref_unique(ix, mass.data(), pid.data(), o.data(), l.data(), oo.data(), occ.data()) == 0);
            CHECK(oref_entry_keys(ix, keys.data()) == 0);
            CHECK(oo[U] == K);
            for (uint64_t u = 1; u < U; ++u) CHECK(oo[u] > oo[u - 1]);
            std::vector<double> qm(500), qt(500);
            for (int i = 0; i < 500; ++i) {
                qm[i] = U ? mass[rng() % U] : 1000.0;
                qt[i] = (i % 50 == 0) ? 3000.0 : 0.01;
            }
            qm[0] = -5.0;
            qm[1] = 8000.0;
            std::vector<uint64_t> f(500), c(500);
            CHECK(oref_query_batch(ix, qm.data(), qt.data(), 500, f.data(), c.data()) == 0);
            uint64_t n = 0;
            CHECK(oref_query(ix, qm[7], qt[7], nullptr, 0, &n) == 0 && n == c[7]);
            CHECK(oref_query_ranges(ix, qm.data(), qt.data(), 30, nullptr, 0, &n) == 0);
            oref_free(ix);
            uint64_t tot = 0, drop = 0, n2 = 0;
            CHECK(oref_count(&p, res.data(), off.data(), off.size() - 1, &tot, &drop) == 0);
            CHECK(oref_digest(&p, res.data(), off.data(), off.size() - 1, nullptr, nullptr, nullptr, nullptr,
                              nullptr, 0, &n2) == 0);
            CHECK(n2 == tot);
        }
    oref_set_threads(1);
}

int main() {
    fasta_cases();
    oracle_cases();
    std::puts("sanitized host code: ok");
    return 0;
}
