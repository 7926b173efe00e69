// oracle/cpu_ref.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// CPU restatement of the reference's digestion + index + mass-lookup path,
// written loop-for-loop from the Java sources under /root/reference
// (paths below relative to src/main/java/edu/scripps/yates/dbindex/).
// Used by tests/ as the parity checker, by bench.py as the `cpu_baseline`
// ("port": single-threaded like the reference, and one thread per core over
// protein ranges then row ranges — oref_set_threads), and by
// __graft_entry__.smoke().
//
// Parity pinning: the reference is Java with no tests, no fixtures and no JDK
// in this image, and its residue-mass table / cleavage rule live in the
// un-vendored edu.scripps.yates:utilities:1.6-SNAPSHOT.  This restatement is
// therefore pinned by (i) hand-derived known-answer tests and (ii) an
// independent pure-Python twin (oracle/pyref.py) that must agree bit-exactly;
// the Enzyme/AssignMass boundary is "parity unpinned" (see DESIGN.md §Oracle).
//
// Mirrors:
//   cutSeq loop ............ DBIndexer.java:237-405
//   filterSequence ......... DBIndexStoreSQLiteMult.java:245-268
//   addSequence / bucket ... DBIndexStoreSQLiteMult.java:215-217,271-291
//   row key + record ....... DBIndexStoreSQLiteByte.java:185-226
//   merge per row .......... DBIndexStoreSQLiteByteIndexMerge.java:620-719
//   single-range query ..... DBIndexStoreSQLiteMult.java:315-350 + IndexMerge.java:146-217,386-481
//   multi-range query ...... DBIndexStoreSQLiteMult.java:353-430 + IndexMerge.java:225-375,494-600
//   getNumberSequences ..... DBIndexStoreSQLiteByte.java:667-690 (rows, not peptides)
//   Enzyme.checkCleavage ... external; pinned rule in DESIGN.md (semantics A3)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/dbindex_hip.h"

namespace {

// Java `(int) d` for a double (JLS 5.1.3): NaN -> 0, saturating, truncation.
inline int32_t java_d2i(double d) {
    if (std::isnan(d)) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}

constexpr int MAX_PRECURSOR_INT = 8000;  // (int) Constants.MAX_PRECURSOR_MASS, Constants.java:20

// Enzyme.isEnzyme / checkCleavage — pinned rule.
struct Enzyme {
    const dbi_params* p;
    bool isEnzyme(uint8_t c) const { return p->cleave[c] != 0; }
    bool checkCleavage(const uint8_t* seq, int len, int start, int end) const {
        bool n_ok = (start == 0) || (p->cleave[seq[start - 1]] && !p->nocut[seq[start]]);
        bool c_ok = (end == len - 1) || (p->cleave[seq[end]] && !p->nocut[seq[end + 1]]);
        return p->semi ? (n_ok || c_ok) : (n_ok && c_ok);
    }
};

struct Occ {
    double mass;
    uint32_t pid;
    uint32_t offset;
    uint32_t length;
    uint32_t dropped;
};

// DBIndexStoreSQLiteMult.filterSequence (:245-268)
int filter_sequence(const dbi_params* p, double precMass, const uint8_t* pep, int len) {
    if (p->mandatory_mode && p->mandatory_count > 0) {
        // "exclude the last AA, which is the cleavage site" (:258-259)
        for (int c = 0; c < 256; ++c) {
            if (!p->mandatory[c]) continue;
            for (int i = 0; i < len - 1; ++i)
                if (pep[i] == c) return DBI_FILTER_INCLUDE;
        }
        return DBI_FILTER_SKIP;
    }
    if (p->max_mh < precMass || p->min_mh > precMass) return DBI_FILTER_SKIP;
    return DBI_FILTER_INCLUDE;
}

// FormulaCalculator.calculateMass (external jar, not vendored): the restated
// monoisotopic element sum the product uses too (dbi_engine.hip formula_mass);
// NaN = unknown element (UnknownElementMassException).  Parity unpinned.
double formula_mass(const std::string& f) {
    static const std::pair<const char*, double> kEl[] = {
        {"H", 1.00782503207}, {"D", 2.0141017778}, {"C", 12.0}, {"N", 14.0030740048}, {"O", 15.99491461956},
        {"P", 30.97376163}, {"S", 31.97207100}, {"Se", 79.9165213}, {"Na", 22.9897692809}, {"K", 38.96370668},
        {"Li", 7.01600455}, {"Mg", 23.9850417}, {"Ca", 39.96259098}, {"Fe", 55.9349375}, {"Zn", 63.9291422},
        {"Cu", 62.9295975}, {"Cl", 34.96885268}, {"Br", 78.9183371}, {"I", 126.904473}, {"F", 18.99840322},
        {"Si", 27.9769265325}, {"B", 11.0093054}, {"Hg", 201.970643}};
    double mass = 0.0;
    size_t i = 0;
    while (i < f.size()) {
        if (!(f[i] >= 'A' && f[i] <= 'Z')) return NAN;
        size_t j = i + 1;
        while (j < f.size() && f[j] >= 'a' && f[j] <= 'z') ++j;
        const std::string el = f.substr(i, j - i);
        bool neg = false;
        if (j < f.size() && f[j] == '-') {
            neg = true;
            ++j;
        }
        long cnt = 0;
        size_t k = j;
        while (k < f.size() && f[k] >= '0' && f[k] <= '9' && cnt < 100000000) cnt = cnt * 10 + (f[k++] - '0');
        if (k == j) {
            if (neg) return NAN;
            cnt = 1;
        }
        double em = NAN;
        for (const auto& e : kEl)
            if (el == e.first) em = e.second;
        if (std::isnan(em)) return NAN;
        mass = mass + (double)(neg ? -cnt : cnt) * em;
        i = k;
    }
    return mass;
}

// Java String.replace(CharSequence, CharSequence): every non-overlapping copy, left to right
void replace_all(std::string& s, const std::string& pat) {
    std::string r;
    size_t i = 0;
    for (size_t at; (at = s.find(pat, i)) != std::string::npos; i = at + pat.size()) r.append(s, i, at - i);
    r.append(s, i, std::string::npos);
    s.swap(r);
}

// cutSeq over a protein carrying inline '[formula]' PTMs, literally: the
// protein string is mutated as the reference does (:288-303).  Returns false
// where the reference throws StringIndexOutOfBoundsException out of cutSeq
// (a formula before the first residue, '[' without ']').
bool cut_seq_literal(const dbi_params* p, std::string protSeq, uint32_t proteinId, std::vector<Occ>& out) {
    Enzyme enz{p};
    const int maxIntCleavage = p->max_missed;
    const int bucketRange = MAX_PRECURSOR_INT / p->index_factor;
    int length = (int)protSeq.size();
    for (int start = 0; start < length; ++start) {
        int end = start;
        double precMass = 0;
        if (p->add_h2o_proton) precMass += p->h2o_proton;
        precMass += p->cterm;
        precMass += p->nterm;
        int pepSize = 0;
        int intMisCleavageCount = -1;
        std::string pepSeq;
        while (precMass <= p->max_mh && end < length) {
            pepSize++;
            const char curIon = protSeq[end];
            double aaMass;
            if (curIon == '[') {
                std::string formula;
                for (;;) {
                    if (++end >= length) return false;  // charAt past the end
                    if (protSeq[end] == ']') break;
                    formula += protSeq[end];
                }
                aaMass = formula_mass(formula);
                if (std::isnan(aaMass)) return true;  // UnknownElementMassException: caught, cutSeq ends (:400-403)
                replace_all(protSeq, "[" + formula + "]");
                end -= (int)formula.size() + 2;
                length = (int)protSeq.size();
            } else {
                pepSeq += curIon;
                aaMass = p->mass[(uint8_t)curIon];
            }
            precMass = precMass + aaMass;
            if (end < 0) return false;  // charAt(-1)
            const uint8_t* seq = (const uint8_t*)protSeq.data();
            if (enz.isEnzyme(seq[end])) intMisCleavageCount++;
            if (enz.checkCleavage(seq, length, start, end)) {
                if (intMisCleavageCount > maxIntCleavage) break;
                if (precMass > p->max_mh) break;
                const int curSeqI = (int)pepSeq.size();
                if (pepSize >= p->min_len && precMass >= p->min_mh) {
                    const uint8_t* pep = (const uint8_t*)pepSeq.data();
                    if (p->mandatory_mode) {
                        bool found = false;
                        for (int c = 0; c < 256 && !found; ++c) {
                            if (!p->mandatory[c]) continue;
                            for (int i = 0; i < curSeqI; ++i)
                                if (pep[i] == c) { found = true; break; }
                        }
                        if (!found) break;
                    }
                    int fr = filter_sequence(p, precMass, pep, curSeqI);
                    if (fr == DBI_FILTER_SKIP_PROTEIN_START) break;
                    if (fr == DBI_FILTER_INCLUDE) {
                        int bucket = java_d2i(precMass) / bucketRange;
                        out.push_back(Occ{precMass, proteinId, (uint32_t)start, (uint32_t)curSeqI,
                                          (uint32_t)(bucket > p->index_factor - 1)});
                    }
                }
            }
            ++end;
        }
    }
    return true;
}

std::atomic<bool> g_ptm_fatal{false};  // a protein the reference's cutSeq throws on

// DBIndexer.cutSeq(String,String) (:237-405), with the SQLiteMult store behind it.
// Appends every INCLUDE'd occurrence (incl. bucket-dropped ones, flagged) in
// insertion order.
void cut_seq(const dbi_params* p, const uint8_t* seq, int length, uint32_t proteinId,
             std::vector<Occ>& out) {
    if (length > 0 && std::memchr(seq, '[', (size_t)length)) {
        if (!cut_seq_literal(p, std::string((const char*)seq, (size_t)length), proteinId, out)) g_ptm_fatal = true;
        return;
    }
    Enzyme enz{p};
    const int maxIntCleavage = p->max_missed;
    const int bucketRange = MAX_PRECURSOR_INT / p->index_factor;  // SQLiteMult:56
    for (int start = 0; start < length; ++start) {
        int end = start;
        int curSeqI = 0;
        double precMass = 0;
        if (p->add_h2o_proton) precMass += p->h2o_proton;  // :268-269
        precMass += p->cterm;                              // :270
        precMass += p->nterm;                              // :271
        int pepSize = 0;
        int intMisCleavageCount = -1;                      // :280
        while (precMass <= p->max_mh && end < length) {    // :284
            pepSize++;
            const uint8_t curIon = seq[end];
            ++curSeqI;                                     // pepSeq[curSeqI++] = curIon (:305)
            double aaMass = p->mass[curIon];               // :306
            precMass = precMass + aaMass;                  // :308
            if (enz.isEnzyme(seq[end])) intMisCleavageCount++;        // :314-316
            const bool cleavageStatus = enz.checkCleavage(seq, length, start, end);  // :318
            if (cleavageStatus) {
                if (intMisCleavageCount > maxIntCleavage) break;      // :322-324
                if (precMass > p->max_mh) break;                      // :326-329
                if (pepSize >= p->min_len && precMass >= p->min_mh) { // :331
                    const uint8_t* pep = seq + start;
                    if (p->mandatory_mode) {                          // :334-344
                        bool found = false;
                        for (int c = 0; c < 256 && !found; ++c) {
                            if (!p->mandatory[c]) continue;
                            for (int i = 0; i < curSeqI; ++i)
                                if (pep[i] == c) { found = true; break; }
                        }
                        if (!found) break;
                    }
                    int fr = filter_sequence(p, precMass, pep, curSeqI);   // :349
                    if (fr == DBI_FILTER_SKIP_PROTEIN_START) break;
                    if (fr == DBI_FILTER_INCLUDE) {
                        // SQLiteMult.addSequence: totalSeqCount++ then bucket check (:277-288)
                        int bucket = java_d2i(precMass) / bucketRange;
                        Occ o{precMass, proteinId, (uint32_t)start, (uint32_t)curSeqI,
                              (uint32_t)(bucket > p->index_factor - 1)};
                        out.push_back(o);
                    }
                }
            }
            ++end;
        }
    }
}

// ---------------------------------------------------------------------------
// Store: buckets -> rows keyed by (int)(mass*factor) -> merged peptide entries
// ---------------------------------------------------------------------------
// A row is one (bucket, key) pair: SQLiteMult routes a peptide to bucket
// (int)m / BUCKET_MASS_RANGE (:215-217) and SQLiteByte appends it to the row
// of key (int)(m*factor) in that bucket's database (Byte:185-226).  Both are
// monotone in m, so (bucket, key) rows in lexicographic order are the rows of
// bucket 0, 1, ... each in rowid (= key) order.  Merged entries are stored
// flattened in that order: unique id = position (uid).
struct RowRef {
    int32_t bucket;
    int32_t key;
    uint64_t ub, ue;  // uids [ub, ue)
};

int g_threads = 1;  // oref_set_threads: worker threads of build / query_batch

template <typename F>
void parallel_for(int nt, F&& f) {
    if (nt <= 1) {
        f(0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&f, t] { f(t); });
    for (auto& x : th) x.join();
}

}  // namespace

struct oref_index {
    dbi_params p;
    std::vector<uint8_t> residues;
    std::vector<uint64_t> off;
    uint64_t n_total = 0, n_dropped = 0;
    // unique table in (bucket, key, row) order + occurrence CSR
    std::vector<double> umass;
    std::vector<uint32_t> upid, uoff, ulen;
    std::vector<uint64_t> occ_off;  // U + 1
    std::vector<uint32_t> occ_pid;
    std::vector<RowRef> rows;                // lexicographic (bucket, key)
    std::vector<uint64_t> bucket_rows;       // rows of bucket b: [bucket_rows[b], bucket_rows[b+1])
    double build_seconds = 0;
};

namespace {

// Pinned tie-break between different peptides of bit-identical mass
// (semantics A7): a 16-bit hash of the length and the first and
// last (up to) four residues, then first appearance.
uint16_t peptide_tag(std::string_view s) {
    const uint32_t L = (uint32_t)s.size();
    uint32_t head = 0, tail = 0;
    for (uint32_t k = 0; k < 4 && k < L; ++k) {
        head |= (uint32_t)(unsigned char)s[k] << (8 * k);
        tail |= (uint32_t)(unsigned char)s[L - 1 - k] << (8 * k);
    }
    uint32_t x = (head * 0x9E3779B1u) ^ (tail * 0x85EBCA77u) ^ (L * 0xC2B2AE3Du);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return (uint16_t)((x >> 16) ^ (x & 0xFFFFu));
}

int64_t row_of(const dbi_params* p, double mass) {
    const int br = MAX_PRECURSOR_INT / p->index_factor;               // SQLiteMult:56
    const int64_t bucket = java_d2i(mass) / br;                        // getBucketForMass :215-217
    const int64_t key = java_d2i(mass * (double)p->mass_group_factor);  // Byte:187
    return bucket * (int64_t(1) << 32) + key;
}

// One worker's slice of the store: every row whose (bucket, key) lies in
// [lo, hi), merged, with uids local to the slice.
struct Slice {
    std::vector<double> umass;
    std::vector<uint32_t> upid, uoff, ulen;
    std::vector<uint64_t> ucnt;  // occurrences per merged entry
    std::vector<uint32_t> occ_pid;
    std::vector<RowRef> rows;
};

// DBIndexStoreSQLiteByteIndexMerge.getMergedData (:620-719) over the rows of
// one slice.  Per row (records in insertion order, Byte.updateCachedData
// appends): group by peptide string (ProteinCache.getPeptideSequence); the
// first occurrence keeps mass/offset/length; proteinIds = every occurrence's
// protein in insertion order, duplicates kept (:678-681); then
// Collections.sort — stable, by mass (IndexedSeqMerged.compareTo) — with the
// THashMap-order ties pinned to (tag, first appearance).
void merge_slice(const oref_index* ix, const std::vector<Occ>& occ, int64_t lo, int64_t hi, Slice& out) {
    const dbi_params* p = &ix->p;
    std::vector<std::pair<int64_t, uint32_t>> sel;  // (row, occurrence index)
    for (uint32_t i = 0; i < (uint32_t)occ.size(); ++i) {
        if (occ[i].dropped) continue;
        const int64_t r = row_of(p, occ[i].mass);
        if (r >= lo && r < hi) sel.push_back({r, i});
    }
    std::sort(sel.begin(), sel.end());  // by row, insertion order inside
    struct Group {
        double mass;
        uint32_t offset, length, first, n;
        uint16_t tag;
    };
    std::unordered_map<std::string_view, uint32_t> where;
    std::vector<std::string_view> gstr;
    std::vector<Group> groups;
    std::vector<uint32_t> gid, ord, gpos;
    for (size_t a = 0; a < sel.size();) {
        size_t b = a;
        while (b < sel.size() && sel[b].first == sel[a].first) ++b;
        // the THashMap of the row (a linear scan for short rows: same grouping)
        const bool small = b - a <= 32;
        if (!small) {
            std::unordered_map<std::string_view, uint32_t>().swap(where);
            where.reserve(2 * (b - a));
        }
        groups.clear();
        gstr.clear();
        gid.clear();
        for (size_t k = a; k < b; ++k) {
            const Occ& r = occ[sel[k].second];
            const uint8_t* s = ix->residues.data() + ix->off[r.pid] + r.offset;
            const std::string_view pep((const char*)s, r.length);
            uint32_t g = (uint32_t)groups.size();
            if (small) {
                for (uint32_t q = 0; q < gstr.size(); ++q)
                    if (gstr[q] == pep) { g = q; break; }
            } else {
                auto it = where.find(pep);
                if (it != where.end()) g = it->second;
                else where.emplace(pep, g);
            }
            if (g == groups.size()) {
                gstr.push_back(pep);
                groups.push_back(Group{r.mass, r.offset, r.length, r.pid, 1, peptide_tag(pep)});
            } else {
                groups[g].n++;
            }
            gid.push_back(g);
        }
        ord.resize(groups.size());
        for (size_t g = 0; g < ord.size(); ++g) ord[g] = (uint32_t)g;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
            if (groups[x].mass != groups[y].mass) return groups[x].mass < groups[y].mass;
            return groups[x].tag < groups[y].tag;
        });
        // occurrence slots of each group in sorted order
        gpos.assign(groups.size(), 0);
        uint64_t base = out.occ_pid.size();
        for (uint32_t g : ord) {
            gpos[g] = (uint32_t)(base - out.occ_pid.size());
            base += groups[g].n;
        }
        const uint64_t ob = out.occ_pid.size();
        out.occ_pid.resize(base);
        for (size_t k = a; k < b; ++k) out.occ_pid[ob + gpos[gid[k - a]]++] = occ[sel[k].second].pid;
        RowRef row;
        row.bucket = (int32_t)(sel[a].first >> 32);
        row.key = (int32_t)(sel[a].first - ((int64_t)row.bucket << 32));
        row.ub = out.umass.size();
        for (uint32_t g : ord) {
            out.umass.push_back(groups[g].mass);
            out.upid.push_back(groups[g].first);
            out.uoff.push_back(groups[g].offset);
            out.ulen.push_back(groups[g].length);
            out.ucnt.push_back(groups[g].n);
        }
        row.ue = out.umass.size();
        out.rows.push_back(row);
        a = b;
    }
}

void build_store(oref_index* ix, const std::vector<Occ>& occ) {
    const dbi_params* p = &ix->p;
    const int nt = std::max(1, g_threads);
    // row splitters: quantiles of a strided sample (rows never straddle slices)
    std::vector<int64_t> samp;
    const size_t stride = std::max<size_t>(1, occ.size() / 65536);
    for (size_t i = 0; i < occ.size(); i += stride)
        if (!occ[i].dropped) samp.push_back(row_of(p, occ[i].mass));
    std::sort(samp.begin(), samp.end());
    std::vector<int64_t> cut(nt + 1);
    cut[0] = INT64_MIN;
    cut[nt] = INT64_MAX;
    for (int t = 1; t < nt; ++t) cut[t] = samp.empty() ? INT64_MAX : samp[samp.size() * t / nt];
    std::vector<Slice> sl(nt);
    parallel_for(nt, [&](int t) { merge_slice(ix, occ, cut[t], cut[t + 1], sl[t]); });
    // concatenate the slices (rows ascend across them)
    std::vector<uint64_t> ub(nt + 1, 0), ob(nt + 1, 0);
    for (int t = 0; t < nt; ++t) {
        ub[t + 1] = ub[t] + sl[t].umass.size();
        ob[t + 1] = ob[t] + sl[t].occ_pid.size();
    }
    const uint64_t U = ub[nt];
    ix->umass.resize(U);
    ix->upid.resize(U);
    ix->uoff.resize(U);
    ix->ulen.resize(U);
    ix->occ_off.resize(U + 1);
    ix->occ_pid.resize(ob[nt]);
    parallel_for(nt, [&](int t) {
        const Slice& s = sl[t];
        std::copy(s.umass.begin(), s.umass.end(), ix->umass.begin() + ub[t]);
        std::copy(s.upid.begin(), s.upid.end(), ix->upid.begin() + ub[t]);
        std::copy(s.uoff.begin(), s.uoff.end(), ix->uoff.begin() + ub[t]);
        std::copy(s.ulen.begin(), s.ulen.end(), ix->ulen.begin() + ub[t]);
        std::copy(s.occ_pid.begin(), s.occ_pid.end(), ix->occ_pid.begin() + ob[t]);
        uint64_t pos = ob[t];
        for (size_t u = 0; u < s.ucnt.size(); ++u) {
            ix->occ_off[ub[t] + u] = pos;
            pos += s.ucnt[u];
        }
    });
    ix->occ_off[U] = ob[nt];
    ix->rows.clear();
    for (int t = 0; t < nt; ++t)
        for (RowRef r : sl[t].rows) {
            r.ub += ub[t];
            r.ue += ub[t];
            ix->rows.push_back(r);
        }
    ix->bucket_rows.assign(p->index_factor + 1, 0);
    for (int b = 0, r = 0; b <= p->index_factor; ++b) {
        while (r < (int)ix->rows.size() && ix->rows[r].bucket < b) ++r;
        ix->bucket_rows[b] = r;
    }
}

// IndexMerge.getSequences(precMass, tolerance) for one bucket (:146-217)
void bucket_query(const oref_index* ix, int b, double precMass, double tolerance,
                  std::vector<uint64_t>& out) {
    const double f = (double)ix->p.mass_group_factor;
    double minMassF = precMass - tolerance;
    if (minMassF < 0.0) minMassF = 0.0;
    const double maxMassF = precMass + tolerance;
    int32_t minMass = java_d2i(minMassF * f);
    if (minMass < 0) minMass = 0;
    int32_t maxMass = java_d2i(maxMassF * f);
    // SELECT ... WHERE precursor_mass_key BETWEEN minMass AND maxMass (rowid order)
    auto rb = ix->rows.begin() + ix->bucket_rows[b], re = ix->rows.begin() + ix->bucket_rows[b + 1];
    auto it = std::lower_bound(rb, re, minMass, [](const RowRef& r, int32_t k) { return r.key < k; });
    for (; it != re && it->key <= maxMass; ++it) {
        // parseAddPeptideInfo (:386-481): sorted by mass; > max -> break; < min -> skip
        for (uint64_t u = it->ub; u < it->ue; ++u) {
            const double m = ix->umass[u];
            if (m > maxMassF) break;
            if (m < minMassF) continue;
            out.push_back(u);
        }
    }
}

// DBIndexStoreSQLiteMult.getSequences(precMass, tolerance) (:315-350)
void query_one(const oref_index* ix, double precMass, double tolerance, std::vector<uint64_t>& out) {
    const int nb = ix->p.index_factor;
    const int br = MAX_PRECURSOR_INT / nb;
    double minMass = precMass - tolerance;
    if (minMass < 0) minMass = 0;
    const double maxMass = precMass + tolerance;
    int b0 = java_d2i(minMass) / br, b1 = java_d2i(maxMass) / br;  // :226-242
    if (!(b0 > nb - 1 || b1 > nb - 1)) {
        for (int b = b0; b <= b1; ++b) bucket_query(ix, b, precMass, tolerance, out);
    }
}

// cutSeq over proteins [0, n_prot) with worker threads on residue-balanced
// protein ranges, concatenated in protein order = the reference's insertion order
void digest_all(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
                std::vector<Occ>& occ) {
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, g_threads), n_prot));
    std::vector<uint64_t> pb(nt + 1, n_prot);
    pb[0] = 0;
    for (int t = 1; t < nt; ++t)
        pb[t] = (uint64_t)(std::lower_bound(off, off + n_prot + 1, off[n_prot] / nt * t) - off);
    for (int t = 1; t <= nt; ++t) pb[t] = std::max(pb[t], pb[t - 1]);
    std::vector<std::vector<Occ>> part(nt);
    g_ptm_fatal = false;
    parallel_for(nt, [&](int t) {
        for (uint64_t i = pb[t]; i < pb[t + 1]; ++i)
            cut_seq(p, res + off[i], (int)(off[i + 1] - off[i]), (uint32_t)i, part[t]);
    });
    size_t n = 0;
    for (auto& v : part) n += v.size();
    occ.clear();
    occ.reserve(n);
    for (auto& v : part) {
        occ.insert(occ.end(), v.begin(), v.end());
        std::vector<Occ>().swap(v);
    }
}

}  // namespace

extern "C" {

// Worker threads of oref_build*, oref_digest and oref_query_batch (default 1:
// the reference's single-threaded path).
void oref_set_threads(int n) { g_threads = std::max(1, n); }

// Digestion only: every INCLUDE'd occurrence in insertion order.
// Returns count via *n; arrays may be NULL to query the count.
int oref_digest(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
                double* mass, uint32_t* pid, uint32_t* offset, uint32_t* length,
                uint8_t* dropped, uint64_t cap, uint64_t* n) {
    std::vector<Occ> occ;
    digest_all(p, res, off, n_prot, occ);
    if (g_ptm_fatal) return DBI_E_INVALID;
    *n = occ.size();
    if (!mass) return 0;
    if (cap < occ.size()) return DBI_E_INVALID;
    for (size_t i = 0; i < occ.size(); ++i) {
        mass[i] = occ[i].mass;
        pid[i] = occ[i].pid;
        offset[i] = occ[i].offset;
        length[i] = occ[i].length;
        dropped[i] = (uint8_t)occ[i].dropped;
    }
    return 0;
}

// totalSeqCount and bucket drops of cutSeq over every protein, without
// keeping the occurrences (count-only streaming, BASELINE configs[4]).
int oref_count(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
               uint64_t* total, uint64_t* dropped) {
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)g_threads, n_prot));
    std::vector<uint64_t> tot(nt, 0), drop(nt, 0);
    g_ptm_fatal = false;
    parallel_for(nt, [&](int t) {
        std::vector<Occ> occ;
        for (uint64_t i = n_prot * t / nt; i < n_prot * (t + 1) / nt; ++i) {
            occ.clear();
            cut_seq(p, res + off[i], (int)(off[i + 1] - off[i]), (uint32_t)i, occ);
            tot[t] += occ.size();
            for (const Occ& o : occ) drop[t] += o.dropped;
        }
    });
    if (g_ptm_fatal) return DBI_E_INVALID;
    *total = *dropped = 0;
    for (int t = 0; t < nt; ++t) {
        *total += tot[t];
        *dropped += drop[t];
    }
    return 0;
}

// The same count split by SQLiteMult bucket (getBucketForMass, :215-217:
// (int)precMass / BUCKET_MASS_RANGE): hist[b] += the INCLUDE'd occurrences of
// bucket b < NUM_BUCKETS, hist[NUM_BUCKETS] += those past the last bucket
// (addSequence's drops, :283-288).  hist has index_factor + 1 entries.
int oref_count_buckets(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
                       uint64_t* hist) {
    if (p->index_factor <= 0) return DBI_E_INVALID;
    const int nb = p->index_factor;
    const int bucketRange = MAX_PRECURSOR_INT / nb;  // SQLiteMult:56
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)g_threads, n_prot));
    std::vector<std::vector<uint64_t>> part(nt, std::vector<uint64_t>(nb + 1, 0));
    g_ptm_fatal = false;
    parallel_for(nt, [&](int t) {
        std::vector<Occ> occ;
        for (uint64_t i = n_prot * t / nt; i < n_prot * (t + 1) / nt; ++i) {
            occ.clear();
            cut_seq(p, res + off[i], (int)(off[i + 1] - off[i]), (uint32_t)i, occ);
            for (const Occ& o : occ) part[t][std::min(java_d2i(o.mass) / bucketRange, nb)]++;
        }
    });
    if (g_ptm_fatal) return DBI_E_INVALID;
    for (int b = 0; b <= nb; ++b) {
        hist[b] = 0;
        for (int t = 0; t < nt; ++t) hist[b] += part[t][b];
    }
    return 0;
}

int oref_build(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
               oref_index** out) {
    if (p->index_factor <= 0) return DBI_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    oref_index* ix = new oref_index();
    ix->p = *p;
    ix->off.assign(off, off + n_prot + 1);
    ix->residues.assign(res, res + off[n_prot]);
    std::vector<Occ> occ;
    digest_all(p, ix->residues.data(), off, n_prot, occ);
    if (g_ptm_fatal) {
        delete ix;
        return DBI_E_INVALID;
    }
    ix->n_total = occ.size();
    for (const Occ& o : occ) ix->n_dropped += o.dropped;
    build_store(ix, occ);
    auto t1 = std::chrono::steady_clock::now();
    ix->build_seconds = std::chrono::duration<double>(t1 - t0).count();
    *out = ix;
    return 0;
}

// Index from externally supplied occurrences (DBIndexStore.addSequence path).
int oref_build_occurrences(const dbi_params* p, const uint8_t* res, const uint64_t* off,
                           uint64_t n_prot, const double* mass, const uint32_t* pid,
                           const uint32_t* offset, const uint32_t* length, uint64_t n_occ,
                           oref_index** out) {
    if (p->index_factor <= 0) return DBI_E_INVALID;
    oref_index* ix = new oref_index();
    ix->p = *p;
    ix->off.assign(off, off + n_prot + 1);
    ix->residues.assign(res, res + off[n_prot]);
    const int bucketRange = MAX_PRECURSOR_INT / p->index_factor;
    std::vector<Occ> occ;
    for (uint64_t i = 0; i < n_occ; ++i) {
        int bucket = java_d2i(mass[i]) / bucketRange;
        Occ o{mass[i], pid[i], offset[i], length[i], (uint32_t)(bucket > p->index_factor - 1)};
        occ.push_back(o);
    }
    ix->n_total = occ.size();
    for (const Occ& o : occ) ix->n_dropped += o.dropped;
    build_store(ix, occ);
    *out = ix;
    return 0;
}

void oref_free(oref_index* ix) { delete ix; }

double oref_build_seconds(const oref_index* ix) { return ix->build_seconds; }
uint64_t oref_n_total(const oref_index* ix) { return ix->n_total; }
uint64_t oref_n_dropped(const oref_index* ix) { return ix->n_dropped; }
uint64_t oref_n_unique(const oref_index* ix) { return ix->umass.size(); }
uint64_t oref_n_kept(const oref_index* ix) { return ix->n_total - ix->n_dropped; }

// getNumberSequences(): number of rows summed over buckets (SQLiteMult:182-192)
uint64_t oref_n_keys(const oref_index* ix) { return ix->rows.size(); }

// getEntryKeys(): rows of bucket 0, 1, ... in rowid order
int oref_entry_keys(const oref_index* ix, int32_t* keys) {
    for (size_t i = 0; i < ix->rows.size(); ++i) keys[i] = ix->rows[i].key;
    return 0;
}

// Flattened unique table in (bucket, key, row) order + occurrence CSR.
int oref_unique(const oref_index* ix, double* mass, uint32_t* pid, uint32_t* offset,
                uint32_t* length, uint64_t* occ_off, uint32_t* occ_pid) {
    const size_t U = ix->umass.size();
    if (mass) std::copy(ix->umass.begin(), ix->umass.end(), mass);
    if (pid) std::copy(ix->upid.begin(), ix->upid.end(), pid);
    if (offset) std::copy(ix->uoff.begin(), ix->uoff.end(), offset);
    if (length) std::copy(ix->ulen.begin(), ix->ulen.end(), length);
    if (occ_off) std::copy(ix->occ_off.begin(), ix->occ_off.begin() + U + 1, occ_off);
    if (occ_pid) std::copy(ix->occ_pid.begin(), ix->occ_pid.end(), occ_pid);
    return 0;
}

// DBIndexStoreSQLiteMult.getSequences(precMass, tolerance) (:315-350).
// Writes unique ids in result order; *n = count (ids may be NULL).
int oref_query(const oref_index* ix, double precMass, double tolerance, uint64_t* ids,
               uint64_t cap, uint64_t* n) {
    std::vector<uint64_t> out;
    query_one(ix, precMass, tolerance, out);
    *n = out.size();
    if (ids) {
        if (cap < out.size()) return DBI_E_INVALID;
        std::copy(out.begin(), out.end(), ids);
    }
    return 0;
}

// A batch of single-range queries as (first uid, count) per query — the
// result of every query is a run of consecutive uids (rows ascend in uid
// order and each row's entries are mass-sorted); DBI_E_STATE if one is not.
int oref_query_batch(const oref_index* ix, const double* mass, const double* tol, uint64_t nq,
                     uint64_t* first, uint64_t* count) {
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)g_threads, nq / 4096 + 1));
    std::vector<int> bad(nt, 0);
    parallel_for(nt, [&](int t) {
        std::vector<uint64_t> out;
        for (uint64_t i = nq * t / nt; i < nq * (t + 1) / nt; ++i) {
            out.clear();
            query_one(ix, mass[i], tol[i], out);
            count[i] = out.size();
            first[i] = out.empty() ? 0 : out[0];
            for (size_t k = 1; k < out.size(); ++k)
                if (out[k] != out[0] + k) bad[t] = 1;
        }
    });
    for (int b : bad)
        if (b) return DBI_E_STATE;
    return 0;
}

// getSequences(List<MassRange>) (SQLiteMult:353-430): one range delegates to
// the single-range query; >1 ranges reproduce the reference's row selection,
// which binds Da-valued interval bounds to the integer key column
// (IndexMerge.java:300-312 via `(int) minMassF`, `(int) (maxMassF + rows)`;
// for >24 ranges the bounds are the raw doubles, :267-274).
int oref_query_ranges(const oref_index* ix, const double* mass, const double* tol, uint64_t nr,
                      uint64_t* ids, uint64_t cap, uint64_t* n) {
    if (nr == 1) return oref_query(ix, mass[0], tol[0], ids, cap, n);
    std::vector<uint64_t> out;
    if (nr == 0) { *n = 0; return 0; }
    const int nb = ix->p.index_factor;
    const int br = MAX_PRECURSOR_INT / nb;
    // Interval.massRangeToInterval + MergeIntervals.mergeIntervals
    std::vector<std::pair<double, double>> iv;
    for (uint64_t i = 0; i < nr; ++i) {
        double lo = mass[i] - tol[i];
        if (lo < 0.0f) lo = 0.0f;
        iv.push_back({lo, mass[i] + tol[i]});
    }
    std::vector<std::pair<double, double>> merged;
    if (iv.size() < 2) {
        merged = iv;
    } else {
        std::stable_sort(iv.begin(), iv.end(),
                         [](const std::pair<double, double>& a, const std::pair<double, double>& b) {
                             return a.first < b.first;  // Double.compareTo (no NaNs expected)
                         });
        double s = iv[0].first, e = iv[0].second;
        for (size_t i = 1; i < iv.size(); ++i) {
            if (e >= iv[i].first) {
                e = std::max(e, iv[i].second);
            } else {
                merged.push_back({s, e});
                s = iv[i].first;
                e = iv[i].second;
            }
        }
        merged.push_back({s, e});
    }
    std::vector<std::vector<std::pair<double, double>>> per_bucket(nb);
    for (auto& m : merged) {
        int b0 = java_d2i(m.first) / br, b1 = java_d2i(m.second) / br;
        if (b0 > nb - 1 || b1 > nb - 1) { *n = 0; return 0; }  // `return ret` (empty)
        for (int b = b0; b <= b1; ++b) {
            auto& v = per_bucket[b];
            if (std::find(v.begin(), v.end(), m) == v.end()) v.push_back(m);
        }
    }
    for (int b = 0; b < nb; ++b) {
        const auto& ranges = per_bucket[b];
        if (ranges.empty()) continue;
        // IndexMerge.getSequencesIntervals: <=24 intervals use the prepared
        // integer statements, more use an ad-hoc statement with double bounds.
        const size_t k = ranges.size();
        // rows selected by the OR of BETWEEN clauses over the integer key
        for (uint64_t ri = ix->bucket_rows[b]; ri < ix->bucket_rows[b + 1]; ++ri) {
            const RowRef& row = ix->rows[ri];
            const int32_t key = row.key;
            bool sel = false;
            for (auto& r : ranges) {
                if (k <= 24) {
                    int32_t lo = java_d2i(r.first) - 0;          // (int) minMassF - rows(0)
                    int32_t hi = java_d2i(r.second + 0);         // (int) (maxMassF + rows)
                    if (key >= lo && key <= hi) sel = true;
                } else {
                    if ((double)key >= r.first && (double)key <= r.second) sel = true;
                }
            }
            if (!sel) continue;
            // parseAddPeptideInfo(data, ret, minMasses, maxMasses) (:494-600)
            for (uint64_t u = row.ub; u < row.ue; ++u) {
                const double m = ix->umass[u];
                bool greaterThanMax = true, qualifies = false;
                for (auto& r : ranges) {
                    if (m < r.second) greaterThanMax = false;
                    if (m >= r.first && m <= r.second) qualifies = true;
                    if (qualifies) break;
                }
                if (greaterThanMax && !qualifies) break;
                if (!qualifies) continue;
                out.push_back(u);
            }
        }
    }
    *n = out.size();
    if (ids) {
        if (cap < out.size()) return DBI_E_INVALID;
        std::copy(out.begin(), out.end(), ids);
    }
    return 0;
}

// IndexUtil.calculateMass(seq, h2o) (IndexUtil.java:197-208)
// the formula mass the literal PTM walk adds (cut_seq_literal)
double oref_formula_mass(const char* f, uint64_t len) { return formula_mass(std::string(f, len)); }

double oref_calculate_mass(const dbi_params* p, const uint8_t* seq, uint64_t len) {
    double mass = 0;
    if (p->add_h2o_proton) mass += p->h2o_proton;
    mass += p->cterm;
    mass += p->nterm;
    for (uint64_t i = 0; i < len; ++i) mass += p->mass[seq[i]];
    return mass;
}

// IndexUtil.getToleranceInDalton (:238-240)
double oref_tolerance_in_dalton(double actualMass, double ppm) {
    return actualMass * (1 - 1 / (ppm / 1000000 + 1));
}

}  // extern "C"
