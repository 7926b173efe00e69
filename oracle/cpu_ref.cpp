// oracle/cpu_ref.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// CPU restatement of the reference's digestion + index + mass-lookup path,
// written loop-for-loop from the Java sources under /root/reference
// (paths below relative to src/main/java/edu/scripps/yates/dbindex/).
// Used by tests/ as the parity checker, by bench.py as the `cpu_baseline`
// ("port": single-threaded, like the reference), and by __graft_entry__.smoke().
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
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
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

// DBIndexer.cutSeq(String,String) (:237-405), with the SQLiteMult store behind it.
// Appends every INCLUDE'd occurrence (incl. bucket-dropped ones, flagged) in
// insertion order.
void cut_seq(const dbi_params* p, const uint8_t* seq, int length, uint32_t proteinId,
             std::vector<Occ>& out) {
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
struct Merged {
    double mass;
    uint32_t offset;
    uint32_t length;
    std::vector<uint32_t> pids;
    uint64_t uid;  // position in the flattened (bucket, key, row-order) table
};

struct Row {
    int32_t key;
    std::vector<Occ> recs;        // insertion order (Byte.updateCachedData appends)
    std::vector<Merged> merged;   // after getMergedData
};

}  // namespace

struct oref_index {
    dbi_params p;
    std::vector<uint8_t> residues;
    std::vector<uint64_t> off;
    std::vector<Occ> occ;  // all INCLUDE'd occurrences, insertion order
    uint64_t n_total = 0, n_dropped = 0;
    // buckets[b] : key -> row (std::map keeps ascending key = rowid order)
    std::vector<std::map<int32_t, Row>> buckets;
    std::vector<const Merged*> flat;  // uid -> entry
    double build_seconds = 0;
};

namespace {

std::string pep_string(const oref_index* ix, uint32_t pid, uint32_t off, uint32_t len) {
    // ProteinCache.getPeptideSequence (ProteinCache.java:112-127)
    const uint8_t* s = ix->residues.data() + ix->off[pid] + off;
    return std::string((const char*)s, len);
}

// Pinned tie-break between different peptides of bit-identical mass
// (semantics A7): the 32-bit FNV-1a of the peptide string folded
// to 16 bits, then first appearance.
uint16_t peptide_tag(const std::string& s) {
    uint32_t h = 2166136261u;
    for (unsigned char c : s) {
        h ^= c;
        h *= 16777619u;
    }
    return (uint16_t)((h >> 16) ^ (h & 0xFFFFu));
}

// DBIndexStoreSQLiteByteIndexMerge.getMergedData (:620-719).  The reference
// groups through a THashMap (iteration order unspecified) and then stable-sorts
// by mass (IndexedSeqMerged.compareTo); we pin the order of equal-mass groups to
// (16-bit FNV-1a tag of the string, first appearance) (semantics A7).
void merge_row(const oref_index* ix, Row& row) {
    std::unordered_map<std::string, size_t> where;
    std::vector<Merged> groups;
    std::vector<uint16_t> gtag;
    where.reserve(row.recs.size() * 2);
    for (const Occ& r : row.recs) {
        std::string pep = pep_string(ix, r.pid, r.offset, r.length);
        auto it = where.find(pep);
        if (it == where.end()) {
            gtag.push_back(peptide_tag(pep));
            where.emplace(std::move(pep), groups.size());
            // first occurrence keeps mass/offset/length; its protein id is first
            groups.push_back(Merged{r.mass, r.offset, r.length, {r.pid}, 0});
        } else {
            groups[it->second].pids.push_back(r.pid);
        }
    }
    // Collections.sort(sortedMerged) — stable, by mass (IndexedSeqMerged.compareTo),
    // ties pinned to (tag, first appearance)
    std::vector<size_t> ord(groups.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        if (groups[a].mass != groups[b].mass) return groups[a].mass < groups[b].mass;
        return gtag[a] < gtag[b];
    });
    row.merged.clear();
    row.merged.reserve(groups.size());
    for (size_t i : ord) row.merged.push_back(std::move(groups[i]));
    row.recs.clear();
    row.recs.shrink_to_fit();
}

void build_store(oref_index* ix) {
    const dbi_params* p = &ix->p;
    ix->buckets.assign(p->index_factor, {});
    const int bucketRange = MAX_PRECURSOR_INT / p->index_factor;
    for (const Occ& o : ix->occ) {
        if (o.dropped) continue;
        int bucket = java_d2i(o.mass) / bucketRange;
        int32_t key = java_d2i(o.mass * (double)p->mass_group_factor);  // Byte:187
        Row& row = ix->buckets[bucket][key];
        row.key = key;
        row.recs.push_back(o);
    }
    for (auto& b : ix->buckets)
        for (auto& kv : b) merge_row(ix, kv.second);
    ix->flat.clear();
    for (auto& b : ix->buckets)
        for (auto& kv : b)
            for (auto& m : kv.second.merged) {
                m.uid = ix->flat.size();
                ix->flat.push_back(&m);
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
    const auto& rows = ix->buckets[b];
    for (auto it = rows.lower_bound(minMass); it != rows.end() && it->first <= maxMass; ++it) {
        // parseAddPeptideInfo (:386-481): sorted by mass; > max -> break; < min -> skip
        for (const Merged& m : it->second.merged) {
            if (m.mass > maxMassF) break;
            if (m.mass < minMassF) continue;
            out.push_back(m.uid);
        }
    }
}

}  // namespace

extern "C" {

// Digestion only: every INCLUDE'd occurrence in insertion order.
// Returns count via *n; arrays may be NULL to query the count.
int oref_digest(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
                double* mass, uint32_t* pid, uint32_t* offset, uint32_t* length,
                uint8_t* dropped, uint64_t cap, uint64_t* n) {
    std::vector<Occ> occ;
    for (uint64_t i = 0; i < n_prot; ++i)
        cut_seq(p, res + off[i], (int)(off[i + 1] - off[i]), (uint32_t)i, occ);
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

int oref_build(const dbi_params* p, const uint8_t* res, const uint64_t* off, uint64_t n_prot,
               oref_index** out) {
    if (p->index_factor <= 0) return DBI_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    oref_index* ix = new oref_index();
    ix->p = *p;
    ix->off.assign(off, off + n_prot + 1);
    ix->residues.assign(res, res + off[n_prot]);
    for (uint64_t i = 0; i < n_prot; ++i)
        cut_seq(p, ix->residues.data() + off[i], (int)(off[i + 1] - off[i]), (uint32_t)i, ix->occ);
    ix->n_total = ix->occ.size();
    for (const Occ& o : ix->occ) ix->n_dropped += o.dropped;
    build_store(ix);
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
    for (uint64_t i = 0; i < n_occ; ++i) {
        int bucket = java_d2i(mass[i]) / bucketRange;
        Occ o{mass[i], pid[i], offset[i], length[i], (uint32_t)(bucket > p->index_factor - 1)};
        ix->occ.push_back(o);
    }
    ix->n_total = ix->occ.size();
    for (const Occ& o : ix->occ) ix->n_dropped += o.dropped;
    build_store(ix);
    *out = ix;
    return 0;
}

void oref_free(oref_index* ix) { delete ix; }

double oref_build_seconds(const oref_index* ix) { return ix->build_seconds; }
uint64_t oref_n_total(const oref_index* ix) { return ix->n_total; }
uint64_t oref_n_dropped(const oref_index* ix) { return ix->n_dropped; }
uint64_t oref_n_unique(const oref_index* ix) { return ix->flat.size(); }
uint64_t oref_n_kept(const oref_index* ix) { return ix->n_total - ix->n_dropped; }

// getNumberSequences(): number of rows summed over buckets (SQLiteMult:182-192)
uint64_t oref_n_keys(const oref_index* ix) {
    uint64_t n = 0;
    for (auto& b : ix->buckets) n += b.size();
    return n;
}

// getEntryKeys(): rows of bucket 0, 1, ... in rowid order
int oref_entry_keys(const oref_index* ix, int32_t* keys) {
    uint64_t i = 0;
    for (auto& b : ix->buckets)
        for (auto& kv : b) keys[i++] = kv.first;
    return 0;
}

// Flattened unique table in (bucket, key, row) order + occurrence CSR.
int oref_unique(const oref_index* ix, double* mass, uint32_t* pid, uint32_t* offset,
                uint32_t* length, uint64_t* occ_off, uint32_t* occ_pid) {
    uint64_t pos = 0;
    for (size_t u = 0; u < ix->flat.size(); ++u) {
        const Merged* m = ix->flat[u];
        if (mass) mass[u] = m->mass;
        if (pid) pid[u] = m->pids[0];
        if (offset) offset[u] = m->offset;
        if (length) length[u] = m->length;
        if (occ_off) occ_off[u] = pos;
        for (uint32_t q : m->pids) {
            if (occ_pid) occ_pid[pos] = q;
            ++pos;
        }
    }
    if (occ_off) occ_off[ix->flat.size()] = pos;
    return 0;
}

// DBIndexStoreSQLiteMult.getSequences(precMass, tolerance) (:315-350).
// Writes unique ids in result order; *n = count (ids may be NULL).
int oref_query(const oref_index* ix, double precMass, double tolerance, uint64_t* ids,
               uint64_t cap, uint64_t* n) {
    std::vector<uint64_t> out;
    const int nb = ix->p.index_factor;
    const int br = MAX_PRECURSOR_INT / nb;
    double minMass = precMass - tolerance;
    if (minMass < 0) minMass = 0;
    const double maxMass = precMass + tolerance;
    int b0 = java_d2i(minMass) / br, b1 = java_d2i(maxMass) / br;  // :226-242
    if (!(b0 > nb - 1 || b1 > nb - 1)) {
        for (int b = b0; b <= b1; ++b) bucket_query(ix, b, precMass, tolerance, out);
    }
    *n = out.size();
    if (ids) {
        if (cap < out.size()) return DBI_E_INVALID;
        std::copy(out.begin(), out.end(), ids);
    }
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
        const auto& rows = ix->buckets[b];
        for (auto it = rows.begin(); it != rows.end(); ++it) {
            const int32_t key = it->first;
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
            for (const Merged& m : it->second.merged) {
                bool greaterThanMax = true, qualifies = false;
                for (auto& r : ranges) {
                    if (m.mass < r.second) greaterThanMax = false;
                    if (m.mass >= r.first && m.mass <= r.second) qualifies = true;
                    if (qualifies) break;
                }
                if (greaterThanMax && !qualifies) break;
                if (!qualifies) continue;
                out.push_back(m.uid);
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
