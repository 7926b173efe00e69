// dbi_store.cpp — the DBIndexStore mirror (include/dbindex_hip.h, dbi_store_*).
//
// Behaviour follows DBIndexStoreSQLiteMult (the store the reference's DBIndexer
// builds, DBIndexStoreSQLiteMult.java) with the SQLite persistence replaced by
// the HBM-resident index of the batch engine:
//   init/startAddSeq/stopAddSeq state machine ... SQLiteMult.java:92-176,
//                                                 SQLiteAbstract.java:235-325
//   addProteinDef returns num ....................... SQLiteMult.java:446-450
//   filterSequence .................................. SQLiteMult.java:245-268
//   addSequence (totalSeqCount, bucket drop) ........ SQLiteMult.java:271-291
//   getSequences(m, tol) ............................ SQLiteMult.java:315-350
//   getSequences(List<MassRange>) ................... SQLiteMult.java:353-430
//   getNumberSequences (rows, not peptides) ......... SQLiteByte.java:667-690
//   IndexedSequence materialisation + flanks ........ IndexMerge.java:386-481,
//                                                     Util.getResidues Util.java:130-162
// The GPU engine is opened lazily at the first stopAddSeq(), so the host-side
// contract is usable (and tested) on machines without a GPU.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dbi_internal.h"

namespace dbi {
int engine_key_range(dbi_handle* h, int32_t klo, int32_t khi, uint64_t* b, uint64_t* e);
bool engine_built(const dbi_handle* h);
}  // namespace dbi

using namespace dbi;

struct dbi_store {
    dbi_params p;
    int device = 0;
    dbi_handle* eng = nullptr;
    bool inited = false, in_tx = false, device_digest = false, persist = false;
    int unindexed = 0;          // MassRangeFilteringIndex mode (SEARCH_UNINDEXED): 0 off, 1 resident, 2 stream
    uint64_t last_matches = 0;  // unindexed: size of the last cutAndSearch result
    std::mutex search_mu;       // STREAM searches rebuild the engine's index: one at a time
    std::string db_id;
    // ProteinCache (ProteinCache.java:24-95): defs + sequences in id order
    std::vector<std::string> defs;
    std::vector<uint8_t> residues;
    std::vector<uint64_t> off{0};
    // occurrences from addSequence (insertion order)
    std::vector<double> om;
    std::vector<uint32_t> opid, ooff, olen;
    uint64_t dropped = 0;
    int64_t total_seq_count = 0;
};

namespace {

int br_of(const dbi_params& p) { return MAX_PRECURSOR_INT / p.index_factor; }

struct ListBuilder {
    std::vector<double> mass;
    std::vector<uint64_t> seq_off{0};
    std::string chars;
    std::string left, right;
    std::vector<uint64_t> prot_off{0};
    std::vector<uint32_t> prot_ids, offset, length;
    std::vector<uint64_t> uid;

    int finish(dbi_seq_list** out) {
        dbi_seq_list* l = (dbi_seq_list*)std::calloc(1, sizeof(dbi_seq_list));
        if (!l) return set_error(DBI_E_OOM, "calloc");
        const uint64_t n = mass.size();
        l->n = n;
        auto dup = [](const void* src, size_t bytes) -> void* {
            void* d = std::malloc(bytes ? bytes : 1);
            if (d && bytes) std::memcpy(d, src, bytes);
            return d;
        };
        l->mass = (double*)dup(mass.data(), 8 * n);
        l->seq_off = (uint64_t*)dup(seq_off.data(), 8 * (n + 1));
        l->seq_chars = (char*)dup(chars.data(), chars.size());
        l->res_left = (char*)dup(left.data(), left.size());
        l->res_right = (char*)dup(right.data(), right.size());
        l->prot_off = (uint64_t*)dup(prot_off.data(), 8 * (n + 1));
        l->prot_ids = (uint32_t*)dup(prot_ids.data(), 4 * prot_ids.size());
        l->offset = (uint32_t*)dup(offset.data(), 4 * n);
        l->length = (uint32_t*)dup(length.data(), 4 * n);
        l->unique_id = (uint64_t*)dup(uid.data(), 8 * n);
        if (!l->mass || !l->seq_off || !l->seq_chars || !l->res_left || !l->res_right || !l->prot_off ||
            !l->prot_ids || !l->offset || !l->length || !l->unique_id) {
            dbi_seq_list_free(l);
            return set_error(DBI_E_OOM, "malloc");
        }
        *out = l;
        return 0;
    }
};

// Util.getResidues(peptide, seqOffset, seqLen, proteinSequence) (Util.java:130-162);
// cut_flanks: the flanks cutSeq itself computes (DBIndexer.java:356-383, end
// inclusive there, so no one-short right flank), kept by MassRangeFilteringIndex
void get_residues(const uint8_t* prot, uint64_t protLen, uint64_t seqOffset, uint64_t seqLen, std::string& left,
                  std::string& right, bool cut_flanks = false) {
    const uint64_t L = 3;  // Constants.MAX_INDEX_RESIDUE_LEN
    const uint64_t resLeftI = seqOffset >= L ? seqOffset - L : 0;
    const uint64_t resLeftLen = std::min<uint64_t>(L, seqOffset);
    std::string sl((const char*)prot + resLeftI, resLeftLen);
    const uint64_t end = seqOffset + seqLen;
    const int64_t rr = (int64_t)protLen - (int64_t)end - (cut_flanks ? 0 : 1);  // protLen - end - 1 (quirk)
    const int64_t resRightLen = std::min<int64_t>((int64_t)L, rr);
    std::string sr;
    if (end < protLen && resRightLen > 0) sr.assign((const char*)prot + end, (size_t)resRightLen);
    while (sl.size() < L) sl.insert(sl.begin(), '-');
    while (sr.size() < L) sr.push_back('-');
    left += sl;
    right += sr;
}

// materialise unique ids [first, first+count) (contiguous, ascending) into lb
// filtering: MassRangeFilteringIndex entries -- protein ids without repeats
// (addSequence :124-127, `!protIds.contains`; occurrences are in protein order,
// so repeats are adjacent) and cutSeq's own flanks (IndexedSequence resLeft/resRight)
int materialise(dbi_store* s, const std::vector<uint64_t>& ids, ListBuilder& lb, bool filtering = false) {
    const uint64_t n = ids.size();
    if (n == 0) return 0;
    std::vector<double> mass(n);
    std::vector<uint32_t> pid(n), off(n), len(n);
    std::vector<uint64_t> ob(n), oe(n);
    int rc = dbi_peptides(s->eng, ids.data(), n, mass.data(), pid.data(), off.data(), len.data(), ob.data(), oe.data());
    if (rc) return rc;
    // occurrence lists of consecutive ids are adjacent: one read per run of ids
    std::vector<uint32_t> run;
    uint64_t run_b = 0, run_e = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (i == 0 || ids[i] != ids[i - 1] + 1) {
            uint64_t j = i;
            while (j + 1 < n && ids[j + 1] == ids[j] + 1) ++j;
            run_b = ob[i];
            run_e = oe[j];
            run.resize(run_e - run_b);
            if (!run.empty() && (rc = dbi_occurrences(s->eng, run_b, run_e, run.data()))) return rc;
        }
        std::vector<uint32_t> occ(run.begin() + (ob[i] - run_b), run.begin() + (oe[i] - run_b));
        const uint8_t* prot = s->residues.data() + s->off[pid[i]];
        const uint64_t plen = s->off[pid[i] + 1] - s->off[pid[i]];
        lb.mass.push_back(mass[i]);
        lb.chars.append((const char*)prot + off[i], len[i]);
        lb.seq_off.push_back(lb.chars.size());
        get_residues(prot, plen, off[i], len[i], lb.left, lb.right, filtering);
        if (filtering) occ.erase(std::unique(occ.begin(), occ.end()), occ.end());
        lb.prot_ids.insert(lb.prot_ids.end(), occ.begin(), occ.end());
        lb.prot_off.push_back(lb.prot_ids.size());
        lb.offset.push_back(off[i]);
        lb.length.push_back(len[i]);
        lb.uid.push_back(ids[i]);
    }
    return 0;
}

int ensure_engine(dbi_store* s) {
    if (s->eng) return 0;
    int rc = dbi_open(&s->p, s->device, &s->eng);
    if (!rc && s->unindexed) rc = dbi_set_bucket_drop(s->eng, 0);
    return rc;
}

}  // namespace

extern "C" {

int dbi_store_create(const dbi_params* params, int device, dbi_store** out) {
    if (!params || !out) return set_error(DBI_E_INVALID, "NULL argument");
    if (params->index_factor <= 0) return set_error(DBI_E_INVALID, "index_factor must be > 0");
    if (params->mass_group_factor <= 0) return set_error(DBI_E_INVALID, "mass_group_factor must be > 0");
    dbi_store* s = new dbi_store();
    s->p = *params;
    s->device = device;
    *out = s;
    return 0;
}

void dbi_store_close(dbi_store* s) {
    if (!s) return;
    if (s->eng) dbi_close(s->eng);
    delete s;
}

int dbi_store_set_device_digest(dbi_store* s, int on) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (!on && s->unindexed) return set_error(DBI_E_STATE, "the unindexed store digests on the device");
    if (s->in_tx && !s->om.empty()) return set_error(DBI_E_STATE, "occurrences already added in this transaction");
    s->device_digest = on != 0;
    return 0;
}

int dbi_store_set_persist(dbi_store* s, int on) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (s->inited) return set_error(DBI_E_STATE, "set persistence before init()");
    if (on && s->unindexed) return set_error(DBI_E_STATE, "the unindexed store keeps no index on disk");
    s->persist = on != 0;
    return 0;
}

int dbi_store_set_unindexed(dbi_store* s, int on) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (s->inited) return set_error(DBI_E_STATE, "set the unindexed mode before init()");
    if (on) {
        // SKIP_PROTEIN_START ends a start's walk once its mass passes every range
        // (DBIndexer.java:351-354); that drops nothing only while masses never decrease
        for (int c = 0; c < 256; ++c)
            if (!(s->p.mass[c] >= 0.0))
                return set_error(DBI_E_INVALID, "unindexed search needs non-negative residue masses");
        if (!(s->p.max_mh < 65536.0))
            return set_error(DBI_E_INVALID, "unindexed search needs a max precursor mass < 65536 Da");
        s->device_digest = true;
        s->persist = false;
        // MassRangeFilteringIndex.filterSequence has no mandatory-residue test;
        // cutSeq's own test (DBIndexer.java:334-344, mandatory[]) stays
        s->p.mandatory_count = 0;
    }
    if (on < 0 || on > DBI_UNINDEXED_STREAM) return set_error(DBI_E_INVALID, "unknown unindexed mode");
    s->unindexed = on;
    return 0;
}

int dbi_store_init(dbi_store* s, const char* database_id) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (!database_id || !*database_id)
        return set_error(DBI_E_INVALID, "Index path is missing, cannot initialize the indexer.");
    if (s->inited) return set_error(DBI_E_STATE, "Already intialized");
    s->db_id = database_id;
    if (s->persist) {
        // an index of these parameters on disk: load it (DBIndexStoreSQLiteMult.init :92-149)
        const std::string path = s->db_id + ".dbihip";
        bool match = false;
        int rc = index_file_matches(s->p, path.c_str(), &match);
        if (rc) return rc;
        if (match) {
            if ((rc = ensure_engine(s))) return rc;
            std::string defs;
            std::vector<uint64_t> doff;
            if ((rc = index_load(s->eng, path.c_str(), &s->residues, &s->off, &defs, &doff))) return rc;
            s->defs.clear();
            for (size_t i = 0; i + 1 < doff.size(); ++i) s->defs.emplace_back(defs, doff[i], doff[i + 1] - doff[i]);
            dbi_stats st{};
            dbi_stats_get(s->eng, &st);
            s->total_seq_count = (int64_t)st.n_total;
        }
    }
    s->inited = true;
    return 0;
}

int dbi_store_start_add_seq(dbi_store* s) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    if (s->in_tx) return set_error(DBI_E_STATE, "In transaction already");
    s->in_tx = true;
    return 0;
}

int dbi_store_stop_add_seq(dbi_store* s) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    if (!s->in_tx) return set_error(DBI_E_STATE, "Not in transaction.");
    int rc = ensure_engine(s);
    if (rc) return rc;
    const uint64_t P = s->defs.size();
    if (s->unindexed == DBI_UNINDEXED_STREAM) {
        // proteins to HBM once; each search digests them through its windows
        if (!s->residues.empty() && std::memchr(s->residues.data(), '[', s->residues.size()))
            return set_error(DBI_E_INVALID, "inline '[formula]' PTMs need the resident unindexed mode (the streaming "
                                            "search re-digests the proteins as stored)");
        if ((rc = dbi_set_windows(s->eng, nullptr, nullptr, 0, 1))) return rc;
        rc = dbi_build(s->eng, s->residues.data(), s->residues.size(), s->off.data(), P);
    } else if (s->device_digest) {
        rc = dbi_build(s->eng, s->residues.data(), s->residues.size(), s->off.data(), P);
    } else {
        rc = dbi_build_occurrences(s->eng, s->residues.data(), s->residues.size(), s->off.data(), P, s->om.data(),
                                   s->opid.data(), s->ooff.data(), s->olen.data(), s->om.size(), s->dropped);
    }
    if (rc) return rc;
    s->in_tx = false;
    if (s->persist) {  // commit to disk (DBIndexStoreSQLiteMult.stopAddSeq -> commitCachedData)
        std::string defs;
        std::vector<uint64_t> doff{0};
        for (const auto& d : s->defs) {
            defs += d;
            doff.push_back(defs.size());
        }
        const std::string path = s->db_id + ".dbihip";
        if ((rc = index_save(s->eng, path.c_str(), &defs, &doff))) return rc;
    }
    return 0;
}

int dbi_store_index_exists(dbi_store* s, int* out) {
    if (!s || !out) return set_error(DBI_E_INVALID, "NULL argument");
    if (!s->inited) return set_error(DBI_E_STATE, "Not intialized");
    if (s->unindexed) {  // MassRangeFilteringIndex.indexExists (:83-87)
        *out = 0;
        return 0;
    }
    dbi_stats st{};
    if (s->eng && engine_built(s->eng)) dbi_stats_get(s->eng, &st);
    *out = st.n_keys > 0;  // hasSequences(): any bucket with rows (SQLiteMult:204-213)
    return 0;
}

int dbi_store_add_protein_def(dbi_store* s, int64_t num, const char* def, const char* seq, uint64_t seq_len,
                              int64_t* out_id) {
    if (!s || (!seq && seq_len)) return set_error(DBI_E_INVALID, "NULL argument");
    if (num != (int64_t)s->defs.size())
        return set_error(DBI_E_INVALID, "protein numbers must be 0,1,2,... in FASTA order (ProteinCache ids)");
    std::string d = def ? def : "";
    std::replace(d.begin(), d.end(), '\t', ' ');  // ProteinCache.addProtein (:84-90)
    s->defs.push_back(std::move(d));
    s->residues.insert(s->residues.end(), (const uint8_t*)seq, (const uint8_t*)seq + seq_len);
    s->off.push_back(s->residues.size());
    if (out_id) *out_id = num;
    return 0;
}

int dbi_store_filter_sequence(dbi_store* s, double mass, const char* seq, uint64_t seq_len, int* out_result) {
    if (!s || !out_result) return set_error(DBI_E_INVALID, "NULL argument");
    if (s->device_digest) {  // digestion happens on the device at stopAddSeq()
        *out_result = DBI_FILTER_SKIP_PROTEIN_START;
        return 0;
    }
    const dbi_params& p = s->p;
    if (p.mandatory_mode && p.mandatory_count > 0) {
        for (uint64_t i = 0; i + 1 < seq_len; ++i)
            if (p.mandatory[(uint8_t)seq[i]]) {
                *out_result = DBI_FILTER_INCLUDE;
                return 0;
            }
        *out_result = DBI_FILTER_SKIP;
        return 0;
    }
    *out_result = (p.max_mh < mass || p.min_mh > mass) ? DBI_FILTER_SKIP : DBI_FILTER_INCLUDE;
    return 0;
}

int dbi_store_add_sequence(dbi_store* s, double mass, int32_t offset, int32_t length, int64_t protein_id) {
    if (!s) return set_error(DBI_E_INVALID, "NULL store");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    if (s->device_digest) return set_error(DBI_E_STATE, "device digestion is on: occurrences are produced on the GPU");
    s->total_seq_count++;
    const int bucket = java_d2i(mass) / br_of(s->p);
    if (!(mass >= 0.0) || bucket < 0) return set_error(DBI_E_INVALID, "negative or NaN precursor mass");
    if (bucket > s->p.index_factor - 1) {  // "Cannot add to index, unsupported precursor mass"
        s->dropped++;
        return 0;
    }
    if (protein_id < 0 || (uint64_t)protein_id >= s->defs.size())
        return set_error(DBI_E_INVALID, "protein id not added with addProteinDef");
    const uint64_t plen = s->off[protein_id + 1] - s->off[protein_id];
    if (offset < 0 || length <= 0 || (uint64_t)offset + (uint64_t)length > plen)
        return set_error(DBI_E_INVALID, "sequence offset/length outside its protein");
    s->om.push_back(mass);
    s->opid.push_back((uint32_t)protein_id);
    s->ooff.push_back((uint32_t)offset);
    s->olen.push_back((uint32_t)length);
    return 0;
}

int dbi_store_get_number_sequences(dbi_store* s, int64_t* out) {
    if (!s || !out) return set_error(DBI_E_INVALID, "NULL argument");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    if (s->unindexed) {  // MassRangeFilteringIndex.getNumberSequences (:181-183): the last result's size
        *out = (int64_t)s->last_matches;
        return 0;
    }
    dbi_stats st{};
    if (s->eng && engine_built(s->eng)) dbi_stats_get(s->eng, &st);
    *out = (int64_t)st.n_keys;
    return 0;
}

int dbi_store_get_total_seq_count(dbi_store* s, int64_t* out) {
    if (!s || !out) return set_error(DBI_E_INVALID, "NULL argument");
    if (s->device_digest) {
        dbi_stats st{};
        if (s->eng && engine_built(s->eng)) dbi_stats_get(s->eng, &st);
        *out = (int64_t)st.n_total;
    } else {
        *out = s->total_seq_count;
    }
    return 0;
}

int dbi_store_get_entry_keys(dbi_store* s, int32_t* keys, uint64_t cap, uint64_t* n) {
    if (!s || !n) return set_error(DBI_E_INVALID, "NULL argument");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    if (s->unindexed) return set_error(DBI_E_STATE, "Method not implemented");  // MassRangeFilteringIndex:212-215
    if (!s->eng || !engine_built(s->eng)) {
        *n = 0;
        return 0;
    }
    return dbi_entry_keys(s->eng, keys, cap, n);
}

dbi_handle* dbi_store_engine(dbi_store* s) { return s ? s->eng : nullptr; }

int dbi_store_cut_and_search(dbi_store* s, const double* mass, const double* tol, uint64_t n_ranges,
                             dbi_seq_list** out) {
    if (!s || !out || (n_ranges && (!mass || !tol))) return set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    if (!s->unindexed) return set_error(DBI_E_STATE, "Cut and search only supported for SEARCH_UNINDEXED mode !");
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    std::lock_guard<std::mutex> lock(s->search_mu);
    ListBuilder lb;
    s->last_matches = 0;
    const bool stream = s->unindexed == DBI_UNINDEXED_STREAM;
    if (n_ranges == 0 || !s->eng || (!stream && !engine_built(s->eng))) return lb.finish(out);
    // every range is one window of the mass-sorted unique table (the engine
    // is built without buckets); their union, each sequence once
    int rc;
    if (stream) {  // cut the cached proteins through these ranges
        if ((rc = dbi_set_windows(s->eng, mass, tol, n_ranges, 1)) || (rc = dbi_rebuild(s->eng))) return rc;
    }
    std::vector<uint64_t> first(n_ranges), count(n_ranges);
    rc = dbi_query(s->eng, mass, tol, n_ranges, first.data(), count.data());
    if (rc) return rc;
    std::vector<std::pair<uint64_t, uint64_t>> iv;
    for (uint64_t i = 0; i < n_ranges; ++i)
        if (count[i]) iv.push_back({first[i], first[i] + count[i]});
    std::sort(iv.begin(), iv.end());
    std::vector<uint64_t> ids;
    uint64_t next = 0;
    for (auto& r : iv) {
        for (uint64_t u = std::max(r.first, next); u < r.second; ++u) ids.push_back(u);
        next = std::max(next, r.second);
    }
    if ((rc = materialise(s, ids, lb, true))) return rc;
    s->last_matches = ids.size();
    return lb.finish(out);
}

int dbi_store_get_sequences(dbi_store* s, double mass, double tol, dbi_seq_list** out) {
    if (!s || !out) return set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    if (s->unindexed) return dbi_store_cut_and_search(s, &mass, &tol, 1, out);
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    ListBuilder lb;
    if (s->eng && engine_built(s->eng)) {
        uint64_t first = 0, count = 0;
        int rc = dbi_query(s->eng, &mass, &tol, 1, &first, &count);
        if (rc) return rc;
        std::vector<uint64_t> ids(count);
        for (uint64_t i = 0; i < count; ++i) ids[i] = first + i;
        if ((rc = materialise(s, ids, lb))) return rc;
    }
    return lb.finish(out);
}

int dbi_store_get_sequences_ranges(dbi_store* s, const double* mass, const double* tol, uint64_t n_ranges,
                                   dbi_seq_list** out) {
    if (!s || !out || (n_ranges && (!mass || !tol))) return set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    if (s->unindexed) return dbi_store_cut_and_search(s, mass, tol, n_ranges, out);
    if (n_ranges == 1) return dbi_store_get_sequences(s, mass[0], tol[0], out);
    if (!s->inited) return set_error(DBI_E_STATE, "Indexer is not initialized");
    ListBuilder lb;
    if (n_ranges == 0 || !s->eng || !engine_built(s->eng)) return lb.finish(out);
    const int nb = s->p.index_factor, br = br_of(s->p);
    const double f = (double)s->p.mass_group_factor;
    // Interval.massRangeToInterval + MergeIntervals.mergeIntervals
    std::vector<std::pair<double, double>> iv;
    for (uint64_t i = 0; i < n_ranges; ++i) {
        double lo = mass[i] - tol[i];
        if (lo < 0.0f) lo = 0.0f;
        iv.push_back({lo, mass[i] + tol[i]});
    }
    std::stable_sort(iv.begin(), iv.end(), [](const std::pair<double, double>& a, const std::pair<double, double>& b) {
        return a.first < b.first;
    });
    std::vector<std::pair<double, double>> merged;
    double cs = iv[0].first, ce = iv[0].second;
    for (size_t i = 1; i < iv.size(); ++i) {
        if (ce >= iv[i].first) {
            ce = std::max(ce, iv[i].second);
        } else {
            merged.push_back({cs, ce});
            cs = iv[i].first;
            ce = iv[i].second;
        }
    }
    merged.push_back({cs, ce});
    std::vector<std::vector<std::pair<double, double>>> per_bucket(nb);
    for (auto& m : merged) {
        const int b0 = java_d2i(m.first) / br, b1 = java_d2i(m.second) / br;
        if (b0 > nb - 1 || b1 > nb - 1) return lb.finish(out);  // "Cannot query, unsupported precursor mass"
        for (int b = b0; b <= b1; ++b) {
            auto& v = per_bucket[b];
            if (std::find(v.begin(), v.end(), m) == v.end()) v.push_back(m);
        }
    }
    // Rows are selected by BETWEEN on the integer key column with Da-valued
    // bounds (IndexMerge.java:300-312; raw doubles beyond 24 ranges :267-274).
    std::vector<uint64_t> ids;
    for (int b = 0; b < nb; ++b) {
        const auto& ranges = per_bucket[b];
        if (ranges.empty()) continue;
        const bool prepared = ranges.size() <= 24;
        std::vector<std::pair<int64_t, int64_t>> kr;
        for (auto& r : ranges) {
            int64_t klo, khi;
            if (prepared) {
                klo = java_d2i(r.first);
                khi = java_d2i(r.second);
            } else {
                klo = (int64_t)std::ceil(r.first);
                khi = (int64_t)std::floor(r.second);
            }
            klo = std::max<int64_t>(klo, INT32_MIN);
            khi = std::min<int64_t>(khi, INT32_MAX);
            if (klo <= khi) kr.push_back({klo, khi});
        }
        std::sort(kr.begin(), kr.end());
        std::vector<std::pair<int64_t, int64_t>> ku;
        for (auto& k : kr) {
            if (!ku.empty() && k.first <= ku.back().second + 1) ku.back().second = std::max(ku.back().second, k.second);
            else ku.push_back(k);
        }
        for (auto& k : ku) {
            uint64_t ub = 0, ue = 0;
            int rc = engine_key_range(s->eng, (int32_t)k.first, (int32_t)k.second, &ub, &ue);
            if (rc) return rc;
            if (ue <= ub) continue;
            std::vector<uint64_t> cand(ue - ub);
            for (uint64_t i = 0; i < cand.size(); ++i) cand[i] = ub + i;
            std::vector<double> cm(cand.size());
            if ((rc = dbi_peptides(s->eng, cand.data(), cand.size(), cm.data(), nullptr, nullptr, nullptr, nullptr,
                                   nullptr)))
                return rc;
            int32_t row_key = 0;
            bool skip_row = false;
            for (uint64_t i = 0; i < cand.size(); ++i) {
                const double m = cm[i];
                if (java_d2i(m) / br != b) continue;  // row lives in another bucket
                const int32_t key = java_d2i(m * f);
                if (i == 0 || key != row_key) {
                    row_key = key;
                    skip_row = false;
                }
                if (skip_row) continue;
                // parseAddPeptideInfo(data, ret, minMasses, maxMasses) (IndexMerge:494-600)
                bool greaterThanMax = true, qualifies = false;
                for (auto& r : ranges) {
                    if (m < r.second) greaterThanMax = false;
                    if (m >= r.first && m <= r.second) qualifies = true;
                    if (qualifies) break;
                }
                if (greaterThanMax && !qualifies) {
                    skip_row = true;
                    continue;
                }
                if (!qualifies) continue;
                ids.push_back(cand[i]);
            }
        }
    }
    int rc = materialise(s, ids, lb);
    if (rc) return rc;
    return lb.finish(out);
}

void dbi_seq_list_free(dbi_seq_list* l) {
    if (!l) return;
    std::free(l->mass);
    std::free(l->seq_off);
    std::free(l->seq_chars);
    std::free(l->res_left);
    std::free(l->res_right);
    std::free(l->prot_off);
    std::free(l->prot_ids);
    std::free(l->offset);
    std::free(l->length);
    std::free(l->unique_id);
    std::free(l);
}

int dbi_store_protein_count(dbi_store* s, uint64_t* out) {
    if (!s || !out) return set_error(DBI_E_INVALID, "NULL argument");
    *out = s->defs.size();
    return 0;
}

int dbi_store_protein_def(dbi_store* s, uint64_t id, const char** def, uint64_t* len) {
    if (!s || !def || !len) return set_error(DBI_E_INVALID, "NULL argument");
    if (id >= s->defs.size()) return set_error(DBI_E_INVALID, "protein id out of range");
    *def = s->defs[id].c_str();
    *len = s->defs[id].size();
    return 0;
}

int dbi_store_protein_sequence(dbi_store* s, uint64_t id, const char** seq, uint64_t* len) {
    if (!s || !seq || !len) return set_error(DBI_E_INVALID, "NULL argument");
    if (id >= s->defs.size()) return set_error(DBI_E_INVALID, "protein id out of range");
    *seq = (const char*)s->residues.data() + s->off[id];
    *len = s->off[id + 1] - s->off[id];
    return 0;
}

}  // extern "C"
