/*
 * dbindex_hip.h — C-ABI of the MI355X-native peptide-index engine.
 *
 * This is the drop-in boundary for dbIndex's digestion + index + mass-lookup
 * hot path.  A JNI shim binds these symbols one-for-one to
 * the Java extension points of the reference:
 *
 *   DBIndexStore            /root/reference/src/main/java/edu/scripps/yates/dbindex/DBIndexStore.java:19-194
 *   DBIndexStoreSQLiteMult  (the store the reference builds)   DBIndexStoreSQLiteMult.java:23-637
 *   DBIndexer.cutSeq        (digestion loop, run on device)    DBIndexer.java:237-405
 *
 * Two layers are exported:
 *   - dbi_store_*  : one function per DBIndexStore method (init, startAddSeq,
 *                    addProteinDef, filterSequence, addSequence, stopAddSeq,
 *                    indexExists, getSequences(m,tol), getSequences(List),
 *                    getNumberSequences, getEntryKeys, getProteins, ...).
 *   - dbi_*        : the batch engine underneath (build from a packed residue
 *                    array, batched mass-window queries, peptide gathers),
 *                    usable on host buffers or on buffers already in HBM.
 *
 * Conventions: plain C types only, no torch types.  Every function returns an
 * int status: 0 = OK, negative = error class (DBI_E_*); the message of the
 * last error on the calling thread is in dbi_last_error().  Nothing is
 * swallowed (unlike DBIndexer.cutSeq, DBIndexer.java:398-403).
 * Library-allocated results are freed by the caller with the matching *_free.
 */
#ifndef DBINDEX_HIP_H
#define DBINDEX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DBI_OK 0
#define DBI_E_INVALID (-1) /* invalid argument / unsupported input     */
#define DBI_E_OOM (-2)     /* host or device allocation failed          */
#define DBI_E_HIP (-3)     /* HIP runtime error (kernel launch, copy)   */
#define DBI_E_RCCL (-4)    /* collective error (sharded build)          */
#define DBI_E_STATE (-5)   /* call not valid in the current state       */

#define DBI_ABI_VERSION 1

/* DBIndexStore.FilterResult (DBIndexStore.java:22-24) */
#define DBI_FILTER_INCLUDE 0
#define DBI_FILTER_SKIP 1
#define DBI_FILTER_SKIP_PROTEIN_START 2

/*
 * Flat parameter block: the handful of DBIndexSearchParams / AssignMass /
 * Enzyme values the hot loop reads.
 * The Java side fills mass[] from AssignMass.getMass(char) for every char,
 * cleave[] from the Enzyme residues and nocut[] from getEnzymeNocutResidues(),
 * so residue arithmetic and the cleavage sets are identical by construction.
 */
typedef struct dbi_params {
    double min_mh;       /* getMinPrecursorMass()          DBIndexer.java:331        */
    double max_mh;       /* getMaxPrecursorMass()          DBIndexer.java:284,325    */
    double h2o_proton;   /* AssignMass.H2O_PROTON          DBIndexer.java:269        */
    double cterm;        /* AssignMass.getcTerm()          DBIndexer.java:270        */
    double nterm;        /* AssignMass.getnTerm()          DBIndexer.java:271        */
    double mass[256];    /* AssignMass.getMass(char)       DBIndexer.java:306        */
    uint8_t cleave[256]; /* Enzyme.isEnzyme(char)          DBIndexer.java:314        */
    uint8_t nocut[256];  /* getEnzymeNocutResidues()       DBIndexer.java:318-319    */
    uint8_t mandatory[256]; /* getMandatoryInternalAAs()   DBIndexer.java:334-344    */
    int32_t max_missed;        /* getMaxMissedCleavages()  DBIndexer.java:246,322    */
    int32_t semi;              /* isSemiCleavage()  (Enzyme semi flag)               */
    int32_t add_h2o_proton;    /* isH2OPlusProtonAdded()   DBIndexer.java:268        */
    int32_t min_len;           /* Constants.MIN_PEP_LENGTH = 6   Constants.java:10    */
    int32_t mass_group_factor; /* getMassGroupFactor() = 10000  DBIndexStoreSQLiteByte.java:187 */
    int32_t index_factor;      /* getIndexFactor() = NUM_BUCKETS  DBIndexStoreSQLiteMult.java:55 */
    int32_t mandatory_mode;    /* 0: getMandatoryInternalAAs()==null, 1: non-null    */
    int32_t mandatory_count;   /* its length (filterSequence tests length>0)         */
    int32_t reserved[8];
} dbi_params;

/* Fills *p with the reference defaults (dbindex.properties:6-22 + Constants):
 * trypsin "KR", empty nocut, mc=max_missed, 500..6000 Da, H2O+H+ added,
 * factor 10000, index_factor 8, min length 6, pinned monoisotopic table. */
void dbi_params_default(dbi_params* p, int32_t max_missed, int32_t semi);

/* ------------------------------------------------------------------------ */
/* Batch engine                                                             */
/* ------------------------------------------------------------------------ */
typedef struct dbi_handle dbi_handle;

typedef struct dbi_stats {
    uint64_t n_residues;     /* R                                                  */
    uint64_t n_proteins;     /* P                                                  */
    uint64_t n_total;        /* N: occurrences passing all filters = totalSeqCount */
                             /*    (DBIndexStoreSQLiteMult.java:277)               */
    uint64_t n_dropped;      /* of N, bucket > NUM_BUCKETS-1 (SQLiteMult:283-288)  */
    uint64_t n_kept;         /* N - n_dropped: occurrences stored in the index     */
    uint64_t n_unique;       /* U: unique peptide sequences (IndexMerge:620-719)   */
    uint64_t n_keys;         /* distinct mass-key rows = getNumberSequences()      */
    uint64_t n_bins;         /* device mass bins used by the build                 */
    uint64_t n_big_bins;     /* bins sorted by the large-bin path                  */
    uint64_t device_bytes;   /* HBM held by the index + workspace                  */
    double build_ms;         /* device time of the last build (HIP events)         */
    double digest_ms;        /* of which: digest count + emit kernels              */
} dbi_stats;

/* Opens an engine on HIP device `device` (ordinal as seen by this process). */
int dbi_open(const dbi_params* params, int device, dbi_handle** out);
void dbi_close(dbi_handle* h);

/* Build the index from a packed FASTA: residues[0..n_res) = all protein
 * sequences concatenated in FASTA order, prot_off[0..n_prot] = start offsets
 * (prot_off[0]=0, prot_off[n_prot]=n_res).  Protein id = 0-based position
 * (DBIndexer.java:251,418 + DBIndexStoreSQLiteMult.addProteinDef:446-450).
 * Proteins may carry inline '[formula]' PTMs, digested as DBIndexer.cutSeq
 * does (:288-303; offsets of the stripped protein, identity and text from the
 * protein as given); a formula before a protein's first residue or a '['
 * without ']' is DBI_E_INVALID (the reference throws out of cutSeq).
 * Host pointers; copied to HBM.  Replaces any previous index of the handle. */
int dbi_build(dbi_handle* h, const uint8_t* residues, uint64_t n_res,
              const uint64_t* prot_off, uint64_t n_prot);

/* Same, with residues / offsets already resident in HBM (device pointers),
 * work ordered on `stream` (a hipStream_t, NULL = default stream). */
int dbi_build_device(dbi_handle* h, const uint8_t* d_residues, uint64_t n_res,
                     const uint64_t* d_prot_off, uint64_t n_prot, void* stream);

/* Build from externally supplied occurrences (DBIndexStore.addSequence path):
 * mass / protein id / offset-in-protein / length per occurrence, in insertion
 * order, over the protein residues given as above.  Dedup + sort + query are
 * identical to the device-digest build. */
int dbi_build_occurrences(dbi_handle* h, const uint8_t* residues, uint64_t n_res,
                          const uint64_t* prot_off, uint64_t n_prot,
                          const double* mass, const uint32_t* prot_id,
                          const uint32_t* offset, const uint32_t* length,
                          uint64_t n_occ, uint64_t n_dropped_extra);

int dbi_stats_get(dbi_handle* h, dbi_stats* out);

/* Bucket switch (default on = the SQLite store: peptides with bucket >
 * NUM_BUCKETS-1 are dropped, DBIndexStoreSQLiteMult.java:282-288, and queries
 * reaching such a bucket are empty).  Off = MassRangeFilteringIndex semantics
 * (SEARCH_UNINDEXED): every peptide is kept and queries are plain
 * minMass <= m <= maxMass windows (MassRangeFilteringIndex.java:90-108).
 * Clears the built index. */
int dbi_set_bucket_drop(dbi_handle* h, int on);

/* Mass-window filter for the next builds (needs the bucket drop off): with
 * on = 1 a build keeps only the peptides with m - tol <= mass <= m + tol for
 * some i (MassRangeFilteringIndex.filterSequence, :90-108; a NaN bound
 * includes nothing, n = 0 includes nothing) and ends a start's walk once its
 * mass passes every window (SKIP_PROTEIN_START, DBIndexer.java:351-354): the
 * SEARCH_UNINDEXED cut-and-search without a resident full index.  on = 0
 * removes the filter.  Clears the built index. */
int dbi_set_windows(dbi_handle* h, const double* mass, const double* tol, uint64_t n, int on);

/* Build again over the inputs of the last dbi_build (still resident in HBM),
 * under the current windows / bucket setting. */
int dbi_rebuild(dbi_handle* h);

/* Threading: a build (dbi_build*, dbi_rebuild, dbi_count,
 * dbi_index_load, the dbi_shard_* phases) is exclusive per handle.  Query-side
 * calls (dbi_query*, dbi_peptides, dbi_occurrences, dbi_export,
 * dbi_entry_keys) may come from several threads at once: they serialise on
 * the handle's scratch buffers; dbi_query_device on caller buffers and its
 * own stream only for the one-off query directory. */

/* Batched single-range mass-window queries, getSequences(m, tol) semantics
 * (DBIndexStoreSQLiteMult.java:315-350 + IndexMerge.java:146-217,386-481):
 * for query i, the unique peptides with lo<=mass<=hi, lo=max(0,m-tol),
 * hi=m+tol, empty when a bucket of lo or hi exceeds NUM_BUCKETS-1.
 * Results are contiguous in the mass-sorted unique table: ids
 * first[i] .. first[i]+count[i]-1, ascending mass.  Host arrays. */
int dbi_query(dbi_handle* h, const double* mass, const double* tol, uint64_t nq,
              uint64_t* first, uint64_t* count);

/* Same on device arrays (stream = hipStream_t or NULL). */
int dbi_query_device(dbi_handle* h, const double* d_mass, const double* d_tol, uint64_t nq,
                     uint64_t* d_first, uint64_t* d_count, void* stream);

/* Materialised CSR form of a query batch: row_ptr[nq+1] and ids[] (H ids). */
typedef struct dbi_query_result {
    uint64_t nq;
    uint64_t n_hits;
    uint64_t* row_ptr; /* nq+1 */
    uint64_t* ids;     /* n_hits, unique-peptide ids */
} dbi_query_result;
int dbi_query_csr(dbi_handle* h, const double* mass, const double* tol, uint64_t nq,
                  dbi_query_result** out);
void dbi_query_result_free(dbi_query_result* r);

/* Builds the query directory of the current index now (otherwise the first
 * query after a build or load does); lets a caller time or overlap it. */
int dbi_query_prepare(dbi_handle* h);

/* Materialised hits of a query batch, all in HBM (getSequences(m, tol) per
 * query, DBIndexStoreSQLiteMult.java:315-350: every peptide with its protein
 * ids, IndexMerge.parseAddPeptideInfo :386-481).  Hits of query i:
 * ids[row[i] .. row[i+1]) (unique-peptide ids, ascending mass).  Protein ids
 * of those hits: prot[occ_row[i] .. occ_row[i+1]), hit h's own list starting
 * at prot[occ_row[i] + hit_occ[h]] and ending where the next hit's (or the
 * query's) starts (insertion order, duplicates kept, IndexMerge.java:676-681).
 * The buffers belong to the handle and stay valid until its next query-side
 * call or build; the call returns once they are complete. */
typedef struct dbi_device_hits {
    const uint64_t* row;      /* nq + 1 */
    const uint32_t* ids;      /* n_hits */
    const uint64_t* occ_row;  /* nq + 1 */
    const uint32_t* hit_occ;  /* n_hits */
    const uint32_t* prot;     /* n_prot_ids */
    uint64_t nq;
    uint64_t n_hits;
    uint64_t n_prot_ids;
} dbi_device_hits;
int dbi_query_hits_device(dbi_handle* h, const double* d_mass, const double* d_tol, uint64_t nq,
                          dbi_device_hits* out);

/* Gather per-unique-peptide data for ids[0..n): mass, representative
 * (first-occurrence) protein id + offset + length (IndexMerge.java:671-675),
 * and the occurrence range [occ_begin, occ_end) into dbi_occurrences().
 * Any output pointer may be NULL. */
int dbi_peptides(dbi_handle* h, const uint64_t* ids, uint64_t n, double* mass,
                 uint32_t* prot_id, uint32_t* offset, uint32_t* length,
                 uint64_t* occ_begin, uint64_t* occ_end);

/* Protein ids of occurrences [begin, end) (insertion order, duplicates kept,
 * IndexMerge.java:676-681). */
int dbi_occurrences(dbi_handle* h, uint64_t begin, uint64_t end, uint32_t* prot_id);

/* Copy the whole index to host (any pointer may be NULL):
 * mass[U], prot_id[U], offset[U], length[U], occ_off[U+1], occ_prot[n_kept]. */
int dbi_export(dbi_handle* h, double* mass, uint32_t* prot_id, uint32_t* offset,
               uint32_t* length, uint64_t* occ_off, uint32_t* occ_prot);

/* Distinct mass keys (int)(mass*factor), ascending = getEntryKeys()
 * (DBIndexStoreSQLiteByte.java:693-716 summed over buckets).  keys may be
 * NULL to query the count only. */
int dbi_entry_keys(dbi_handle* h, int32_t* keys, uint64_t cap, uint64_t* n);

/* Device pointers of the resident index (for in-HBM consumers / bench).
 * d_mass[U] f64 ascending; others as dbi_export. */
typedef struct dbi_device_index {
    const double* mass;
    const uint32_t* prot_id;
    const uint32_t* offset;
    const uint32_t* length;
    const uint32_t* occ_off;   /* U+1 */
    const uint32_t* occ_prot;  /* n_kept */
    uint64_t n_unique;
    uint64_t n_kept;
} dbi_device_index;
int dbi_device_view(dbi_handle* h, dbi_device_index* out);

/* Per-kernel device times of the last build.  With timing on (the default)
 * every launch carries HIP start/stop events in its own dispatch packet
 * (hipExtLaunchKernelGGL on the engine stream), so timing inserts no marker
 * packets and no idle gaps between kernels.  names[i] are static strings
 * ("digest_slots", "digest", "radix_scatter", "chunk_sort", ...);
 * ms[i] = 0 for a stage that launched nothing or with timing off;
 * bytes[i] = algorithmic HBM bytes of that launch.
 * Arrays may be NULL to query *n. */
/* Tuning switches and test hooks of one handle -- experiments and the test
 * suite; the defaults are the measured best, and nothing is read from the
 * environment.  Integer options: "build_graph", "digest_hist",
 * "semi_bounded", "depth_bins", "semi_part" (0 / 1: the warm build's hipGraph,
 * the digest-counted first radix histogram of small tails, the bounded
 * semi-specific digest, depth bins, the semi-specific digest partitioning by
 * the first radix digit); "depth_map_reuse" (1: the depth-bin map
 * is sampled again only when the resident index changes size, 0: every
 * build); "big_split" (-1: by the list length, 0,
 * 1: the big chunk tier's two size classes); "bin_bits_max", "split_above",
 * "chunk_target" (0: by size); "shard_full_path", "shard_dev_digest",
 * "shard_resample" (0 / 1, dbi_build_sharded); "owner_depth" (0 / 1: warm
 * owner merges on depth bins, else the radix tail); "big_side" (0 / 1: a
 * depth-bin tail's big chunk tier on a second stream beside the chunk sort); "part_stage" (0 / 1: the
 * partitioning digest keeps a tile's records in LDS, 1, or writes them
 * through HBM slots, 0).  Test-build library only
 * (libdbindex_hip_hooks.so, -DDBI_TEST_HOOKS; the product library answers
 * DBI_E_INVALID): "test_split_skew" (a rank, -1 off: that rank's reused owner
 * split is skewed) and string option "test_fail" = "<phase>@<rank>" (or ""):
 * an injected local failure of a sharded build or query.  DBI_E_INVALID for
 * an unknown name or value. */
int dbi_set_option(dbi_handle* h, const char* name, int64_t value);
int dbi_set_option_str(dbi_handle* h, const char* name, const char* value);

/* The next build starts cold, as the one-off build of DBIndexer.run
 * (DBIndexer.java:508-684) does: no capacity, chunk-list grids, depth-bin map
 * or build graph carried over from earlier builds (the bounded digest's slot
 * count then its pass -- count + emit for the other digests -- and the radix
 * tail), but the device buffers are kept -- the cold pipeline timed
 * without its allocations (bench.py cold_ms). */
int dbi_set_cold(dbi_handle* h);

/* on = 0: no events (wall clock only); on = 1: time every stage, or only the
 * stages named `only` (NULL or "" = all) — each timed stage costs a few us. */
int dbi_set_timing(dbi_handle* h, int on, const char* only);
int dbi_stage_times(dbi_handle* h, const char** names, double* ms, double* bytes, uint64_t cap,
                    uint64_t* n);

/* ------------------------------------------------------------------------ */
/* Sharded build: one index over the proteins of every shard (GPU)           */
/* ------------------------------------------------------------------------ */
/*
 * The proteome is split into contiguous protein ranges, one per shard (one
 * shard per GPU, one process per GPU).  Every shard digests its own proteins
 * (DBIndexer.cutSeq, DBIndexer.java:237-405); the records are then routed to
 * the shard that OWNS their mass key (int)(mass*factor) — owners hold
 * contiguous key ranges chosen from a sample of every shard's masses — and each
 * owner sorts, de-duplicates across shards and finalises its key range
 * (IndexMerge.getMergedData, DBIndexStoreSQLiteByteIndexMerge.java:620-719).
 * The owners' unique tables, concatenated in shard order, ARE the index of the
 * whole proteome: identical, row for row, to a single-device build.  Protein
 * ids are global (FASTA order, DBIndexer.java:251,418).
 *
 * Every shard must hold the residues and offsets of the WHOLE proteome in HBM
 * (the owner merge compares peptide strings of any shard); dbi_comm_allgatherv
 * assembles them from per-shard pieces.
 *
 * Phases (each call is per handle; dbi_build_sharded runs them all over RCCL):
 *   dbi_shard_digest     digest proteins [p_begin, p_end) of the global arrays
 *   dbi_shard_samples    DBI_SHARD_SAMPLES masses of this shard's records + weight
 *   dbi_shard_splitters  (host only) owner key ranges from every shard's samples
 *   dbi_shard_partition  route records by owner; per-owner send counts
 *   dbi_shard_exchange_local / RCCL exchange   records to their owners
 *   dbi_shard_merge      owner sort + cross-shard dedup + finalize
 * After the merge the handle answers dbi_query / dbi_peptides / dbi_export for
 * its own key range (ids are local to the owner's table).
 */
#define DBI_SHARD_SAMPLES 4096
typedef struct dbi_comm dbi_comm; /* RCCL communicator, below */
#define DBI_MAX_SHARDS 64

typedef struct dbi_shard_stats {
    int32_t rank, nshards;
    uint64_t p_begin, p_end;      /* this shard's proteins (global ids)                   */
    int32_t key_lo, key_hi;       /* owned mass keys [key_lo, key_hi) (INT32_MIN/MAX ends)  */
    uint64_t n_total;             /* this shard's digest: totalSeqCount                    */
    uint64_t n_dropped;           /*   of which bucket drops (not routed)                  */
    uint64_t n_sent;              /*   records routed to other owners                      */
    uint64_t n_received;          /* records this owner merged (from every shard, incl. self) */
    uint64_t n_unique, n_keys;    /* this owner's unique peptides / distinct mass keys     */
    /* whole-index totals (sums over shards; filled by dbi_build_sharded) */
    uint64_t g_total, g_dropped, g_kept, g_unique, g_keys;
    double digest_ms, partition_ms, exchange_ms, merge_ms; /* wall time of each phase      */
    double merge_gpu_ms;          /* device time of this owner's merge kernels             */
    int32_t split_sampled;        /* dbi_build_sharded: 1 = this build gathered samples for its
                                     owner split, 0 = it reused the previous build's split  */
    int32_t split_rounds;         /* count-matrix rounds (2: a rank lacked or disagreed on the
                                     split, every rank sampled and partitioned again)       */
    int32_t split_held;           /* 1 = the next build keeps this build's split: the owners'
                                     merge times were balanced (max <= 1.1 x mean)          */
    int32_t reserved0;
} dbi_shard_stats;

/* Digest proteins [p_begin, p_end) of the global arrays (device pointers:
 * d_residues[n_res], d_prot_off[n_prot+1]) as shard `rank` of `nshards`. */
int dbi_shard_digest(dbi_handle* h, const uint8_t* d_residues, uint64_t n_res, const uint64_t* d_prot_off,
                     uint64_t n_prot, uint64_t p_begin, uint64_t p_end, int rank, int nshards);
/* samples[0..DBI_SHARD_SAMPLES) = masses of evenly spaced records (NaN = no
 * record there), samples[DBI_SHARD_SAMPLES] = records per valid sample. */
int dbi_shard_samples(dbi_handle* h, double* samples);
/* Host only.  samples = nshards blocks of DBI_SHARD_SAMPLES+1 (dbi_shard_samples
 * of every shard, in shard order); split[0..nshards-1) = first key of owners
 * 1..nshards-1 (weighted quantiles: balanced record counts).  Deterministic: every
 * shard computes the same split from the same samples. */
int dbi_shard_splitters(const double* samples, int nshards, int32_t factor, int32_t* split);
/* The same with a cost profile: nbands key bands (band_split[0..nbands-1)
 * their boundaries, ascending) of cost per record band_cost[0..nbands): the
 * splitters balance sum(records x cost of their band) instead of records.
 * band_cost NULL: dbi_shard_splitters. */
int dbi_shard_splitters_cost(const double* samples, int nshards, int32_t factor, int nbands,
                             const int32_t* band_split, const double* band_cost, int32_t* split);
/* The handle's own merge-cost profile (the one dbi_build_sharded keeps): a
 * smoothed cost per record over DBI_COST_BANDS fixed key bands of
 * [minMH, maxMH], updated from one build's owners (their key ranges = split,
 * their merge device time and records); dbi_shard_splitters_profiled then
 * balances that cost.  A profile only steers the splitters: any split gives
 * the same index. */
#define DBI_COST_BANDS 256
int dbi_shard_cost_update(dbi_handle* h, int nshards, const int32_t* split, const double* merge_ms,
                          const uint64_t* records);
int dbi_shard_splitters_profiled(dbi_handle* h, const double* samples, int nshards, int32_t* split);
/* Route this shard's records by owner (stable; global protein ids);
 * send_count[0..nshards) = records for each owner. */
int dbi_shard_partition(dbi_handle* h, const int32_t* split, uint64_t* send_count);
/* Single-process exchange between the handles of all shards (same device or
 * peer-accessible devices): hs[i] = shard i. */
int dbi_shard_exchange_local(dbi_handle* const* hs, int nshards);
/* Owner merge of the received records: the index of this owner's key range. */
int dbi_shard_merge(dbi_handle* h);
int dbi_shard_stats_get(dbi_handle* h, dbi_shard_stats* out);

/* Mass-window queries against a sharded index, getSequences(m, tol) semantics
 * (DBIndexStoreSQLiteMult.java:315-350): each rank passes its own batch
 * (device arrays); every window goes to the owners whose key range it meets,
 * is answered there, and comes back as ids first..first+count-1 of the WHOLE
 * index (the owners' unique tables concatenated in shard order). */
int dbi_query_sharded(dbi_handle* h, dbi_comm* c, const double* d_mass, const double* d_tol, uint64_t nq,
                      uint64_t* d_first, uint64_t* d_count);
/* Replicated index — BASELINE.json north_star's all-gatherv of the sorted
 * mass index over xGMI: after a sharded build (phase 4 on every rank), every
 * rank receives every owner's unique table and occurrence CSR (one group of
 * point-to-point transfers over all peers).  The handle then holds the index
 * of the whole proteome, identical to a single-device build, and answers every
 * query locally (dbi_query*, dbi_query_hits_device, dbi_export, dbi_peptides,
 * dbi_entry_keys) with no exchange per batch; routed queries
 * (dbi_query_sharded) no longer apply.  At most 2^32-2 occurrences per device.
 * Collective: every rank calls it.  _local: the shards' handles of one
 * process, by device copies (tests). */
int dbi_shard_replicate(dbi_handle* h, dbi_comm* c);
int dbi_shard_replicate_local(dbi_handle* const* hs, int nshards);

/* The same over the handles of one process: shard i's batch is
 * (d_mass[i], d_tol[i], nq[i]) with results in (d_first[i], d_count[i]). */
int dbi_query_sharded_local(dbi_handle* const* hs, int nshards, const double* const* d_mass,
                            const double* const* d_tol, const uint64_t* nq, uint64_t* const* d_first,
                            uint64_t* const* d_count);

/* RCCL communicator (one rank per GPU, xGMI).  The 128-byte id comes from
 * rank 0's dbi_comm_unique_id and is passed to every rank out of band. */
int dbi_comm_unique_id(uint8_t* id128);
int dbi_comm_init(const uint8_t* id128, int nranks, int rank, int device, dbi_comm** out);
/* TESTS ONLY: the same communicator over a host-staged transport -- POSIX
 * shared memory `name` ("/..."; rank 0 creates it, the others attach) between
 * the processes of one node, device -> host -> shared memory -> host ->
 * device with a barrier between, slot_bytes per rank slot and per (source,
 * destination) mailbox -- so that N processes on ONE GPU run the N-rank
 * driver (RCCL refuses two ranks on one device).  Every product run is RCCL. */
int dbi_comm_init_host(const char* name, int nranks, int rank, int device, uint64_t slot_bytes, dbi_comm** out);
void dbi_comm_destroy(dbi_comm* c);
/* d_recv = concatenation over ranks of rank_bytes[r] bytes; this rank's piece
 * (rank_bytes[rank] bytes at d_send) lands at its offset (d_send may be that
 * spot).  Point-to-point sends/receives grouped over all peers. */
int dbi_comm_allgatherv(dbi_comm* c, const void* d_send, void* d_recv, const uint64_t* rank_bytes, void* stream);
/* Small host-buffer all-reduce over RCCL (bench / driver coordination: the
 * barrier, max-over-ranks times, summed counts): out[i] = op over ranks of
 * in[i], n <= 4096, op DBI_OP_SUM / DBI_OP_MAX / DBI_OP_MIN.  Blocking; a
 * call with n = 0 is a barrier.  in may alias out. */
#define DBI_OP_SUM 0
#define DBI_OP_MAX 1
#define DBI_OP_MIN 2
int dbi_comm_allreduce_f64(dbi_comm* c, const double* in, double* out, uint32_t n, int op);
/* Device-buffer sum all-reduce of n u64 values (a count histogram), in place
 * allowed; stream NULL = the communicator's own stream (blocking). */
int dbi_comm_allreduce_u64(dbi_comm* c, const uint64_t* d_in, uint64_t* d_out, uint64_t n, void* stream);
/* All phases over RCCL: digest, sample all-gather, splitters, partition,
 * count all-gather, grouped send/recv exchange, owner merge, totals all-reduce. */
int dbi_build_sharded(dbi_handle* h, dbi_comm* c, const uint8_t* d_residues, uint64_t n_res,
                      const uint64_t* d_prot_off, uint64_t n_prot, uint64_t p_begin, uint64_t p_end);

/* ------------------------------------------------------------------------ */
/* Count-only streaming (proteomes too large to index: TrEMBL scale)         */
/* ------------------------------------------------------------------------ */
/* Seeded synthetic proteome generated on the device: protein p has length
 * len_table[fmix64(seed*G + p + 1) >> 52] (4096 entries), the residue at
 * global residue index g is res_table[fmix64((seed ^ S)*G + g) >> 48] (65536
 * entries), G = 0x9E3779B97F4A7C15, S = 0xD1B54A32D192ED03, fmix64 = the
 * MurmurHash3 finaliser.  Writes proteins [p_begin, p_begin+n_prot), whose
 * first residue has global index res_base, into buffers owned by the handle
 * (valid until the next call on it): *d_residues[*n_res], *d_prot_off[n_prot+1]
 * (offsets from 0).  dbindex_amd/fasta.py holds the numpy twin. */
int dbi_synth_proteome(dbi_handle* h, uint64_t seed, uint64_t p_begin, uint64_t n_prot, uint64_t res_base,
                       const uint16_t* len_table, const uint8_t* res_table, const uint8_t** d_residues,
                       const uint64_t** d_prot_off, uint64_t* n_res);
/* Digest proteins in COUNT mode (device pointers, < 2^32 residues): the
 * cutSeq loop (DBIndexer.java:237-405) without records.  *n_total =
 * totalSeqCount (DBIndexStoreSQLiteMult.java:277), *n_dropped = its bucket
 * drops.  Builds no index (the handle's index, if any, is discarded). */
int dbi_count(dbi_handle* h, const uint8_t* d_residues, uint64_t n_res, const uint64_t* d_prot_off,
              uint64_t n_prot, uint64_t* n_total, uint64_t* n_dropped);
/* dbi_count, and the occurrences per SQLiteMult bucket (getBucketForMass,
 * DBIndexStoreSQLiteMult.java:215-217: (int)m / BUCKET_MASS_RANGE, the store
 * each one goes to, :277-288): d_bucket_counts[b] += those of bucket b <
 * NUM_BUCKETS, d_bucket_counts[NUM_BUCKETS] += those past the last bucket
 * (the drops of :283-288).  d_bucket_counts: device array of index_factor + 1
 * u64 (index_factor <= 64) on the handle's device, accumulated (+=) so
 * chunks of one proteome add up; dbi_comm_allreduce_u64 sums it over ranks. */
int dbi_count_buckets(dbi_handle* h, const uint8_t* d_residues, uint64_t n_res, const uint64_t* d_prot_off,
                      uint64_t n_prot, uint64_t* d_bucket_counts, uint64_t* n_total, uint64_t* n_dropped);

/* ------------------------------------------------------------------------ */
/* Persisted index (the reference's SQLite index files + indexExists reuse)  */
/* ------------------------------------------------------------------------ */
/* One binary file: the proteome the index refers to + the unique table and
 * occurrence CSR; the header fingerprints every build parameter (the role of
 * the params md5 in the reference's file name, IndexUtil.java:270-324), and a
 * file is only loaded under the same parameters. */
int dbi_index_save(dbi_handle* h, const char* path);
int dbi_index_load(dbi_handle* h, const char* path);  /* replaces the handle's index */
/* *out = 1 when `path` holds an index built with exactly these parameters (host only) */
int dbi_index_file_matches(const dbi_params* params, const char* path, int* out);

/* ------------------------------------------------------------------------ */
/* DBIndexStore mirror                                                      */
/* ------------------------------------------------------------------------ */
typedef struct dbi_store dbi_store;

/* new DBIndexStoreSQLiteMult(sparam, inMemory) (DBIndexStoreSQLiteMult.java:47-64) */
int dbi_store_create(const dbi_params* params, int device, dbi_store** out);
void dbi_store_close(dbi_store* s);

/* Device digestion switch (the DBIndexerHip hook): when on, stopAddSeq runs
 * the cutSeq loop on the GPU over every protein given to addProteinDef, and
 * filterSequence answers SKIP_PROTEIN_START so a stock DBIndexer.cutSeq bails
 * out of every start (DBIndexer.java:351-354).  When off (default), the store
 * indexes exactly the occurrences passed to addSequence, like the reference. */
int dbi_store_set_device_digest(dbi_store* s, int on);

/* Persistence switch (default off): when on, init(database_id) loads
 * `<database_id>.dbihip` if it holds an index built with the store's
 * parameters (then indexExists() is true and DBIndexer.run skips indexing,
 * DBIndexer.java:522-527), and stopAddSeq() writes it (index + ProteinCache). */
int dbi_store_set_persist(dbi_store* s, int on);

/* SEARCH_UNINDEXED switch (before init; default 0 = off): the store becomes the
 * MassRangeFilteringIndex (DBIndexer.java:175-200, MassRangeFilteringIndex.java):
 * device digestion over the ProteinCache (addProteinDef) without buckets and
 * without the SQLite store's mandatory-residue filter; getSequences and
 * cutAndSearch return every peptide with a mass in any [m - tol, m + tol],
 * one entry per sequence (first occurrence), protein ids without repeats;
 * indexExists() is false, getNumberSequences() is the last result's size,
 * getEntryKeys() is not supported.  Needs non-negative residue masses and a
 * max precursor mass < 65536 Da. */
int dbi_store_set_unindexed(dbi_store* s, int mode);
#define DBI_UNINDEXED_RESIDENT 1 /* one device index of every peptide; searches are windows over it  */
#define DBI_UNINDEXED_STREAM   2 /* proteins resident; every search re-digests them through its       */
                                 /* ranges (dbi_set_windows): memory for the matches only, for        */
                                 /* proteomes/enzymes whose full index does not fit in HBM            */

int dbi_store_init(dbi_store* s, const char* database_id);              /* init(String)      */
int dbi_store_start_add_seq(dbi_store* s);                              /* startAddSeq()     */
int dbi_store_stop_add_seq(dbi_store* s);                               /* stopAddSeq()      */
int dbi_store_index_exists(dbi_store* s, int* out);                     /* indexExists()     */
/* addProteinDef(long num, String def, String seq): returns num (SQLiteMult:446-450) */
int dbi_store_add_protein_def(dbi_store* s, int64_t num, const char* def, const char* seq,
                              uint64_t seq_len, int64_t* out_id);
/* filterSequence(double, String) (DBIndexStoreSQLiteMult.java:245-268) */
int dbi_store_filter_sequence(dbi_store* s, double mass, const char* seq, uint64_t seq_len,
                              int* out_result);
/* addSequence(double, int, int, String, String, String, long) (SQLiteMult:271-291) */
int dbi_store_add_sequence(dbi_store* s, double mass, int32_t offset, int32_t length,
                           int64_t protein_id);
int dbi_store_get_number_sequences(dbi_store* s, int64_t* out);         /* getNumberSequences */
int dbi_store_get_total_seq_count(dbi_store* s, int64_t* out);          /* totalSeqCount      */
int dbi_store_get_entry_keys(dbi_store* s, int32_t* keys, uint64_t cap, uint64_t* n);
dbi_handle* dbi_store_engine(dbi_store* s);                             /* batch engine view  */

/* A materialised List<IndexedSequence> (IndexMerge.parseAddPeptideInfo:386-481). */
typedef struct dbi_seq_list {
    uint64_t n;
    double* mass;          /* n                                              */
    uint64_t* seq_off;     /* n+1: sequence i = seq_chars[seq_off[i]..seq_off[i+1]) */
    char* seq_chars;
    char* res_left;        /* n*3: Util.getResidues left flank (Util.java:130-162)  */
    char* res_right;       /* n*3: right flank, '-' padded                   */
    uint64_t* prot_off;    /* n+1: protein ids of i = prot_ids[prot_off[i]..)       */
    uint32_t* prot_ids;
    uint32_t* offset;      /* n: representative offset  (IndexedSequence offset)    */
    uint32_t* length;      /* n                                              */
    uint64_t* unique_id;   /* n: id in the mass-sorted unique table          */
} dbi_seq_list;

/* getSequences(double precMass, double tolerance) */
int dbi_store_get_sequences(dbi_store* s, double mass, double tol, dbi_seq_list** out);
/* getSequences(List<MassRange>) (DBIndexStoreSQLiteMult.java:353-430) */
int dbi_store_get_sequences_ranges(dbi_store* s, const double* mass, const double* tol,
                                   uint64_t n_ranges, dbi_seq_list** out);
/* DBIndexer.cutAndSearch(List<MassRange>) (DBIndexer.java:707-747) over the
 * unindexed store: ranges minMass = m - tol, maxMass = m + tol; results in
 * ascending mass (the reference returns THashMap order, i.e. unspecified). */
int dbi_store_cut_and_search(dbi_store* s, const double* mass, const double* tol,
                             uint64_t n_ranges, dbi_seq_list** out);
void dbi_seq_list_free(dbi_seq_list* l);

/* ProteinCache accessors (ProteinCache.java:60-127) */
int dbi_store_protein_count(dbi_store* s, uint64_t* out);
int dbi_store_protein_def(dbi_store* s, uint64_t id, const char** def, uint64_t* len);
int dbi_store_protein_sequence(dbi_store* s, uint64_t id, const char** seq, uint64_t* len);

/* ------------------------------------------------------------------------ */
/* FASTA parsing (host, multi-threaded): the packed layout the builds read   */
/* ------------------------------------------------------------------------ */
/* Records start at a '>' at a line start (DBIndexer.run / FastaReader,
 * DBIndexer.java:546-616); definition = the rest of that line without
 * trailing CR/LF; sequence = the following lines with ASCII whitespace
 * removed; text before the first record is ignored.  Protein id = position
 * (ProteinCache.addProtein, ProteinCache.java:84-95). */
typedef struct dbi_fasta {
    uint64_t n_proteins;
    uint64_t n_residues;
    uint8_t* residues;  /* n_residues (+16 zero bytes of padding)              */
    uint64_t* offsets;  /* n_proteins + 1                                      */
    char* defs;         /* definitions, concatenated                           */
    uint64_t* def_off;  /* n_proteins + 1: definition i = defs[def_off[i]..)  */
    uint64_t n_uniprot; /* definitions with a UniProt accession (sp|ACC|/tr|ACC|):
                           DBIndexer.run rejects a FASTA with none (:560-565) */
} dbi_fasta;
/* threads <= 0: one per hardware thread.  Free with dbi_fasta_free. */
int dbi_fasta_parse(const char* buf, uint64_t len, int threads, dbi_fasta** out);
int dbi_fasta_read(const char* path, int threads, dbi_fasta** out);
void dbi_fasta_free(dbi_fasta* f);

/* The one-off build from a FASTA file (DBIndexer.run, DBIndexer.java:546-616)
 * in one call: dbi_fasta_read, then dbi_build of its output (whose 2-MiB-page
 * residue buffer is pinned and DMA'd to HBM without a staging copy).  *out
 * (optional; free with dbi_fasta_free) gets the parsed file -- definitions
 * and offsets for the ProteinCache.  (Streaming each parse thread's residues
 * to HBM during the parse measured slower: DESIGN.md §7.) */
int dbi_build_fasta(dbi_handle* h, const char* path, int threads, dbi_fasta** out);

/* ------------------------------------------------------------------------ */
/* Device memory helpers (so host code needs no other HIP runtime binding)  */
/* ------------------------------------------------------------------------ */
int dbi_dev_alloc(int device, uint64_t bytes, void** out);
int dbi_dev_free(int device, void* p);
int dbi_dev_copy_h2d(int device, void* dst, const void* src, uint64_t bytes);
int dbi_dev_copy_d2h(int device, void* dst, const void* src, uint64_t bytes);
int dbi_dev_copy_d2d(int device, void* dst, const void* src, uint64_t bytes);
int dbi_dev_synchronize(int device);
/* STREAM-like device copy of `bytes` (read + write counted: 2 x bytes per
   pass), `reps` timed passes on a stream of its own: the measured HBM ceiling
   the bench prints next to the 8 TB/s peak. */
int dbi_hbm_copy_bandwidth(int device, uint64_t bytes, int reps, double* gbps);

/* ------------------------------------------------------------------------ */
/* Misc                                                                     */
/* ------------------------------------------------------------------------ */
const char* dbi_last_error(void); /* thread-local; "" when no error */
int dbi_abi_version(void);
/* The HIP runtime and RCCL this library is bound to in this process: versions
 * and the shared objects that provide hipMalloc / ncclGetVersion (dladdr), so
 * a caller can check that one HIP runtime and one RCCL are in play. */
typedef struct dbi_runtime_info {
    int hip_runtime_version;  /* hipRuntimeGetVersion */
    int hip_driver_version;   /* hipDriverGetVersion */
    int rccl_version;         /* ncclGetVersion: major*10000 + minor*100 + patch */
    char libamdhip64[512];
    char librccl[512];
} dbi_runtime_info;
int dbi_runtime_info_get(dbi_runtime_info* out);
int dbi_device_count(int* out);

#ifdef __cplusplus
}
#endif
#endif /* DBINDEX_HIP_H */
