// dbi_engine.h — the engine handle and the build phases shared by the
// single-device build (dbi_engine.hip) and the sharded build (dbi_shard.hip).
// Internal: not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dbi_internal.h"

namespace dbi {

// Bumped by every device (re)allocation: a captured build graph holds buffer
// pointers, so it is replayed only while this has not moved.
inline std::atomic<uint64_t> g_alloc_gen{0};

// Growable device buffer.
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;  // elements
    int ensure(size_t n) {
        if (n <= cap && p) return 0;
        g_alloc_gen.fetch_add(1, std::memory_order_relaxed);
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1);
        hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            return hip_fail(e, "hipMalloc");
        }
        cap = want;
        return 0;
    }
    // look-back status words: a fresh allocation may hold words of an earlier
    // (freed) status array whose epoch tags match; start from zero
    int ensure_zeroed(size_t n, hipStream_t s) {
        if (n <= cap && p) return 0;
        int rc = ensure(n);
        if (rc) return rc;
        const hipError_t e = hipMemsetAsync(p, 0, cap * sizeof(T), s);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    void release() {  // (a freed pointer in a captured graph: the graph is stale too)
        if (p) {
            g_alloc_gen.fetch_add(1, std::memory_order_relaxed);
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    size_t bytes() const { return cap * sizeof(T); }
};

// Owner-splitter samples of a sharded build, sorted by mass key (dbi_shard.hip)
struct SampleKeys {
    std::vector<int32_t> key;
    std::vector<double> w;  // records per sample of the shard it came from
};

// State of a sharded build on this handle (dbi_shard_* phases, dbi_shard.hip).
struct ShardState {
    int phase = 0;  // 0 none, 1 digested, 2 partitioned, 3 exchanged, 4 merged, 5 replicated
    int rank = 0, nshards = 1;
    uint64_t p_begin = 0, p_end = 0;        // this shard's proteins (global ids)
    uint64_t n_res_global = 0, n_prot_global = 0;
    const uint8_t* d_res_global = nullptr;  // every shard's residues (owner merge reads any peptide)
    uint64_t n_digest = 0, n_in = 0;        // digest records / slots in recA
    bool sparse = false;
    bool dev = false;  // device-sized digest: n_digest / n_in are the capacity until the count-matrix sync
    uint64_t n_total = 0, n_dropped = 0;    // this shard's digest: totalSeqCount, bucket drops
    uint32_t width = 0;                     // global record field width W
    int32_t split[MAX_SHARDS - 1] = {};
    std::vector<uint64_t> send_count, send_off;  // per owner, location words in xsend
    uint64_t part_blocks = 0;                    // radix blocks of the owner partition (hist stride)
    std::vector<uint64_t> recv_count;            // per source shard
    uint64_t n_recv = 0;
    double ms_digest = 0, ms_partition = 0, ms_exchange = 0, ms_merge = 0;
    double ms_merge_gpu = 0;                // device time of the owner merge's kernels
    int split_sampled = 0, split_rounds = 0;  // dbi_build_sharded: the owner split's provenance
    bool split_held = false;                // ... and the next build keeps it (balanced owners)
    dbi_shard_stats global{};               // filled by dbi_build_sharded (RCCL sums)
    uint64_t u_base = 0;                    // first global id of this owner's unique table
    bool u_base_known = false;
    // routed query batch (dbi_query_sharded*)
    uint64_t q_n = 0, q_pairs = 0, q_recv = 0;
    std::vector<uint64_t> qsend_count, qsend_off, qrecv_count, qrecv_off;
};

}  // namespace dbi

// the C-ABI handle (include/dbindex_hip.h)
struct dbi_handle {
    template <typename T>
    using DevBuf = dbi::DevBuf<T>;
    using DevParams = dbi::DevParams;
    using Counters = dbi::Counters;
    using Rec = dbi::Rec;

    dbi_params params;
    DevParams dp;
    int device = 0;
    hipStream_t stream = nullptr;
    int bin_bits_max = 24;               // fine mass bins <= 2^bin_bits_max (radix passes of <= 8 bits)
    uint32_t split_above = dbi::BIG_CAP; // chunks above this many records take the MSD split path
    uint32_t chunk_t = 0;                // target records per chunk-sort block (DBI_CHUNK_T; 0: chunk_target())
    bool timing = true;                  // per-stage kernel-attached events (dbi_set_timing)
    std::string timing_only;             // "" = every stage
    std::chrono::steady_clock::time_point t0;

    DevBuf<double> mass_tab;
    DevBuf<uint8_t> flags_tab;
    DevBuf<Counters> ctr;

    // inputs (owned copies for host builds)
    DevBuf<uint8_t> res;
    // host residues -> HBM through a pinned staging ring (upload_inputs):
    // UP_THREADS copy threads, two slots of UP_SLOT bytes each, a copy event per slot
    uint8_t* up_host = nullptr;
    std::vector<hipEvent_t> up_ev;
    DevBuf<uint64_t> poff64;
    DevBuf<uint32_t> poff;
    DevBuf<uint32_t> poff_g;            // sharded build: global u32 offsets (owner merge)
    const uint32_t* d_poff = nullptr;   // offsets the current stage reads (poff or poff_g)
    const uint8_t* d_res = nullptr;  // residues the index refers to
    uint64_t n_res = 0, n_prot = 0;

    // workspace
    DevBuf<uint32_t> blk;       // digest tile counts / offsets
    DevBuf<unsigned long long> status;  // fused digest: per-tile look-back words
    uint32_t epoch = 0;                 // tag of the current fused launch in `status`
    DevBuf<uint32_t> thr;       // digest per-thread counts
    DevBuf<uint32_t> tile_pf;   // first protein of every digest tile (+1)
    DevBuf<uint32_t> scan_tmp;
    DevBuf<Rec> recA, recB;
    DevBuf<uint32_t> hist;
    DevBuf<uint8_t> digits;             // radix: next pass's digit per record
    // inline '[formula]' PTM builds (dbi_build): the digest input (formulas
    // stripped, PTM proteins masked), those proteins stripped, their formula
    // events, and the mass table with the mask residue
    DevBuf<uint8_t> res_dig, ptm_res;
    DevBuf<uint32_t> poff_dig, ptm_soff, ptm_pid, ptm_evoff, ptm_evpos, ptm_cnt;
    DevBuf<double> ptm_evmass, mass_tab_x;
    DevBuf<unsigned long long> ptm_total;
    DevBuf<uint32_t> ucount, big_list, mid_list, giant_list, chunk_lo;
    DevBuf<uint4> segs;                 // giant-chunk split: segment lists
    DevBuf<uint16_t> synth_len;         // dbi_synth_proteome: length quantile table
    DevBuf<uint8_t> synth_res;          //   residue table
    DevBuf<uint8_t> synth_out;          //   generated residues (valid until the next dbi_synth_proteome)
    DevBuf<uint64_t> synth_off;         //   generated offsets
    DevBuf<unsigned long long> ws_key;
    DevBuf<uint32_t> ws_k2;

    // index
    DevBuf<double> umass;
    DevBuf<uint32_t> upid, uoff, ulen, occ_off, occ_pid;
    bool built = false;

    // host-input occurrences (addSequence path)
    DevBuf<double> o_mass;
    DevBuf<uint32_t> o_pid, o_off, o_len;

    // query scratch
    std::recursive_mutex qmu;           // query-side calls share scratch buffers and the stream
    DevBuf<double> win_lo, win_hi;      // dbi_set_windows: merged mass windows
    DevBuf<uint32_t> qdir;              // query directory (launch_qdir), rebuilt per index
    DevBuf<dbi::QueryDir> qdir_par;
    uint64_t build_serial = 0, qdir_serial = 0;
    bool inputs_resident = false;       // res/poff hold the last host build's inputs (dbi_rebuild)
    bool inputs_ptm = false;            // ... and they carry inline '[formula]' PTMs (no dbi_rebuild)
    bool hc_final = false;              // hc holds the counters after the build's last kernel
    uint64_t last_kept = 0;             // the previous build's records (bins of a device-sized tail)
    uint32_t grid_split = 0;              // depth bins: k_chunk_sort's front blocks for split pairs (previous build's count + a margin)
    uint32_t grid_mid = 0, grid_big = 0;  // list-kernel grids of a device-sized tail, from the previous build (0: one block per possible entry; GRID_NONE: that list was empty, the kernel is not launched)
    bool skip_mid = false, skip_big = false;  // the last tail did not launch that list kernel (GRID_NONE)
    // records of this build may repeat exactly (the addSequence flow: the same occurrence added
    // twice, DBIndexStoreSQLiteMult.java:521-523): the chunk sort's ranks break ties by position
    bool exact_dups = false;
    bool lists_short = false;             // the last tail's chunk lists outgrew their grids (set by finish_build)
    bool giants_seen = true;              // the previous build had giant chunks (or none yet): run the giant pass
    DevBuf<double> q_mass, q_tol;
    DevBuf<uint64_t> q_first, q_count, q_row, q_ids;
    DevBuf<uint32_t> h_nh, h_no, h_ids, h_hocc, h_prot;  // dbi_query_hits_device
    DevBuf<uint64_t> h_row, h_orow;
    DevBuf<unsigned long long> h_sums;
    DevBuf<uint64_t> kr_scratch;        // engine_key_range result (2 words)
    DevBuf<double> r_mass;              // dbi_shard_replicate: the whole index being assembled
    DevBuf<uint32_t> r_pid, r_off, r_len, r_occ_off, r_occ;
    DevBuf<double> g_mass;
    DevBuf<uint32_t> g_pid, g_off, g_len;
    DevBuf<uint64_t> g_b, g_e;

    dbi_stats stats{};
    dbi::ShardState shard;
    // merge-cost profile kept across dbi_build_sharded calls (fixed key bands,
    // smoothed over builds): the next build's splitters balance that cost
    // instead of record counts
    struct {
        bool valid = false;
        int32_t split[DBI_COST_BANDS - 1] = {};  // fixed key bands over [minMH, maxMH]
        double cost[DBI_COST_BANDS] = {};        // smoothed merge time per record
        // the owner split whose slowest merge was the fastest so far, and the
        // profile updates since one beat it: after SPLIT_TRIES the next builds
        // keep that split (the profile's re-splits stop chasing spikes)
        bool has_best = false;
        int best_n = 0, since_best = 0;
        int32_t best_split[dbi::MAX_SHARDS - 1] = {};
        double best_max = 0.0;
        uint64_t best_records = 0;  // records of the build that set the best split (another proteome: forgotten)
    } shard_prof;
    // what a warm dbi_build_sharded reuses: the sorted sample keys of the last
    // sampled build (every rank's: all-gathered) and the split the previous
    // build left for the next one (its cost profile applied); valid for a
    // communicator of n ranks.  The count matrix carries a hash of each rank's
    // split: ranks holding different ones sample again.
    struct {
        bool valid = false;
        int n = 0;
        int32_t split[DBI_MAX_SHARDS - 1] = {};
        dbi::SampleKeys keys;
        uint64_t sampled_kept = 0;  // whole-index records of the sampled build
        // the last build's owner split, this owner's merge device time and records
        // received: the next build's totals row carries them (the cost profile)
        int32_t prev_split[DBI_MAX_SHARDS - 1] = {};
        double prev_merge_ms = 0;
        uint64_t prev_recv = 0;
    } shard_warm;
    // the shard the last dbi_build_sharded digested: a warm build of the same
    // shard digests without a host round trip (residue range and record width
    // from here; the device checks them against the offsets, k_shard_flags)
    struct {
        bool valid = false;
        const void* d_res = nullptr;
        const void* d_poff = nullptr;
        uint64_t n_res = 0, n_prot = 0, p_begin = 0, p_end = 0;
        uint64_t e0 = 0, e1 = 0;  // the shard's first / one-past-last residue
        uint32_t width = 0;       // record field width W of the whole proteome
    } shard_dev;
    hipEvent_t ev_merge[2] = {nullptr, nullptr};  // owner merge device time
    DevBuf<uint64_t> xsend, xrecv;      // sharded build: 8-B location words to / from the owners
    DevBuf<double> samp;                // sharded build: mass samples (splitters)
    DevBuf<unsigned long long> xcount;  // sharded build: send counts of every shard (RCCL all-gather)
    DevBuf<uint32_t> qcnt;              // sharded queries: owners per query -> pair offsets
    DevBuf<Rec> qpairA, qpairB;         //   (owner, query) pairs, then grouped by owner
    DevBuf<Rec> qsend, qrecv;           //   (mass, tol) out / in
    DevBuf<Rec> qres, qback;            //   (first, count) answered here / returned to the origin
    Counters hc{};
    uint64_t n_total_extra = 0;

    // per-launch HIP events on the engine stream (dbi_stage_times)
    struct Stage {
        const char* name;
        int eb, ee;                     // event pool slots
        double cR, cN, cU, cP, cB;      // algorithmic bytes = cR*R + cN*N + cU*U + cP*P + cB*nbins
        double ms, bytes;
        double c0;                      // + fixed bytes (exchange)
        bool launched;
    };
    static constexpr int MAX_STAGES = 48;
    hipEvent_t evpool[2 * MAX_STAGES] = {};
    Stage stages[MAX_STAGES];
    int nstage = 0;

    // The warm device-sized build (digest + tail, bounded digest) as one
    // hipGraph: captured on the second warm build with the same key, replayed
    // while the key holds.  The key is everything baked into the captured
    // kernel arguments: inputs, sizes, buffers (g_alloc_gen), parameters,
    // timing mode.
    struct GraphKey {
        const void* d_res = nullptr;
        const void* d_poff = nullptr;
        uint64_t n_res = 0, n_prot = 0, cap = 0, last_kept = 0, alloc_gen = 0, dp_gen = 0;
        uint64_t prev_unique = 0;         // depth bins: the sampled index
        uint32_t depth_cap = 0;           // depth bins: region capacity (0: the radix tail)
        uint32_t lsd_cap = 0;             // semi builds' first-digit partition: region capacity (0: none)
        bool depth_fresh = false;         // depth bins: the map is sampled in this build
        bool tail_local = false;          // the previous build's tail (its list grids)
        uint32_t grid_mid = 0, grid_big = 0, grid_split = 0;
        bool giants = true;
        bool timing = false;
        char timing_only[32] = {};
        // field by field: the struct's padding bytes are not guaranteed zero
        bool operator==(const GraphKey& o) const {
            return d_res == o.d_res && d_poff == o.d_poff && n_res == o.n_res && n_prot == o.n_prot &&
                   cap == o.cap && last_kept == o.last_kept && alloc_gen == o.alloc_gen && dp_gen == o.dp_gen &&
                   prev_unique == o.prev_unique && depth_cap == o.depth_cap && lsd_cap == o.lsd_cap &&
                   depth_fresh == o.depth_fresh &&
                   tail_local == o.tail_local &&
                   grid_mid == o.grid_mid && grid_big == o.grid_big && grid_split == o.grid_split &&
                   giants == o.giants && timing == o.timing &&
                   std::strncmp(timing_only, o.timing_only, sizeof(timing_only)) == 0;
        }
    };
    uint64_t dp_gen = 0;                  // bumped when dp changes (dbi_set_windows, bucket drop)
    bool use_graph = true;                // DBI_BUILD_GRAPH=0: never
    bool use_h1 = true;                   // DBI_DIGEST_HIST=0: the first radix histogram as its own kernel
    bool use_semi_bounded = true;         // DBI_SEMI_BOUNDED=0: warm semi builds by the fused count + emit digest
    int big_split = -1;                   // DBI_BIG_SPLIT: big tier in two size classes (1 always, 0 never, -1 long lists)
    bool h1_on = false;                   // this warm build's digest counts the first radix histogram (h1plan)
    // depth bins (warm lean builds: dbi_engine.hip warm_body_depth)
    bool use_depth = true;                // option depth_bins=0: the radix tail always
    bool use_semi_part = true;            // option semi_part=0: warm semi builds' first radix pass as its own kernels
    bool use_part_stage = true;           // option part_stage=0: the partitioning digest's records go through HBM slots
    bool depth_off = false;               // this build's retry takes the radix tail (a region overflowed)
    bool depth_keep_map = false;          // this build's retry keeps the depth map it computed
    const uint4* depth_map_of = nullptr;  // the map buffer a complete map was last enqueued into
    uint64_t depth_map_unique = 0;        // ... sampled from an index of this many unique peptides
    uint32_t depth_map_nbins = 0;         // ... for this many bins
    double depth_map_lo = 0, depth_map_scale = 0;  // ... over these sub-bins (BinMap lo, scale)
    // owner merges on depth bins (dbi_shard.hip merge_body): the index the map samples is this
    // owner's own slice, left by its last merge (not a replica, not a single-device build)
    bool opt_owner_depth = true;          // option owner_depth=0: owner merges by the radix tail
    bool opt_big_side = true;             // option big_side=0: depth tails' big tier after the mid tier, not beside the chunk sort
    hipStream_t side = nullptr;           // the big tier's stream (sort_chunks), created on first use
    hipEvent_t ev_side[2] = {nullptr, nullptr};  // its fork / join
    hipStream_t stage_stream = nullptr;   // set while stages are enqueued on the side stream (graph timing events)
    uint64_t owner_serial = ~0ull;        // build_serial after this handle's last owner merge
    const void* owner_umass = nullptr;    // ... and its index buffers
    const void* owner_occ = nullptr;
    double owner_lo = 0, owner_hi = 0;    // ... and its mass range
    double owner_us_radix = 0, owner_us_depth = 0;  // merge device time per 1000 records received, by tail (averaged)
    bool opt_depth_map_reuse = true;      // option depth_map_reuse: keep the map while the index's size holds
    bool cur_local = false, tail_local = false;  // this / the last finished build's chunk sort took depth-bin chunks
    bool force_cold = false;              // dbi_set_cold: the next build takes the cold path (buffers kept)
    // dbi_set_option: sharded-build switches and test hooks
    bool opt_shard_full_path = false;     // one rank takes the general path (partition, exchange, agreement)
    bool opt_shard_dev_digest = true;     // warm shard digests device-sized
    bool opt_shard_resample = false;      // every sharded build samples its split again
    int opt_test_split_skew = -1;         // this rank's reused split is skewed (a forced resample)
    std::string opt_test_fail;            // "<phase>@<rank>": an injected local failure
    // region capacity / its share of the previous build's records (doubled after an overflow):
    // the depth bins' regions, the semi builds' low-digit regions
    double depth_slack = 1.25;
    double lsd_slack = 1.25;
    int slack_ok = 0;                     // warm region builds since the last overflow (or the last decay)
    uint64_t prev_unique = 0;             // uniques of the resident index (the depth map's sample)
    DevBuf<Rec> recR;                     // the digest's regions
    DevBuf<uint8_t> rdig;                 //   each record's low bin digit
    DevBuf<uint32_t> rcur, dsub, dpre, desc, d1c, hist2, bstart;  // dsub / dpre: the map's samples
    DevBuf<uint32_t> split_list;          // depth bins: the split chunk pairs
    DevBuf<uint4> dmap;                   // the depth map (DepthMap)
    DevBuf<uint32_t> dheavy;              // its heavy sub-bins (the next map's room for them)
    const dbi::PartOut* part_now = nullptr;  // run_digest: partition the warm digest's records (warm_body_depth)
    dbi::Hist1Plan h1plan{};
    bool capturing = false;               // stage events become event nodes
    GraphKey prev_key{};                  // the last plain warm build's key
    bool prev_key_valid = false;
    struct {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        GraphKey key{};
        Stage stages[MAX_STAGES];
        int nstage = 0;
        uint64_t n_bins = 0, n_in = 0;
        bool sparse = false;
    } bgraph;
    // The owner merge of a warm sharded build (dbi_shard.hip merge_enqueue),
    // captured the same way: the second identical merge is captured, later
    // ones replay it.  Key: everything its kernels bake in.
    struct MergeKey {
        GraphKey g{};             // inputs, buffers, grids, parameters, timing
        uint64_t n_recv = 0;
        double lo = 0, hi = 0;
        const void* xrecv = nullptr;
        uint32_t width = 0;
        int nstage0 = 0;          // stage slots (event pool) the merge's stages start at
        uint32_t depth_cap = 0;   // depth bins: region capacity (0: the radix tail)
        bool depth_fresh = false; // depth bins: the map is sampled in this merge
        bool operator==(const MergeKey& o) const {
            return g == o.g && n_recv == o.n_recv && lo == o.lo && hi == o.hi && xrecv == o.xrecv &&
                   width == o.width && nstage0 == o.nstage0 && depth_cap == o.depth_cap &&
                   depth_fresh == o.depth_fresh;
        }
    };
    struct {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        MergeKey key{};
        Stage stages[MAX_STAGES];
        int nstage = 0;
        uint64_t n_bins = 0;
    } mgraph;
    MergeKey prev_mkey{};
    bool prev_mkey_valid = false;
};


namespace dbi {

struct Bytes {
    double cR = 0, cN = 0, cU = 0, cP = 0, cB = 0;
};

inline int stage_begin(dbi_handle* h, const char* name, Bytes b) {
    if (h->nstage >= dbi_handle::MAX_STAGES) return -1;
    const int i = h->nstage++;
    auto& st = h->stages[i];
    st.name = name;
    st.eb = 2 * i;
    st.ee = 2 * i + 1;
    st.cR = b.cR; st.cN = b.cN; st.cU = b.cU; st.cP = b.cP; st.cB = b.cB;
    st.ms = 0;
    st.c0 = 0;
    st.bytes = 0;
    st.launched = false;
    t_launch_ev = LaunchEvents{};
    // the stage's two events are created on first use (an untimed engine --
    // a one-off build -- creates none: 96 hipEventCreate took ms at dbi_open)
    if (h->timing && (h->timing_only.empty() || h->timing_only == name) &&
        ((h->evpool[st.eb] || hipEventCreate(&h->evpool[st.eb]) == hipSuccess) &&
         (h->evpool[st.ee] || hipEventCreate(&h->evpool[st.ee]) == hipSuccess))) {
        if (h->capturing) {  // a graph: event-record nodes around the stage's kernels (on their stream)
            st.launched = hipEventRecord(h->evpool[st.eb], h->stage_stream ? h->stage_stream : h->stream) == hipSuccess;
        } else {             // events in the kernels' own dispatch packets
            t_launch_ev = LaunchEvents{h->evpool[st.eb], h->evpool[st.ee]};
        }
    }
    return i;
}

inline void stage_end(dbi_handle* h, int i) {
    if (i >= 0 && h->capturing) {
        auto& st = h->stages[i];
        if (st.launched)
            st.launched = hipEventRecord(h->evpool[st.ee], h->stage_stream ? h->stage_stream : h->stream) == hipSuccess;
    } else if (i >= 0) {
        // the first launch of the stage consumed `start`: otherwise nothing ran
        h->stages[i].launched = t_launch_ev.stop != nullptr && t_launch_ev.start == nullptr;
    }
    t_launch_ev = LaunchEvents{};
}

#define STAGE(h, NAME, BYTES, EXPR)                  \
    do {                                             \
        const int _si = stage_begin(h, NAME, BYTES); \
        const hipError_t _stage_err = (EXPR);        \
        stage_end(h, _si);                           \
        DBI_HIP(_stage_err);                         \
    } while (0)

inline Bytes by(double cR, double cN, double cU, double cP, double cB) {
    Bytes b;
    b.cR = cR; b.cN = cN; b.cU = cU; b.cP = cP; b.cB = cB;
    return b;
}

int read_counters(dbi_handle* h);
const char* ptm_device_msg();  // ERR_PTM's message
int begin_build(dbi_handle* h, uint64_t n_res, uint64_t n_prot, bool zero_ctr = true);  // zero_ctr false: the caller zeroes the counters on the stream itself
int prepare_tiles(dbi_handle* h);
// digest of h->d_res / h->d_poff into recA: *n records (*n_in slots, REC_SENTINEL
// in the unused ones when *sparse)
int run_digest(dbi_handle* h, uint64_t* n, uint64_t* n_in, bool* sparse, bool* dev_sized = nullptr);
int tail_buffers(dbi_handle* h, uint64_t n, uint64_t n_in, bool sparse);  // build_tail's allocations, ahead
int build_tail(dbi_handle* h, uint64_t n, double lo, double hi, uint64_t n_in, bool sparse,
               const unsigned long long* d_n_in = nullptr, const unsigned long long* d_n = nullptr, uint64_t n_est = 0, bool est = false);
int ensure_qdir(dbi_handle* h, hipStream_t s);  // query directory of the current index
void drop_graph(dbi_handle* h);                 // the captured warm build graphs (build, owner merge), if any
dbi_handle::GraphKey graph_key(const dbi_handle* h);
uint32_t choose_nbins(uint64_t n, int max_bits);  // fine mass bins of a tail over n records
int radix_plan(uint32_t nbins, bool sparse, int* width);  // LSD digit widths; returns the passes
int finish_build(dbi_handle* h);
bool bounded_digest(const dbi_handle* h);  // a warm build digests into bounded slots (device-sized)
// depth-bin tails (dbi_engine.hip): the bins and regions for about n records,
// the map's reuse test, the allocations, the map, and the tail from the
// filled regions (the lean warm build's, and the owner merge's: dbi_shard.hip)
struct DepthPlan {
    bool on = false;
    uint32_t b1 = 0, b2 = 0, nbins = 0, cap = 0, nreg = 0, max_chunks = 0;
};
DepthPlan depth_plan_n(const dbi_handle* h, uint64_t n, uint64_t slots);
bool depth_map_reusable(const dbi_handle* h, uint32_t nbins, const BinMap& sub);
int depth_buffers(dbi_handle* h, const DepthPlan& pl, uint32_t nchunks);
int depth_map_enqueue(dbi_handle* h, const DepthPlan& pl, const BinMap& sub, uint64_t U);
int depth_tail(dbi_handle* h, const DepthPlan& pl, const BinMap& sub, uint64_t cap, uint32_t T, uint32_t nchunks,
               bool est);
uint32_t chunk_target(const dbi_handle* h, uint64_t n);

}  // namespace dbi
