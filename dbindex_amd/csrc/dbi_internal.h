// dbi_internal.h — shared between the device kernels (dbi_device.hip) and the
// host orchestration (dbi_engine.hip, dbi_store.cpp).  Not part of the C-ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/dbindex_hip.h"

namespace dbi {

// Occurrence record as it moves through the build: 16 B, two u64 words.
//   q0 = enc(mass) << 8 | tag >> 8
//   q1 = (tag & 0xFF) << 56 | pid << 2W | off << W | len
// enc(m) = bits(m) - bits(1.0): exact and order-preserving for 1 <= m < 65536
// Da (every kept mass: >= max(minMH, m0) >= 1 is checked at dbi_open, and
// < NUM_BUCKETS * BUCKET_MASS_RANGE <= 8000).  W = bits(longest protein), read
// by every kernel from Counters::max_plen, so off < plen and len <= plen
// always fit; pid gets 56 - 2W bits (ERR_LAYOUT otherwise).  Ordering records
// by q0 then (q1 >> 56) is ordering by (mass, peptide tag); pid/off locate
// the occurrence directly, so nothing downstream looks proteins up.
//   tag : digest -> chunk sort: peptide_tag() of the string (tie-break key);
//         chunk sort -> finalize: the low byte of q0 = 1 for the first
//         occurrence of its unique peptide, else 0
struct alignas(16) Rec {
    uint64_t q0;
    uint64_t q1;
};
static_assert(sizeof(Rec) == 16, "Rec must be 16 bytes");

constexpr uint64_t MASS_BIAS = 0x3FF0000000000000ull;  // bits(1.0)
__host__ __device__ inline uint64_t rec_q0(double m, uint32_t tag) {
    uint64_t b;
    __builtin_memcpy(&b, &m, 8);
    return ((b - MASS_BIAS) << 8) | (tag >> 8);
}
__host__ __device__ inline double q0_mass(uint64_t q0) {
    const uint64_t b = (q0 >> 8) + MASS_BIAS;
    double m;
    __builtin_memcpy(&m, &b, 8);
    return m;
}
// pid << 2W | off << W (the per-start part of q1)
__host__ __device__ inline uint64_t rec_loc(uint32_t pid, uint32_t off, uint32_t w) {
    return ((uint64_t)pid << (2 * w)) | ((uint64_t)off << w);
}
__host__ __device__ inline uint64_t rec_q1(uint32_t tag, uint64_t loc, uint32_t len) {
    return ((uint64_t)(tag & 0xFFu) << 56) | loc | len;
}
__host__ __device__ inline uint32_t q1_len(uint64_t q1, uint32_t w) { return (uint32_t)(q1 & ((1ull << w) - 1)); }
__host__ __device__ inline uint32_t q1_off(uint64_t q1, uint32_t w) {
    return (uint32_t)((q1 >> w) & ((1ull << w) - 1));
}
__host__ __device__ inline uint32_t q1_pid(uint64_t q1, uint32_t w) {
    return (uint32_t)((q1 >> (2 * w)) & ((1ull << (56 - 2 * w)) - 1));
}
// field width W from the longest protein (>= 1)
__host__ __device__ inline uint32_t rec_width(uint32_t max_plen) {
    uint32_t w = 1;
    while (w < 32 && (max_plen >> w) != 0) ++w;
    return w;
}
// pid of every protein fits in 56 - 2W bits
__host__ __device__ inline bool rec_layout_ok(uint32_t w, uint64_t n_prot) {
    return 2 * w < 56 && (n_prot == 0 || ((n_prot - 1) >> (56 - 2 * w)) == 0);
}

// Pinned order of different peptides with bit-identical mass:
// (16-bit tag, first appearance).  The tag hashes the peptide's length and its
// first and last (up to) four residues, so a digest walk reads residue bytes
// only at the two ends of a peptide, never per residue step:
//   head = s[0] | s[1] << 8 | s[2] << 16 | s[3] << 24        (bytes past the end: 0)
//   tail = s[L-1] | s[L-2] << 8 | s[L-3] << 16 | s[L-4] << 24 (bytes before the start: 0)
// (a walk keeps tail as tail << 8 | c).  oracle/cpu_ref.cpp peptide_tag and
// oracle/pyref.py peptide_tag restate it over the string.
__host__ __device__ inline uint32_t tag_keep(uint32_t len) { return len >= 4 ? ~0u : (1u << (8 * len)) - 1u; }
__host__ __device__ inline uint16_t peptide_tag(uint32_t head, uint32_t tail, uint32_t len) {
    const uint32_t k = tag_keep(len);
    uint32_t x = ((head & k) * 0x9E3779B1u) ^ ((tail & k) * 0x85EBCA77u) ^ (len * 0xC2B2AE3Du);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return (uint16_t)((x >> 16) ^ (x & 0xFFFFu));
}
// the tag of the len residues at s (reads s[0, len) only)
__host__ __device__ inline uint16_t peptide_tag_of(const uint8_t* s, uint32_t len) {
    uint32_t head = 0, tail = 0;
    for (uint32_t k = 0; k < 4 && k < len; ++k) {
        head |= (uint32_t)s[k] << (8 * k);
        tail |= (uint32_t)s[len - 1 - k] << (8 * k);
    }
    return peptide_tag(head, tail, len);
}

constexpr int MAX_PRECURSOR_INT = 8000;  // (int) Constants.MAX_PRECURSOR_MASS

// Residue class bits, one byte per char, staged in LDS by the digest kernels.
constexpr uint8_t F_CLEAVE = 1;
constexpr uint8_t F_NOCUT = 2;
constexpr uint8_t F_MAND = 4;
constexpr uint8_t F_CUT = 8;    // window only: checkCleavage C-side ok at this residue (or protein end)
constexpr uint8_t F_LAST = 16;  // window only: last residue of its protein
constexpr uint8_t F_PTM = 32;   // '[': an inline formula (DBIndexer.java:288-303) where none may be

struct BinMap {
    double lo;
    double scale;     // nbins / (hi - lo)
    uint32_t nbins;
};

// Device-side copy of the parameters the kernels need (kernel argument).
struct DevParams {
    double min_mh, max_mh;
    double m0;                // ((0 + H2O_PROTON) + cTerm) + nTerm, Java order
    int32_t max_missed;
    int32_t min_len;
    int32_t nb;               // NUM_BUCKETS
    int32_t br;               // BUCKET_MASS_RANGE
    int32_t mand_mode;        // 0 null, 1 non-null
    int32_t mand_filter;      // mand_mode && count > 0 (filterSequence path)
    int32_t semi;
    double drop_mass;         // bucket > NUM_BUCKETS-1  <=>  (int)m >= nb*br  <=>  m >= nb*br
    int32_t cut_count;        // count by cut stepping (full enzyme, no mandatory AAs, residue masses < 1024 Da)
    int32_t buckets;          // 1: bucketed store (drop + query bucket test); 0: MassRangeFilteringIndex (none)
    // mass-window filter (dbi_set_windows): keep only peptides inside one of
    // n_win sorted disjoint closed intervals; a start's walk ends once its mass
    // passes win_max (SKIP_PROTEIN_START, DBIndexer.java:351-354)
    int32_t filter;
    uint32_t n_win;
    double win_max;           // +inf without a filter
    const double* win_lo;     // device arrays, n_win each
    const double* win_hi;
};

// fine mass bins of a build: the one place the map's fields are computed
inline BinMap make_binmap(double lo, double hi, uint32_t nbins) {
    BinMap bm;
    bm.lo = lo;
    bm.nbins = nbins;
    bm.scale = (hi > lo) ? (double)nbins / (hi - lo) : 0.0;
    return bm;
}

constexpr int HIST_MAX_BUCKETS = 64;  // dbi_count_buckets: index_factor (NUM_BUCKETS) at most
constexpr int GIANT_PASSES = 5;  // MSD split passes over chunks above BIG_CAP (then the global-memory fallback)

// Device counters block (one per engine), read back once per build.
struct Counters {
    unsigned long long n_kept;     // occurrences stored
    unsigned long long n_dropped;  // bucket > NUM_BUCKETS-1
    unsigned long long n_unique;
    unsigned long long n_keys;
    unsigned long long n_keys_shard[8];  // per-XCD-group partial key counts (summed on readback)
    unsigned int n_big;            // chunks above CHUNK_CAP (sorted by the 1024-thread LDS kernel)
    unsigned int n_mid;            // chunks with a bin above WAVE_SORT_MAX (block-level compact sort)
    unsigned int err;              // device error bits
    unsigned int n_giant;          // chunks above BIG_CAP (MSD split into LDS-sized leaves)
    unsigned int n_seg[GIANT_PASSES + 1];  // giant split: segments in work list p
    unsigned int n_leaf_small, n_leaf_big, n_fallback;
    unsigned long long n_big_recs, n_giant_recs;  // records in chunks sorted by the big / giant paths
    unsigned long long n_mid_recs;                // records in chunks sorted by the mid path (chunk_sort_mid)
    // what the tail of a device-sized warm build sorts (k_tail_counts): the
    // digest's slots / records, or 0 when they did not fit the buffer (the
    // skipped tiles left stale slots behind; the build is redone)
    unsigned long long tail_in, tail_n;
    unsigned long long depth_w;    // depth bins: the sampled occurrence weight (the map's total)
    unsigned int part_chunks;      // depth bins: pass-2 chunks over the digest's regions (k_part_plan)
    unsigned int depth_h;          // depth bins: heavy sub-bins of this map (k_depth_mark)
    unsigned int depth_hc;         // depth bins: the same, from the map's counting pass (room for them)
    unsigned int n_split;          // depth bins: chunk pairs split in two (k_depth_chunks' split_list)
    // hot lines apart: the digest's per-tile ticket (every block, waits for
    // the result), and the layout word every block of every kernel reads
    // (sharing the ticket's line cost the digest 30%)
    alignas(256) unsigned int tile_ticket;  // k_digest_fused: tiles in dispatch order
    alignas(256) unsigned long long n_slots;  // k_digest_bounded: record slots reserved (kept + sentinels), the
                                              // cursor every tile takes its output region from
    alignas(256) unsigned int max_plen;     // longest protein (k_tile_proteins): the record field width
};
constexpr unsigned ERR_LAYOUT = 1;  // 2*bits(longest protein) + bits(proteins) > 56
constexpr unsigned ERR_SEGS = 2;    // giant split: a segment list overflowed (internal)
constexpr unsigned ERR_SLOTS = 4;   // bounded digest: a thread emitted more records than it reserved (internal)
constexpr unsigned ERR_PTM = 8;     // a device digest met '[' (inline PTMs are only digested from host input)
constexpr uint32_t GRID_NONE = 0xFFFFFFFFu;  // list grid: the previous build's list was empty (no launch)
constexpr unsigned ERR_GRID = 16;   // a chunk list outgrew its kernel's grid (estimated from the previous build): redo
constexpr unsigned ERR_PART = 32;   // depth bins: a digest region outgrew its capacity: redo by the radix tail

// Tunables
constexpr int DIGEST_THREADS = 256;
constexpr int DIGEST_TILE = 4096;   // starts per digest block
constexpr int DIGEST_HALO = 256;    // residues staged past the tile
constexpr int RADIX_BITS = 8;        // max digit width (256 buckets; 3 passes cover the 2^24 bins)
constexpr int RADIX_THREADS = 512;
constexpr int RADIX_ITEMS = 8;      // records per thread per radix block (4096: 64 KiB LDS exchange)
constexpr int CHUNK_THREADS = 512;
constexpr int CHUNK_CAP = 1984;     // records per chunk sorted in LDS (20 B each: 4 blocks per CU)
constexpr int CHUNK_T = 1536;       // target chunk size (whole mass bins; DBI_CHUNK_T A/B, round 3: 1024-1792 measured, 1536 best since the chunk pairs)
constexpr int CHUNK_T_SMALL = 1280;  // below CHUNK_T_MIN_RECS records (human scale: 0.059 vs 0.069 ms, more blocks to fill 256 CUs)
constexpr uint64_t CHUNK_T_MIN_RECS = 8ull << 20;
constexpr int CHUNK_T_DEPTH = 1792;  // depth-bin chunks from CHUNK_T_MIN_RECS records (SwissProt: 3.75-3.83 -> 3.73-3.76 ms, r05s / r05t)
constexpr int BIN_AVG = 8;          // target records per fine mass bin (rank-sorted by one wave)
#ifndef DBI_WAVE_SORT_LIMIT
#define DBI_WAVE_SORT_LIMIT 512
#endif
constexpr int WAVE_SORT_LIMIT = DBI_WAVE_SORT_LIMIT;  // bins up to this size: one wave in k_chunk_sort (more: chunk_sort_mid)
// chunk_sort_mid entries (single bins above WAVE_SORT_LIMIT) per chunk pair: the
// wide bins of a chunk of <= CHUNK_CAP records plus the pair's straddling bin
constexpr uint32_t MID_PER_PAIR = CHUNK_CAP / (WAVE_SORT_LIMIT + 1) + 1;
constexpr int BIG_THREADS = 1024;
constexpr int BIG_CAP = 7936;       // records per oversize chunk sorted in LDS (1 block per CU)

// ---- launchers (dbi_device.hip) -------------------------------------------------
// All return hipError_t of the launch.
// tile_pf[t] = protein holding residue min(t*DIGEST_TILE, R-1); ctr->max_plen
// = longest protein (the record field width, see Rec)
hipError_t launch_tile_proteins(const uint32_t* d_poff, uint32_t n_prot, uint32_t n_res, uint32_t* d_tile_pf,
                                Counters* d_ctr, hipStream_t s, uint32_t* d_zero = nullptr, uint32_t n_zero = 0);
hipError_t launch_digest_count(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                               const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot,
                               uint32_t n_res, const uint32_t* d_tile_pf, uint32_t* d_blk, uint32_t* d_thr,
                               Counters* d_ctr, hipStream_t s);
// One pass: count, decoupled look-back for the tile's output offset, emit.
// Records past `cap` are not written (the exact total still lands in
// ctr->n_kept: the caller grows the buffer and runs it again).  status:
// ntiles words tagged with `epoch` (never 0; reset the words when it wraps).
hipError_t launch_digest_fused(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                               const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot, uint32_t n_res,
                               const uint32_t* d_tile_pf, unsigned long long* d_status, uint32_t epoch,
                               Rec* d_out, uint32_t cap, Counters* d_ctr, hipStream_t s);
// Full-enzyme digest without mandatory residues, <= 2 missed cleavages, in one
// walk: each tile reserves the exact number of candidate ends of its starts
// (mass filters only lower the real count) with one atomic add on
// ctr->n_slots (tiles in arrival order), fills them in its own order and
// marks unused slots with REC_SENTINEL (q0 == ~0).  ctr->n_slots = slots
// reserved, ctr->n_kept = records kept; nothing is written when n_slots > cap
// (the caller grows the buffer and runs it again).
constexpr unsigned long long REC_SENTINEL = ~0ull;
// h1p (warm device-sized builds): the digest also counts the first radix
// pass's histogram -- hist[d * G + slot / RADIX_CHUNK] of every record it
// writes, d = bin_of(mass, bm) & (2^bits - 1) -- into a zeroed `hist`, so the
// tail skips that pass's histogram kernel (a read of every slot's mass)
struct Hist1Plan {
    uint32_t* hist;
    BinMap bm;
    int bits;
    uint32_t G;  // radix blocks over cap slots
};
// ---- depth bins (warm lean builds) ----------------------
// 2^(b1 + b2) mass bins of about equal record counts: a monotone map of
// 2^DEPTH_SUB_BITS linear sub-bins of [minMH, maxMH], built from a sample of the
// previous build's index (occurrence-weighted; a heuristic: a stale or poor
// map costs speed, never correctness).  The digest partitions its records by
// the bin's high b1 bits into (digit, XCD) regions; one radix pass over the
// low b2 bits orders them by bin; the chunk sort bins each chunk locally.
// The map is a bit per sub-bin (1: a bin starts there) plus the starts before
// each 64-sub-bin word, 16 B per word {mask lo, mask hi, base, 0}: bin = base
// + popcount of the word's bits up to the sub-bin -- one 16-B load per record
// (1 MiB at 2^22 sub-bins: L2-resident, where a u16 table of 2^22 entries was
// 8 MiB).
#ifndef DBI_DEPTH_SUB_BITS
#define DBI_DEPTH_SUB_BITS 22
#endif
constexpr int DEPTH_SUB_BITS = DBI_DEPTH_SUB_BITS;
constexpr uint32_t DEPTH_XCDS = 8;        // regions per high digit: one per XCD (block b on XCD b % 8)
constexpr uint32_t PART_CHUNK = 4096;     // records per pass-2 block (RADIX_THREADS * RADIX_ITEMS)
struct DepthMap {
    const uint4* map;      // per 64 sub-bins: bit s of (y:x) -- sub-bin s starts a bin (s > 0); z: the bin before them
    BinMap sub;            // the linear sub-bins
    uint32_t b2;           // low bits of a bin (the pass-2 digit); the high bits: the digest's partition
    uint32_t last;         // the last bin (2^(b1 + b2) - 1)
};
struct PartOut {          // the digest's partition (k_digest_bounded / k_digest_semi_bounded PART)
    Rec* recs;            // region r = d1 * DEPTH_XCDS + xcd at [r * cap, r * cap + cur[r])
    uint8_t* dig;         // each record's pass-2 digit (b2 bits), same positions
    uint32_t* cur;        // per region: records placed (zeroed before the digest)
    DepthMap dm;          // depth bins: d1 = the bin's high b1 bits, the digit its low b2 bits
    uint32_t cap;         // records per region (a multiple of 64)
    uint32_t b1;
    // lsd (linear fine bins, semi-specific builds): d1 = the bin's LOW b1 bits
    // (the first LSD pass), the digit the next dm.b2 bits (the second)
    uint32_t lsd;
    BinMap lin;
    uint32_t stage;       // lean digest: tiles that fit keep their records in LDS until partitioned
};
// the map: ns evenly spaced uniques of the previous index (mass order) -> their
// sub-bins and occurrence weights; the weights' scan (total -> ctr->depth_w);
// the bin starts (zeroed d_map, nsub / 64 entries), then the word bases;
// *d_heavy carries the map's heavy sub-bin count to the next map
hipError_t launch_depth_sample(const double* d_umass, const uint32_t* d_occ_off, uint64_t n_unique, uint32_t ns,
                               const BinMap& sub, uint32_t* d_ss, uint32_t* d_sw, hipStream_t s);
hipError_t launch_depth_map(const uint32_t* d_ss, const uint32_t* d_pre, uint32_t ns, uint32_t nbins, uint32_t nsub,
                            uint4* d_map, uint32_t* d_heavy, Counters* d_ctr, hipStream_t s);
hipError_t launch_digest_bounded(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                                 const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot, uint32_t n_res,
                                 const uint32_t* d_tile_pf, Rec* d_out, uint64_t cap, Counters* d_ctr, hipStream_t s,
                                 const Hist1Plan* h1p = nullptr, const PartOut* part = nullptr);
// pass-2 plan over the regions: desc[c] = region << 16 | piece for every
// PART_CHUNK-record piece, d1c[d] / d1c[D1 + d] = first chunk / chunks of high
// digit d, ctr->part_chunks; ctr->tail_n = the records (0 when the digest's
// slots or a region overflowed: nothing downstream runs, the host redoes it)
hipError_t launch_part_plan(const uint32_t* d_cur, uint32_t cap, uint32_t b1, uint64_t slot_cap, uint32_t* d_desc,
                            uint32_t* d_d1c, Counters* d_ctr, hipStream_t s);
// hist[(first(d1) << b2) + d2 * nch(d1) + (c - first(d1))] = records of chunk c with digit d2
// (records ordered by (d1, d2): depth bins); lsd: hist[d2 * max_chunks + c]
// (ordered by (d2, d1): the second LSD pass of linear bins; the chunks past
// ctr->part_chunks write zeros)
hipError_t launch_part_hist(const uint8_t* d_dig, const uint32_t* d_cur, uint32_t cap, const uint32_t* d_desc,
                            const uint32_t* d_d1c, uint32_t b1, uint32_t b2, uint32_t max_chunks, uint32_t* d_hist,
                            const Counters* d_ctr, hipStream_t s, bool lsd = false);
// lsd: also each record's next-pass digit ((bin_of(m, bm) >> nshift) & (2^nbits - 1)) into d_ndig
hipError_t launch_part_scatter(const Rec* d_recs, const uint8_t* d_dig, const uint32_t* d_cur, uint32_t cap,
                               const uint32_t* d_desc, const uint32_t* d_d1c, uint32_t b1, uint32_t b2,
                               uint32_t max_chunks, const uint32_t* d_offs, Rec* d_out, const Counters* d_ctr,
                               hipStream_t s, bool lsd = false, uint8_t* d_ndig = nullptr, BinMap bm = BinMap{},
                               uint32_t nshift = 0, uint32_t nbits = 0);
// chunk pairs over the bin-ordered records from the pass-2 offsets: bin
// starts (bstart: nbins + 1), then chunk_lo[2c] = first bin start at or after
// c*T, chunk_lo[2c+1] = the last bin's start when the chunk exceeds CHUNK_CAP
// (those pairs c listed in d_split_list[0, ctr->n_split)); d_big_list: the
// chunks above CHUNK_CAP listed too (ctr->n_big), for a big tier launched
// beside the chunk sort (launch_chunk_sort big_listed)
hipError_t launch_depth_bounds(const uint32_t* d_offs, const uint32_t* d_d1c, uint32_t b1, uint32_t b2,
                               uint32_t* d_bstart, uint32_t T, uint32_t nchunks, uint32_t* d_chunk_lo,
                               Counters* d_ctr, hipStream_t s, uint32_t* d_split_list,
                               uint32_t* d_big_list = nullptr);
// semi-specific enzymes (no mandatory residues, no windows): one walk per start
// into slots bounded by the bit maps (REC_SENTINEL in the unused ones)
hipError_t launch_digest_semi_bounded(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                                      const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot, uint32_t n_res,
                                      const uint32_t* d_tile_pf, Rec* d_out, uint64_t cap, Counters* d_ctr,
                                      hipStream_t s, const PartOut* part = nullptr);
// tail_in / tail_n of a device-sized build: the digest's slot and record
// counts, or 0 / 0 when the slots needed exceed cap
hipError_t launch_tail_counts(Counters* d_ctr, uint64_t cap, bool sparse, hipStream_t s);
// COUNT with SQLiteMult bucket counts: d_hist[min((int)m / BUCKET_MASS_RANGE,
// NUM_BUCKETS)] += each INCLUDE'd occurrence (NUM_BUCKETS <= HIST_MAX_BUCKETS)
hipError_t launch_digest_count_hist(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                                    const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot, uint32_t n_res,
                                    const uint32_t* d_tile_pf, uint32_t* d_blk, uint32_t* d_thr, Counters* d_ctr,
                                    unsigned long long* d_hist, hipStream_t s);
hipError_t launch_digest_emit(const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                              const uint8_t* d_res, const uint32_t* d_poff, uint32_t n_prot,
                              uint32_t n_res, const uint32_t* d_tile_pf, uint32_t* d_blk_off, uint32_t* d_thr,
                              Rec* d_out, Counters* d_ctr, hipStream_t s);
// exclusive scan of n u32 values into out (may alias), total written to *d_total
hipError_t launch_scan_u32(const uint32_t* d_in, uint32_t* d_out, uint64_t n, uint32_t* d_block_tmp,
                           uint64_t tmp_elems, unsigned long long* d_total, hipStream_t s);
size_t scan_u32_tmp_elems(uint64_t n);
// inline-PTM proteins, one thread each (COUNT: per-protein kept counts into
// d_cnt; EMIT: d_cnt = exclusive offsets into d_out, counters updated)
hipError_t launch_ptm_digest(bool emit, const DevParams& dp, const double* d_mass_tab, const uint8_t* d_flags,
                             const uint8_t* d_sres, const uint32_t* d_soff, const uint8_t* d_ores,
                             const uint32_t* d_ooff, const uint32_t* d_pid, const uint32_t* d_ev_off,
                             const uint32_t* d_ev_pos, const double* d_ev_mass, uint32_t n_ptm, uint32_t* d_cnt,
                             Rec* d_out, Counters* d_ctr, hipStream_t s);

// Owner map of a sharded build (dbi_shard_*): shard d owns the mass keys
// (int)(m * factor) in [split[d-1], split[d]) (split[-1] = -inf, split[n-1] =
// +inf), so a key, and every occurrence of a peptide, has exactly one owner.
// pid_add = (first global protein id of the sending shard) << 2W.
constexpr int MAX_SHARDS = 64;
struct OwnerMap {
    int32_t split[MAX_SHARDS - 1];
    uint32_t nshards;
    int32_t factor;
    uint64_t pid_add;
};
inline int owner_bits(uint32_t nshards) {
    int b = 0;
    while ((1u << b) < nshards) ++b;
    return b;
}
// Query routing of a sharded index: a window [lo, hi] goes to every owner
// whose key range meets [(int)(lo*factor), (int)(hi*factor)].
struct RouteMap {
    int32_t split[MAX_SHARDS - 1];
    uint32_t nshards;
    int32_t factor;
    int32_t nb, br;  // NUM_BUCKETS / BUCKET_MASS_RANGE: windows past the last bucket are empty
};
// sparse: the input holds REC_SENTINEL slots (bounded digest), left out of the output
// d_n (optional, every launcher below): the real count on the device, n its
// upper bound (a device-sized build sizes its grids by capacity)
hipError_t launch_radix_hist(const Rec* d_in, uint32_t n, const BinMap& bm, int shift, int bits, bool sparse,
                             uint32_t* d_hist, hipStream_t s, const unsigned long long* d_n = nullptr);
// d_next_dig (optional): the record's digit of the next pass, one byte per
// output position, counted by launch_radix_hist_u8 instead of re-reading records
hipError_t launch_radix_scatter(const Rec* d_in, Rec* d_out, uint32_t n, const BinMap& bm, int shift, int bits,
                                bool sparse, const uint32_t* d_hist, hipStream_t s, uint8_t* d_next_dig = nullptr,
                                int next_shift = 0, int next_bits = 0, const unsigned long long* d_n = nullptr);
hipError_t launch_radix_hist_u8(const uint8_t* d_dig, uint32_t n, int bits, uint32_t* d_hist, hipStream_t s,
                                const unsigned long long* d_n = nullptr);
uint64_t radix_blocks(uint32_t n);
// stable partition pass by owner shard (digit = OwnerDigit), global protein ids out
// (d_n: the slot count on the device, n its upper bound -- a device-sized shard digest)
hipError_t launch_owner_hist(const Rec* d_in, uint32_t n, const OwnerMap& om, bool sparse, uint32_t* d_hist,
                             hipStream_t s, const unsigned long long* d_n = nullptr);
// writes the second record word only (global protein | offset | length), 8 B
// per record: the owner recomputes mass and tag from the residues
hipError_t launch_owner_scatter(const Rec* d_in, uint64_t* d_out, uint32_t n, const OwnerMap& om, bool sparse,
                                const uint32_t* d_hist, hipStream_t s, const unsigned long long* d_n = nullptr);
// owner side: 8-B location words -> 16-B records (mass and tag from the residues)
hipError_t launch_expand_locs(const uint64_t* d_locs, uint64_t n, const uint8_t* d_res, const uint32_t* d_poff,
                              const double* d_mass_tab, double m0, uint32_t w, Rec* d_out, hipStream_t s);
// the same, counting the first radix pass's histogram (digit bin_of(m, bm) &
// (2^bits - 1), hist[d * G + radix chunk], G = radix_blocks(n)) of the tail
hipError_t launch_expand_locs_hist(const uint64_t* d_locs, uint32_t n, const uint8_t* d_res, const uint32_t* d_poff,
                                   const double* d_mass_tab, double m0, uint32_t w, Rec* d_out, const BinMap& bm,
                                   int bits, uint32_t* d_hist, hipStream_t s);
// the same, partitioned by the depth bin's high digit into po's (digit, XCD)
// regions with each record's low digit (the owner merge on depth bins;
// po.cur zeroed, ctr->n_kept = n for k_part_plan's check)
hipError_t launch_expand_locs_part(const uint64_t* d_locs, uint32_t n, const uint8_t* d_res, const uint32_t* d_poff,
                                   const double* d_mass_tab, double m0, uint32_t w, const PartOut& po,
                                   Counters* d_ctr, hipStream_t s);
// stable partition of query routing pairs (q0 = owner, q1 = query index) by owner
hipError_t launch_pair_hist(const Rec* d_in, uint32_t n, uint32_t nshards, uint32_t* d_hist, hipStream_t s);
hipError_t launch_pair_scatter(const Rec* d_in, Rec* d_out, uint32_t n, uint32_t nshards, const uint32_t* d_hist,
                               hipStream_t s);
// cnt[i] = owners query i's window meets (0: empty window)
hipError_t launch_qroute_count(const double* d_qm, const double* d_qt, uint64_t nq, const RouteMap& rm,
                               uint32_t* d_cnt, hipStream_t s);
// pairs[offs[i] + k] = (owner o0 + k, i)
hipError_t launch_qroute_emit(const double* d_qm, const double* d_qt, uint64_t nq, const RouteMap& rm,
                              const uint32_t* d_offs, Rec* d_pairs, hipStream_t s);
// out[p] = (mass, tol) bits of pair p's query
hipError_t launch_qpack(const Rec* d_pairs, uint64_t np, const double* d_qm, const double* d_qt, Rec* d_out,
                        hipStream_t s);
// owner side: (mass, tol) -> (base + first, count), first = ~0 when count = 0
struct QueryDir {  // query directory over the unique masses (launch_qdir)
    double lo, scale;
    uint32_t nb;
};
hipError_t launch_query_pairs(const DevParams& dp, int32_t factor, const double* d_umass, uint32_t n_unique,
                              const Rec* d_in, uint64_t n, uint64_t base, Rec* d_out, const QueryDir* d_qd,
                              const uint32_t* d_dir, hipStream_t s);
// origin side: fold the owners' answers into per-query (first, count)
hipError_t launch_qcombine(const Rec* d_pairs, const Rec* d_res, uint64_t np, uint64_t* d_first,
                           uint64_t* d_count, uint64_t nq, hipStream_t s);
// out[i] = mass of slot i * n / ns (NaN for a sentinel slot), i < ns
hipError_t launch_sample_masses(const Rec* d_recs, uint64_t n, uint32_t ns, double* d_out, hipStream_t s);
// out[i] = in[i] - base (u64 -> u32 offsets of a protein range)
hipError_t launch_off_rebase(const uint64_t* d_in, uint64_t base, uint64_t hi, uint32_t* d_out, uint64_t n,
                             hipStream_t s);  // out = clamp(in - base, 0, hi)
// ctr->max_plen = max(ctr->max_plen, longest protein of poff[0..n_prot])
hipError_t launch_max_plen(const uint32_t* d_poff, uint32_t n_prot, Counters* d_ctr, hipStream_t s);
size_t radix_hist_elems(uint32_t n, int bits);
// chunk pairs over the bin-sorted records (2*nchunks+1 entries): chunk_lo[2c] =
// first bin start at or after c*T, chunk_lo[2c+1] = the start of a big bin
// straddling (c+1)*T (its own chunk), else chunk_lo[2c+2]
hipError_t launch_chunk_bounds(const Rec* d_recs, uint32_t n, const BinMap& bm, uint32_t T, uint32_t nchunks,
                               uint32_t* d_chunk_lo, hipStream_t s, const unsigned long long* d_n = nullptr);
// local: depth-bin chunks (launch_depth_bounds), each binned in LDS by its own
// mass range; one block per chunk (2 * nchunks), the wide local bins written
// unsorted for chunk_sort_mid, which then sorts `out` in place (d_in == d_out)
hipError_t launch_chunk_sort(const Rec* d_in, Rec* d_out, const BinMap& bm, const uint32_t* d_chunk_lo,
                             uint32_t nchunks, const uint8_t* d_res, const uint32_t* d_poff, uint32_t* d_ucount,
                             uint32_t* d_big_list, uint32_t* d_mid_list, bool ties, Counters* d_ctr, hipStream_t s,
                             bool local = false, const uint32_t* d_split_list = nullptr, uint32_t nfront = 0,
                             bool big_listed = false);
hipError_t launch_chunk_sort_mid(const Rec* d_in, Rec* d_out, const BinMap& bm, const uint32_t* d_chunk_lo,
                                 const uint8_t* d_res, const uint32_t* d_poff, uint32_t* d_ucount,
                                 const uint32_t* d_mid_list, uint32_t max_blocks, Counters* d_ctr, hipStream_t s);
hipError_t launch_chunk_sort_big(const Rec* d_in, Rec* d_out, const BinMap& bm, const uint32_t* d_chunk_lo,
                                 const uint8_t* d_res, const uint32_t* d_poff, uint32_t* d_ucount,
                                 const uint32_t* d_big_list, uint32_t* d_giant_list, uint32_t max_blocks,
                                 uint32_t split_above, bool ties, Counters* d_ctr, hipStream_t s,
                                 int split = -1, bool local = false);
// chunks above BIG_CAP listed in d_giant_list: MSD split on the (mass, tag)
// key into leaves sorted in LDS; a segment of one (mass, tag) key above
// BIG_CAP falls back to global-memory scratch (ws_key / ws_k2).  segs: 5 lists
// of seg_cap entries (two work lists, small leaves, big leaves, fallback).
size_t giant_seg_cap(uint64_t n);
hipError_t launch_giant_chunks(const Rec* d_in, Rec* d_out, const uint32_t* d_chunk_lo, const uint8_t* d_res,
                               const uint32_t* d_poff, uint32_t* d_ucount, const uint32_t* d_giant_list,
                               uint4* d_segs, size_t seg_cap, unsigned long long* d_ws_key, uint32_t* d_ws_k2,
                               Counters* d_ctr, hipStream_t s);
hipError_t launch_finalize(const Rec* d_recs, const uint32_t* d_chunk_lo, uint32_t nchunks, const uint32_t* d_ubase,
                           double* d_umass, uint32_t* d_upid, uint32_t* d_uoff, uint32_t* d_ulen,
                           uint32_t* d_occ_off, uint32_t* d_occ_pid, int32_t factor, uint32_t ucap, uint32_t cstride,
                           uint32_t n_kept, const unsigned long long* d_n, Counters* d_ctr, hipStream_t s);
hipError_t launch_key_flags(const double* d_umass, uint32_t n_unique, int32_t factor, uint32_t* d_flags,
                            hipStream_t s);
hipError_t launch_write_tail(uint32_t* d_occ_off, uint32_t n_kept, const Counters* d_ctr, hipStream_t s,
                             const unsigned long long* d_n = nullptr);
hipError_t launch_hbm_copy(const void* d_in, void* d_out, uint64_t n16, hipStream_t s);
hipError_t launch_gather(const uint64_t* d_ids, uint64_t n, const double* d_umass, const uint32_t* d_upid,
                         const uint32_t* d_uoff, const uint32_t* d_ulen, const uint32_t* d_occ_off,
                         double* o_mass, uint32_t* o_pid, uint32_t* o_off, uint32_t* o_len, uint64_t* o_b,
                         uint64_t* o_e, hipStream_t s);
hipError_t launch_write_keys(const double* d_umass, uint32_t n_unique, int32_t factor,
                             const uint32_t* d_pos, int32_t* d_keys, hipStream_t s);
hipError_t launch_qdir(const double* d_umass, uint32_t nu, uint32_t nb, QueryDir* d_qd, uint32_t* d_dir,
                       hipStream_t s);
hipError_t launch_query(const DevParams& dp, int32_t factor, const double* d_umass, uint32_t n_unique,
                        const double* d_qmass, const double* d_qtol, uint64_t nq,
                        uint64_t* d_first, uint64_t* d_count, const QueryDir* d_qd, const uint32_t* d_dir,
                        hipStream_t s);
hipError_t launch_key_range(const double* d_umass, uint32_t n_unique, int32_t factor, int32_t klo,
                            int32_t khi, uint64_t* d_out2, hipStream_t s);
hipError_t launch_occ_to_recs(const double* d_mass, const uint32_t* d_pid, const uint32_t* d_off,
                              const uint32_t* d_len, const uint32_t* d_poff, const uint8_t* d_res, uint64_t n,
                              uint64_t n_prot, Rec* d_out, Counters* d_ctr, hipStream_t s);
hipError_t launch_off64_to_32(const uint64_t* d_in, uint32_t* d_out, uint64_t n, hipStream_t s,
                              Counters* d_ctr = nullptr);  // d_ctr: zeroed too
// query hits: per-query hit / protein-id counts -> u64 offsets (row, occ_row:
// nq + 1 entries each, totals also at tot[0..1]); sums: scan2_tmp_elems(nq)
size_t scan2_tmp_elems(uint64_t n);
hipError_t launch_hits_offsets(const uint64_t* d_first, const uint64_t* d_count, const uint32_t* d_occ_off,
                               uint64_t nq, uint32_t* d_nh, uint32_t* d_no, unsigned long long* d_sums,
                               uint64_t* d_row, uint64_t* d_occ_row, unsigned long long* d_tot, hipStream_t s);
hipError_t launch_hits_expand(const uint64_t* d_first, const uint64_t* d_count, const uint64_t* d_row,
                              const uint64_t* d_occ_row, const uint32_t* d_occ_off, const uint32_t* d_occ_pid,
                              uint64_t nq, uint32_t* d_ids, uint32_t* d_hit_occ, uint32_t* d_prot, hipStream_t s);
hipError_t launch_expand_csr(const uint64_t* d_first, const uint64_t* d_count, const uint64_t* d_row,
                             uint64_t nq, uint64_t* d_ids, hipStream_t s);

// ---- per-stage timing ----------------------------------------------------------
// Events of the stage being launched, attached to the dispatch packets
// themselves (hipExtLaunchKernelGGL): timing adds no marker packets, hence no
// idle gaps, between kernels.  `start` is consumed by the first launch of the
// stage; every launch re-records `stop`, so it ends up at the stage's last
// kernel.  Both null = untimed.
struct LaunchEvents {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};
extern thread_local LaunchEvents t_launch_ev;

// ---- persistence (dbi_persist.hip) ---------------------------------------------------
int index_save(dbi_handle* h, const char* path, const std::string* defs, const std::vector<uint64_t>* def_off);
int index_load(dbi_handle* h, const char* path, std::vector<uint8_t>* res_out, std::vector<uint64_t>* off_out,
               std::string* defs_out, std::vector<uint64_t>* def_off_out);
int index_file_matches(const dbi_params& p, const char* path, bool* out);

// ---- error plumbing (dbi_engine.hip) ------------------------------------------------
int set_error(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Java (int) cast of a double (JLS 5.1.3), host+device.
__host__ __device__ inline int32_t java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
}

}  // namespace dbi

#define DBI_LAUNCH(KERNEL, GRID, BLOCK, SHMEM, STREAM, ...)                                                  \
    do {                                                                                                   \
        hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, STREAM, ::dbi::t_launch_ev.start,                \
                              ::dbi::t_launch_ev.stop, 0u, __VA_ARGS__);                                   \
        ::dbi::t_launch_ev.start = nullptr;                                                                \
    } while (0)

#define DBI_HIP(expr)                                          \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return ::dbi::hip_fail(_e, #expr); \
    } while (0)
