// dbi_engine.hip — host orchestration of the device build and queries behind
// the batch C-ABI (include/dbindex_hip.h).  One engine = one HIP device, one
// stream, an HBM-resident index and a workspace that grows but never shrinks
// (steady-state rebuilds allocate nothing).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <limits>
#include <cstdlib>
#include <string>
#include <thread>

#include <sys/mman.h>
#include <vector>

#include "dbi_engine.h"
#include "dbi_fasta.h"

namespace dbi {

static thread_local std::string g_err;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_err = std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ") in " + what;
    return e == hipErrorOutOfMemory ? DBI_E_OOM : DBI_E_HIP;
}

}  // namespace dbi

using namespace dbi;

namespace dbi {
thread_local LaunchEvents t_launch_ev;
}

namespace dbi {

int check_params(const dbi_params* p) {
    if (!p) return set_error(DBI_E_INVALID, "params is NULL");
    if (p->index_factor <= 0 || p->index_factor > MAX_PRECURSOR_INT)
        return set_error(DBI_E_INVALID, "index_factor must be in [1, 8000] (BUCKET_MASS_RANGE = 8000/index_factor)");
    if (!(p->min_mh >= 0.0)) return set_error(DBI_E_INVALID, "min precursor mass must be >= 0");
    if (!(p->max_mh == p->max_mh)) return set_error(DBI_E_INVALID, "max precursor mass is NaN");
    if (p->mass_group_factor <= 0) return set_error(DBI_E_INVALID, "mass_group_factor must be > 0");
    for (int c = 0; c < 256; ++c)
        if (!(p->mass[c] >= 0.0) || std::isinf(p->mass[c]))
            return set_error(DBI_E_INVALID, "residue masses must be finite and >= 0");
    return 0;
}

// every kept mass is >= max(minMH, m0) (residue masses are >= 0): the 16-B
// record encodes masses in [1, 65536) Da exactly (Rec)
int check_mass_floor(const dbi_params* p, double m0) {
    if (!(std::max(p->min_mh, m0) >= 1.0))
        return set_error(DBI_E_INVALID, "peptide masses below 1 Da are not supported (min precursor mass and "
                                        "H2O + proton + termini both < 1)");
    return 0;
}

DevParams make_dev_params(const dbi_params& p) {
    DevParams d{};
    d.min_mh = p.min_mh;
    d.max_mh = p.max_mh;
    // DBIndexer.java:265-271: precMass = 0; (+= H2O_PROTON); += cTerm; += nTerm
    volatile double m = 0;
    if (p.add_h2o_proton) m = m + p.h2o_proton;
    m = m + p.cterm;
    m = m + p.nterm;
    d.m0 = m;
    d.max_missed = p.max_missed;
    d.min_len = p.min_len;
    d.nb = p.index_factor;
    d.br = MAX_PRECURSOR_INT / p.index_factor;
    d.mand_mode = p.mandatory_mode ? 1 : 0;
    d.mand_filter = (p.mandatory_mode && p.mandatory_count > 0) ? 1 : 0;
    d.semi = p.semi ? 1 : 0;
    d.drop_mass = (double)(d.nb * d.br);
    d.buckets = 1;
    d.filter = 0;
    d.n_win = 0;
    d.win_max = INFINITY;
    d.win_lo = d.win_hi = nullptr;
    double mmax = 0.0;
    for (int c = 0; c < 256; ++c) mmax = std::max(mmax, p.mass[c]);
    d.cut_count = (!p.semi && !p.mandatory_mode && mmax < 1024.0) ? 1 : 0;  // fixed-point prefix tables fit u32
    return d;
}

// LSD digit widths over log2(nbins) bits: the first (lowest) digit takes the
// remainder, the others RADIX_BITS-wide digits; returns the number of passes
int radix_plan(uint32_t nbins, bool sparse, int* width) {
    int total = 0;
    while ((1ull << total) < nbins) ++total;
    const int passes = std::max((total + RADIX_BITS - 1) / RADIX_BITS, sparse ? 1 : 0);
    const int per = total ? (total + passes - 1) / passes : 0;
    for (int p = 0; p < passes; ++p) width[p] = p == 0 ? total - (passes - 1) * per : per;
    return passes;
}

uint32_t choose_nbins(uint64_t n, int max_bits) {
    uint64_t want = n / BIN_AVG;  // fine mass bins; chunks group them to ~CHUNK_T records
    uint32_t b = 1;
    while (b < want && b < (1u << max_bits)) b <<= 1;
    return b;
}

int log2_ceil(uint32_t x) {
    int r = 0;
    while ((1ull << r) < x) ++r;
    return r;
}

const char* ptm_device_msg() {
    return "inline '[formula]' PTMs in device-resident residues: digested only from host input (dbi_build), "
           "which strips and walks them (DBIndexer.java:288-303)";
}

int read_counters(dbi_handle* h) {
    DBI_HIP(hipMemcpyAsync(&h->hc, h->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    h->hc_final = false;
    return 0;
}

// Steps 4-6 over n records in recA: partition by mass bin, per-bin sort +
// dedup, finalize.  lo/hi bound every record mass.  sparse: recA holds n_in
// slots, n of them records and the rest REC_SENTINEL (bounded digest); the
// first radix pass leaves the sentinels behind.  Device-sized (d_n_in / d_n
// set: the counts the digest left on the device): n_in and n are upper bounds
// that size the grids and buffers, every kernel reads the real count itself,
// and n_est (the previous build's count) chooses the bins -- no host sync
// between the digest and the tail.
// Every buffer the tail over n records (n_in slots) uses; build_tail calls it
// before its first launch (a reallocation must never free a buffer that queued
// kernels still use), callers that time the tail call it first.
// records per chunk-sort block: DBI_CHUNK_T, else by the tail's size
uint32_t chunk_target(const dbi_handle* h, uint64_t n) {
    return h->chunk_t ? h->chunk_t : (uint32_t)(n >= CHUNK_T_MIN_RECS ? CHUNK_T : CHUNK_T_SMALL);
}

int tail_buffers(dbi_handle* h, uint64_t n, uint64_t n_in, bool sparse, int passes, int bits_per) {
    int rc;
    const uint32_t n_in32 = sparse ? (uint32_t)n_in : (uint32_t)n;
    const size_t hist_elems = passes ? radix_hist_elems(n_in32, bits_per) : 1;
    const uint32_t T = chunk_target(h, n);
    const uint32_t nchunks = (uint32_t)std::max<uint64_t>((n + T - 1) / T, 1);
    const size_t seg_cap = giant_seg_cap(n);
    const size_t scan_need = std::max(scan_u32_tmp_elems(hist_elems), scan_u32_tmp_elems(2 * (uint64_t)nchunks));
    if ((rc = h->scan_tmp.ensure(std::max<size_t>(scan_need, h->scan_tmp.cap)))) return rc;
    if ((rc = h->recB.ensure(n)) || (rc = h->hist.ensure(hist_elems)) ||
        (rc = h->ucount.ensure(2 * (size_t)nchunks)) || (rc = h->chunk_lo.ensure(2 * (size_t)nchunks + 1)) ||
        (rc = h->big_list.ensure(2 * (size_t)nchunks)) || (rc = h->mid_list.ensure(2 * MID_PER_PAIR * (size_t)nchunks)) ||
        (rc = h->giant_list.ensure(2 * (size_t)nchunks)) || (rc = h->segs.ensure((GIANT_PASSES + 4) * seg_cap)) ||
        (rc = h->ws_key.ensure(4 * n)) || (rc = h->ws_k2.ensure(4 * n)) ||
        (rc = h->umass.ensure(n)) || (rc = h->upid.ensure(n)) || (rc = h->uoff.ensure(n)) ||
        (rc = h->ulen.ensure(n)) || (rc = h->occ_off.ensure(n + 1)) || (rc = h->occ_pid.ensure(n)))
        return rc;
    // stable LSD passes over the bin id write the next pass's digit of each record
    if (passes > 1 && (rc = h->digits.ensure(std::max<uint64_t>(n, h->digits.cap)))) return rc;
    return 0;
}

int tail_buffers(dbi_handle* h, uint64_t n, uint64_t n_in, bool sparse) {
    int width[8] = {};
    const int passes = radix_plan(choose_nbins(n, h->bin_bits_max), sparse, width);
    return tail_buffers(h, n, n_in, sparse, passes, passes ? width[passes - 1] : 0);
}

int sort_chunks(dbi_handle* h, Rec* src, Rec* dst, const BinMap& bm, uint32_t nchunks, uint64_t n,
                const unsigned long long* d_n, bool est, bool local, bool big_listed = false);

int build_tail(dbi_handle* h, uint64_t n, double lo, double hi, uint64_t n_in, bool sparse,
               const unsigned long long* d_n_in, const unsigned long long* d_n, uint64_t n_est, bool est) {
    hipStream_t s = h->stream;
    int rc;
    const uint32_t n32 = (uint32_t)n;
    const uint32_t nbins = choose_nbins(d_n && n_est ? std::min(n_est, n) : n, h->bin_bits_max);
    const BinMap bm = make_binmap(lo, hi, nbins);
    int width[8] = {};
    const int passes = radix_plan(nbins, sparse, width);
    const int bits_per = passes ? width[passes - 1] : 0;  // the widest digit
    const uint32_t n_in32 = sparse ? (uint32_t)n_in : n32;
    const uint32_t T = chunk_target(h, n);
    const uint32_t nchunks = (uint32_t)std::max<uint64_t>((n + T - 1) / T, 1);
    if ((rc = tail_buffers(h, n, n_in, sparse, passes, bits_per))) return rc;

    // stable LSD passes over the bin id; every pass but the last writes the
    // next pass's digit of each record (1 B) next to its output, so the next
    // histogram reads bytes instead of records
    Rec* src = h->recA.p;
    Rec* dst = h->recB.p;
    int shift = 0;
    for (int ps = 0; ps < passes; ++ps) {
        const int bits = width[ps];
        const bool sp = sparse && ps == 0;
        const uint32_t nin = sp ? n_in32 : n32;
        const double hbytes = 8.0 * (double)radix_blocks(nin) * (double)(1u << bits);  // hist write + scan
        const unsigned long long* dn = sp ? d_n_in : d_n;
        if (ps == 0 && h->h1_on) {  // counted by the digest (warm_body) or the owner's expansion (dbi_shard_merge)
        } else if (ps == 0) {            // the 8-B mass of every record
            STAGE(h, "radix_hist", by(0, 8, 0, 0, 0),
                  launch_radix_hist(src, nin, bm, shift, bits, sp, h->hist.p, s, dn));
        } else {                         // the digit bytes of the previous pass
            STAGE(h, "radix_hist", by(0, 1, 0, 0, 0),
                  launch_radix_hist_u8(h->digits.p, nin, bits, h->hist.p, s, dn));
        }
        STAGE(h, "radix_scan", by(0, 0, 0, 0, 0),
              launch_scan_u32(h->hist.p, h->hist.p, (uint64_t)radix_blocks(nin) << bits, h->scan_tmp.p,
                              h->scan_tmp.cap, nullptr, s));
        h->stages[h->nstage - 1].cB = hbytes / std::max<double>(nbins, 1.0);
        // scatter moves 16 B in + 16 B out (+ 1 B next digit)
        const bool more = ps + 1 < passes;
        const int nbits = more ? width[ps + 1] : 0;
        STAGE(h, "radix_scatter", by(0, more ? 33 : 32, 0, 0, 0),
              launch_radix_scatter(src, dst, nin, bm, shift, bits, sp, h->hist.p, s, more ? h->digits.p : nullptr,
                                   shift + bits, nbits, dn));
        std::swap(src, dst);
        shift += bits;
    }
    // src: records grouped by bin, insertion order inside each bin
    // chunk sort: 16 B in + 16 B out per record (+ the residues of every peptide for its hash)
    STAGE(h, "chunk_bounds", by(0, 0, 0, 0, 0),
          launch_chunk_bounds(src, n32, bm, T, nchunks, h->chunk_lo.p, s, d_n));
    if ((rc = sort_chunks(h, src, dst, bm, nchunks, n, d_n, est, false))) return rc;
    h->stats.n_bins = nbins;
    return 0;
}

// The chunk sort tiers, the unique counts' scan and finalize over the chunk
// pairs in h->chunk_lo (src: records in bin order; the index from dst).
// local: depth-bin chunks (sort_chunk LOCAL; chunk_sort_mid sorts dst in place).
// the side stream and its fork / join events (created on first use)
int ensure_side(dbi_handle* h) {
    if (!h->side && hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess) {
        h->side = nullptr;
        return set_error(DBI_E_HIP, "hipStreamCreate (side stream) failed");
    }
    for (auto& ev : h->ev_side)
        if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
            return set_error(DBI_E_HIP, "hipEventCreate (side stream) failed");
        }
    return 0;
}

// big_listed (depth-bin tails): k_depth_chunks listed the chunks above
// CHUNK_CAP, so the big tier and the giant pass run on the side stream beside
// the chunk sort and the mid tier (forked after the chunk bounds, joined
// before the unique counts' scan): the big tier is ~420 blocks of one wave
// each at SwissProt scale, its time the slowest chunk's, and beside the chunk
// sort's ~30 k blocks it fills CUs instead of idling most of the chip.
int sort_chunks(dbi_handle* h, Rec* src, Rec* dst, const BinMap& bm, uint32_t nchunks, uint64_t n,
                const unsigned long long* d_n, bool est, bool local, bool big_listed) {
    hipStream_t s = h->stream;
    const uint32_t n32 = (uint32_t)n;
    const size_t seg_cap = giant_seg_cap(n);
    // depth bins: the split pairs' second chunks in front blocks (the previous
    // depth build's count + a margin; more, and the pairs' own blocks sort them)
    const uint32_t nfront = local && (est || d_n) && h->tail_local ? std::min(h->grid_split, nchunks) : 0u;
    // (the list grids below, from the previous build, are host values: computed first)
    // one block per listed bin (mid: every bin above the wave sort's reach) or
    // chunk (big: above CHUNK_CAP); the lists are filled on the device.  A device-sized tail
    // launches the previous build's list lengths plus a margin instead (a grid
    // of every possible entry spent most of these launches dispatching blocks
    // with nothing to do, the big tier's at one 155-KiB block per CU at a
    // time); a longer list sets ERR_GRID and the build is redone with full grids.
    uint32_t max_mid = (uint32_t)std::min<uint64_t>(MID_PER_PAIR * (uint64_t)nchunks, n / (WAVE_SORT_LIMIT + 1) + 1);
    uint32_t max_big = (uint32_t)std::min<uint64_t>(2 * (uint64_t)nchunks, n / (CHUNK_CAP + 1) + 1);
    // the list grids of the previous build hold for the same tail only (the
    // depth bins' chunks and lists differ from the radix tail's)
    est = (est || d_n) && h->tail_local == local;
    h->cur_local = local;
    // (a list that was empty last time is not launched at all: ~4 us of an
    // empty grid plus its launch gap; entries there redo the build as above)
    h->skip_mid = est && h->grid_mid == GRID_NONE;
    h->skip_big = est && h->grid_big == GRID_NONE;
    if (est && h->grid_mid) max_mid = h->skip_mid ? 0u : std::min(max_mid, h->grid_mid);
    if (est && h->grid_big) max_big = h->skip_big ? 0u : std::min(max_big, h->grid_big);
    // the giant-chunk pass (seven launches) only when the last build had giant
    // chunks: a giant chunk otherwise sets ERR_GRID and the build is redone
    const bool giants = !est || h->giants_seen;
    int rc;
    // (a big tier that is not launched -- its list was empty last build -- needs no fork)
    const bool fork = big_listed && max_big > 0;
    if (fork && (rc = ensure_side(h))) return rc;
    // beside the chunk sort the big tier takes its two size classes whatever
    // the list's length (the 512-thread, half-LDS blocks of the small class
    // interleave with the chunk sort's: SwissProt 3.40-3.43 -> 3.35-3.36 ms,
    // `profiles/r06bsp_big_split_ab.txt`); option big_split overrides
    const int big_split = h->big_split >= 0 ? h->big_split : fork ? 1 : -1;
    // the big tier (and the giant pass) on stream bs: the side stream, forked here, or the build's own after the mid tier
    auto big_tiers = [&](hipStream_t bs) -> int {
        h->stage_stream = bs;
        struct Reset {
            dbi_handle* h;
            ~Reset() { h->stage_stream = nullptr; }
        } reset{h};
        STAGE(h, "chunk_sort_big", by(0, 0, 0, 0, 0),
              launch_chunk_sort_big(src, dst, bm, h->chunk_lo.p, h->d_res, h->d_poff, h->ucount.p, h->big_list.p,
                                    giants ? h->giant_list.p : nullptr, max_big, h->split_above, h->exact_dups,
                                    h->ctr.p, bs, big_split, local));
        if (giants)
            STAGE(h, "chunk_sort_giant", by(0, 0, 0, 0, 0),
                  launch_giant_chunks(src, dst, h->chunk_lo.p, h->d_res, h->d_poff, h->ucount.p, h->giant_list.p,
                                      h->segs.p, seg_cap, h->ws_key.p, h->ws_k2.p, h->ctr.p, bs));
        return 0;
    };
    if (fork) {
        DBI_HIP(hipEventRecord(h->ev_side[0], s));
        DBI_HIP(hipStreamWaitEvent(h->side, h->ev_side[0], 0));
        if ((rc = big_tiers(h->side))) return rc;
        DBI_HIP(hipEventRecord(h->ev_side[1], h->side));
    }
    STAGE(h, "chunk_sort", by(0, 32, 0, 0, 0),
          launch_chunk_sort(src, dst, bm, h->chunk_lo.p, nchunks, h->d_res, h->d_poff, h->ucount.p, h->big_list.p,
                            h->mid_list.p, h->exact_dups, h->ctr.p, s, local, local ? h->split_list.p : nullptr,
                            nfront, big_listed));
    STAGE(h, "chunk_sort_mid", by(0, 0, 0, 0, 0),
          launch_chunk_sort_mid(local ? dst : src, dst, bm, h->chunk_lo.p, h->d_res, h->d_poff, h->ucount.p,
                                h->mid_list.p, max_mid, h->ctr.p, s));
    if (fork) DBI_HIP(hipStreamWaitEvent(s, h->ev_side[1], 0));  // join
    else if ((rc = big_tiers(s))) return rc;
    // unique offsets per chunk
    STAGE(h, "ucount_scan", by(0, 0, 0, 0, 0),
          launch_scan_u32(h->ucount.p, h->ucount.p, 2 * (uint64_t)nchunks, h->scan_tmp.p, h->scan_tmp.cap,
                          &h->ctr.p->n_unique, s));
    // finalize: 16 B record in, 4 B occurrence protein id out, 24 B per unique out
    STAGE(h, "finalize", by(0, 20, 24, 0, 0),
          launch_finalize(dst, h->chunk_lo.p, nchunks, h->ucount.p, h->umass.p, h->upid.p, h->uoff.p, h->ulen.p,
                          h->occ_off.p, h->occ_pid.p, h->params.mass_group_factor,
                          (uint32_t)std::min<size_t>(h->umass.cap, 0xFFFFFFFFu), 2u, n32, d_n, h->ctr.p, s));
    return 0;
}

// did the last tail's chunk lists outgrow their grids (a launched list kernel
// sets ERR_GRID; a list not launched because it was empty last time must be
// empty again)?
bool chunk_lists_short(const dbi_handle* h) {
    return (h->hc.err & ERR_GRID) || (h->skip_mid && h->hc.n_mid) || (h->skip_big && h->hc.n_big);
}

int finish_build(dbi_handle* h) {
    int rc = h->hc_final ? 0 : read_counters(h);  // a device-sized build has read them after its last kernel
    if (rc) return rc;
    if (h->hc.err & ERR_SEGS) return set_error(DBI_E_STATE, "internal: giant-chunk segment list overflow");
    if (h->hc.err & ERR_SLOTS) return set_error(DBI_E_STATE, "internal: digest slot bound exceeded");
    if (h->hc.err & ERR_PTM) return set_error(DBI_E_INVALID, ptm_device_msg());
    if (h->hc.err & ERR_LAYOUT)
        return set_error(DBI_E_INVALID, "2 x bits(longest protein) + bits(protein count) exceeds the 56 bits of the "
                                        "16-B occurrence record: shard the FASTA");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h->t0).count();
    dbi_stats& st = h->stats;
    st.n_residues = h->n_res;
    st.n_proteins = h->n_prot;
    st.n_kept = h->hc.n_kept;
    st.n_dropped = h->hc.n_dropped + h->n_total_extra;
    st.n_total = st.n_kept + st.n_dropped;
    st.n_unique = h->hc.n_unique;
    st.n_keys = h->hc.n_keys;
    for (int i = 0; i < 8; ++i) st.n_keys += h->hc.n_keys_shard[i];
    st.n_big_bins = h->hc.n_big;  // chunks above CHUNK_CAP (of which n_giant above BIG_CAP)
    st.build_ms = ms;
    st.digest_ms = 0;
    for (int i = 0; i < h->nstage; ++i) {
        auto& sg = h->stages[i];
        float t = 0;
        if (!sg.launched || hipEventElapsedTime(&t, h->evpool[sg.eb], h->evpool[sg.ee]) != hipSuccess) t = 0;
        sg.ms = t;
        if (std::strncmp(sg.name, "digest", 6) == 0) st.digest_ms += t;
        sg.bytes = sg.cR * (double)h->n_res + sg.cN * (double)st.n_kept + sg.cU * (double)st.n_unique +
                   sg.cP * (double)(h->n_prot + 1) + sg.cB * (double)st.n_bins + sg.c0;
        // the chunk-sort tiers split the records: 16 B in + 16 B out each, in the tier that sorted it
        // (chunk_sort's read of a chunk it hands to the mid tier is overhead, not credited)
        const double big = (double)h->hc.n_big_recs, giant = (double)h->hc.n_giant_recs;
        const double mid = (double)h->hc.n_mid_recs;
        if (std::strcmp(sg.name, "chunk_sort") == 0)
            sg.bytes = 32.0 * std::max(0.0, (double)st.n_kept - mid - big - giant);
        else if (std::strcmp(sg.name, "chunk_sort_mid") == 0) sg.bytes = 32.0 * mid;
        else if (std::strcmp(sg.name, "chunk_sort_big") == 0) sg.bytes = 32.0 * big;
        else if (std::strcmp(sg.name, "chunk_sort_giant") == 0) sg.bytes = 32.0 * giant;
    }
    size_t bytes = 0;
    bytes += h->res.bytes() + h->poff64.bytes() + h->poff.bytes() + h->poff_g.bytes() + h->blk.bytes() + h->scan_tmp.bytes();
    bytes += h->thr.bytes() + h->tile_pf.bytes() + h->chunk_lo.bytes();
    bytes += h->recA.bytes() + h->recB.bytes() + h->hist.bytes() + h->ucount.bytes();
    bytes += h->big_list.bytes() + h->mid_list.bytes() + h->giant_list.bytes() + h->segs.bytes() + h->ws_key.bytes() + h->ws_k2.bytes() + h->umass.bytes() + h->upid.bytes();
    bytes += h->uoff.bytes() + h->ulen.bytes() + h->occ_off.bytes() + h->occ_pid.bytes();
    // the digest's regions and the depth-bin plan (they were left out)
    bytes += h->recR.bytes() + h->rdig.bytes() + h->rcur.bytes() + h->dsub.bytes() + h->dpre.bytes() + h->desc.bytes();
    bytes += h->d1c.bytes() + h->hist2.bytes() + h->bstart.bytes() + h->split_list.bytes() + h->dmap.bytes();
    bytes += h->dheavy.bytes() + h->digits.bytes();
    st.device_bytes = bytes;
    h->built = true;
    h->last_kept = st.n_kept;
    h->prev_unique = st.n_unique;
    // the next device-sized tail's list grids: this build's lists plus a
    // margin, or no launch for an empty list
    h->lists_short = chunk_lists_short(h);
    h->grid_mid = h->hc.n_mid ? h->hc.n_mid + h->hc.n_mid / 8 + 32 : GRID_NONE;
    h->grid_big = h->hc.n_big ? h->hc.n_big + h->hc.n_big / 8 + 16 : GRID_NONE;
    h->grid_split = h->cur_local ? h->hc.n_split + h->hc.n_split / 8 + 32 : 0u;
    h->giants_seen = h->hc.n_giant > 0;
    h->tail_local = h->cur_local;
    h->force_cold = false;
    ++h->build_serial;
    return 0;
}

// per-tile first-protein table (digest tiles) + the longest protein (record layout)
int prepare_tiles(dbi_handle* h) {
    const uint32_t ntiles = (uint32_t)((h->n_res + DIGEST_TILE - 1) / DIGEST_TILE);
    int rc;
    if ((rc = h->tile_pf.ensure(2 * ((size_t)ntiles + 2)))) return rc;  // first + last protein of every tile
    // (a partitioning digest's region cursors are zeroed by the same kernel)
    STAGE(h, "tile_proteins", by(0, 0, 0, 4, 0),
          launch_tile_proteins(h->d_poff, (uint32_t)h->n_prot, (uint32_t)h->n_res, h->tile_pf.p, h->ctr.p,
                               h->stream, h->part_now ? h->part_now->cur : nullptr, DEPTH_XCDS * 256));
    return 0;
}

// Warm builds digest into bounded slots: the lean kernel (full enzyme, no
// mandatory residues, <= 2 missed cleavages) or the semi-specific one (no
// mandatory residues); both without the unindexed search's windows.
bool lean_digest(const dbi_handle* h) {
    return !h->dp.semi && !h->dp.mand_mode && h->dp.max_missed <= 2 && !h->dp.filter;
}
bool bounded_digest(const dbi_handle* h) {
    return lean_digest(h) || (h->dp.semi && !h->dp.mand_mode && !h->dp.filter && h->use_semi_bounded);
}

// Device digest over residues at d_res (n_res) with u32 offsets at h->d_poff.
// Warm builds with dev_sized: the digest into the previous build's capacity,
// and no host sync: *n = *n_in = that capacity (upper bounds), *dev_sized set;
// the caller checks the real need once the whole build has run (build_digest).
int run_digest(dbi_handle* h, uint64_t* n_out, uint64_t* n_in_out, bool* sparse_out, bool* dev_sized) {
    hipStream_t s = h->stream;
    int rc;
    const uint64_t R = h->n_res;
    const uint32_t nblk = (uint32_t)((R + DIGEST_TILE - 1) / DIGEST_TILE);
    if ((rc = h->blk.ensure(std::max<uint32_t>(nblk, 1))) || (rc = h->thr.ensure((size_t)nblk * DIGEST_THREADS + 1)))
        return rc;
    if ((rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(nblk), h->scan_tmp.cap)))) return rc;
    if ((rc = prepare_tiles(h))) return rc;
    uint64_t n;
    // full enzyme, no mandatory residues, <= 2 missed cleavages: one walk into
    // per-tile reservations of exactly each start's candidate ends
    const bool lean = lean_digest(h), bounded = bounded_digest(h);
    // cold builds of a bounded digest take the same pass: a first attempt into
    // no capacity is its slot count (every tile reserves its bound and stops
    // before its walks: the bit maps, no mass walk), then the pass into that
    // (SwissProt: 0.3 + 0.85 ms instead of the count and emit walks' 0.7 + 2.1)
    const bool cold = h->recA.cap < 1024 || h->force_cold;
    if (!cold || (bounded && !dev_sized)) {
        // warm: one pass into the capacity of the previous build; the exact
        // need comes back with the counters, and a short buffer is grown and
        // the pass run again
        if (!bounded && (rc = h->status.ensure_zeroed(nblk, s))) return rc;
        const bool dev = dev_sized != nullptr;
        for (int attempt = 0;; ++attempt) {
            if (!bounded && ++h->epoch >= 0xFFFFu) {
                DBI_HIP(hipMemsetAsync(h->status.p, 0, sizeof(unsigned long long) * h->status.cap, s));
                h->epoch = 1;
            }
            const uint64_t cap = cold && attempt == 0 ? 0 : std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
            const char* stage = cold && attempt == 0 ? "digest_slots" : "digest";
            if (bounded && !lean)
                STAGE(h, stage, by(1, h->part_now ? 17 : 16, 0, 4, 0),
                      launch_digest_semi_bounded(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff,
                                                 (uint32_t)h->n_prot, (uint32_t)R, h->tile_pf.p, h->recA.p, cap,
                                                 h->ctr.p, s, dev_sized ? h->part_now : nullptr));
            else if (bounded)
                STAGE(h, stage, by(1, h->part_now ? 17 : 16, 0, 4, 0),
                      launch_digest_bounded(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff,
                                            (uint32_t)h->n_prot, (uint32_t)R, h->tile_pf.p, h->recA.p, cap, h->ctr.p,
                                            s, dev_sized && h->h1_on ? &h->h1plan : nullptr,
                                            dev_sized ? h->part_now : nullptr));
            else
                STAGE(h, "digest", by(1, 16, 0, 4, 0),
                      launch_digest_fused(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff,
                                          (uint32_t)h->n_prot, (uint32_t)R, h->tile_pf.p, h->status.p, h->epoch,
                                          h->recA.p, (uint32_t)cap, h->ctr.p, s));
            if (dev) {  // no sync: the tail runs on device counts, checked after the build
                *n_out = cap;
                *n_in_out = cap;
                *sparse_out = bounded;
                *dev_sized = true;
                return 0;
            }
            if ((rc = read_counters(h))) return rc;
            n = h->hc.n_kept;
            const uint64_t need = bounded ? std::max<uint64_t>(h->hc.n_slots, n) : n;
            if (need >= (1ull << 32) - 1)
                return set_error(DBI_E_INVALID, "more than 2^32-2 peptide occurrences (or bounded-digest slots) on "
                                                "one device: shard the FASTA");
            if (need <= cap) break;
            if (attempt > 0) return set_error(DBI_E_STATE, "digest output grew between identical passes");
            if ((rc = h->recA.ensure(need + need / 8))) return rc;
            // counters back to zero, except the record layout (max_plen) set by prepare_tiles
            DBI_HIP(hipMemsetAsync(h->ctr.p, 0, offsetof(Counters, max_plen), s));
        }
        if (bounded) {
            *n_out = n;
            *n_in_out = h->hc.n_slots;
            *sparse_out = true;
            return 0;
        }
    } else {
        // cold: count, scan, size the output, emit
        STAGE(h, "digest_count", by(1, 0, 0, 4, 0),
              launch_digest_count(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff, (uint32_t)h->n_prot,
                                  (uint32_t)R, h->tile_pf.p, h->blk.p, h->thr.p, h->ctr.p, s));
        STAGE(h, "digest_scan", by(0, 0, 0, 0, 0),
              launch_scan_u32(h->blk.p, h->blk.p, nblk, h->scan_tmp.p, h->scan_tmp.cap, &h->ctr.p->n_kept, s));
        if ((rc = read_counters(h))) return rc;
        n = h->hc.n_kept;
        if (n >= (1ull << 32) - 1)
            return set_error(DBI_E_INVALID, "more than 2^32-2 peptide occurrences on one device: shard the FASTA");
        if ((rc = h->recA.ensure(n))) return rc;
        // digest emit: residues in, one 16-B record per kept occurrence out
        STAGE(h, "digest_emit", by(1, 16, 0, 4, 0),
              launch_digest_emit(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff, (uint32_t)h->n_prot,
                                 (uint32_t)R, h->tile_pf.p, h->blk.p, h->thr.p, h->recA.p, h->ctr.p, s));
    }
    *n_out = n;
    *n_in_out = n;
    *sparse_out = false;
    return 0;
}

// Depth bins of a warm lean build: 2^B bins of about
// DEPTH_BIN_AVG records each -- the high b1 bits partitioned by the digest into
// (digit, XCD) regions, the low b2 by one radix pass -- then chunks of whole
// bins, binned again in LDS by the chunk sort.  Replaces the radix tail's
// first histogram and two of its three full passes over the records.
constexpr uint64_t DEPTH_BIN_AVG = 768;     // records per depth bin (~1 chunk-sort chunk per 2 bins)
constexpr uint64_t DEPTH_MIN_RECS = 1u << 14;
#ifndef DBI_DEPTH_SAMPLES
#define DBI_DEPTH_SAMPLES (1u << 19)
#endif
constexpr uint32_t DEPTH_SAMPLES = DBI_DEPTH_SAMPLES;  // uniques of the previous index sampled for the map
// the bins and regions of a depth-bin tail over about n records (slots: the
// record buffers' capacity)
DepthPlan depth_plan_n(const dbi_handle* h, uint64_t n, uint64_t slots) {
    DepthPlan p;
    if (n < DEPTH_MIN_RECS || slots < 1024) return p;
    int B = 9;
    while (B < 16 && (DEPTH_BIN_AVG << (B + 1)) <= n) ++B;
    p.b1 = (uint32_t)std::max(1, std::min(8, B - 8));  // the pass over the low digit: 8 bits when B >= 9
    p.b2 = (uint32_t)B - p.b1;
    p.nbins = 1u << B;
    p.nreg = (1u << p.b1) * DEPTH_XCDS;
    const double share = (double)n / (double)p.nreg * h->depth_slack;
    p.cap = (uint32_t)std::min<double>((share + 256.0 + 63.0) / 64.0, (double)(1u << 26)) * 64u;
    if ((uint64_t)p.nreg * p.cap >= (1ull << 32) - 1 || p.cap / PART_CHUNK >= 65536u) return DepthPlan{};
    p.max_chunks = (uint32_t)std::min<uint64_t>((uint64_t)p.nreg * ((p.cap + PART_CHUNK - 1) / PART_CHUNK),
                                                 slots / PART_CHUNK + p.nreg);
    p.on = true;
    return p;
}

DepthPlan depth_plan(const dbi_handle* h) {
    if (!h->use_depth || h->depth_off || !lean_digest(h) || h->prev_unique == 0) return DepthPlan{};
    return depth_plan_n(h, h->last_kept, std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull));
}

// the map of the last depth build still fits: sampled from an index of the
// same size (the previous build's, the one this build would sample), for the
// same bin count and sub-bin range.  The map is a plan, never a result (any
// monotone map gives the exact index): it is sampled again when the index
// changes size, after a region overflow, and on cold builds; option
// depth_map_reuse=0 samples every build (0.08 ms at SwissProt scale).
bool depth_map_reusable(const dbi_handle* h, uint32_t nbins, const BinMap& sub) {
    return h->opt_depth_map_reuse && h->depth_map_of != nullptr && h->depth_map_of == h->dmap.p &&
           h->prev_unique != 0 && h->depth_map_unique == h->prev_unique && h->depth_map_nbins == nbins &&
           h->depth_map_lo == sub.lo && h->depth_map_scale == sub.scale;
}
bool depth_map_reusable(const dbi_handle* h, uint32_t nbins) {
    return depth_map_reusable(h, nbins, make_binmap(h->params.min_mh, h->params.max_mh, 1u << DEPTH_SUB_BITS));
}

// every buffer of a depth-bin tail past the record buffers (tail_buffers)
int depth_buffers(dbi_handle* h, const DepthPlan& pl, uint32_t nchunks) {
    const uint64_t nreg_slots = (uint64_t)pl.nreg * pl.cap;
    int rc;
    if ((rc = h->recR.ensure(nreg_slots)) || (rc = h->rdig.ensure(nreg_slots + 16)) ||
        (rc = h->rcur.ensure(DEPTH_XCDS * 256)) || (rc = h->dsub.ensure(DEPTH_SAMPLES)) ||
        (rc = h->dpre.ensure(DEPTH_SAMPLES)) || (rc = h->dmap.ensure((1u << DEPTH_SUB_BITS) / 64)) ||
        (rc = h->dheavy.ensure_zeroed(1, h->stream)) || (rc = h->desc.ensure(pl.max_chunks)) ||
        (rc = h->d1c.ensure(512)) || (rc = h->hist2.ensure((size_t)pl.max_chunks << pl.b2)) ||
        (rc = h->bstart.ensure(pl.nbins + 1)) || (rc = h->split_list.ensure(nchunks)) ||
        (rc = h->scan_tmp.ensure(std::max({scan_u32_tmp_elems(DEPTH_SAMPLES),
                                           scan_u32_tmp_elems((uint64_t)pl.max_chunks << pl.b2), h->scan_tmp.cap}))))
        return rc;
    return 0;
}

// the map over sub's sub-bins, sampled from the resident index's U uniques
int depth_map_enqueue(dbi_handle* h, const DepthPlan& pl, const BinMap& sub, uint64_t U) {
    hipStream_t s = h->stream;
    const uint32_t nsub = 1u << DEPTH_SUB_BITS;
    const uint32_t ns = (uint32_t)std::min<uint64_t>(DEPTH_SAMPLES, U);
    DBI_HIP(hipMemsetAsync(h->dmap.p, 0, sizeof(uint4) * (nsub / 64), s));
    STAGE(h, "depth_map", by(0, 0, 0, 0, 0), ([&]() -> hipError_t {
              hipError_t e = launch_depth_sample(h->umass.p, h->occ_off.p, U, ns, sub, h->dsub.p, h->dpre.p, s);
              if (e == hipSuccess)
                  e = launch_scan_u32(h->dpre.p, h->dpre.p, ns, h->scan_tmp.p, h->scan_tmp.cap, &h->ctr.p->depth_w, s);
              return e == hipSuccess
                         ? launch_depth_map(h->dsub.p, h->dpre.p, ns, pl.nbins, nsub, h->dmap.p, h->dheavy.p, h->ctr.p, s)
                         : e;
          }()));
    h->depth_map_of = h->dmap.p;
    h->depth_map_unique = h->prev_unique;
    h->depth_map_nbins = pl.nbins;
    h->depth_map_lo = sub.lo;
    h->depth_map_scale = sub.scale;
    return 0;
}

// the regions (filled: the digest's or the owner expansion's partition) ->
// one radix pass over the low digit into bin order (recA), the chunks of whole
// bins, the chunk sort and finalize over cap record slots (the records: the
// device count ctr->tail_n, 0 when a region overflowed)
int depth_tail(dbi_handle* h, const DepthPlan& pl, const BinMap& sub, uint64_t cap, uint32_t T, uint32_t nchunks,
               bool est) {
    hipStream_t s = h->stream;
    STAGE(h, "part_plan", by(0, 0, 0, 0, 0),
          launch_part_plan(h->rcur.p, pl.cap, pl.b1, cap, h->desc.p, h->d1c.p, h->ctr.p, s));
    STAGE(h, "part_hist", by(0, 1, 0, 0, 0),
          launch_part_hist(h->rdig.p, h->rcur.p, pl.cap, h->desc.p, h->d1c.p, pl.b1, pl.b2, pl.max_chunks, h->hist2.p,
                           h->ctr.p, s));
    STAGE(h, "part_scan", by(0, 0, 0, 0, 0),
          launch_scan_u32(h->hist2.p, h->hist2.p, (uint64_t)pl.max_chunks << pl.b2, h->scan_tmp.p, h->scan_tmp.cap,
                          nullptr, s));
    STAGE(h, "bin_scatter", by(0, 33, 0, 0, 0),
          launch_part_scatter(h->recR.p, h->rdig.p, h->rcur.p, pl.cap, h->desc.p, h->d1c.p, pl.b1, pl.b2,
                              pl.max_chunks, h->hist2.p, h->recA.p, h->ctr.p, s));
    // the big tier beside the chunk sort (sort_chunks); not when every stage is
    // timed: the per-stage breakdown's event spans would overlap (the big
    // tier's span then covers the chunk sort's), so such builds serialise
    const bool big_side = h->opt_big_side && !(h->timing && h->timing_only.empty());
    STAGE(h, "chunk_bounds", by(0, 0, 0, 0, 0),
          launch_depth_bounds(h->hist2.p, h->d1c.p, pl.b1, pl.b2, h->bstart.p, T, nchunks, h->chunk_lo.p, h->ctr.p, s,
                              h->split_list.p, big_side ? h->big_list.p : nullptr));
    int rc;
    if ((rc = sort_chunks(h, h->recA.p, h->recB.p, sub, nchunks, cap, &h->ctr.p->tail_n, est, true, big_side)))
        return rc;
    h->stats.n_bins = pl.nbins;
    return 0;
}

// Warm semi-specific builds: the radix tail's first
// LSD pass -- its histogram over the sparse slots and its scatter, two full
// passes over 16-B records -- fused into the digest: each tile partitions its
// records by the low digit (b1 bits) of their linear fine bin into (digit,
// XCD) regions (part_tile, PartOut::lsd), one pass over the regions by the
// second digit (k_part_hist / k_part_scatter, digit-major: a stable LSD pass)
// writes them dense, with each record's third digit beside it, and the radix
// tail goes on from its third pass.  Any order inside a digit is fine for an
// LSD pass; the chunk sort orders every bin by the full record key.
constexpr uint64_t LSD_MIN_RECS = 1u << 16;
struct LsdPlan {
    bool on = false;
    uint32_t nbins = 0, b1 = 0, b2 = 0, cap = 0, nreg = 0, max_chunks = 0;
    int passes = 0;
    int width[8] = {};
};

LsdPlan lsd_plan(const dbi_handle* h) {
    LsdPlan p;
    const uint64_t n = h->last_kept, slots = std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
    if (!h->use_semi_part || h->depth_off || !h->dp.semi || lean_digest(h) || !bounded_digest(h) ||
        n < LSD_MIN_RECS || slots < 1024)
        return p;
    p.nbins = choose_nbins(std::min(n, slots), h->bin_bits_max);  // build_tail's bins (n_est = the last count)
    p.passes = radix_plan(p.nbins, true, p.width);
    if (p.passes < 2 || p.width[0] < 1 || p.width[0] > 8 || p.width[1] < 1 || p.width[1] > RADIX_BITS) return LsdPlan{};
    p.b1 = (uint32_t)p.width[0];
    p.b2 = (uint32_t)p.width[1];
    p.nreg = (1u << p.b1) * DEPTH_XCDS;
    const double share = (double)n / (double)p.nreg * h->lsd_slack;
    p.cap = (uint32_t)std::min<double>((share + 256.0 + 63.0) / 64.0, (double)(1u << 26)) * 64u;
    if ((uint64_t)p.nreg * p.cap >= (1ull << 32) - 1 || p.cap / PART_CHUNK >= 65536u) return LsdPlan{};
    p.max_chunks = (uint32_t)std::min<uint64_t>((uint64_t)p.nreg * ((p.cap + PART_CHUNK - 1) / PART_CHUNK),
                                                 slots / PART_CHUNK + p.nreg);
    p.on = true;
    return p;
}

int warm_body_lsd(dbi_handle* h, const LsdPlan& pl, uint64_t* n_in, bool* sparse) {
    hipStream_t s = h->stream;
    int rc;
    const uint64_t cap = std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
    const uint32_t cap32 = (uint32_t)cap;
    const uint64_t nreg_slots = (uint64_t)pl.nreg * pl.cap;
    const uint32_t ntiles = (uint32_t)((h->n_res + DIGEST_TILE - 1) / DIGEST_TILE);
    const BinMap bm = make_binmap(h->params.min_mh, h->params.max_mh, pl.nbins);
    const uint32_t T = chunk_target(h, cap);
    const uint32_t nchunks = (uint32_t)std::max<uint64_t>((cap + T - 1) / T, 1);
    // every allocation before the first launch
    if ((rc = tail_buffers(h, cap, cap, true, pl.passes, pl.width[pl.passes - 1])) ||
        (rc = h->recR.ensure(nreg_slots)) || (rc = h->rdig.ensure(nreg_slots + 16)) ||
        (rc = h->rcur.ensure(DEPTH_XCDS * 256)) || (rc = h->desc.ensure(pl.max_chunks)) || (rc = h->d1c.ensure(512)) ||
        (rc = h->hist2.ensure((size_t)pl.max_chunks << pl.b2)) || (rc = h->blk.ensure(std::max<uint32_t>(ntiles, 1))) ||
        (rc = h->thr.ensure((size_t)ntiles * DIGEST_THREADS + 1)) || (rc = h->tile_pf.ensure(2 * ((size_t)ntiles + 2))) ||
        (rc = h->scan_tmp.ensure(std::max({scan_u32_tmp_elems((uint64_t)pl.max_chunks << pl.b2),
                                           scan_u32_tmp_elems(ntiles), h->scan_tmp.cap}))))
        return rc;
    PartOut po{};
    po.recs = h->recR.p;
    po.dig = h->rdig.p;
    po.cur = h->rcur.p;
    po.dm.b2 = pl.b2;
    po.cap = pl.cap;
    po.b1 = pl.b1;
    po.lsd = 1;
    po.lin = bm;
    h->part_now = &po;
    uint64_t n = 0;
    bool dev = false;
    rc = run_digest(h, &n, n_in, sparse, &dev);
    h->part_now = nullptr;
    if (rc) return rc;
    if (!dev) return set_error(DBI_E_STATE, "internal: warm build without device sizing");
    const unsigned long long* d_n = &h->ctr.p->tail_n;  // k_part_plan: the records, 0 when anything overflowed
    // the second LSD pass, region by region, into recA (dense), with the third digit of each record
    const int nshift = pl.width[0] + pl.width[1], nbits = pl.passes > 2 ? pl.width[2] : 0;
    STAGE(h, "part_plan", by(0, 0, 0, 0, 0),
          launch_part_plan(h->rcur.p, pl.cap, pl.b1, cap, h->desc.p, h->d1c.p, h->ctr.p, s));
    STAGE(h, "part_hist", by(0, 1, 0, 0, 0),
          launch_part_hist(h->rdig.p, h->rcur.p, pl.cap, h->desc.p, h->d1c.p, pl.b1, pl.b2, pl.max_chunks, h->hist2.p,
                           h->ctr.p, s, true));
    STAGE(h, "part_scan", by(0, 0, 0, 0, 0),
          launch_scan_u32(h->hist2.p, h->hist2.p, (uint64_t)pl.max_chunks << pl.b2, h->scan_tmp.p, h->scan_tmp.cap,
                          nullptr, s));
    STAGE(h, "bin_scatter", by(0, nbits ? 33 : 32, 0, 0, 0),
          launch_part_scatter(h->recR.p, h->rdig.p, h->rcur.p, pl.cap, h->desc.p, h->d1c.p, pl.b1, pl.b2,
                              pl.max_chunks, h->hist2.p, h->recA.p, h->ctr.p, s, true,
                              nbits ? h->digits.p : nullptr, bm, (uint32_t)nshift, (uint32_t)nbits));
    // the radix tail's remaining passes (build_tail's, from the third)
    Rec* src = h->recA.p;
    Rec* dst = h->recB.p;
    int shift = nshift;
    for (int ps = 2; ps < pl.passes; ++ps) {
        const int bits = pl.width[ps];
        const double hbytes = 8.0 * (double)radix_blocks(cap32) * (double)(1u << bits);
        STAGE(h, "radix_hist", by(0, 1, 0, 0, 0), launch_radix_hist_u8(h->digits.p, cap32, bits, h->hist.p, s, d_n));
        STAGE(h, "radix_scan", by(0, 0, 0, 0, 0),
              launch_scan_u32(h->hist.p, h->hist.p, (uint64_t)radix_blocks(cap32) << bits, h->scan_tmp.p,
                              h->scan_tmp.cap, nullptr, s));
        h->stages[h->nstage - 1].cB = hbytes / std::max<double>(pl.nbins, 1.0);
        const bool more = ps + 1 < pl.passes;
        const int nb = more ? pl.width[ps + 1] : 0;
        STAGE(h, "radix_scatter", by(0, more ? 33 : 32, 0, 0, 0),
              launch_radix_scatter(src, dst, cap32, bm, shift, bits, false, h->hist.p, s, more ? h->digits.p : nullptr,
                                   shift + bits, nb, d_n));
        std::swap(src, dst);
        shift += bits;
    }
    STAGE(h, "chunk_bounds", by(0, 0, 0, 0, 0),
          launch_chunk_bounds(src, cap32, bm, T, nchunks, h->chunk_lo.p, s, d_n));
    if ((rc = sort_chunks(h, src, dst, bm, nchunks, cap, d_n, false, false))) return rc;
    h->stats.n_bins = pl.nbins;
    return 0;
}

dbi_handle::GraphKey graph_key(const dbi_handle* h) {
    dbi_handle::GraphKey k{};
    k.d_res = h->d_res;
    k.d_poff = h->d_poff;
    k.n_res = h->n_res;
    k.n_prot = h->n_prot;
    k.cap = h->recA.cap;
    k.last_kept = h->last_kept;
    k.grid_mid = h->grid_mid;
    k.grid_big = h->grid_big;
    k.grid_split = h->grid_split;
    k.prev_unique = h->prev_unique;
    k.tail_local = h->tail_local;
    const DepthPlan dpl = depth_plan(h);
    k.depth_cap = dpl.on ? dpl.cap : 0u;
    k.depth_fresh = dpl.on && !depth_map_reusable(h, dpl.nbins);
    const LsdPlan lpl = lsd_plan(h);
    k.lsd_cap = lpl.on ? lpl.cap : 0u;
    k.giants = h->giants_seen;
    k.alloc_gen = g_alloc_gen.load(std::memory_order_relaxed);
    k.dp_gen = h->dp_gen;
    k.timing = h->timing;
    std::strncpy(k.timing_only, h->timing_only.c_str(), sizeof(k.timing_only) - 1);
    return k;
}

void drop_graph(dbi_handle* h) {
    if (h->bgraph.exec) (void)hipGraphExecDestroy(h->bgraph.exec);
    if (h->bgraph.graph) (void)hipGraphDestroy(h->bgraph.graph);
    h->bgraph.exec = nullptr;
    h->bgraph.graph = nullptr;
    if (h->mgraph.exec) (void)hipGraphExecDestroy(h->mgraph.exec);
    if (h->mgraph.graph) (void)hipGraphDestroy(h->mgraph.graph);
    h->mgraph.exec = nullptr;
    h->mgraph.graph = nullptr;
    h->prev_mkey_valid = false;
}

// DEPTH_FALLBACK: no map to use (the index it samples was reallocated on the
// way here and no earlier map is in place): the caller runs the radix tail
constexpr int DEPTH_FALLBACK = 1;
constexpr double SLACK_MIN = 1.25;  // region room / the region's share of the previous build's records
constexpr int SLACK_DECAY = 8;      // builds without an overflow before the room is halved back toward SLACK_MIN

int warm_body_depth(dbi_handle* h, const DepthPlan& pl, bool index_kept, uint64_t* n_in, bool* sparse) {
    int rc;
    const uint64_t cap = std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
    const uint32_t T = h->chunk_t ? h->chunk_t : cap >= CHUNK_T_MIN_RECS ? (uint32_t)CHUNK_T_DEPTH : chunk_target(h, cap);
    const uint32_t nchunks = (uint32_t)std::max<uint64_t>((cap + T - 1) / T, 1);
    const uint32_t ntiles = (uint32_t)((h->n_res + DIGEST_TILE - 1) / DIGEST_TILE);
    // every allocation before the first launch (a reallocation must never free
    // a buffer that queued kernels use): the tail's (chunk sort, index), the
    // depth bins', the digest's (run_digest finds them in place)
    if ((rc = tail_buffers(h, cap, cap, true)) || (rc = depth_buffers(h, pl, nchunks)) ||
        (rc = h->blk.ensure(std::max<uint32_t>(ntiles, 1))) ||
        (rc = h->thr.ensure((size_t)ntiles * DIGEST_THREADS + 1)) || (rc = h->tile_pf.ensure(2 * ((size_t)ntiles + 2))) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(ntiles), h->scan_tmp.cap))))
        return rc;
    // the map, from a sample of the resident index (the previous build's)
    const uint64_t U = std::min<uint64_t>({h->prev_unique, h->umass.cap, h->occ_off.cap ? h->occ_off.cap - 1 : 0});
    const BinMap sub = make_binmap(h->params.min_mh, h->params.max_mh, 1u << DEPTH_SUB_BITS);
    // a redo keeps the map its first attempt computed (that attempt may have
    // overwritten the index, or the redo's larger buffers moved it); any
    // complete map is monotone in the mass, so it is exact, only its balance
    // may be off
    const bool keep = (h->depth_keep_map && h->depth_map_of == h->dmap.p) || depth_map_reusable(h, pl.nbins);
    if (!keep && !index_kept) return DEPTH_FALLBACK;
    if (!keep && (rc = depth_map_enqueue(h, pl, sub, U))) return rc;
    // the digest, partitioned into the regions
    PartOut po{};
    po.recs = h->recR.p;
    po.dig = h->rdig.p;
    po.cur = h->rcur.p;
    po.dm = DepthMap{h->dmap.p, sub, pl.b2, pl.nbins - 1};
    po.cap = pl.cap;
    po.b1 = pl.b1;
    po.stage = h->use_part_stage ? 1u : 0u;
    h->part_now = &po;
    uint64_t n = 0;
    bool dev = false;
    rc = run_digest(h, &n, n_in, sparse, &dev);
    h->part_now = nullptr;
    if (rc) return rc;
    if (!dev) return set_error(DBI_E_STATE, "internal: warm build without device sizing");
    return depth_tail(h, pl, sub, cap, T, nchunks, true);
}

// digest + tail of a warm device-sized build, enqueued (or captured)
int warm_body(dbi_handle* h, uint64_t* n_in, bool* sparse) {
    const DepthPlan dpl = depth_plan(h);
    if (dpl.on) {
        // (the map samples the resident index: a reallocation of it on the way
        // here -- the tail's buffers grown -- and the radix tail runs instead)
        const double* um = h->umass.p;
        const uint32_t* oo = h->occ_off.p;
        int rc0;
        if ((rc0 = tail_buffers(h, std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull),
                                std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull), true)))
            return rc0;
        const int rd = warm_body_depth(h, dpl, um == h->umass.p && oo == h->occ_off.p, n_in, sparse);
        if (rd != DEPTH_FALLBACK) return rd;
    }
    const LsdPlan lpl = lsd_plan(h);
    if (lpl.on) return warm_body_lsd(h, lpl, n_in, sparse);
    // small tails: the bounded digest counts the first radix pass's histogram
    // as it writes the records (one kernel and its launch gap fewer, human
    // scale 0.33 -> 0.31 ms).  Bins and buffers planned here from what
    // build_tail will use -- cap slots, the previous build's count,
    // minMH..maxMH -- and the histogram zeroed.  Not above H1_MAX_SLOTS: the
    // tiles' flushes are ~200 global atomics each (SwissProt: 10 M, the digest
    // +0.1 ms against the 0.19 ms histogram kernel, measured: no gain).
    h->h1_on = false;
    const bool lean = lean_digest(h);
    constexpr uint64_t H1_MAX_SLOTS = 16ull << 20;
    if (lean && h->use_h1 && std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull) <= H1_MAX_SLOTS) {
        const uint64_t cap = std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
        const uint32_t nbins = choose_nbins(h->last_kept ? std::min<uint64_t>(h->last_kept, cap) : cap, h->bin_bits_max);
        int width[8] = {};
        const int passes = radix_plan(nbins, true, width);
        if (passes >= 1 && width[0] >= 1) {
            int rc0;
            if ((rc0 = tail_buffers(h, cap, cap, true, passes, width[passes - 1]))) return rc0;
            h->h1plan = Hist1Plan{h->hist.p, make_binmap(h->params.min_mh, h->params.max_mh, nbins), width[0],
                                  (uint32_t)radix_blocks((uint32_t)cap)};
            DBI_HIP(hipMemsetAsync(h->hist.p, 0, sizeof(uint32_t) * ((size_t)h->h1plan.G << width[0]), h->stream));
            h->h1_on = true;
        }
    }
    uint64_t n = 0;
    bool dev = false;
    int rc = run_digest(h, &n, n_in, sparse, &dev);
    if (!rc && !dev) rc = set_error(DBI_E_STATE, "internal: warm build without device sizing");
    if (!rc && h->h1_on && (!*sparse || n != std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull)))
        rc = set_error(DBI_E_STATE, "internal: first radix histogram planned for another tail");
    // the tail sorts what the digest wrote -- nothing when its slots did not
    // fit (tiles that found no room left stale slots; build_digest redoes it)
    if (!rc) {
        const hipError_t e = launch_tail_counts(h->ctr.p, *n_in, *sparse, h->stream);
        rc = e == hipSuccess ? build_tail(h, n, h->params.min_mh, h->params.max_mh, *n_in, *sparse,
                                          &h->ctr.p->tail_in, &h->ctr.p->tail_n, h->last_kept)
                             : hip_fail(e, "launch_tail_counts");
    }
    h->h1_on = false;
    return rc;
}

int build_digest(dbi_handle* h) {
    for (int attempt = 0;; ++attempt) {
        const bool warm = h->recA.cap >= 1024 && !h->force_cold;
        uint64_t n_in = 0;
        bool sparse = false;
        int rc;
        if (!warm) {  // cold: host-sized (the bounded digest's slot count, or count / emit)
            uint64_t n = 0;
            if ((rc = run_digest(h, &n, &n_in, &sparse, nullptr))) return rc;
            // the tail's buffers (the index among them) as the next, warm build
            // sizes them -- by the slot capacity -- so that its depth map can
            // sample this index where it lies
            const uint64_t cap = std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull);
            if (sparse && cap > n && (rc = tail_buffers(h, cap, cap, true))) return rc;
            return build_tail(h, n, h->params.min_mh, h->params.max_mh, n_in, sparse);
        }
        // graphs for the bounded digest's builds, untimed or timing one stage
        // (every stage timed: events in the dispatch packets, no graph)
        const bool bounded = bounded_digest(h) && !(h->timing && h->timing_only.empty());
        const dbi_handle::GraphKey key = graph_key(h);
        if (bounded && h->use_graph && attempt == 0 && h->bgraph.exec && h->bgraph.key == key) {
            // replay the captured build; its host-side results come with it
            DBI_HIP(hipGraphLaunch(h->bgraph.exec, h->stream));
            h->nstage = h->bgraph.nstage;
            std::copy(h->bgraph.stages, h->bgraph.stages + h->bgraph.nstage, h->stages);
            h->stats.n_bins = h->bgraph.n_bins;
            h->skip_mid = h->grid_mid == GRID_NONE;  // as when it was captured (the grids are in the key)
            h->skip_big = h->grid_big == GRID_NONE;
            n_in = h->bgraph.n_in;
            sparse = h->bgraph.sparse;
        } else if (bounded && h->use_graph && attempt == 0 && h->prev_key_valid && h->prev_key == key) {
            // the same build as last time: capture it, then run the graph
            drop_graph(h);
            DBI_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
            h->capturing = true;
            rc = warm_body(h, &n_in, &sparse);
            h->capturing = false;
            hipGraph_t g = nullptr;
            const hipError_t ec = hipStreamEndCapture(h->stream, &g);
            if (rc || ec != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                return rc ? rc : hip_fail(ec, "hipStreamEndCapture");
            }
            hipGraphExec_t ex = nullptr;
            const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
            if (ei != hipSuccess) {
                (void)hipGraphDestroy(g);
                return hip_fail(ei, "hipGraphInstantiate");
            }
            DBI_HIP(hipGraphLaunch(ex, h->stream));
            h->bgraph.graph = g;
            h->bgraph.exec = ex;
            h->bgraph.key = key;
            h->bgraph.nstage = h->nstage;
            std::copy(h->stages, h->stages + h->nstage, h->bgraph.stages);
            h->bgraph.n_bins = h->stats.n_bins;
            h->bgraph.n_in = n_in;
            h->bgraph.sparse = sparse;
            if (graph_key(h).alloc_gen != key.alloc_gen) drop_graph(h);  // buffers moved while capturing: once only
        } else {
            if ((rc = warm_body(h, &n_in, &sparse))) return rc;
            h->prev_key = graph_key(h);
            h->prev_key_valid = bounded;
        }
        // the one host sync of a warm build: did the digest fit the capacity,
        // and the chunk lists their grids?
        if ((rc = read_counters(h))) return rc;
        // (a digest tile staged in LDS reserves no slots: n_kept can exceed n_slots)
        const uint64_t need = sparse ? std::max<uint64_t>(h->hc.n_slots, h->hc.n_kept) : h->hc.n_kept;
        if (need >= (1ull << 32) - 1)
            return set_error(DBI_E_INVALID, "more than 2^32-2 peptide occurrences (or bounded-digest slots) on "
                                            "one device: shard the FASTA");
        const bool grid_short = chunk_lists_short(h);
        const bool part_over = (h->hc.err & ERR_PART) != 0;
        if (need <= n_in && !grid_short && !part_over) {
            h->hc_final = true;
            h->depth_off = false;
            h->depth_keep_map = false;
            // the regions' room comes back down after SLACK_DECAY builds without an
            // overflow (one transient spike does not size them at 8x for good)
            if ((depth_plan(h).on || lsd_plan(h).on) && ++h->slack_ok >= SLACK_DECAY) {
                h->slack_ok = 0;
                h->depth_slack = std::max(SLACK_MIN, 0.5 * h->depth_slack);
                h->lsd_slack = std::max(SLACK_MIN, 0.5 * h->lsd_slack);
            }
            return 0;
        }
        if (part_over) {  // a depth-bin region overflowed: this build by the radix tail, the next with more room
            h->depth_off = true;
            h->depth_map_unique = 0;  // (and a freshly sampled map)
            h->depth_slack = std::min(8.0, 2.0 * h->depth_slack);
            h->lsd_slack = std::min(8.0, 2.0 * h->lsd_slack);
            h->slack_ok = 0;
        }
        // a redo of a depth-bin build keeps its map (this attempt's finalize may have overwritten the index)
        h->depth_keep_map = !part_over && !h->depth_off;
        if (attempt > 2) {
            h->depth_off = false;
            h->depth_keep_map = false;
            return set_error(DBI_E_STATE, "digest output grew between identical passes");
        }
        // grown, or a chunk list longer than its grid: everything again (full
        // list grids; counters back to zero, except the record layout; the
        // stage table restarts)
        drop_graph(h);
        h->prev_key_valid = false;
        h->grid_mid = h->grid_big = h->grid_split = 0;
        h->giants_seen = true;
        if (need > n_in && (rc = h->recA.ensure(need + need / 8))) return rc;
        DBI_HIP(hipMemsetAsync(h->ctr.p, 0, offsetof(Counters, max_plen), h->stream));
        h->nstage = 0;
    }
}

int begin_build(dbi_handle* h, uint64_t n_res, uint64_t n_prot, bool zero_ctr) {
    if (n_res >= (1ull << 32) - 1) return set_error(DBI_E_INVALID, "n_res must be < 2^32-1 per device: shard the FASTA");
    if (n_prot >= (1ull << 32) - 1) return set_error(DBI_E_INVALID, "n_prot must be < 2^32-1");
    DBI_HIP(hipSetDevice(h->device));
    h->built = false;
    h->shard.phase = 0;
    h->n_res = n_res;
    h->n_prot = n_prot;
    h->n_total_extra = 0;
    h->exact_dups = false;
    h->depth_off = false;  // (a depth-bin redo's state never outlives its build)
    h->depth_keep_map = false;
    std::memset(&h->stats, 0, sizeof(h->stats));
    h->nstage = 0;
    h->hc_final = false;
    h->t0 = std::chrono::steady_clock::now();
    if (zero_ctr) DBI_HIP(hipMemsetAsync(h->ctr.p, 0, sizeof(Counters), h->stream));
    return 0;
}

int check_offsets_host(const uint64_t* off, uint64_t n_res, uint64_t n_prot) {
    if (off[0] != 0) return set_error(DBI_E_INVALID, "prot_off[0] must be 0");
    if (off[n_prot] != n_res) return set_error(DBI_E_INVALID, "prot_off[n_prot] must equal n_res");
    for (uint64_t i = 0; i < n_prot; ++i)
        if (off[i + 1] < off[i]) return set_error(DBI_E_INVALID, "prot_off must be non-decreasing");
    return 0;
}

// ---- inline '[formula]' PTMs (DBIndexer.java:288-303) ------------------------
// FormulaCalculator.calculateMass lives in the un-vendored
// edu.scripps.yates.utilities jar: restated as the left-to-right sum of
// count x monoisotopic element mass (element = capital letter + lower-case
// letters, count = optional [-]digits, default 1); an unknown element is NaN
// (UnknownElementMassException).  Parity unpinned.
double formula_mass(const std::string& f) {
    static const std::pair<const char*, double> kEl[] = {
        {"H", 1.00782503207}, {"D", 2.0141017778}, {"C", 12.0}, {"N", 14.0030740048}, {"O", 15.99491461956},
        {"P", 30.97376163}, {"S", 31.97207100}, {"Se", 79.9165213}, {"Na", 22.9897692809}, {"K", 38.96370668},
        {"Li", 7.01600455}, {"Mg", 23.9850417}, {"Ca", 39.96259098}, {"Fe", 55.9349375}, {"Zn", 63.9291422},
        {"Cu", 62.9295975}, {"Cl", 34.96885268}, {"Br", 78.9183371}, {"I", 126.904473}, {"F", 18.99840322},
        {"Si", 27.9769265325}, {"B", 11.0093054}, {"Hg", 201.970643}};
    const double nan = std::numeric_limits<double>::quiet_NaN();
    double mass = 0.0;
    size_t i = 0;
    while (i < f.size()) {
        if (!(f[i] >= 'A' && f[i] <= 'Z')) return nan;
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
            if (neg) return nan;
            cnt = 1;
        }
        double em = nan;
        for (const auto& e : kEl)
            if (el == e.first) em = e.second;
        if (!(em == em)) return nan;
        mass = mass + (double)(neg ? -cnt : cnt) * em;
        i = k;
    }
    return mass;
}

// Formulas out of every protein: the stripped proteome (digest input), and per
// protein carrying formulas its events -- position in the stripped protein
// (the residue that followed ']'), mass (NaN: unknown element).  A formula
// string seen earlier in the same protein is dropped: String.replace removed
// every copy when the first was reached (:298).
struct PtmPlan {
    std::vector<uint8_t> stripped;
    std::vector<uint64_t> soff;
    std::vector<uint32_t> pid, ev_off, ev_pos;
    std::vector<double> ev_mass;
};

int plan_ptms(const uint8_t* res, const uint64_t* off, uint64_t n_prot, PtmPlan& pl) {
    pl.stripped.reserve(off[n_prot]);
    pl.soff.assign(1, 0);
    pl.ev_off.assign(1, 0);
    for (uint64_t i = 0; i < n_prot; ++i) {
        const uint64_t b = off[i], e = off[i + 1];
        if (!std::memchr(res + b, '[', e - b)) {
            pl.stripped.insert(pl.stripped.end(), res + b, res + e);
            pl.soff.push_back(pl.stripped.size());
            continue;
        }
        const size_t p0 = pl.stripped.size();
        std::vector<std::string> seen;
        for (uint64_t x = b; x < e;) {
            if (res[x] != '[') {
                pl.stripped.push_back(res[x++]);
                continue;
            }
            const uint8_t* close = (const uint8_t*)std::memchr(res + x + 1, ']', e - x - 1);
            if (!close)
                return set_error(DBI_E_INVALID, "protein " + std::to_string(i) +
                                                    ": '[' without ']' (the reference reads past the protein: "
                                                    "StringIndexOutOfBoundsException, DBIndexer.java:291)");
            const std::string f((const char*)res + x + 1, (size_t)(close - res) - x - 1);
            x = (uint64_t)(close - res) + 1;
            if (std::find(seen.begin(), seen.end(), f) != seen.end()) continue;
            seen.push_back(f);
            const uint32_t pos = (uint32_t)(pl.stripped.size() - p0);
            const double m = formula_mass(f);
            if (pos == 0 && m == m)
                return set_error(DBI_E_INVALID, "protein " + std::to_string(i) +
                                                    ": a '[formula]' before its first residue (the reference reads "
                                                    "charAt(-1): StringIndexOutOfBoundsException, DBIndexer.java:300-314)");
            pl.ev_pos.push_back(pos);
            pl.ev_mass.push_back(m);
        }
        pl.soff.push_back(pl.stripped.size());
        pl.pid.push_back((uint32_t)i);
        pl.ev_off.push_back((uint32_t)pl.ev_pos.size());
    }
    return 0;
}

int upload_inputs(dbi_handle* h, const uint8_t* residues, uint64_t n_res, const uint64_t* prot_off, uint64_t n_prot,
                  bool* ptm = nullptr);

int build_with_ptms(dbi_handle* h, const uint8_t* residues, uint64_t n_res, const uint64_t* prot_off,
                    uint64_t n_prot) {
    PtmPlan pl;
    int rc;
    if ((rc = plan_ptms(residues, prot_off, n_prot, pl))) return rc;
    const uint64_t Rs = pl.stripped.size();
    const uint32_t n_ptm = (uint32_t)pl.pid.size();
    hipStream_t s = h->stream;
    // the engine keeps the proteins as given (the ProteinCache's strings: tags,
    // string verification and every later lookup read them at the stripped
    // offsets, as IndexMerge does); the digest runs over the stripped proteome
    // with the formula-carrying proteins masked (a residue above maxMH), and
    // those proteins are walked literally by k_ptm_digest
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    if ((rc = upload_inputs(h, residues, n_res, prot_off, n_prot))) return rc;
    h->inputs_ptm = true;  // dbi_rebuild cannot digest this text directly
    std::vector<uint8_t> masked = pl.stripped;
    std::vector<uint8_t> sres;
    std::vector<uint32_t> soff32(1, 0), off32(n_prot + 1);
    for (uint32_t j = 0; j < n_ptm; ++j) {
        const uint64_t b = pl.soff[pl.pid[j]], e = pl.soff[pl.pid[j] + 1];
        sres.insert(sres.end(), pl.stripped.begin() + b, pl.stripped.begin() + e);
        soff32.push_back((uint32_t)sres.size());
        std::memset(masked.data() + b, 1, e - b);
    }
    for (uint64_t i = 0; i <= n_prot; ++i) off32[i] = (uint32_t)pl.soff[i];
    double tab[256];
    DBI_HIP(hipMemcpy(tab, h->mass_tab.p, sizeof(tab), hipMemcpyDeviceToHost));
    tab[1] = 1e300;  // the mask residue: every walk over it ends at its first step
    if ((rc = h->res_dig.ensure(Rs + 16)) || (rc = h->poff_dig.ensure(n_prot + 1)) ||
        (rc = h->mass_tab_x.ensure(256)) || (rc = h->ptm_res.ensure(sres.size() + 16)) ||
        (rc = h->ptm_soff.ensure(n_ptm + 1)) || (rc = h->ptm_pid.ensure(n_ptm)) ||
        (rc = h->ptm_evoff.ensure(n_ptm + 1)) || (rc = h->ptm_evpos.ensure(pl.ev_pos.size())) ||
        (rc = h->ptm_evmass.ensure(pl.ev_mass.size())) || (rc = h->ptm_cnt.ensure(n_ptm + 1)) ||
        (rc = h->ptm_total.ensure(1)) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(n_ptm + 1), h->scan_tmp.cap))))
        return rc;
    if (Rs) DBI_HIP(hipMemcpyAsync(h->res_dig.p, masked.data(), Rs, hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->poff_dig.p, off32.data(), 4 * (n_prot + 1), hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->mass_tab_x.p, tab, sizeof(tab), hipMemcpyHostToDevice, s));
    if (!sres.empty()) DBI_HIP(hipMemcpyAsync(h->ptm_res.p, sres.data(), sres.size(), hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->ptm_soff.p, soff32.data(), 4 * (n_ptm + 1), hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->ptm_pid.p, pl.pid.data(), 4 * n_ptm, hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->ptm_evoff.p, pl.ev_off.data(), 4 * (n_ptm + 1), hipMemcpyHostToDevice, s));
    if (!pl.ev_pos.empty()) {
        DBI_HIP(hipMemcpyAsync(h->ptm_evpos.p, pl.ev_pos.data(), 4 * pl.ev_pos.size(), hipMemcpyHostToDevice, s));
        DBI_HIP(hipMemcpyAsync(h->ptm_evmass.p, pl.ev_mass.data(), 8 * pl.ev_mass.size(), hipMemcpyHostToDevice, s));
    }
    DBI_HIP(hipStreamSynchronize(s));  // host staging vectors die here
    // the digest over the masked stripped proteome (its own offsets, length,
    // mass table; the cut-stepping count assumes residue masses < 1024 Da)
    const uint8_t* o_res = h->d_res;
    const uint32_t* o_off = h->d_poff;
    const int cut_count = h->dp.cut_count;
    h->d_res = h->res_dig.p;
    h->d_poff = h->poff_dig.p;
    h->n_res = Rs;
    h->dp.cut_count = 0;
    std::swap(h->mass_tab, h->mass_tab_x);
    uint64_t n = 0, n_in = 0;
    bool sparse = false;
    rc = run_digest(h, &n, &n_in, &sparse, nullptr);
    std::swap(h->mass_tab, h->mass_tab_x);
    h->dp.cut_count = cut_count;
    h->d_res = o_res;
    h->d_poff = o_off;
    h->n_res = n_res;
    if (rc) return rc;
    // the formula-carrying proteins: count, offsets, emit after the digest's slots
    DBI_HIP(launch_ptm_digest(false, h->dp, h->mass_tab.p, h->flags_tab.p, h->ptm_res.p, h->ptm_soff.p, h->d_res,
                              h->d_poff, h->ptm_pid.p, h->ptm_evoff.p, h->ptm_evpos.p, h->ptm_evmass.p, n_ptm,
                              h->ptm_cnt.p, nullptr, h->ctr.p, s));
    DBI_HIP(launch_scan_u32(h->ptm_cnt.p, h->ptm_cnt.p, n_ptm, h->scan_tmp.p, h->scan_tmp.cap, h->ptm_total.p, s));
    unsigned long long extra = 0;
    DBI_HIP(hipMemcpyAsync(&extra, h->ptm_total.p, sizeof(extra), hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if (n_in + extra >= (1ull << 32) - 1)
        return set_error(DBI_E_INVALID, "more than 2^32-2 peptide occurrences on one device: shard the FASTA");
    if (h->recA.cap < n_in + extra) {  // grow, keeping the digest's records
        DevBuf<Rec> grown;
        if ((rc = grown.ensure(n_in + extra))) return rc;
        if (n_in) DBI_HIP(hipMemcpyAsync(grown.p, h->recA.p, sizeof(Rec) * n_in, hipMemcpyDeviceToDevice, s));
        DBI_HIP(hipStreamSynchronize(s));
        std::swap(h->recA, grown);
        grown.release();
    }
    DBI_HIP(launch_ptm_digest(true, h->dp, h->mass_tab.p, h->flags_tab.p, h->ptm_res.p, h->ptm_soff.p, h->d_res,
                              h->d_poff, h->ptm_pid.p, h->ptm_evoff.p, h->ptm_evpos.p, h->ptm_evmass.p, n_ptm,
                              h->ptm_cnt.p, h->recA.p + n_in, h->ctr.p, s));
    if ((rc = read_counters(h))) return rc;
    return build_tail(h, h->hc.n_kept, h->params.min_mh, h->params.max_mh, n_in + extra, sparse);
}

// Host residues -> HBM.  The first large pageable hipMemcpy of a process pays
// the runtime's one-time setup (~200 ms on MI355X boxes, even for 64 MiB;
// later ones of a fresh 201-MB buffer ~4.5 ms), and registering the caller's
// buffer costs ~0.04 ms a MiB (tools/probe/h2d_probe.hip, h2d_ring.hip).  So
// the copy goes through a pinned ring owned by the handle: UP_THREADS threads each copy
// every UP_THREADS-th slice into one of their two UP_SLOT slots (waiting for
// that slot's previous DMA), look for '[' in it on the way (inline PTMs: the
// caller then takes the PTM path), and queue its DMA on the engine stream.
// Small inputs take one plain copy.
constexpr uint64_t UP_SLOT = 2ull << 20;  // (1 MiB: ~6.7 ms for 201 MB, 2 MiB: ~5.1, tools/probe/h2d_ring.hip)
constexpr int UP_THREADS = 8;
constexpr uint64_t UP_MIN = 16ull << 20;  // below: one pageable copy

// A parser-owned residue buffer goes to HBM without a staging copy: pinned
// in UP_REG pieces (2-MiB pages: ~0.1 ms a piece), each piece's DMA queued as
// soon as it is pinned, all unpinned once the stream has drained (201 MB:
// ~4.3 ms vs ~6.6 ms through the ring; tools/probe/h2d_ring.hip).  Returns
// false (nothing left pinned) when the runtime refuses a registration, e.g.
// of memory the caller registered itself: the ring then copies it.
constexpr uint64_t UP_REG = 32ull << 20;

// The handle's pinned staging ring and its slots' events.  Host pages pinned
// by registration: hipHostMalloc of the same 16 MiB took ~0.15-0.2 ms a MiB
// on MI355X boxes, hipHostRegister ~0.04 (tools/probe/h2d_probe.hip).
constexpr uint64_t UP_RING = UP_SLOT * 2 * UP_THREADS;

int ensure_ring(dbi_handle* h) {
    if (!h->up_host) {
        void* p = nullptr;
        if (posix_memalign(&p, 2ull << 20, UP_RING) != 0) return set_error(DBI_E_OOM, "staging ring");
        (void)madvise(p, UP_RING, MADV_HUGEPAGE);
        if (hipHostRegister(p, UP_RING, hipHostRegisterDefault) != hipSuccess) {
            std::free(p);
            return set_error(DBI_E_HIP, "hipHostRegister of the staging ring failed");
        }
        h->up_host = (uint8_t*)p;
    }
    while (h->up_ev.size() < 2 * UP_THREADS) {
        hipEvent_t ev = nullptr;
        DBI_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        h->up_ev.push_back(ev);
    }
    return 0;
}

bool upload_registered(dbi_handle* h, const uint8_t* residues, uint64_t n_res) {
    const uintptr_t base = (uintptr_t)residues & ~(uintptr_t)((2ull << 20) - 1);  // (the buffer is 2-MiB aligned)
    const uint64_t span = (uint64_t)((uintptr_t)residues + n_res - base);
    std::vector<void*> pinned;
    bool ok = true;
    for (uint64_t o = 0; o < span && ok; o += UP_REG) {
        uint8_t* a = (uint8_t*)(base + o);
        const uint64_t len = std::min(UP_REG, span - o);
        if (hipHostRegister(a, len, hipHostRegisterDefault) != hipSuccess) {
            (void)hipGetLastError();
            ok = false;
            break;
        }
        pinned.push_back(a);
        const uint8_t* lo = std::max<const uint8_t*>(a, residues);
        const uint8_t* hi = std::min<const uint8_t*>(a + len, residues + n_res);
        if (hi > lo && hipMemcpyAsync(h->res.p + (lo - residues), lo, (size_t)(hi - lo), hipMemcpyHostToDevice,
                                      h->stream) != hipSuccess)
            ok = false;
    }
    ok = hipStreamSynchronize(h->stream) == hipSuccess && ok;
    for (void* a : pinned) (void)hipHostUnregister(a);
    return ok;
}

int upload_residues(dbi_handle* h, const uint8_t* residues, uint64_t n_res, bool* ptm) {
    bool ptm_known = false, brackets = false;
    if (n_res >= UP_MIN && fasta_residue_buffer(residues, n_res, &ptm_known, &brackets)) {
        if (ptm && !ptm_known) {  // (a parser without AVX-512 did not look): 8 threads scan
            std::atomic<bool> any{false};
            std::vector<std::thread> th;
            for (int t = 0; t < UP_THREADS; ++t)
                th.emplace_back([&, t] {
                    const uint64_t a = n_res * (uint64_t)t / UP_THREADS, e = n_res * (uint64_t)(t + 1) / UP_THREADS;
                    if (e > a && std::memchr(residues + a, '[', e - a)) any = true;
                });
            for (auto& x : th) x.join();
            brackets = any;
        }
        if (upload_registered(h, residues, n_res)) {
            if (ptm) *ptm = brackets;
            return 0;
        }
    }
    if (n_res < UP_MIN) {
        if (ptm) *ptm = n_res && std::memchr(residues, '[', n_res) != nullptr;
        if (n_res) DBI_HIP(hipMemcpyAsync(h->res.p, residues, n_res, hipMemcpyHostToDevice, h->stream));
        return 0;
    }
    int rc;
    if ((rc = ensure_ring(h))) return rc;
    const uint64_t nslices = (n_res + UP_SLOT - 1) / UP_SLOT;
    const int T = (int)std::min<uint64_t>(UP_THREADS, nslices);
    std::atomic<bool> found{false};
    std::atomic<int> err{0};
    auto work = [&](int t) {
        uint32_t k = 0;
        for (uint64_t c = (uint64_t)t; c < nslices; c += (uint64_t)T, ++k) {
            const int slot = 2 * t + (int)(k & 1u);
            uint8_t* st = h->up_host + UP_SLOT * (uint64_t)slot;
            const uint64_t a = c * UP_SLOT, len = std::min(UP_SLOT, n_res - a);
            if (k >= 2 && hipEventSynchronize(h->up_ev[slot]) != hipSuccess) {  // the slot's last DMA done
                err = 1;
                return;
            }
            std::memcpy(st, residues + a, len);
            if (ptm && !found.load(std::memory_order_relaxed) && std::memchr(st, '[', len)) found = true;
            if (hipMemcpyAsync(h->res.p + a, st, len, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
                hipEventRecord(h->up_ev[slot], h->stream) != hipSuccess) {
                err = 1;
                return;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (err) return set_error(DBI_E_HIP, "staged host-to-device copy of the residues failed");
    if (ptm) *ptm = found;
    return 0;
}

int upload_inputs(dbi_handle* h, const uint8_t* residues, uint64_t n_res, const uint64_t* prot_off, uint64_t n_prot,
                  bool* ptm) {
    int rc;
    DBI_HIP(hipSetDevice(h->device));
    if ((rc = h->res.ensure(n_res + 16))) return rc;
    if ((rc = h->poff.ensure(n_prot + 1))) return rc;
    std::vector<uint32_t> off32(n_prot + 1);
    for (uint64_t i = 0; i <= n_prot; ++i) off32[i] = (uint32_t)prot_off[i];
    if ((rc = upload_residues(h, residues, n_res, ptm))) return rc;
    DBI_HIP(hipMemcpyAsync(h->poff.p, off32.data(), sizeof(uint32_t) * (n_prot + 1), hipMemcpyHostToDevice, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));  // off32 is a stack vector
    h->d_res = h->res.p;
    h->d_poff = h->poff.p;
    h->inputs_resident = true;
    h->inputs_ptm = false;
    return 0;
}

}  // namespace

extern "C" {

const char* dbi_last_error(void) { return g_err.c_str(); }

int dbi_dev_alloc(int device, uint64_t bytes, void** out) {
    if (!out) return set_error(DBI_E_INVALID, "NULL argument");
    DBI_HIP(hipSetDevice(device));
    DBI_HIP(hipMalloc(out, std::max<uint64_t>(bytes, 1)));
    return 0;
}

int dbi_dev_free(int device, void* p) {
    DBI_HIP(hipSetDevice(device));
    if (p) DBI_HIP(hipFree(p));
    return 0;
}

int dbi_dev_copy_h2d(int device, void* dst, const void* src, uint64_t bytes) {
    DBI_HIP(hipSetDevice(device));
    if (bytes) {
        DBI_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        DBI_HIP(hipDeviceSynchronize());  // pageable sources: the DMA may still be in flight on return
    }
    return 0;
}

int dbi_dev_copy_d2h(int device, void* dst, const void* src, uint64_t bytes) {
    DBI_HIP(hipSetDevice(device));
    if (bytes) DBI_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}

int dbi_dev_copy_d2d(int device, void* dst, const void* src, uint64_t bytes) {
    DBI_HIP(hipSetDevice(device));
    if (bytes) {
        // a device-to-device hipMemcpy may return before the copy ran; the source
        // may be an engine buffer its next (non-blocking-stream) call overwrites
        DBI_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
        DBI_HIP(hipDeviceSynchronize());
    }
    return 0;
}

int dbi_dev_synchronize(int device) {
    DBI_HIP(hipSetDevice(device));
    DBI_HIP(hipDeviceSynchronize());
    return 0;
}

int dbi_hbm_copy_bandwidth(int device, uint64_t bytes, int reps, double* gbps) {
    if (!gbps || reps <= 0 || bytes < 16) return set_error(DBI_E_INVALID, "dbi_hbm_copy_bandwidth: bad argument");
    DBI_HIP(hipSetDevice(device));
    const uint64_t n16 = bytes / 16;
    void *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipMalloc(&a, 16 * n16);
    if (e == hipSuccess) e = hipMalloc(&b, 16 * n16);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemsetAsync(a, 1, 16 * n16, s);
    if (e == hipSuccess) e = launch_hbm_copy(a, b, n16, s);  // warm
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    for (int r = 0; r < reps && e == hipSuccess; ++r) e = launch_hbm_copy(r & 1 ? b : a, r & 1 ? a : b, n16, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) *gbps = ms > 0.f ? 2.0 * 16.0 * (double)n16 * reps / (ms * 1e-3) / 1e9 : 0.0;
    if (e1) (void)hipEventDestroy(e1);
    if (e0) (void)hipEventDestroy(e0);
    if (s) (void)hipStreamDestroy(s);
    if (b) (void)hipFree(b);
    if (a) (void)hipFree(a);
    DBI_HIP(e);
    return 0;
}
int dbi_abi_version(void) { return DBI_ABI_VERSION; }

int dbi_device_count(int* out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return 0;
}

void dbi_params_default(dbi_params* p, int32_t max_missed, int32_t semi) {
    std::memset(p, 0, sizeof(*p));
    // pinned monoisotopic residue masses (Unimod), see dbindex_amd/params.py
    static const struct { char c; double m; } tab[] = {
        {'G', 57.021464},  {'A', 71.037114},  {'S', 87.032028},  {'P', 97.052764},  {'V', 99.068414},
        {'T', 101.047679}, {'C', 103.009185}, {'L', 113.084064}, {'I', 113.084064}, {'N', 114.042927},
        {'D', 115.026943}, {'Q', 128.058578}, {'K', 128.094963}, {'E', 129.042593}, {'M', 131.040485},
        {'H', 137.058912}, {'F', 147.068414}, {'R', 156.101111}, {'Y', 163.063329}, {'W', 186.079313},
        {'U', 150.953636}, {'O', 237.147727},
    };
    for (const auto& t : tab) p->mass[(unsigned char)t.c] = t.m;
    p->min_mh = 500.0;    // default_min_precursor_mass (dbindex.properties:9)
    p->max_mh = 6000.0;   // default_max_precursor_mass (dbindex.properties:8)
    p->h2o_proton = 18.0105646863 + 1.00727646688;
    p->cleave[(unsigned char)'K'] = 1;  // default_enzyme_residues=KR (dbindex.properties:12)
    p->cleave[(unsigned char)'R'] = 1;
    p->max_missed = max_missed;
    p->semi = semi;
    p->add_h2o_proton = 1;
    p->min_len = 6;
    p->mass_group_factor = 10000;
    p->index_factor = 8;
}

int dbi_open(const dbi_params* params, int device, dbi_handle** out) {
    if (!out) return set_error(DBI_E_INVALID, "out is NULL");
    *out = nullptr;
    int rc = check_params(params);
    if (rc) return rc;
    if ((rc = check_mass_floor(params, make_dev_params(*params).m0))) return rc;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return set_error(DBI_E_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return set_error(DBI_E_INVALID, "device ordinal out of range");
    DBI_HIP(hipSetDevice(device));
    dbi_handle* h = new dbi_handle();
    h->params = *params;
    h->dp = make_dev_params(*params);
    h->device = device;
    // (tuning switches and test hooks: dbi_set_option; the defaults are the measured best)
    auto fail = [&](int code) {
        dbi_close(h);
        return code;
    };
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(set_error(DBI_E_HIP, "hipStreamCreate failed"));
    if ((rc = h->mass_tab.ensure(256)) || (rc = h->flags_tab.ensure(256)) || (rc = h->ctr.ensure(1)))
        return fail(rc);
    uint8_t fl[256];
    for (int c = 0; c < 256; ++c)
        fl[c] = (params->cleave[c] ? F_CLEAVE : 0) | (params->nocut[c] ? F_NOCUT : 0) |
                (params->mandatory[c] ? F_MAND : 0) | (c == '[' ? F_PTM : 0);
    if (hipMemcpy(h->mass_tab.p, params->mass, sizeof(double) * 256, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->flags_tab.p, fl, 256, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(h->ctr.p, 0, sizeof(Counters)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)  // null-stream work done before the engine's non-blocking stream runs
        return fail(set_error(DBI_E_HIP, "parameter upload failed"));
    *out = h;
    return 0;
}

void dbi_close(dbi_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    h->mass_tab.release(); h->flags_tab.release(); h->ctr.release();
    h->res_dig.release(); h->ptm_res.release(); h->poff_dig.release(); h->ptm_soff.release(); h->ptm_pid.release();
    h->ptm_evoff.release(); h->ptm_evpos.release(); h->ptm_cnt.release(); h->ptm_evmass.release();
    h->mass_tab_x.release(); h->ptm_total.release();
    h->res.release(); h->poff64.release(); h->poff.release(); h->poff_g.release();
    h->samp.release(); h->xcount.release(); h->xsend.release(); h->xrecv.release();
    h->qcnt.release(); h->qpairA.release(); h->qpairB.release(); h->qsend.release(); h->qrecv.release();
    h->qres.release(); h->qback.release(); h->blk.release(); h->scan_tmp.release();
    h->status.release(); h->win_lo.release(); h->win_hi.release(); h->qdir.release(); h->qdir_par.release();
    h->thr.release(); h->tile_pf.release(); h->chunk_lo.release();
    h->recA.release(); h->recB.release(); h->hist.release(); h->ucount.release(); h->digits.release();
    h->big_list.release(); h->mid_list.release(); h->giant_list.release(); h->segs.release(); h->synth_len.release(); h->synth_res.release(); h->synth_out.release(); h->synth_off.release(); h->ws_key.release(); h->ws_k2.release(); h->umass.release(); h->upid.release();
    h->uoff.release(); h->ulen.release(); h->occ_off.release(); h->occ_pid.release();
    h->o_mass.release(); h->o_pid.release(); h->o_off.release(); h->o_len.release();
    h->q_mass.release(); h->q_tol.release(); h->q_first.release(); h->q_count.release(); h->q_row.release();
    h->q_ids.release(); h->g_mass.release(); h->g_pid.release(); h->g_off.release(); h->g_len.release();
    h->g_b.release(); h->g_e.release();
    h->h_nh.release(); h->h_no.release(); h->h_ids.release(); h->h_hocc.release(); h->h_prot.release();
    h->h_row.release(); h->h_orow.release(); h->h_sums.release(); h->kr_scratch.release();
    h->r_mass.release(); h->r_pid.release(); h->r_off.release(); h->r_len.release(); h->r_occ_off.release();
    h->r_occ.release();
    h->recR.release(); h->rdig.release(); h->rcur.release(); h->dsub.release(); h->dpre.release(); h->dmap.release();
    h->dheavy.release(); h->desc.release(); h->d1c.release(); h->hist2.release(); h->bstart.release();
    h->split_list.release();
    drop_graph(h);
    for (auto& ev : h->evpool)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : h->ev_merge)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : h->up_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (h->up_host) {
        (void)hipHostUnregister(h->up_host);
        std::free(h->up_host);
    }
    for (auto& ev : h->ev_side)
        if (ev) (void)hipEventDestroy(ev);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int dbi_build(dbi_handle* h, const uint8_t* residues, uint64_t n_res, const uint64_t* prot_off, uint64_t n_prot) {
    if (!h || (!residues && n_res) || !prot_off) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = check_offsets_host(prot_off, n_res, n_prot))) return rc;
    if (n_res >= (1ull << 32) - 1) return set_error(DBI_E_INVALID, "n_res must be < 2^32-1 per device: shard the FASTA");
    bool ptm = false;  // the upload looks for '[' as it copies
    if ((rc = upload_inputs(h, residues, n_res, prot_off, n_prot, &ptm))) return rc;
    if (ptm) {  // inline '[formula]' PTMs
        if ((rc = build_with_ptms(h, residues, n_res, prot_off, n_prot))) return rc;
        return finish_build(h);
    }
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    if ((rc = build_digest(h))) return rc;
    return finish_build(h);
}

int dbi_build_fasta(dbi_handle* h, const char* path, int threads, dbi_fasta** out) {
    if (out) *out = nullptr;
    if (!h || !path) return set_error(DBI_E_INVALID, "NULL argument");
    dbi_fasta* f = nullptr;
    int rc = dbi_fasta_read(path, threads, &f);
    if (!rc) rc = dbi_build(h, f->residues, f->n_residues, f->offsets, f->n_proteins);
    if (out && !rc) *out = f;
    else dbi_fasta_free(f);
    return rc;
}

int dbi_build_device(dbi_handle* h, const uint8_t* d_residues, uint64_t n_res, const uint64_t* d_prot_off,
                     uint64_t n_prot, void* stream) {
    if (!h || (!d_residues && n_res) || !d_prot_off) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = begin_build(h, n_res, n_prot, false))) return rc;  // (the counters: zeroed by the offsets' conversion)
    hipStream_t user = (hipStream_t)stream;
    if (user) {
        // order the engine stream after the caller's producer work
        hipEvent_t ev;
        DBI_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        DBI_HIP(hipEventRecord(ev, user));
        DBI_HIP(hipStreamWaitEvent(h->stream, ev, 0));
        DBI_HIP(hipEventDestroy(ev));
    }
    if ((rc = h->poff.ensure(n_prot + 1))) return rc;
    DBI_HIP(launch_off64_to_32(d_prot_off, h->poff.p, n_prot + 1, h->stream, h->ctr.p));
    h->d_res = d_residues;
    h->d_poff = h->poff.p;
    if ((rc = build_digest(h))) return rc;
    return finish_build(h);
}

int dbi_build_occurrences(dbi_handle* h, const uint8_t* residues, uint64_t n_res, const uint64_t* prot_off,
                          uint64_t n_prot, const double* mass, const uint32_t* prot_id, const uint32_t* offset,
                          const uint32_t* length, uint64_t n_occ, uint64_t n_dropped_extra) {
    if (!h || (!residues && n_res) || !prot_off || (n_occ && (!mass || !prot_id || !offset || !length)))
        return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = check_offsets_host(prot_off, n_res, n_prot))) return rc;
    if (n_occ >= (1ull << 32) - 1) return set_error(DBI_E_INVALID, "too many occurrences for one device");
    double lo = 0, hi = 0;
    for (uint64_t i = 0; i < n_occ; ++i) {
        if (!(mass[i] >= 1.0 && mass[i] < 65536.0))
            return set_error(DBI_E_INVALID, "occurrence mass must be in [1, 65536) Da");
        if (prot_id[i] >= n_prot) return set_error(DBI_E_INVALID, "occurrence protein id out of range");
        const uint64_t plen = prot_off[prot_id[i] + 1] - prot_off[prot_id[i]];
        if ((uint64_t)offset[i] + length[i] > plen || length[i] == 0)
            return set_error(DBI_E_INVALID, "occurrence offset/length outside its protein");
        if (i == 0 || mass[i] < lo) lo = mass[i];
        if (i == 0 || mass[i] > hi) hi = mass[i];
    }
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    h->exact_dups = true;
    if ((rc = upload_inputs(h, residues, n_res, prot_off, n_prot))) return rc;
    if ((rc = h->o_mass.ensure(n_occ)) || (rc = h->o_pid.ensure(n_occ)) || (rc = h->o_off.ensure(n_occ)) ||
        (rc = h->o_len.ensure(n_occ)) || (rc = h->recA.ensure(n_occ)))
        return rc;
    if (n_occ) {
        DBI_HIP(hipMemcpyAsync(h->o_mass.p, mass, 8 * n_occ, hipMemcpyHostToDevice, h->stream));
        DBI_HIP(hipMemcpyAsync(h->o_pid.p, prot_id, 4 * n_occ, hipMemcpyHostToDevice, h->stream));
        DBI_HIP(hipMemcpyAsync(h->o_off.p, offset, 4 * n_occ, hipMemcpyHostToDevice, h->stream));
        DBI_HIP(hipMemcpyAsync(h->o_len.p, length, 4 * n_occ, hipMemcpyHostToDevice, h->stream));
    }
    if ((rc = prepare_tiles(h))) return rc;  // record layout first
    DBI_HIP(launch_occ_to_recs(h->o_mass.p, h->o_pid.p, h->o_off.p, h->o_len.p, h->d_poff, h->d_res, n_occ, n_prot,
                               h->recA.p, h->ctr.p, h->stream));
    // n_kept known on the host: seed the device counter
    const unsigned long long kept = n_occ;
    DBI_HIP(hipMemcpyAsync(&h->ctr.p->n_kept, &kept, sizeof(kept), hipMemcpyHostToDevice, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    h->n_total_extra = n_dropped_extra;
    if ((rc = build_tail(h, n_occ, lo, hi, n_occ, false))) return rc;
    return finish_build(h);
}

int dbi_stats_get(dbi_handle* h, dbi_stats* out) {
    if (!h || !out) return set_error(DBI_E_INVALID, "NULL argument");
    *out = h->stats;
    return 0;
}

}  // extern "C"

namespace dbi {
// the query directory of the current index, built on first use (once per build / load)
int ensure_qdir(dbi_handle* h, hipStream_t s) {
    if (h->qdir_serial == h->build_serial) return 0;
    const uint32_t nu = (uint32_t)h->stats.n_unique;
    uint32_t nb = 16;  // ~4 uniques per bucket, at most 2^22 buckets
    while (nb < nu / 4 && nb < (1u << 22)) nb <<= 1;
    int rc;
    if ((rc = h->qdir.ensure((size_t)nb + 1)) || (rc = h->qdir_par.ensure(1))) return rc;
    DBI_HIP(launch_qdir(h->umass.p, nu, nb, h->qdir_par.p, h->qdir.p, s));
    DBI_HIP(hipStreamSynchronize(s));  // later queries may come on other streams
    h->qdir_serial = h->build_serial;
    return 0;
}
}  // namespace dbi

extern "C" {

int dbi_query_device(dbi_handle* h, const double* d_mass, const double* d_tol, uint64_t nq, uint64_t* d_first,
                     uint64_t* d_count, void* stream) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    DBI_HIP(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const uint32_t nu = (uint32_t)h->stats.n_unique;
    int rc;
    if ((rc = ensure_qdir(h, s))) return rc;
    DBI_HIP(launch_query(h->dp, h->params.mass_group_factor, h->umass.p, nu, d_mass, d_tol, nq, d_first, d_count,
                         h->qdir_par.p, h->qdir.p, s));
    return 0;
}

int dbi_query(dbi_handle* h, const double* mass, const double* tol, uint64_t nq, uint64_t* first, uint64_t* count) {
    if (!h || (nq && (!mass || !tol || !first || !count))) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    if (nq == 0) return 0;
    DBI_HIP(hipSetDevice(h->device));
    int rc;
    if ((rc = h->q_mass.ensure(nq)) || (rc = h->q_tol.ensure(nq)) || (rc = h->q_first.ensure(nq)) ||
        (rc = h->q_count.ensure(nq)))
        return rc;
    DBI_HIP(hipMemcpyAsync(h->q_mass.p, mass, 8 * nq, hipMemcpyHostToDevice, h->stream));
    DBI_HIP(hipMemcpyAsync(h->q_tol.p, tol, 8 * nq, hipMemcpyHostToDevice, h->stream));
    if ((rc = dbi_query_device(h, h->q_mass.p, h->q_tol.p, nq, h->q_first.p, h->q_count.p, h->stream))) return rc;
    DBI_HIP(hipMemcpyAsync(first, h->q_first.p, 8 * nq, hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipMemcpyAsync(count, h->q_count.p, 8 * nq, hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

int dbi_query_prepare(dbi_handle* h) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    DBI_HIP(hipSetDevice(h->device));
    return ensure_qdir(h, h->stream);
}

int dbi_query_hits_device(dbi_handle* h, const double* d_mass, const double* d_tol, uint64_t nq,
                          dbi_device_hits* out) {
    if (!h || !out || (nq && (!d_mass || !d_tol))) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    DBI_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    int rc;
    if ((rc = h->q_first.ensure(std::max<uint64_t>(nq, 1))) || (rc = h->q_count.ensure(std::max<uint64_t>(nq, 1))) ||
        (rc = h->h_nh.ensure(std::max<uint64_t>(nq, 1))) || (rc = h->h_no.ensure(std::max<uint64_t>(nq, 1))) ||
        (rc = h->h_row.ensure(nq + 1)) || (rc = h->h_orow.ensure(nq + 1)) ||
        (rc = h->h_sums.ensure(scan2_tmp_elems(nq))))
        return rc;
    if ((rc = dbi_query_device(h, d_mass, d_tol, nq, h->q_first.p, h->q_count.p, s))) return rc;
    DBI_HIP(launch_hits_offsets(h->q_first.p, h->q_count.p, h->occ_off.p, nq, h->h_nh.p, h->h_no.p, h->h_sums.p,
                                h->h_row.p, h->h_orow.p, h->h_sums.p + scan2_tmp_elems(nq) - 2, s));
    unsigned long long tot[2];
    DBI_HIP(hipMemcpyAsync(tot, h->h_sums.p + scan2_tmp_elems(nq) - 2, sizeof(tot), hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if ((rc = h->h_ids.ensure(std::max<uint64_t>(tot[0], 1))) || (rc = h->h_hocc.ensure(std::max<uint64_t>(tot[0], 1))) ||
        (rc = h->h_prot.ensure(std::max<uint64_t>(tot[1], 1))))
        return rc;
    DBI_HIP(launch_hits_expand(h->q_first.p, h->q_count.p, h->h_row.p, h->h_orow.p, h->occ_off.p, h->occ_pid.p, nq,
                               h->h_ids.p, h->h_hocc.p, h->h_prot.p, s));
    DBI_HIP(hipStreamSynchronize(s));
    out->row = h->h_row.p;
    out->ids = h->h_ids.p;
    out->occ_row = h->h_orow.p;
    out->hit_occ = h->h_hocc.p;
    out->prot = h->h_prot.p;
    out->nq = nq;
    out->n_hits = tot[0];
    out->n_prot_ids = tot[1];
    return 0;
}

int dbi_query_csr(dbi_handle* h, const double* mass, const double* tol, uint64_t nq, dbi_query_result** out) {
    if (!out || !h) return set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    std::vector<uint64_t> first(nq), count(nq);
    int rc = dbi_query(h, mass, tol, nq, first.data(), count.data());
    if (rc) return rc;
    dbi_query_result* r = (dbi_query_result*)std::calloc(1, sizeof(dbi_query_result));
    if (!r) return set_error(DBI_E_OOM, "calloc");
    r->nq = nq;
    r->row_ptr = (uint64_t*)std::malloc(8 * (nq + 1));
    if (!r->row_ptr) {
        dbi_query_result_free(r);
        return set_error(DBI_E_OOM, "malloc");
    }
    uint64_t tot = 0;
    for (uint64_t i = 0; i < nq; ++i) {
        r->row_ptr[i] = tot;
        tot += count[i];
    }
    r->row_ptr[nq] = tot;
    r->n_hits = tot;
    r->ids = (uint64_t*)std::malloc(8 * std::max<uint64_t>(tot, 1));
    if (!r->row_ptr || !r->ids) {
        dbi_query_result_free(r);
        return set_error(DBI_E_OOM, "malloc");
    }
    if (tot) {
        if ((rc = h->q_row.ensure(nq + 1)) || (rc = h->q_ids.ensure(tot))) {
            dbi_query_result_free(r);
            return rc;
        }
        hipError_t e = hipMemcpyAsync(h->q_row.p, r->row_ptr, 8 * (nq + 1), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = launch_expand_csr(h->q_first.p, h->q_count.p, h->q_row.p, nq, h->q_ids.p, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(r->ids, h->q_ids.p, 8 * tot, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            dbi_query_result_free(r);
            return hip_fail(e, "dbi_query_csr");
        }
    }
    *out = r;
    return 0;
}

void dbi_query_result_free(dbi_query_result* r) {
    if (!r) return;
    std::free(r->row_ptr);
    std::free(r->ids);
    std::free(r);
}

int dbi_peptides(dbi_handle* h, const uint64_t* ids, uint64_t n, double* mass, uint32_t* prot_id, uint32_t* offset,
                 uint32_t* length, uint64_t* occ_begin, uint64_t* occ_end) {
    if (!h || (n && !ids)) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    if (n == 0) return 0;
    for (uint64_t i = 0; i < n; ++i)
        if (ids[i] >= h->stats.n_unique) return set_error(DBI_E_INVALID, "peptide id out of range");
    DBI_HIP(hipSetDevice(h->device));
    int rc;
    if ((rc = h->q_ids.ensure(n)) || (rc = h->g_mass.ensure(n)) || (rc = h->g_pid.ensure(n)) ||
        (rc = h->g_off.ensure(n)) || (rc = h->g_len.ensure(n)) || (rc = h->g_b.ensure(n)) || (rc = h->g_e.ensure(n)))
        return rc;
    hipStream_t s = h->stream;
    DBI_HIP(hipMemcpyAsync(h->q_ids.p, ids, 8 * n, hipMemcpyHostToDevice, s));
    DBI_HIP(launch_gather(h->q_ids.p, n, h->umass.p, h->upid.p, h->uoff.p, h->ulen.p, h->occ_off.p, h->g_mass.p,
                          h->g_pid.p, h->g_off.p, h->g_len.p, h->g_b.p, h->g_e.p, s));
    if (mass) DBI_HIP(hipMemcpyAsync(mass, h->g_mass.p, 8 * n, hipMemcpyDeviceToHost, s));
    if (prot_id) DBI_HIP(hipMemcpyAsync(prot_id, h->g_pid.p, 4 * n, hipMemcpyDeviceToHost, s));
    if (offset) DBI_HIP(hipMemcpyAsync(offset, h->g_off.p, 4 * n, hipMemcpyDeviceToHost, s));
    if (length) DBI_HIP(hipMemcpyAsync(length, h->g_len.p, 4 * n, hipMemcpyDeviceToHost, s));
    if (occ_begin) DBI_HIP(hipMemcpyAsync(occ_begin, h->g_b.p, 8 * n, hipMemcpyDeviceToHost, s));
    if (occ_end) DBI_HIP(hipMemcpyAsync(occ_end, h->g_e.p, 8 * n, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    return 0;
}

int dbi_occurrences(dbi_handle* h, uint64_t begin, uint64_t end, uint32_t* prot_id) {
    if (!h || !prot_id) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    if (begin > end || end > h->stats.n_kept) return set_error(DBI_E_INVALID, "occurrence range out of bounds");
    if (end == begin) return 0;
    DBI_HIP(hipSetDevice(h->device));
    DBI_HIP(hipMemcpyAsync(prot_id, h->occ_pid.p + begin, 4 * (end - begin), hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    return 0;
}

int dbi_export(dbi_handle* h, double* mass, uint32_t* prot_id, uint32_t* offset, uint32_t* length, uint64_t* occ_off,
               uint32_t* occ_prot) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    DBI_HIP(hipSetDevice(h->device));
    const uint64_t U = h->stats.n_unique, K = h->stats.n_kept;
    hipStream_t s = h->stream;
    std::vector<uint32_t> oo;
    if (mass && U) DBI_HIP(hipMemcpyAsync(mass, h->umass.p, 8 * U, hipMemcpyDeviceToHost, s));
    if (prot_id && U) DBI_HIP(hipMemcpyAsync(prot_id, h->upid.p, 4 * U, hipMemcpyDeviceToHost, s));
    if (offset && U) DBI_HIP(hipMemcpyAsync(offset, h->uoff.p, 4 * U, hipMemcpyDeviceToHost, s));
    if (length && U) DBI_HIP(hipMemcpyAsync(length, h->ulen.p, 4 * U, hipMemcpyDeviceToHost, s));
    if (occ_off) {
        oo.resize(U + 1);
        DBI_HIP(hipMemcpyAsync(oo.data(), h->occ_off.p, 4 * (U + 1), hipMemcpyDeviceToHost, s));
    }
    if (occ_prot && K) DBI_HIP(hipMemcpyAsync(occ_prot, h->occ_pid.p, 4 * K, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if (occ_off)
        for (uint64_t i = 0; i <= U; ++i) occ_off[i] = oo[i];
    return 0;
}

int dbi_entry_keys(dbi_handle* h, int32_t* keys, uint64_t cap, uint64_t* n) {
    if (!h || !n) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    *n = h->stats.n_keys;
    if (!keys) return 0;
    if (cap < h->stats.n_keys) return set_error(DBI_E_INVALID, "keys buffer too small");
    const uint64_t U = h->stats.n_unique;
    if (U == 0) return 0;
    DBI_HIP(hipSetDevice(h->device));
    DevBuf<uint32_t> flags, pos;
    DevBuf<int32_t> dk;
    int rc;
    if ((rc = flags.ensure(U)) || (rc = pos.ensure(U)) || (rc = dk.ensure(h->stats.n_keys))) {
        flags.release();
        pos.release();
        dk.release();
        return rc;
    }
    if ((rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(U), h->scan_tmp.cap)))) return rc;
    hipError_t e = launch_key_flags(h->umass.p, (uint32_t)U, h->params.mass_group_factor, flags.p, h->stream);
    if (e == hipSuccess)
        e = launch_scan_u32(flags.p, pos.p, U, h->scan_tmp.p, h->scan_tmp.cap, nullptr, h->stream);
    if (e == hipSuccess)
        e = launch_write_keys(h->umass.p, (uint32_t)U, h->params.mass_group_factor, pos.p, dk.p, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(keys, dk.p, 4 * h->stats.n_keys, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    flags.release();
    pos.release();
    dk.release();
    if (e != hipSuccess) return hip_fail(e, "dbi_entry_keys");
    return 0;
}

int dbi_set_bucket_drop(dbi_handle* h, int on) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    if (!on && !(h->params.max_mh < 65536.0))
        return set_error(DBI_E_INVALID, "without buckets every peptide up to the max precursor mass is kept: "
                                        "max precursor mass must be < 65536 Da");
    h->dp.buckets = on ? 1 : 0;
    h->dp.drop_mass = on ? (double)(h->dp.nb * h->dp.br) : INFINITY;
    ++h->dp_gen;
    h->built = false;  // an index built under the other setting no longer answers
    return 0;
}

int dbi_set_windows(dbi_handle* h, const double* mass, const double* tol, uint64_t n, int on) {
    if (!h || (n && on && (!mass || !tol))) return set_error(DBI_E_INVALID, "NULL argument");
    if (on && h->dp.buckets) return set_error(DBI_E_STATE, "a window filter needs the bucket drop off");
    h->built = false;
    ++h->dp_gen;
    if (!on) {
        h->dp.filter = 0;
        h->dp.n_win = 0;
        h->dp.win_max = INFINITY;
        h->dp.win_lo = h->dp.win_hi = nullptr;
        h->dp.cut_count = make_dev_params(h->params).cut_count;
        return 0;
    }
    // MassRangeFilteringIndex.init (:51-65): [m - tol, m + tol]; a NaN bound
    // includes nothing; sorted and merged into disjoint intervals
    std::vector<std::pair<double, double>> iv;
    for (uint64_t i = 0; i < n; ++i) {
        const double lo = mass[i] - tol[i], hi = mass[i] + tol[i];
        if (lo == lo && hi == hi && lo <= hi) iv.push_back({lo, hi});
    }
    std::sort(iv.begin(), iv.end());
    std::vector<double> wl, wh;
    for (auto& r : iv) {
        if (!wl.empty() && r.first <= wh.back()) wh.back() = std::max(wh.back(), r.second);
        else { wl.push_back(r.first); wh.push_back(r.second); }
    }
    int rc;
    if ((rc = h->win_lo.ensure(std::max<size_t>(wl.size(), 1))) || (rc = h->win_hi.ensure(std::max<size_t>(wh.size(), 1))))
        return rc;
    if (!wl.empty()) {
        DBI_HIP(hipMemcpyAsync(h->win_lo.p, wl.data(), 8 * wl.size(), hipMemcpyHostToDevice, h->stream));
        DBI_HIP(hipMemcpyAsync(h->win_hi.p, wh.data(), 8 * wh.size(), hipMemcpyHostToDevice, h->stream));
        DBI_HIP(hipStreamSynchronize(h->stream));
    }
    h->dp.filter = 1;
    h->dp.n_win = (uint32_t)wl.size();
    h->dp.win_max = wl.empty() ? -INFINITY : wh.back();
    h->dp.win_lo = h->win_lo.p;
    h->dp.win_hi = h->win_hi.p;
    h->dp.cut_count = 0;  // the stepping count does not see masses per peptide
    return 0;
}

int dbi_rebuild(dbi_handle* h) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    if (!h->inputs_resident || h->d_res != h->res.p || h->d_poff != h->poff.p)
        return set_error(DBI_E_STATE, "no resident inputs: dbi_build from host arrays first");
    if (h->inputs_ptm)
        return set_error(DBI_E_INVALID, "dbi_rebuild after a build with inline '[formula]' PTMs: call dbi_build "
                                        "again (the resident text still holds the formulas)");
    int rc;
    const uint64_t n_res = h->n_res, n_prot = h->n_prot;
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    h->d_res = h->res.p;
    h->d_poff = h->poff.p;
    if ((rc = build_digest(h))) return rc;
    return finish_build(h);
}

int dbi_set_option(dbi_handle* h, const char* name, int64_t value) {
    if (!h || !name) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lk(h->qmu);
    const std::string n(name);
    const bool on = value != 0;
    auto ranged = [&](int64_t lo, int64_t hi) { return value >= lo && value <= hi; };
    if (n == "build_graph") h->use_graph = on;
    else if (n == "digest_hist") h->use_h1 = on;
    else if (n == "semi_bounded") h->use_semi_bounded = on;
    else if (n == "depth_bins") h->use_depth = on;
    else if (n == "owner_depth") h->opt_owner_depth = on;
    else if (n == "big_side") h->opt_big_side = on;
    else if (n == "semi_part") h->use_semi_part = on;
    else if (n == "part_stage") h->use_part_stage = on;
    else if (n == "depth_map_reuse") h->opt_depth_map_reuse = on;
    else if (n == "big_split" && ranged(-1, 1)) h->big_split = (int)value;
    else if (n == "bin_bits_max" && ranged(1, 32)) h->bin_bits_max = (int)value;
    else if (n == "split_above" && ranged(1, 1ll << 31)) h->split_above = (uint32_t)value;
    else if (n == "chunk_target" && (value == 0 || ranged(64, CHUNK_CAP))) h->chunk_t = (uint32_t)value;
    else if (n == "shard_full_path") h->opt_shard_full_path = on;
    else if (n == "shard_dev_digest") h->opt_shard_dev_digest = on;
    else if (n == "shard_resample") h->opt_shard_resample = on;
#ifdef DBI_TEST_HOOKS  // (test builds: libdbindex_hip_hooks.so)
    else if (n == "test_split_skew" && ranged(-1, 1 << 20)) h->opt_test_split_skew = (int)value;
#endif
    else return set_error(DBI_E_INVALID, "unknown option or value out of range: " + n);
    drop_graph(h);  // a captured build bakes the old setting in
    h->prev_key_valid = false;
    return 0;
}

int dbi_set_option_str(dbi_handle* h, const char* name, const char* value) {
    if (!h || !name || !value) return set_error(DBI_E_INVALID, "NULL argument");
    std::lock_guard<std::recursive_mutex> lk(h->qmu);
#ifdef DBI_TEST_HOOKS  // (test builds: libdbindex_hip_hooks.so)
    if (std::string(name) == "test_fail") {
        h->opt_test_fail = value;
        return 0;
    }
#endif
    return set_error(DBI_E_INVALID, std::string("unknown string option: ") + name);
}

int dbi_set_cold(dbi_handle* h) {
    if (!h) return set_error(DBI_E_INVALID, "null handle");
    std::lock_guard<std::recursive_mutex> lk(h->qmu);
    drop_graph(h);
    h->force_cold = true;
    h->prev_key_valid = false;
    h->grid_mid = h->grid_big = h->grid_split = 0;
    h->depth_map_of = nullptr;
    h->giants_seen = true;
    return 0;
}

int dbi_set_timing(dbi_handle* h, int on, const char* only) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    h->timing = on != 0;
    h->timing_only = only ? only : "";
    return 0;
}

int dbi_stage_times(dbi_handle* h, const char** names, double* ms, double* bytes, uint64_t cap, uint64_t* n) {
    if (!h || !n) return set_error(DBI_E_INVALID, "NULL argument");
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    *n = (uint64_t)h->nstage;
    for (int i = 0; i < h->nstage && (uint64_t)i < cap; ++i) {
        if (names) names[i] = h->stages[i].name;
        if (ms) ms[i] = h->stages[i].ms;
        if (bytes) bytes[i] = h->stages[i].bytes;
    }
    return 0;
}

int dbi_device_view(dbi_handle* h, dbi_device_index* out) {
    if (!h || !out) return set_error(DBI_E_INVALID, "NULL argument");
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    out->mass = h->umass.p;
    out->prot_id = h->upid.p;
    out->offset = h->uoff.p;
    out->length = h->ulen.p;
    out->occ_off = h->occ_off.p;
    out->occ_prot = h->occ_pid.p;
    out->n_unique = h->stats.n_unique;
    out->n_kept = h->stats.n_kept;
    return 0;
}

}  // extern "C"

// ---- internal accessors used by the store mirror (dbi_store.cpp) ----------------
namespace dbi {
int engine_key_range(dbi_handle* h, int32_t klo, int32_t khi, uint64_t* b, uint64_t* e) {
    // a query-side call: same lock as dbi_query* (shared stream), own scratch
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    if (!h->built) return set_error(DBI_E_STATE, "index not built");
    DBI_HIP(hipSetDevice(h->device));
    int rc;
    if ((rc = h->kr_scratch.ensure(2))) return rc;
    DBI_HIP(launch_key_range(h->umass.p, (uint32_t)h->stats.n_unique, h->params.mass_group_factor, klo, khi,
                             h->kr_scratch.p, h->stream));
    uint64_t r[2];
    DBI_HIP(hipMemcpyAsync(r, h->kr_scratch.p, 16, hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    *b = r[0];
    *e = r[1];
    return 0;
}
bool engine_built(const dbi_handle* h) { return h && h->built; }
const dbi_params& engine_params(const dbi_handle* h) { return h->params; }
}  // namespace dbi
