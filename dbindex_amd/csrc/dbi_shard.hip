// dbi_shard.hip — sharded build: one index over the proteins of every shard.
//
// The reference builds one index over the whole FASTA in one thread
// (DBIndexer.run, DBIndexer.java:508-684).  Here the proteome is split into
// contiguous protein ranges, one per GPU.  Each shard digests its own proteins
// (cutSeq, DBIndexer.java:237-405), then every record goes to the shard that
// OWNS its mass key (int)(mass*factor) (DBIndexStoreSQLiteByte.java:187): the
// owners hold contiguous key ranges, so the same peptide — same string, same
// bit-identical mass, same key — from any shard meets at one owner, which
// sorts, de-duplicates and finalises its range exactly like a single-device
// build (IndexMerge.getMergedData, DBIndexStoreSQLiteByteIndexMerge.java:620-719).
// The record carries (mass, tag, global protein id, offset, length), and the
// owner's result is a pure function of the set of records it receives, so the
// order in which shards' records arrive does not matter.
//
// Exchange: 8 B per record (global protein | offset | length; the owner
// recomputes mass and tag from the residues, k_expand_locs), RCCL
// point-to-point sends/receives grouped over all peers (each
// pair of MI355X GPUs has its own xGMI link, so the grouped exchange drives
// all links at once; a ring would serialise them), or device copies between
// the handles of one process (dbi_shard_exchange_local).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "dbi_engine.h"

using namespace dbi;

struct dbi_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1;
    int rank = 0;
    int device = 0;
    unsigned long long* d_flag = nullptr;  // failure agreement (agree())
    hipStream_t stream = nullptr;          // host-buffer collectives (dbi_comm_allreduce_*)
    double* d_red = nullptr;               // their staging (COMM_RED_MAX values)
    // the sharded build's small collectives (sample blocks, count matrix,
    // totals) stage through these, allocated with the communicator: a rank
    // never fails an allocation between two collectives of a build
    double* d_samp = nullptr;              // nranks x (DBI_SHARD_SAMPLES + 2)
    unsigned long long* d_cnt = nullptr;   // nranks x cnt_row
    int cnt_row = 0;                       // max(nranks + 2, 7)
};
constexpr uint32_t COMM_RED_MAX = 4096;

namespace dbi {
namespace {

constexpr uint32_t NS = DBI_SHARD_SAMPLES;

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int nccl_fail(ncclResult_t r, const char* what) {
    return set_error(DBI_E_RCCL, std::string("RCCL error ") + ncclGetErrorString(r) + " in " + what);
}

#define DBI_NCCL(expr)                                        \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return nccl_fail(_r, #expr);   \
    } while (0)

int need_phase(const dbi_handle* h, int phase, const char* what) {
    if (h->shard.phase != phase)
        return set_error(DBI_E_STATE, std::string(what) + ": sharded build phases must run in order "
                                                          "(digest, samples/splitters, partition, exchange, merge)");
    return 0;
}

__global__ void k_set_u64(unsigned long long* p, unsigned long long v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *p = v;
}

// send counts of a partitioned shard, straight from the scanned owner
// histogram (hist[d * g] = first output position of owner d's run)
__global__ void k_owner_counts(const uint32_t* __restrict__ hist, uint64_t g, uint32_t ns, uint64_t n_total,
                               unsigned long long* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= ns) return;
    const uint64_t a = n_total ? hist[(uint64_t)d * g] : 0u;
    const uint64_t b = (d + 1 < ns && n_total) ? hist[(uint64_t)(d + 1) * g] : n_total;
    out[d] = b - a;
}

// Stage whose time comes from events recorded around non-kernel work (RCCL,
// copies) rather than from a dispatch packet; `bytes` = bytes this rank moves.
struct ManualStage {
    dbi_handle* h;
    int i;
    hipEvent_t e1 = nullptr;
    ManualStage(dbi_handle* hh, const char* name, double bytes) : h(hh) {
        i = stage_begin(h, name, by(0, 0, 0, 0, 0));
        hipEvent_t e0 = t_launch_ev.start;
        e1 = t_launch_ev.stop;
        t_launch_ev = LaunchEvents{};
        if (i >= 0) {
            h->stages[i].c0 = bytes;
            h->stages[i].launched = e0 != nullptr && hipEventRecord(e0, h->stream) == hipSuccess;
        }
    }
    void end() {
        if (i >= 0 && h->stages[i].launched && e1) h->stages[i].launched = hipEventRecord(e1, h->stream) == hipSuccess;
    }
};

// owner key range of shard r under `split`
void key_range(const int32_t* split, int nshards, int r, int32_t* lo, int32_t* hi) {
    *lo = r == 0 ? INT32_MIN : split[r - 1];
    *hi = r == nshards - 1 ? INT32_MAX : split[r];
}

// Items from every rank to every rank: item slices [soff[p], +scnt[p]) of
// `send` go to rank p, which receives them at its roff[me]; one group of
// point-to-point transfers over all peers, the rank's own slice by a copy
template <typename T>
int nccl_alltoallv(dbi_comm* c, const T* send, const std::vector<uint64_t>& soff, const std::vector<uint64_t>& scnt,
                   T* recv, const std::vector<uint64_t>& roff, const std::vector<uint64_t>& rcnt, hipStream_t s) {
    const int me = c->rank;
    if (scnt[me])
        DBI_HIP(hipMemcpyAsync(recv + roff[me], send + soff[me], scnt[me] * sizeof(T), hipMemcpyDeviceToDevice, s));
    DBI_NCCL(ncclGroupStart());
    for (int p = 0; p < c->nranks; ++p) {
        if (p == me) continue;
        if (scnt[p]) DBI_NCCL(ncclSend(send + soff[p], scnt[p] * sizeof(T), ncclUint8, p, c->comm, s));
        if (rcnt[p]) DBI_NCCL(ncclRecv(recv + roff[p], rcnt[p] * sizeof(T), ncclUint8, p, c->comm, s));
    }
    DBI_NCCL(ncclGroupEnd());
    return 0;
}

// Local failures must not strand the other ranks inside the next collective:
// every rank reports its status with the data of a collective it would run
// anyway (a status column in the count matrix and the totals, a status word
// in the samples), or through agree() where no such collective comes first,
// and all ranks return an error together.
int peer_failed(const char* phase) {
    return set_error(DBI_E_STATE, std::string("another rank failed (") + phase + "); see that rank's error");
}

// Test hook: DBI_TEST_FAIL="<phase>@<rank>" makes that rank fail locally at
// that phase (digest, partition, buffers, merge, qroute, qbuffers), so the
// agreement paths run without a real failure.
int injected_failure(const char* phase, int rank) {
    const char* e = std::getenv("DBI_TEST_FAIL");
    if (!e || std::string(e) != std::string(phase) + "@" + std::to_string(rank)) return 0;
    return set_error(DBI_E_STATE, std::string("injected failure (DBI_TEST_FAIL) in ") + phase);
}

// max over ranks of (rc != 0): 0 when every rank succeeded
int agree(dbi_comm* c, int rc, hipStream_t s, bool* any) {
    const unsigned long long mine = rc ? 1ull : 0ull;
    unsigned long long all = 0;
    DBI_HIP(hipMemcpyAsync(c->d_flag, &mine, sizeof(mine), hipMemcpyHostToDevice, s));
    DBI_NCCL(ncclAllReduce(c->d_flag, c->d_flag + 1, 1, ncclUint64, ncclMax, c->comm, s));
    DBI_HIP(hipMemcpyAsync(&all, c->d_flag + 1, sizeof(all), hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    *any = all != 0;
    return 0;
}

// all[i * n + j] = mine_i[j] of every rank i (u64 all-gather through c->d_cnt),
// with each rank's status (rc != 0) in a last column: *any_failed
int nccl_count_matrix(dbi_handle* h, dbi_comm* c, const std::vector<uint64_t>& mine, int status,
                      std::vector<uint64_t>& all, bool* any_failed) {
    const int n = c->nranks, me = c->rank, w = n + 1;
    hipStream_t s = h->stream;
    std::vector<uint64_t> full((size_t)n * w, 0);
    for (int j = 0; j < n && j < (int)mine.size(); ++j) full[(size_t)me * w + j] = mine[j];
    full[(size_t)me * w + n] = status ? 1u : 0u;
    DBI_HIP(hipMemcpyAsync(c->d_cnt + (size_t)me * w, full.data() + (size_t)me * w, sizeof(uint64_t) * w,
                           hipMemcpyHostToDevice, s));
    DBI_NCCL(ncclAllGather(c->d_cnt + (size_t)me * w, c->d_cnt, w, ncclUint64, c->comm, s));
    DBI_HIP(hipMemcpyAsync(full.data(), c->d_cnt, sizeof(uint64_t) * n * w, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    all.assign((size_t)n * n, 0);
    *any_failed = false;
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) all[(size_t)i * n + j] = full[(size_t)i * w + j];
        *any_failed |= full[(size_t)i * w + n] != 0;
    }
    return 0;
}

void offsets_of(const std::vector<uint64_t>& cnt, std::vector<uint64_t>& off) {
    off.assign(cnt.size() + 1, 0);
    for (size_t i = 0; i < cnt.size(); ++i) off[i + 1] = off[i] + cnt[i];
}

// ---- routed queries (the owner slices of a sharded index) ----
int query_route(dbi_handle* h, const double* d_m, const double* d_t, uint64_t nq) {
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;
    if (nq >= (1ull << 31)) return set_error(DBI_E_INVALID, "at most 2^31-1 queries per batch and rank");
    RouteMap rm{};
    for (int j = 0; j + 1 < sh.nshards; ++j) rm.split[j] = sh.split[j];
    rm.nshards = (uint32_t)sh.nshards;
    rm.factor = h->params.mass_group_factor;
    rm.nb = h->dp.nb;
    rm.br = h->dp.br;
    int rc;
    if ((rc = h->qcnt.ensure(nq + 1)) || (rc = h->xcount.ensure(std::max<size_t>(h->xcount.cap, 8))) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(nq + 1), h->scan_tmp.cap))))
        return rc;
    DBI_HIP(launch_qroute_count(d_m, d_t, nq, rm, h->qcnt.p, s));
    unsigned long long np = 0;
    if (nq) {
        DBI_HIP(launch_scan_u32(h->qcnt.p, h->qcnt.p, nq, h->scan_tmp.p, h->scan_tmp.cap, h->xcount.p, s));
        DBI_HIP(hipMemcpyAsync(&np, h->xcount.p, sizeof(np), hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
    }
    const int ns = sh.nshards, bits = owner_bits((uint32_t)ns);
    const uint32_t n32 = (uint32_t)np;
    const uint64_t g = radix_blocks(n32);
    const size_t hist_elems = std::max<size_t>(radix_hist_elems(n32, bits), 1);
    if ((rc = h->qpairA.ensure(np + 1)) || (rc = h->qpairB.ensure(np + 1)) || (rc = h->qsend.ensure(np + 1)) ||
        (rc = h->qback.ensure(np + 1)) || (rc = h->hist.ensure(std::max<size_t>(hist_elems, h->hist.cap))) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(hist_elems), h->scan_tmp.cap))))
        return rc;
    std::vector<uint32_t> start(ns + 1, 0);
    if (np) {
        DBI_HIP(launch_qroute_emit(d_m, d_t, nq, rm, h->qcnt.p, h->qpairA.p, s));
        DBI_HIP(launch_pair_hist(h->qpairA.p, n32, (uint32_t)ns, h->hist.p, s));
        DBI_HIP(launch_scan_u32(h->hist.p, h->hist.p, g << bits, h->scan_tmp.p, h->scan_tmp.cap, nullptr, s));
        DBI_HIP(launch_pair_scatter(h->qpairA.p, h->qpairB.p, n32, (uint32_t)ns, h->hist.p, s));
        DBI_HIP(launch_qpack(h->qpairB.p, np, d_m, d_t, h->qsend.p, s));
        DBI_HIP(hipMemcpy2DAsync(start.data(), sizeof(uint32_t), h->hist.p, g * sizeof(uint32_t), sizeof(uint32_t),
                                 (size_t)ns, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
    }
    start[ns] = n32;
    sh.q_n = nq;
    sh.q_pairs = np;
    sh.qsend_count.assign(ns, 0);
    for (int d = 0; d < ns; ++d) sh.qsend_count[d] = (uint64_t)start[d + 1] - start[d];
    offsets_of(sh.qsend_count, sh.qsend_off);
    return 0;
}

int query_answer(dbi_handle* h) {
    ShardState& sh = h->shard;
    int rc;
    if ((rc = h->qres.ensure(sh.q_recv + 1)) || (rc = ensure_qdir(h, h->stream))) return rc;
    DBI_HIP(launch_query_pairs(h->dp, h->params.mass_group_factor, h->umass.p, (uint32_t)h->stats.n_unique,
                               h->qrecv.p, sh.q_recv, sh.u_base, h->qres.p, h->qdir_par.p, h->qdir.p, h->stream));
    return 0;
}

// ---- replicated index (every owner's slice on every rank) ----
__global__ void k_add_u32(uint32_t* __restrict__ p, uint64_t n, uint32_t add) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += add;
}

struct SliceSizes {
    std::vector<uint64_t> u, k;  // per shard: unique peptides, occurrences
    std::vector<uint64_t> ub, kb; // their bases in the whole index (nshards + 1)
};

void slice_bases(SliceSizes& z) {
    const size_t n = z.u.size();
    z.ub.assign(n + 1, 0);
    z.kb.assign(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
        z.ub[i + 1] = z.ub[i] + z.u[i];
        z.kb[i + 1] = z.kb[i] + z.k[i];
    }
}

int replica_check(const SliceSizes& z) {
    if (z.kb.back() >= (1ull << 32) - 1 || z.ub.back() >= (1ull << 32) - 1)
        return set_error(DBI_E_INVALID, "a replicated index holds at most 2^32-2 occurrences per device");
    return 0;
}

int replica_alloc(dbi_handle* h, const SliceSizes& z) {
    const uint64_t U = z.ub.back(), K = z.kb.back();
    int rc;
    if ((rc = h->r_mass.ensure(std::max<uint64_t>(U, 1))) || (rc = h->r_pid.ensure(std::max<uint64_t>(U, 1))) ||
        (rc = h->r_off.ensure(std::max<uint64_t>(U, 1))) || (rc = h->r_len.ensure(std::max<uint64_t>(U, 1))) ||
        (rc = h->r_occ_off.ensure(U + 1)) || (rc = h->r_occ.ensure(std::max<uint64_t>(K, 1))))
        return rc;
    return 0;
}

// slice i's occurrence offsets are local to it: add the occurrences of the
// slices before it; the table ends at K
int replica_rebase(dbi_handle* h, const SliceSizes& z, hipStream_t s) {
    const size_t n = z.u.size();
    for (size_t i = 0; i < n; ++i)
        if (z.u[i] && z.kb[i]) {
            hipLaunchKernelGGL(k_add_u32, dim3((uint32_t)((z.u[i] + 255) / 256)), dim3(256), 0, s,
                               h->r_occ_off.p + z.ub[i], z.u[i], (uint32_t)z.kb[i]);
            DBI_HIP(hipGetLastError());
        }
    const uint32_t K = (uint32_t)z.kb.back();
    DBI_HIP(hipMemcpyAsync(h->r_occ_off.p + z.ub.back(), &K, 4, hipMemcpyHostToDevice, s));
    DBI_HIP(hipStreamSynchronize(s));  // K is a stack value
    return 0;
}

// the replica becomes the handle's index: the whole proteome, queried locally
void replica_install(dbi_handle* h, const SliceSizes& z, uint64_t g_total, uint64_t g_dropped, uint64_t g_keys) {
    // a captured build graph writes the index buffers being swapped out here
    drop_graph(h);
    h->prev_key_valid = false;
    g_alloc_gen.fetch_add(1, std::memory_order_relaxed);
    std::swap(h->umass, h->r_mass);
    std::swap(h->upid, h->r_pid);
    std::swap(h->uoff, h->r_off);
    std::swap(h->ulen, h->r_len);
    std::swap(h->occ_off, h->r_occ_off);
    std::swap(h->occ_pid, h->r_occ);
    h->r_mass.release(); h->r_pid.release(); h->r_off.release(); h->r_len.release();
    h->r_occ_off.release(); h->r_occ.release();
    dbi_stats& st = h->stats;
    st.n_unique = z.ub.back();
    st.n_kept = z.kb.back();
    st.n_total = g_total;
    st.n_dropped = g_dropped;
    st.n_keys = g_keys;
    st.n_residues = h->n_res;
    st.n_proteins = h->n_prot;
    ++h->build_serial;  // a new query directory
    h->shard.phase = 5;
}

int query_need(const dbi_handle* h) {
    if (h->shard.phase != 4 || !h->built || !h->shard.u_base_known)
        return set_error(DBI_E_STATE, "sharded queries need a finished sharded build (dbi_build_sharded, or the "
                                      "phases through dbi_shard_merge on every shard)");
    return 0;
}

}  // namespace
}  // namespace dbi

extern "C" {

int dbi_shard_digest(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_poff, uint64_t n_prot,
                     uint64_t p_begin, uint64_t p_end, int rank, int nshards) {
    if (!h || (!d_res && n_res) || !d_poff) return set_error(DBI_E_INVALID, "NULL argument");
    if (nshards < 1 || nshards > MAX_SHARDS || rank < 0 || rank >= nshards)
        return set_error(DBI_E_INVALID, "shard rank / count out of range (1..64 shards)");
    if (p_begin > p_end || p_end > n_prot) return set_error(DBI_E_INVALID, "shard protein range out of bounds");
    int rc;
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    const double t0 = now_ms();
    hipStream_t s = h->stream;
    uint64_t ends[2] = {0, 0};
    DBI_HIP(hipMemcpyAsync(&ends[0], d_poff + p_begin, 8, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipMemcpyAsync(&ends[1], d_poff + p_end, 8, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if (ends[0] > ends[1] || ends[1] > n_res) return set_error(DBI_E_INVALID, "prot_off is not a valid offset table");
    const uint64_t np = p_end - p_begin;
    if ((rc = h->poff_g.ensure(n_prot + 1)) || (rc = h->poff.ensure(np + 1))) return rc;
    // global u32 offsets (owner merge) + this shard's offsets rebased to its first residue
    DBI_HIP(launch_off_rebase(d_poff, 0, h->poff_g.p, n_prot + 1, s));
    DBI_HIP(launch_off_rebase(d_poff + p_begin, ends[0], h->poff.p, np + 1, s));
    // the record field width W comes from the longest protein of the WHOLE
    // proteome, so every shard packs records the same way
    DBI_HIP(launch_max_plen(h->poff_g.p, (uint32_t)n_prot, h->ctr.p, s));

    ShardState& sh = h->shard;
    sh = ShardState{};
    sh.rank = rank;
    sh.nshards = nshards;
    sh.p_begin = p_begin;
    sh.p_end = p_end;
    sh.n_res_global = n_res;
    sh.n_prot_global = n_prot;
    sh.d_res_global = d_res;
    h->d_res = d_res + ends[0];
    h->d_poff = h->poff.p;
    h->n_res = ends[1] - ends[0];
    h->n_prot = np;
    uint64_t n = 0, n_in = 0;
    bool sparse = false;
    if (h->n_res > 0) {
        if ((rc = run_digest(h, &n, &n_in, &sparse, nullptr))) return rc;
    } else if ((rc = read_counters(h))) {
        return rc;
    }
    if (h->hc.err & ERR_LAYOUT) return set_error(DBI_E_INVALID, "record layout overflow in the shard digest");
    if (h->hc.err & ERR_PTM) return set_error(DBI_E_INVALID, ptm_device_msg());
    // the digest stages' algorithmic bytes are this shard's (the handle turns
    // into the owner of a slice of the whole proteome at the merge)
    for (int i = 0; i < h->nstage; ++i) {
        auto& st = h->stages[i];
        st.c0 += st.cR * (double)h->n_res + st.cN * (double)h->hc.n_kept + st.cP * (double)(np + 1);
        st.cR = st.cN = st.cU = st.cP = st.cB = 0;
    }
    sh.width = rec_width(h->hc.max_plen);
    if (!rec_layout_ok(sh.width, n_prot))
        return set_error(DBI_E_INVALID, "2 x bits(longest protein) + bits(protein count) of the whole proteome "
                                        "exceeds the 56 bits of the 16-B occurrence record");
    sh.n_digest = n;
    sh.n_in = n_in;
    sh.sparse = sparse;
    sh.n_total = h->hc.n_kept + h->hc.n_dropped;
    sh.n_dropped = h->hc.n_dropped;
    sh.ms_digest = now_ms() - t0;
    sh.phase = 1;
    return 0;
}

int dbi_shard_samples(dbi_handle* h, double* samples) {
    if (!h || !samples) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = need_phase(h, 1, "dbi_shard_samples"))) return rc;
    if ((rc = h->samp.ensure(NS))) return rc;
    DBI_HIP(launch_sample_masses(h->recA.p, h->shard.n_in, NS, h->samp.p, h->stream));
    DBI_HIP(hipMemcpyAsync(samples, h->samp.p, sizeof(double) * NS, hipMemcpyDeviceToHost, h->stream));
    DBI_HIP(hipStreamSynchronize(h->stream));
    uint64_t valid = 0;
    for (uint32_t i = 0; i < NS; ++i) valid += samples[i] == samples[i];
    samples[NS] = valid ? (double)h->shard.n_digest / (double)valid : 0.0;
    return 0;
}

int dbi_shard_splitters(const double* samples, int nshards, int32_t factor, int32_t* split) {
    return dbi_shard_splitters_cost(samples, nshards, factor, 0, nullptr, nullptr, split);
}

int dbi_shard_splitters_cost(const double* samples, int nshards, int32_t factor, int nbands,
                             const int32_t* band_split, const double* band_cost, int32_t* split) {
    if (!samples || (!split && nshards > 1)) return set_error(DBI_E_INVALID, "NULL argument");
    if (nshards < 1 || nshards > MAX_SHARDS) return set_error(DBI_E_INVALID, "1..64 shards");
    if (factor <= 0) return set_error(DBI_E_INVALID, "mass_group_factor must be > 0");
    if (band_cost) {
        if (nbands < 1 || (nbands > 1 && !band_split)) return set_error(DBI_E_INVALID, "bad band profile");
        for (int r = 0; r < nbands; ++r)
            if (!(band_cost[r] > 0.0) || !std::isfinite(band_cost[r]))
                return set_error(DBI_E_INVALID, "band costs must be finite and > 0");
        for (int r = 0; r + 2 < nbands; ++r)
            if (band_split[r] > band_split[r + 1]) return set_error(DBI_E_INVALID, "band splits must ascend");
    }
    std::vector<std::pair<int32_t, double>> ks;
    for (int r = 0; r < nshards; ++r) {
        const double* b = samples + (size_t)r * (NS + 1);
        const double w = b[NS];
        if (!(w > 0.0)) continue;
        for (uint32_t i = 0; i < NS; ++i) {
            if (b[i] != b[i]) continue;
            const int32_t k = java_d2i(b[i] * (double)factor);
            double c = 1.0;
            if (band_cost)  // band of k: the number of band boundaries <= k
                c = band_cost[std::upper_bound(band_split, band_split + (nbands - 1), k) - band_split];
            ks.emplace_back(k, w * c);
        }
    }
    std::sort(ks.begin(), ks.end());
    double total = 0.0;
    for (const auto& k : ks) total += k.second;
    // split[j-1] = first key whose preceding weight reaches j/n of the total
    size_t i = 0;
    double cum = 0.0;
    for (int j = 1; j < nshards; ++j) {
        const double target = total * (double)j / (double)nshards;
        int32_t sp = INT32_MAX;
        for (; i < ks.size(); ++i) {
            if (cum >= target && (i == 0 || ks[i].first != ks[i - 1].first)) {
                sp = ks[i].first;
                break;
            }
            cum += ks[i].second;
        }
        split[j - 1] = sp;
    }
    return 0;
}

namespace {
constexpr int CB = DBI_COST_BANDS;
// the fixed key bands of the cost profile: CB equal key ranges of [minMH, maxMH]
void cost_bands(const dbi_handle* h, int32_t* bsplit) {
    const double f = (double)h->params.mass_group_factor;
    const double k0 = h->params.min_mh * f, k1 = h->params.max_mh * f;
    for (int b = 1; b < CB; ++b) bsplit[b - 1] = (int32_t)std::floor(k0 + (k1 - k0) * (double)b / (double)CB);
}
}  // namespace

int dbi_shard_cost_update(dbi_handle* h, int nshards, const int32_t* split, const double* merge_ms,
                          const uint64_t* records) {
    if (!h || !merge_ms || !records || (nshards > 1 && !split)) return set_error(DBI_E_INVALID, "NULL argument");
    if (nshards < 2 || nshards > MAX_SHARDS) return 0;  // one owner: nothing to balance
    for (int r = 0; r < nshards; ++r)
        if (!(merge_ms[r] > 0.0) || records[r] == 0) return 0;  // an owner without a measurement: keep the profile
    int32_t bs[CB - 1];
    cost_bands(h, bs);
    // each band takes the cost per record of the owner holding its middle key,
    // averaged with what it had (the owners' ranges move between builds, so
    // the bands see different owners: the average settles instead of swinging)
    auto& pf = h->shard_prof;
    const double f = (double)h->params.mass_group_factor;
    const double k0 = h->params.min_mh * f, k1 = h->params.max_mh * f;
    for (int b = 0; b < CB; ++b) {
        const double mid = k0 + (k1 - k0) * ((double)b + 0.5) / (double)CB;
        int r = 0;
        while (r + 1 < nshards && (double)split[r] <= mid) ++r;
        const double c = merge_ms[r] / (double)records[r];
        pf.cost[b] = pf.valid ? 0.5 * pf.cost[b] + 0.5 * c : c;
    }
    std::copy(bs, bs + CB - 1, pf.split);
    pf.valid = true;
    return 0;
}

int dbi_shard_splitters_profiled(dbi_handle* h, const double* samples, int nshards, int32_t* split) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    const auto& pf = h->shard_prof;
    return dbi_shard_splitters_cost(samples, nshards, h->params.mass_group_factor, pf.valid ? CB : 0,
                                    pf.valid ? pf.split : nullptr, pf.valid ? pf.cost : nullptr, split);
}

}  // extern "C"

namespace dbi {
namespace {
// The partition's kernels (no host synchronisation): records routed to
// xsend by owner; the scanned owner histogram is left in h->hist
int partition_launch(dbi_handle* h, const int32_t* split) {
    int rc;
    if ((rc = need_phase(h, 1, "dbi_shard_partition"))) return rc;
    ShardState& sh = h->shard;
    const int ns = sh.nshards;
    for (int j = 0; j + 2 < ns; ++j)
        if (split[j] > split[j + 1]) return set_error(DBI_E_INVALID, "splitter keys must be non-decreasing");
    hipStream_t s = h->stream;
    OwnerMap om{};
    for (int j = 0; j + 1 < ns; ++j) om.split[j] = sh.split[j] = split[j];
    om.nshards = (uint32_t)ns;
    om.factor = h->params.mass_group_factor;
    om.pid_add = sh.p_begin << (2 * sh.width);
    const int bits = owner_bits((uint32_t)ns);
    const uint32_t n_in = (uint32_t)sh.n_in;
    const uint64_t g = radix_blocks(n_in);
    const size_t hist_elems = std::max<size_t>(radix_hist_elems(n_in, bits), 1);
    if ((rc = h->hist.ensure(hist_elems)) || (rc = h->xsend.ensure(std::max<uint64_t>(sh.n_digest, 1))) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(hist_elems), h->scan_tmp.cap))))
        return rc;
    if (n_in > 0) {
        STAGE(h, "owner_hist", by(0, 0, 0, 0, 0), launch_owner_hist(h->recA.p, n_in, om, sh.sparse, h->hist.p, s));
        h->stages[h->nstage - 1].c0 = 8.0 * (double)n_in;
        STAGE(h, "owner_scan", by(0, 0, 0, 0, 0),
              launch_scan_u32(h->hist.p, h->hist.p, g << bits, h->scan_tmp.p, h->scan_tmp.cap, nullptr, s));
        STAGE(h, "owner_scatter", by(0, 0, 0, 0, 0),
              launch_owner_scatter(h->recA.p, h->xsend.p, n_in, om, sh.sparse, h->hist.p, s));
        h->stages[h->nstage - 1].c0 = 16.0 * (double)(sh.sparse ? n_in : sh.n_digest) + 8.0 * (double)sh.n_digest;
    }
    sh.part_blocks = g;
    return 0;
}

// send counts / offsets from the whole count matrix's row of this shard
void send_plan(ShardState& sh, const std::vector<uint64_t>& counts) {
    const int ns = sh.nshards;
    sh.send_count.assign(ns, 0);
    sh.send_off.assign(ns, 0);
    for (int d = 0; d < ns; ++d) sh.send_count[d] = counts[(size_t)sh.rank * ns + d];
    for (int d = 1; d < ns; ++d) sh.send_off[d] = sh.send_off[d - 1] + sh.send_count[d - 1];
}
}  // namespace
}  // namespace dbi

extern "C" {

int dbi_shard_partition(dbi_handle* h, const int32_t* split, uint64_t* send_count) {
    if (!h || (!split && h->shard.nshards > 1)) return set_error(DBI_E_INVALID, "NULL argument");
    const double t0 = now_ms();
    int rc;
    if ((rc = partition_launch(h, split))) return rc;
    ShardState& sh = h->shard;
    const int ns = sh.nshards;
    hipStream_t s = h->stream;
    const uint64_t g = sh.part_blocks;
    std::vector<uint32_t> start(ns + 1, 0);
    if (sh.n_in > 0) {
        // first output position of every owner's run: hist[d * g] after the scan
        DBI_HIP(hipMemcpy2DAsync(start.data(), sizeof(uint32_t), h->hist.p, g * sizeof(uint32_t), sizeof(uint32_t),
                                 (size_t)ns, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
    }
    start[ns] = (uint32_t)sh.n_digest;
    sh.send_count.assign(ns, 0);
    sh.send_off.assign(ns, 0);
    for (int d = 0; d < ns; ++d) {
        sh.send_off[d] = start[d];
        sh.send_count[d] = (uint64_t)start[d + 1] - start[d];
        if (send_count) send_count[d] = sh.send_count[d];
    }
    sh.ms_partition = now_ms() - t0;
    sh.phase = 2;
    return 0;
}

int dbi_shard_exchange_local(dbi_handle* const* hs, int nshards) {
    if (!hs || nshards < 1) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    for (int i = 0; i < nshards; ++i) {
        if (!hs[i]) return set_error(DBI_E_INVALID, "NULL handle");
        if ((rc = need_phase(hs[i], 2, "dbi_shard_exchange_local"))) return rc;
        if (hs[i]->shard.nshards != nshards || hs[i]->shard.rank != i)
            return set_error(DBI_E_INVALID, "hs[i] must be shard i of nshards");
    }
    for (int j = 0; j < nshards; ++j) {
        dbi_handle* o = hs[j];
        const double t0 = now_ms();
        ShardState& sh = o->shard;
        sh.recv_count.assign(nshards, 0);
        uint64_t tot = 0, from_others = 0;
        for (int i = 0; i < nshards; ++i) {
            sh.recv_count[i] = hs[i]->shard.send_count[j];
            tot += sh.recv_count[i];
            if (i != j) from_others += sh.recv_count[i];
        }
        DBI_HIP(hipSetDevice(o->device));
        DBI_HIP(hipStreamSynchronize(o->stream));
        if ((rc = o->xrecv.ensure(std::max<uint64_t>(tot, 1)))) return rc;
        ManualStage ms(o, "exchange", 8.0 * (double)(from_others + (sh.n_digest - sh.send_count[j])));
        uint64_t off = 0;
        for (int i = 0; i < nshards; ++i) {
            const uint64_t c = sh.recv_count[i];
            if (c)
                DBI_HIP(hipMemcpyAsync(o->xrecv.p + off, hs[i]->xsend.p + hs[i]->shard.send_off[j],
                                       c * sizeof(uint64_t), hipMemcpyDeviceToDevice, o->stream));
            off += c;
        }
        ms.end();
        DBI_HIP(hipStreamSynchronize(o->stream));
        sh.n_recv = tot;
        sh.ms_exchange = now_ms() - t0;
    }
    for (int j = 0; j < nshards; ++j) hs[j]->shard.phase = 3;
    return 0;
}

int dbi_shard_merge(dbi_handle* h) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    int rc;
    if ((rc = need_phase(h, 3, "dbi_shard_merge"))) return rc;
    ShardState& sh = h->shard;
    const double t0 = now_ms();
    DBI_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    // from here on the handle describes the owner's slice of the whole proteome
    h->d_res = sh.d_res_global;
    h->d_poff = h->poff_g.p;
    h->n_res = sh.n_res_global;
    h->n_prot = sh.n_prot_global;
    h->n_total_extra = 0;
    if ((rc = h->recA.ensure(std::max<uint64_t>(sh.n_recv, 1)))) return rc;
    int32_t klo, khi;
    key_range(sh.split, sh.nshards, sh.rank, &klo, &khi);
    const double f = (double)h->params.mass_group_factor;
    const double lo = klo == INT32_MIN ? h->params.min_mh : std::max(h->params.min_mh, (double)klo / f);
    const double hi = khi == INT32_MAX ? h->params.max_mh : std::min(h->params.max_mh, (double)khi / f);
    // the chunk-list grids (and whether to run the giant pass) from this
    // owner's previous merge; lists that outgrow them (ERR_GRID) and the
    // merge runs again from the received words, with this merge's lists
    for (int e = 0; e < 2; ++e)
        if (!h->ev_merge[e]) DBI_HIP(hipEventCreate(&h->ev_merge[e]));
    // every buffer of the tail first: the merge's device time (the cost
    // profile's measure) then has no host allocation inside it
    if ((rc = tail_buffers(h, sh.n_recv, sh.n_recv, false))) return rc;
    const bool first = h->build_serial == 0;  // the handle's first build also loads the code objects: not timed
    for (int attempt = 0;; ++attempt) {
        const int nstage0 = h->nstage;
        DBI_HIP(hipEventRecord(h->ev_merge[0], s));
        // counters back to zero (the layout word max_plen stays), n_kept = records received
        DBI_HIP(hipMemsetAsync(h->ctr.p, 0, offsetof(Counters, max_plen), s));
        hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(64), 0, s, &h->ctr.p->n_kept, (unsigned long long)sh.n_recv);
        DBI_HIP(hipGetLastError());
        // the received location words -> records (mass + tag from the residues);
        // recA is free (the partition read it before the exchange was enqueued)
        STAGE(h, "owner_expand", by(0, 0, 0, 0, 0),
              launch_expand_locs(h->xrecv.p, sh.n_recv, h->d_res, h->d_poff, h->mass_tab.p, h->dp.m0, sh.width,
                                 h->recA.p, s));
        h->stages[h->nstage - 1].c0 = 24.0 * (double)sh.n_recv;  // 8 B in, 16 B out (+ the residues)
        if ((rc = build_tail(h, sh.n_recv, lo, std::max(hi, lo), sh.n_recv, false, nullptr, nullptr, 0,
                             attempt == 0)))
            return rc;
        DBI_HIP(hipEventRecord(h->ev_merge[1], s));
        if ((rc = finish_build(h))) return rc;  // (synchronises)
        float mg = 0.f;
        sh.ms_merge_gpu =
            !first && hipEventElapsedTime(&mg, h->ev_merge[0], h->ev_merge[1]) == hipSuccess ? (double)mg : 0.0;
        if (!h->lists_short) break;
        if (attempt > 0) return set_error(DBI_E_STATE, "internal: chunk lists outgrew full grids");
        h->nstage = nstage0;
        h->giants_seen = true;
    }
    sh.ms_merge = now_ms() - t0;
    sh.phase = 4;
    return 0;
}

int dbi_shard_stats_get(dbi_handle* h, dbi_shard_stats* out) {
    if (!h || !out) return set_error(DBI_E_INVALID, "NULL argument");
    const ShardState& sh = h->shard;
    if (sh.phase < 1) return set_error(DBI_E_STATE, "no sharded build on this handle");
    dbi_shard_stats st = sh.global;
    st.merge_gpu_ms = sh.ms_merge_gpu;
    st.rank = sh.rank;
    st.nshards = sh.nshards;
    st.p_begin = sh.p_begin;
    st.p_end = sh.p_end;
    key_range(sh.split, sh.nshards, sh.rank, &st.key_lo, &st.key_hi);
    st.n_total = sh.n_total;
    st.n_dropped = sh.n_dropped;
    st.n_sent = sh.phase >= 2 ? sh.n_digest - sh.send_count[sh.rank] : 0;
    st.n_received = sh.n_recv;
    st.n_unique = sh.phase >= 4 ? h->stats.n_unique : 0;
    st.n_keys = sh.phase >= 4 ? h->stats.n_keys : 0;
    st.digest_ms = sh.ms_digest;
    st.partition_ms = sh.ms_partition;
    st.exchange_ms = sh.ms_exchange;
    st.merge_ms = sh.ms_merge;
    *out = st;
    return 0;
}

int dbi_query_sharded_local(dbi_handle* const* hs, int nshards, const double* const* d_mass,
                            const double* const* d_tol, const uint64_t* nq, uint64_t* const* d_first,
                            uint64_t* const* d_count) {
    if (!hs || !d_mass || !d_tol || !nq || !d_first || !d_count || nshards < 1)
        return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    uint64_t base = 0;
    for (int i = 0; i < nshards; ++i)
        if (!hs[i]) return set_error(DBI_E_INVALID, "NULL handle");
    // every handle's query lock, in shard order (handles are distinct)
    std::vector<std::unique_lock<std::recursive_mutex>> locks;
    for (int i = 0; i < nshards; ++i) locks.emplace_back(hs[i]->qmu);
    for (int i = 0; i < nshards; ++i) {
        dbi_handle* h = hs[i];
        if (h->shard.nshards != nshards || h->shard.rank != i)
            return set_error(DBI_E_INVALID, "hs[i] must be shard i of nshards");
        h->shard.u_base = base;  // owners' tables concatenate in shard order
        h->shard.u_base_known = h->shard.phase == 4;
        base += h->stats.n_unique;
        if ((rc = query_need(h))) return rc;
    }
    for (int i = 0; i < nshards; ++i) {
        DBI_HIP(hipSetDevice(hs[i]->device));
        if ((rc = query_route(hs[i], d_mass[i], d_tol[i], nq[i]))) return rc;
    }
    // forward: origin i's pairs for owner j -> owner j; answer; back to the origins
    for (int j = 0; j < nshards; ++j) {
        dbi_handle* o = hs[j];
        ShardState& sh = o->shard;
        sh.qrecv_count.assign(nshards, 0);
        for (int i = 0; i < nshards; ++i) sh.qrecv_count[i] = hs[i]->shard.qsend_count[j];
        offsets_of(sh.qrecv_count, sh.qrecv_off);
        sh.q_recv = sh.qrecv_off[nshards];
        DBI_HIP(hipSetDevice(o->device));
        if ((rc = o->qrecv.ensure(sh.q_recv + 1))) return rc;
        for (int i = 0; i < nshards; ++i)
            if (sh.qrecv_count[i])
                DBI_HIP(hipMemcpyAsync(o->qrecv.p + sh.qrecv_off[i], hs[i]->qsend.p + hs[i]->shard.qsend_off[j],
                                       sh.qrecv_count[i] * sizeof(Rec), hipMemcpyDeviceToDevice, o->stream));
        if ((rc = query_answer(o))) return rc;
        DBI_HIP(hipStreamSynchronize(o->stream));
    }
    for (int i = 0; i < nshards; ++i) {
        dbi_handle* h = hs[i];
        ShardState& sh = h->shard;
        DBI_HIP(hipSetDevice(h->device));
        for (int j = 0; j < nshards; ++j)
            if (sh.qsend_count[j])
                DBI_HIP(hipMemcpyAsync(h->qback.p + sh.qsend_off[j], hs[j]->qres.p + hs[j]->shard.qrecv_off[i],
                                       sh.qsend_count[j] * sizeof(Rec), hipMemcpyDeviceToDevice, h->stream));
        DBI_HIP(launch_qcombine(h->qpairB.p, h->qback.p, sh.q_pairs, d_first[i], d_count[i], sh.q_n, h->stream));
        DBI_HIP(hipStreamSynchronize(h->stream));
    }
    return 0;
}

int dbi_query_sharded(dbi_handle* h, dbi_comm* c, const double* d_mass, const double* d_tol, uint64_t nq,
                      uint64_t* d_first, uint64_t* d_count) {
    if (!h || !c || (nq && (!d_mass || !d_tol || !d_first || !d_count))) return set_error(DBI_E_INVALID, "NULL argument");
    // argument and state errors are the same on every rank of a consistent job
    // (same build, same communicator); the rest is agreed on below
    int rc;
    if ((rc = query_need(h))) return rc;
    if (h->shard.nshards != c->nranks || h->shard.rank != c->rank)
        return set_error(DBI_E_INVALID, "communicator does not match the sharded build");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    DBI_HIP(hipSetDevice(h->device));
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;
    const int n = c->nranks, me = c->rank;
    int rc_route = query_route(h, d_mass, d_tol, nq);
    if (!rc_route) rc_route = injected_failure("qroute", me);
    if (rc_route) sh.qsend_count.assign(n, 0);
    std::vector<uint64_t> counts;
    bool failed = false;
    if ((rc = nccl_count_matrix(h, c, sh.qsend_count, rc_route, counts, &failed))) return rc;
    if (rc_route) return rc_route;
    if (failed) return peer_failed("query routing");
    sh.qrecv_count.assign(n, 0);
    for (int i = 0; i < n; ++i) sh.qrecv_count[i] = counts[(size_t)i * n + me];
    offsets_of(sh.qrecv_count, sh.qrecv_off);
    sh.q_recv = sh.qrecv_off[n];
    // every local allocation of the batch before the exchange, then agree
    int rc_local = h->qrecv.ensure(sh.q_recv + 1);
    if (!rc_local) rc_local = h->qres.ensure(sh.q_recv + 1);
    if (!rc_local) rc_local = ensure_qdir(h, s);
    if (!rc_local) rc_local = injected_failure("qbuffers", me);
    if ((rc = agree(c, rc_local, s, &failed))) return rc;
    if (rc_local) return rc_local;
    if (failed) return peer_failed("query buffers");
    if ((rc = nccl_alltoallv(c, h->qsend.p, sh.qsend_off, sh.qsend_count, h->qrecv.p, sh.qrecv_off, sh.qrecv_count, s)))
        return rc;
    if ((rc = query_answer(h))) return rc;
    if ((rc = nccl_alltoallv(c, h->qres.p, sh.qrecv_off, sh.qrecv_count, h->qback.p, sh.qsend_off, sh.qsend_count, s)))
        return rc;
    DBI_HIP(launch_qcombine(h->qpairB.p, h->qback.p, sh.q_pairs, d_first, d_count, sh.q_n, s));
    DBI_HIP(hipStreamSynchronize(s));
    return 0;
}

int dbi_shard_replicate_local(dbi_handle* const* hs, int nshards) {
    if (!hs || nshards < 1) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    SliceSizes z;
    uint64_t g_total = 0, g_dropped = 0, g_keys = 0;
    for (int i = 0; i < nshards; ++i) {
        if (!hs[i]) return set_error(DBI_E_INVALID, "NULL handle");
        if (hs[i]->shard.phase != 4 || hs[i]->shard.nshards != nshards || hs[i]->shard.rank != i)
            return set_error(DBI_E_STATE, "dbi_shard_replicate_local: hs[i] must be merged shard i of nshards");
        z.u.push_back(hs[i]->stats.n_unique);
        z.k.push_back(hs[i]->stats.n_kept);
        g_total += hs[i]->shard.n_total;
        g_dropped += hs[i]->shard.n_dropped;
        g_keys += hs[i]->stats.n_keys;
    }
    slice_bases(z);
    if ((rc = replica_check(z))) return rc;
    std::vector<std::unique_lock<std::recursive_mutex>> locks;
    for (int i = 0; i < nshards; ++i) locks.emplace_back(hs[i]->qmu);
    for (int j = 0; j < nshards; ++j) {
        dbi_handle* o = hs[j];
        DBI_HIP(hipSetDevice(o->device));
        if ((rc = replica_alloc(o, z))) return rc;
        hipStream_t s = o->stream;
        for (int i = 0; i < nshards; ++i) {
            const dbi_handle* src = hs[i];
            const uint64_t u = z.u[i], k = z.k[i], ub = z.ub[i];
            if (u) {
                DBI_HIP(hipMemcpyAsync(o->r_mass.p + ub, src->umass.p, 8 * u, hipMemcpyDeviceToDevice, s));
                DBI_HIP(hipMemcpyAsync(o->r_pid.p + ub, src->upid.p, 4 * u, hipMemcpyDeviceToDevice, s));
                DBI_HIP(hipMemcpyAsync(o->r_off.p + ub, src->uoff.p, 4 * u, hipMemcpyDeviceToDevice, s));
                DBI_HIP(hipMemcpyAsync(o->r_len.p + ub, src->ulen.p, 4 * u, hipMemcpyDeviceToDevice, s));
                DBI_HIP(hipMemcpyAsync(o->r_occ_off.p + ub, src->occ_off.p, 4 * u, hipMemcpyDeviceToDevice, s));
            }
            if (k) DBI_HIP(hipMemcpyAsync(o->r_occ.p + z.kb[i], src->occ_pid.p, 4 * k, hipMemcpyDeviceToDevice, s));
        }
        if ((rc = replica_rebase(o, z, s))) return rc;
    }
    for (int j = 0; j < nshards; ++j) replica_install(hs[j], z, g_total, g_dropped, g_keys);
    return 0;
}

int dbi_shard_replicate(dbi_handle* h, dbi_comm* c) {
    if (!h || !c) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = query_need(h))) return rc;  // same verdict on every rank of a consistent job
    if (h->shard.nshards != c->nranks || h->shard.rank != c->rank)
        return set_error(DBI_E_INVALID, "communicator does not match the sharded build");
    std::lock_guard<std::recursive_mutex> lock(h->qmu);
    DBI_HIP(hipSetDevice(h->device));
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;
    const int n = c->nranks, me = c->rank;
    // every slice's size (two columns of the count matrix)
    std::vector<uint64_t> mine(n, 0), all;
    mine[0] = h->stats.n_unique;
    if (n > 1) mine[1] = h->stats.n_kept;
    bool failed = false;
    SliceSizes z;
    if (n > 1) {
        if ((rc = nccl_count_matrix(h, c, mine, 0, all, &failed))) return rc;
        for (int i = 0; i < n; ++i) {
            z.u.push_back(all[(size_t)i * n]);
            z.k.push_back(all[(size_t)i * n + 1]);
        }
    } else {
        z.u.push_back(h->stats.n_unique);
        z.k.push_back(h->stats.n_kept);
    }
    slice_bases(z);
    if ((rc = replica_check(z))) return rc;
    const int rc_local = replica_alloc(h, z);
    if ((rc = agree(c, rc_local, s, &failed))) return rc;
    if (rc_local) return rc_local;
    if (failed) return peer_failed("replica buffers");
    // every array of every slice to every rank: one group of point-to-point
    // transfers over all xGMI links; the own slice by a copy
    struct Arr { void* src; uint8_t* dst; size_t esz; bool occ; };
    const Arr arrs[] = {
        {h->umass.p, (uint8_t*)h->r_mass.p, 8, false}, {h->upid.p, (uint8_t*)h->r_pid.p, 4, false},
        {h->uoff.p, (uint8_t*)h->r_off.p, 4, false},   {h->ulen.p, (uint8_t*)h->r_len.p, 4, false},
        {h->occ_off.p, (uint8_t*)h->r_occ_off.p, 4, false}, {h->occ_pid.p, (uint8_t*)h->r_occ.p, 4, true},
    };
    for (const Arr& a : arrs) {
        const uint64_t cnt = a.occ ? z.k[me] : z.u[me], base = a.occ ? z.kb[me] : z.ub[me];
        if (cnt) DBI_HIP(hipMemcpyAsync(a.dst + base * a.esz, a.src, cnt * a.esz, hipMemcpyDeviceToDevice, s));
    }
    DBI_NCCL(ncclGroupStart());
    for (const Arr& a : arrs)
        for (int p = 0; p < n; ++p) {
            if (p == me) continue;
            const uint64_t mc = a.occ ? z.k[me] : z.u[me];
            const uint64_t pc = a.occ ? z.k[p] : z.u[p], pb = a.occ ? z.kb[p] : z.ub[p];
            if (mc) DBI_NCCL(ncclSend(a.src, mc * a.esz, ncclUint8, p, c->comm, s));
            if (pc) DBI_NCCL(ncclRecv(a.dst + pb * a.esz, pc * a.esz, ncclUint8, p, c->comm, s));
        }
    DBI_NCCL(ncclGroupEnd());
    if ((rc = replica_rebase(h, z, s))) return rc;
    replica_install(h, z, sh.global.g_total, sh.global.g_dropped, sh.global.g_keys);
    return 0;
}

// ---- RCCL -------------------------------------------------------------------------

int dbi_comm_unique_id(uint8_t* id128) {
    if (!id128) return set_error(DBI_E_INVALID, "NULL argument");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    DBI_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id128, &id, sizeof(id));
    return 0;
}

int dbi_comm_init(const uint8_t* id128, int nranks, int rank, int device, dbi_comm** out) {
    if (!id128 || !out) return set_error(DBI_E_INVALID, "NULL argument");
    *out = nullptr;
    if (nranks < 1 || nranks > MAX_SHARDS || rank < 0 || rank >= nranks)
        return set_error(DBI_E_INVALID, "rank / nranks out of range (1..64 ranks)");
    DBI_HIP(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    dbi_comm* c = new dbi_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    if (hipMalloc((void**)&c->d_flag, 2 * sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return set_error(DBI_E_OOM, "hipMalloc (communicator status word)");
    }
    c->cnt_row = std::max(nranks + 2, 7);  // count matrix row | the totals row (7)
    if (hipMalloc((void**)&c->d_red, COMM_RED_MAX * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&c->d_samp, sizeof(double) * (size_t)nranks * (NS + 2)) != hipSuccess ||
        hipMalloc((void**)&c->d_cnt, sizeof(unsigned long long) * (size_t)nranks * c->cnt_row) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        dbi_comm_destroy(c);
        return set_error(DBI_E_HIP, "communicator stream / staging buffer");
    }
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        dbi_comm_destroy(c);
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
    return 0;
}

void dbi_comm_destroy(dbi_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->d_flag) (void)hipFree(c->d_flag);
    if (c->d_red) (void)hipFree(c->d_red);
    if (c->d_samp) (void)hipFree(c->d_samp);
    if (c->d_cnt) (void)hipFree(c->d_cnt);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int dbi_comm_allreduce_f64(dbi_comm* c, const double* in, double* out, uint32_t n, int op) {
    if (!c || (n && (!in || !out))) return set_error(DBI_E_INVALID, "NULL argument");
    if (n > COMM_RED_MAX) return set_error(DBI_E_INVALID, "dbi_comm_allreduce_f64: at most 4096 values");
    if (op != DBI_OP_SUM && op != DBI_OP_MAX && op != DBI_OP_MIN)
        return set_error(DBI_E_INVALID, "dbi_comm_allreduce_f64: unknown op");
    DBI_HIP(hipSetDevice(c->device));
    const ncclRedOp_t rop = op == DBI_OP_SUM ? ncclSum : op == DBI_OP_MAX ? ncclMax : ncclMin;
    const uint32_t m = n ? n : 1u;  // n = 0: a barrier (one value, ignored)
    if (n) DBI_HIP(hipMemcpyAsync(c->d_red, in, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    else DBI_HIP(hipMemsetAsync(c->d_red, 0, sizeof(double), c->stream));
    DBI_NCCL(ncclAllReduce(c->d_red, c->d_red, m, ncclFloat64, rop, c->comm, c->stream));
    if (n) DBI_HIP(hipMemcpyAsync(out, c->d_red, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    DBI_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int dbi_comm_allreduce_u64(dbi_comm* c, const uint64_t* d_in, uint64_t* d_out, uint64_t n, void* stream) {
    if (!c || (n && (!d_in || !d_out))) return set_error(DBI_E_INVALID, "NULL argument");
    DBI_HIP(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (n) DBI_NCCL(ncclAllReduce(d_in, d_out, n, ncclUint64, ncclSum, c->comm, s));
    if (!stream) DBI_HIP(hipStreamSynchronize(s));
    return 0;
}

int dbi_runtime_info_get(dbi_runtime_info* out) {
    if (!out) return set_error(DBI_E_INVALID, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    (void)hipRuntimeGetVersion(&out->hip_runtime_version);
    (void)hipDriverGetVersion(&out->hip_driver_version);
    (void)ncclGetVersion(&out->rccl_version);
    Dl_info di;
    if (dladdr(reinterpret_cast<void*>(static_cast<hipError_t (*)(void**, size_t)>(&hipMalloc)), &di) && di.dli_fname)
        std::strncpy(out->libamdhip64, di.dli_fname, sizeof(out->libamdhip64) - 1);
    if (dladdr(reinterpret_cast<void*>(&ncclGetVersion), &di) && di.dli_fname)
        std::strncpy(out->librccl, di.dli_fname, sizeof(out->librccl) - 1);
    return 0;
}

int dbi_comm_allgatherv(dbi_comm* c, const void* d_send, void* d_recv, const uint64_t* rank_bytes, void* stream) {
    if (!c || !d_recv || !rank_bytes) return set_error(DBI_E_INVALID, "NULL argument");
    DBI_HIP(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    std::vector<uint64_t> off(c->nranks + 1, 0);
    for (int r = 0; r < c->nranks; ++r) off[r + 1] = off[r] + rank_bytes[r];
    uint8_t* recv = static_cast<uint8_t*>(d_recv);
    uint8_t* mine = recv + off[c->rank];
    const uint64_t my_bytes = rank_bytes[c->rank];
    if (d_send && d_send != mine && my_bytes)
        DBI_HIP(hipMemcpyAsync(mine, d_send, my_bytes, hipMemcpyDeviceToDevice, s));
    DBI_NCCL(ncclGroupStart());
    for (int p = 0; p < c->nranks; ++p) {
        if (p == c->rank) continue;
        if (my_bytes) DBI_NCCL(ncclSend(mine, my_bytes, ncclUint8, p, c->comm, s));
        if (rank_bytes[p]) DBI_NCCL(ncclRecv(recv + off[p], rank_bytes[p], ncclUint8, p, c->comm, s));
    }
    DBI_NCCL(ncclGroupEnd());
    DBI_HIP(hipStreamSynchronize(s));
    return 0;
}

}  // extern "C"

namespace dbi {
namespace {
// One rank owning the whole proteome: its owner slice is the whole index and
// every record would be routed to itself, so the sharded build is the
// single-device build (digest, one sort, finalise; no sample gather,
// partition, exchange or second sort; warm builds replay its graph) plus the
// shard bookkeeping the routed queries and the replica read.
int build_single_owner(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_poff, uint64_t n_prot) {
    const double t0 = now_ms();
    int rc;
    if ((rc = dbi_build_device(h, d_res, n_res, d_poff, n_prot, nullptr))) return rc;
    ShardState& sh = h->shard;
    sh = ShardState{};
    sh.rank = 0;
    sh.nshards = 1;
    sh.p_end = n_prot;
    sh.n_res_global = n_res;
    sh.n_prot_global = n_prot;
    sh.d_res_global = d_res;
    sh.n_total = h->stats.n_total;
    sh.n_dropped = h->stats.n_dropped;
    sh.n_digest = sh.n_recv = h->stats.n_kept;
    sh.send_count.assign(1, sh.n_recv);
    sh.send_off.assign(1, 0);
    sh.recv_count.assign(1, sh.n_recv);
    sh.ms_merge = now_ms() - t0;
    sh.u_base = 0;
    sh.u_base_known = true;
    sh.global.g_total = h->stats.n_total;
    sh.global.g_dropped = h->stats.n_dropped;
    sh.global.g_kept = h->stats.n_kept;
    sh.global.g_unique = h->stats.n_unique;
    sh.global.g_keys = h->stats.n_keys;
    sh.phase = 4;
    return 0;
}
}  // namespace
}  // namespace dbi

extern "C" {

int dbi_build_sharded(dbi_handle* h, dbi_comm* c, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_poff,
                      uint64_t n_prot, uint64_t p_begin, uint64_t p_end) {
    if (!h || !c) return set_error(DBI_E_INVALID, "NULL argument");
    if (c->device != h->device) return set_error(DBI_E_INVALID, "communicator and engine on different devices");
    const int n = c->nranks, me = c->rank;
    // DBI_SHARD_FULL_PATH=1: one rank takes the general path too (tests of the
    // partition / exchange / agreement code at N=1)
    const char* full_path = std::getenv("DBI_SHARD_FULL_PATH");
    if (n == 1 && p_begin == 0 && p_end == n_prot && !(full_path && full_path[0] == '1'))
        return build_single_owner(h, d_res, n_res, d_poff, n_prot);
    int rc;
    // a rank that fails locally still takes part in the next collective, with
    // its status, so that every rank returns an error (never a hang)
    const double t_digest = now_ms();
    int rc_digest = dbi_shard_digest(h, d_res, n_res, d_poff, n_prot, p_begin, p_end, me, n);
    if (!rc_digest) rc_digest = injected_failure("digest", me);
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;

    // samples of every shard -> the same owner splitters everywhere.  Block
    // of rank r: NS record masses (written on the device), its record count,
    // its status; the sample weight (records per valid sample) on the host
    const size_t blk = NS + 2;
    int rc_local = rc_digest;
    double* my_blk = c->d_samp + (size_t)me * blk;
    if (!rc_local) {
        if ((rc = launch_sample_masses(h->recA.p, sh.n_in, NS, my_blk, s)) != hipSuccess)
            rc_local = hip_fail((hipError_t)rc, "launch_sample_masses");
    }
    std::vector<double> samples((size_t)n * blk, 0.0);
    samples[(size_t)me * blk + NS] = rc_local ? 0.0 : (double)sh.n_digest;
    samples[(size_t)me * blk + NS + 1] = rc_local ? 1.0 : 0.0;
    DBI_HIP(hipMemcpyAsync(my_blk + NS, &samples[(size_t)me * blk + NS], 2 * sizeof(double), hipMemcpyHostToDevice,
                           s));
    DBI_NCCL(ncclAllGather(my_blk, c->d_samp, blk, ncclFloat64, c->comm, s));
    DBI_HIP(hipMemcpyAsync(samples.data(), c->d_samp, sizeof(double) * n * blk, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if (rc_local) return rc_local;
    std::vector<double> packed((size_t)n * (NS + 1));
    for (int r = 0; r < n; ++r) {
        const double* b = samples.data() + (size_t)r * blk;
        if (b[NS + 1] != 0.0) return peer_failed("shard digest");
        uint64_t valid = 0;
        for (uint32_t i = 0; i < NS; ++i) valid += b[i] == b[i];
        std::copy(b, b + NS, packed.begin() + (size_t)r * (NS + 1));
        packed[(size_t)r * (NS + 1) + NS] = valid ? b[NS] / (double)valid : 0.0;  // as dbi_shard_samples
    }
    int32_t split[MAX_SHARDS - 1] = {};
    // the same everywhere: every rank holds the same samples and cost profile
    if ((rc = dbi_shard_splitters_profiled(h, packed.data(), n, split))) return rc;
    sh.ms_digest = now_ms() - t_digest;
    const double t_part = now_ms();
    int rc_part = partition_launch(h, split);
    if (!rc_part) rc_part = injected_failure("partition", me);

    // count matrix: row r = records shard r sends each owner (from its owner
    // histogram, on the device) | its status | its receive capacity
    const double t0 = now_ms();
    const int w = n + 2;
    unsigned long long* my_row = c->d_cnt + (size_t)me * w;
    if (!rc_part && sh.n_in > 0) {
        hipLaunchKernelGGL(k_owner_counts, dim3(1), dim3(64), 0, s, h->hist.p, sh.part_blocks, (uint32_t)n,
                           sh.n_digest, my_row);
        if ((rc = hipGetLastError()) != hipSuccess) rc_part = hip_fail((hipError_t)rc, "k_owner_counts");
    } else if ((rc = hipMemsetAsync(my_row, 0, sizeof(unsigned long long) * n, s)) != hipSuccess && !rc_part) {
        rc_part = hip_fail((hipError_t)rc, "hipMemsetAsync");
    }
    std::vector<unsigned long long> full((size_t)n * w, 0);
    full[(size_t)me * w + n] = rc_part ? 1u : 0u;
    full[(size_t)me * w + n + 1] = h->xrecv.cap;
    DBI_HIP(hipMemcpyAsync(my_row + n, &full[(size_t)me * w + n], 2 * sizeof(unsigned long long), hipMemcpyHostToDevice, s));
    DBI_NCCL(ncclAllGather(my_row, c->d_cnt, w, ncclUint64, c->comm, s));
    DBI_HIP(hipMemcpyAsync(full.data(), c->d_cnt, sizeof(unsigned long long) * n * w, hipMemcpyDeviceToHost, s));
    DBI_HIP(hipStreamSynchronize(s));
    if (rc_part) return rc_part;
    std::vector<uint64_t> counts((size_t)n * n);
    bool failed = false, grow = false;
    for (int i = 0; i < n; ++i) {
        failed |= full[(size_t)i * w + n] != 0;
        for (int j = 0; j < n; ++j) counts[(size_t)i * n + j] = full[(size_t)i * w + j];
    }
    if (failed) return peer_failed("owner partition");
    // checks on the whole matrix: every rank reaches the same verdict
    for (int j = 0; j < n; ++j) {
        uint64_t tot = 0;
        for (int i = 0; i < n; ++i) tot += counts[(size_t)i * n + j];
        if (tot >= (1ull << 32) - 1)
            return set_error(DBI_E_INVALID, "more than 2^32-2 records for one owner: use more shards");
        grow |= std::max<uint64_t>(tot, 1) > full[(size_t)j * w + n + 1];
    }
    send_plan(sh, counts);
    sh.ms_partition = now_ms() - t_part;
    sh.recv_count.assign(n, 0);
    uint64_t from_others = 0;
    for (int i = 0; i < n; ++i) {
        sh.recv_count[i] = counts[(size_t)i * n + me];
        if (i != me) from_others += sh.recv_count[i];
    }
    std::vector<uint64_t> roff;
    offsets_of(sh.recv_count, roff);
    // an owner that must grow its receive buffer may fail to: then every rank
    // learns it before the exchange (a collective only when someone grows)
    if (grow) {
        rc_local = h->xrecv.ensure(std::max<uint64_t>(roff[n], 1));
        if (!rc_local) rc_local = injected_failure("buffers", me);
        if ((rc = agree(c, rc_local, s, &failed))) return rc;
        if (rc_local) return rc_local;
        if (failed) return peer_failed("owner buffers");
    }

    // records to their owners: one group of point-to-point transfers over all peers
    {
        ManualStage ms(h, "exchange", 8.0 * (double)(from_others + (sh.n_digest - sh.send_count[me])));
        if ((rc = nccl_alltoallv(c, h->xsend.p, sh.send_off, sh.send_count, h->xrecv.p, roff, sh.recv_count, s)))
            return rc;
        ms.end();
    }
    // the owner merge runs behind the exchange on the same stream; only a
    // per-phase breakdown (every stage timed) waits for it here
    if (h->timing && h->timing_only.empty()) DBI_HIP(hipStreamSynchronize(s));
    sh.n_recv = roff[n];
    sh.ms_exchange = now_ms() - t0;
    sh.phase = 3;
    int rc_merge = dbi_shard_merge(h);
    if (!rc_merge) rc_merge = injected_failure("merge", me);

    // whole-index totals (+ status), and where this owner's rows start in the whole index
    std::vector<uint64_t> tot(5, 0);
    {
        const int wt = 7;
        std::vector<unsigned long long> row(wt, 0), rows((size_t)n * wt);
        row[0] = sh.n_total; row[1] = sh.n_dropped; row[2] = sh.n_recv; row[3] = h->stats.n_unique;
        row[4] = h->stats.n_keys;
        row[5] = rc_merge ? 1u : 0u;
        row[6] = rc_merge ? 0u : (unsigned long long)(sh.ms_merge_gpu * 1e6);  // ns
        DBI_HIP(hipMemcpyAsync(c->d_cnt + (size_t)me * wt, row.data(), sizeof(uint64_t) * wt, hipMemcpyHostToDevice, s));
        DBI_NCCL(ncclAllGather(c->d_cnt + (size_t)me * wt, c->d_cnt, wt, ncclUint64, c->comm, s));
        DBI_HIP(hipMemcpyAsync(rows.data(), c->d_cnt, sizeof(uint64_t) * n * wt, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
        if (rc_merge) return rc_merge;
        sh.u_base = 0;
        for (int i = 0; i < n; ++i) {
            if (rows[(size_t)i * wt + 5]) return peer_failed("owner merge");
            for (int k = 0; k < 5; ++k) tot[k] += rows[(size_t)i * wt + k];
            if (i < me) sh.u_base += rows[(size_t)i * wt + 3];
        }
        sh.u_base_known = true;
        // the cost profile for the next build: every owner's merge device time
        // and records over its key range (the same numbers, hence the same
        // profile, on every rank)
        std::vector<double> mms(n);
        std::vector<uint64_t> recs(n);
        for (int i = 0; i < n; ++i) {
            mms[i] = (double)rows[(size_t)i * wt + 6] * 1e-6;
            recs[i] = rows[(size_t)i * wt + 2];
        }
        if ((rc = dbi_shard_cost_update(h, n, sh.split, mms.data(), recs.data()))) return rc;
    }
    sh.global.g_total = tot[0];
    sh.global.g_dropped = tot[1];
    sh.global.g_kept = tot[2];
    sh.global.g_unique = tot[3];
    sh.global.g_keys = tot[4];
    return 0;
}

}  // extern "C"
