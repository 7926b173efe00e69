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
#include <thread>
#include <utility>
#include <vector>
#include <atomic>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "dbi_engine.h"

using namespace dbi;

namespace dbi {
// Host-staged transport (dbi_comm_init_host, TESTS ONLY): the same collectives
// through POSIX shared memory between the processes of one node -- device ->
// host -> shm slot or mailbox -> host -> device, a barrier between -- so the
// N-rank driver (warm splits, the count-matrix rounds, failure agreement, the
// exchange, totals, replica, routed queries) runs with N processes on ONE GPU,
// where RCCL refuses two ranks on one device.  Every product run is RCCL.
struct ShmHeader {
    std::atomic<uint32_t> ready, count, gen;
    uint32_t nranks;
    uint64_t slot;  // bytes per rank slot and per (src, dst) mailbox
};
struct HostXport {
    int fd = -1;
    uint8_t* base = nullptr;
    size_t bytes = 0;
    uint64_t slot = 0;
    std::string name;
    ShmHeader* hdr() const { return reinterpret_cast<ShmHeader*>(base); }
    uint8_t* rank_slot(int r) const { return base + 4096 + (size_t)r * slot; }
    uint8_t* mailbox(int src, int dst, int n) const {
        return base + 4096 + (size_t)n * slot + ((size_t)src * n + dst) * slot;
    }
};
}  // namespace dbi

struct dbi_comm {
    ncclComm_t comm = nullptr;
    dbi::HostXport* host = nullptr;        // the test transport instead of RCCL
    int nranks = 1;
    int rank = 0;
    int device = 0;
    unsigned long long* d_flag = nullptr;  // failure agreement (agree())
    hipStream_t stream = nullptr;          // host-buffer collectives (dbi_comm_allreduce_*)
    double* d_red = nullptr;               // their staging (COMM_RED_MAX values)
    // the sharded build's small collectives (sample blocks, count matrix,
    // totals) stage through these, allocated with the communicator: a rank
    // never fails an allocation between two collectives of a build
    double* d_samp = nullptr;              // nranks x (DBI_SHARD_SAMPLES + 3)
    unsigned long long* d_cnt = nullptr;   // nranks x cnt_row
    int cnt_row = 0;                       // max(nranks + 4, TOTALS_W)
};
constexpr uint32_t COMM_RED_MAX = 4096;
// totals row of a sharded build: n_total, n_dropped, n_recv, n_unique, n_keys,
// status, the previous build's merge ns and records received, merge flags
constexpr int TOTALS_W = 9;

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

// ---- collectives: RCCL, or the host-staged test transport ----
int shm_barrier(dbi_comm* c) {
    ShmHeader* h = c->host->hdr();
    const uint32_t g = h->gen.load(std::memory_order_acquire);
    if (h->count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
        h->count.store(0, std::memory_order_relaxed);
        h->gen.fetch_add(1, std::memory_order_release);
        return 0;
    }
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    while (h->gen.load(std::memory_order_acquire) == g) {
        if (std::chrono::steady_clock::now() > t_end)
            return set_error(DBI_E_RCCL, "host transport: barrier timed out (a peer process is gone)");
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return 0;
}

int shm_check(const dbi_comm* c, uint64_t bytes) {
    if (bytes > c->host->slot)
        return set_error(DBI_E_INVALID, "host transport: a message of " + std::to_string(bytes) +
                                            " B exceeds its mailbox (" + std::to_string(c->host->slot) + " B)");
    return 0;
}

// every rank's `bytes` from send -> recv (rank order), device buffers
int c_allgather(dbi_comm* c, const void* send, void* recv, uint64_t bytes, hipStream_t s) {
    if (!c->host) {
        DBI_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, c->comm, s));
        return 0;
    }
    int rc;
    if ((rc = shm_check(c, bytes))) return rc;
    DBI_HIP(hipStreamSynchronize(s));
    DBI_HIP(hipMemcpy(c->host->rank_slot(c->rank), send, bytes, hipMemcpyDeviceToHost));
    if ((rc = shm_barrier(c))) return rc;
    std::vector<uint8_t> all((size_t)bytes * c->nranks);
    for (int r = 0; r < c->nranks; ++r) std::memcpy(all.data() + (size_t)r * bytes, c->host->rank_slot(r), bytes);
    if ((rc = shm_barrier(c))) return rc;  // the slots are free again
    DBI_HIP(hipMemcpy(recv, all.data(), all.size(), hipMemcpyHostToDevice));
    return 0;
}

// element-wise reduction over the ranks (u64 sum / max, f64 sum / max / min)
int c_allreduce(dbi_comm* c, const void* send, void* recv, uint64_t count, ncclDataType_t t, ncclRedOp_t op,
                hipStream_t s) {
    if (!c->host) {
        DBI_NCCL(ncclAllReduce(send, recv, count, t, op, c->comm, s));
        return 0;
    }
    if (t != ncclUint64 && t != ncclFloat64) return set_error(DBI_E_INVALID, "host transport: u64 / f64 only");
    const uint64_t bytes = 8 * count;
    std::vector<uint8_t> all((size_t)bytes * c->nranks);
    int rc;
    if ((rc = shm_check(c, bytes))) return rc;
    DBI_HIP(hipStreamSynchronize(s));
    DBI_HIP(hipMemcpy(c->host->rank_slot(c->rank), send, bytes, hipMemcpyDeviceToHost));
    if ((rc = shm_barrier(c))) return rc;
    for (int r = 0; r < c->nranks; ++r) std::memcpy(all.data() + (size_t)r * bytes, c->host->rank_slot(r), bytes);
    if ((rc = shm_barrier(c))) return rc;
    std::vector<uint8_t> out(bytes);
    for (uint64_t i = 0; i < count; ++i) {
        if (t == ncclUint64) {
            uint64_t v;
            std::memcpy(&v, all.data() + 8 * i, 8);
            for (int r = 1; r < c->nranks; ++r) {
                uint64_t x;
                std::memcpy(&x, all.data() + (size_t)r * bytes + 8 * i, 8);
                v = op == ncclSum ? v + x : op == ncclMax ? std::max(v, x) : std::min(v, x);
            }
            std::memcpy(out.data() + 8 * i, &v, 8);
        } else {
            double v;
            std::memcpy(&v, all.data() + 8 * i, 8);
            for (int r = 1; r < c->nranks; ++r) {
                double x;
                std::memcpy(&x, all.data() + (size_t)r * bytes + 8 * i, 8);
                v = op == ncclSum ? v + x : op == ncclMax ? std::max(v, x) : std::min(v, x);
            }
            std::memcpy(out.data() + 8 * i, &v, 8);
        }
    }
    DBI_HIP(hipMemcpy(recv, out.data(), bytes, hipMemcpyHostToDevice));
    return 0;
}

// point-to-point transfers of one group: to peer p from the rank's device
// buffers; matched by order per peer pair, as RCCL's grouped send / receive
struct Xfer {
    int peer;
    void* ptr;
    uint64_t bytes;
};

int c_group(dbi_comm* c, const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
    if (!c->host) {
        DBI_NCCL(ncclGroupStart());
        for (const Xfer& x : sends)
            if (x.bytes) DBI_NCCL(ncclSend(x.ptr, x.bytes, ncclUint8, x.peer, c->comm, s));
        for (const Xfer& x : recvs)
            if (x.bytes) DBI_NCCL(ncclRecv(x.ptr, x.bytes, ncclUint8, x.peer, c->comm, s));
        DBI_NCCL(ncclGroupEnd());
        return 0;
    }
    const int n = c->nranks, me = c->rank;
    int rc;
    DBI_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> cur(n, 0);
    for (const Xfer& x : sends) {
        if (!x.bytes) continue;
        if ((rc = shm_check(c, cur[x.peer] + x.bytes))) return rc;
        DBI_HIP(hipMemcpy(c->host->mailbox(me, x.peer, n) + cur[x.peer], x.ptr, x.bytes, hipMemcpyDeviceToHost));
        cur[x.peer] += x.bytes;
    }
    if ((rc = shm_barrier(c))) return rc;
    std::fill(cur.begin(), cur.end(), 0);
    for (const Xfer& x : recvs) {
        if (!x.bytes) continue;
        if ((rc = shm_check(c, cur[x.peer] + x.bytes))) return rc;
        DBI_HIP(hipMemcpy(x.ptr, c->host->mailbox(x.peer, me, n) + cur[x.peer], x.bytes, hipMemcpyHostToDevice));
        cur[x.peer] += x.bytes;
    }
    return shm_barrier(c);  // the mailboxes are free again
}

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
// d_total: the record count on the device (a device-sized digest), else n_total
__global__ void k_owner_counts(const uint32_t* __restrict__ hist, uint64_t g, uint32_t ns, uint64_t n_total,
                               const unsigned long long* __restrict__ d_total, unsigned long long* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= ns) return;
    if (d_total) n_total = *d_total;
    const uint64_t a = n_total ? hist[(uint64_t)d * g] : 0u;
    const uint64_t b = (d + 1 < ns && n_total) ? hist[(uint64_t)(d + 1) * g] : n_total;
    out[d] = b - a;
}

// The count-matrix row's device flags of a device-sized shard digest: bit 0
// its slots overflowed the buffer (nothing was partitioned: k_tail_counts),
// bit 1 the offsets no longer give the shard's residue range or record width
// the digest ran with, or the digest raised a layout / PTM error.  Either way
// this rank digests again, synchronously (dbi_shard_digest).
constexpr unsigned long long SHARD_REDO_SLOTS = 1, SHARD_REDO_RANGE = 2;
__global__ void k_shard_flags(const uint64_t* __restrict__ poff, uint64_t p_begin, uint64_t p_end, uint64_t e0,
                              uint64_t e1, uint32_t width, const Counters* __restrict__ ctr, uint64_t cap,
                              unsigned long long* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned long long f = ctr->n_slots > cap ? SHARD_REDO_SLOTS : 0ull;
    if (poff[p_begin] != e0 || poff[p_end] != e1 || rec_width(ctr->max_plen) != width) f |= SHARD_REDO_RANGE;
    if (ctr->err & (ERR_LAYOUT | ERR_PTM)) f |= SHARD_REDO_RANGE;  // the synchronous digest reports it to every rank
    *out = f;
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
    std::vector<Xfer> sends, recvs;
    for (int p = 0; p < c->nranks; ++p) {
        if (p == me) continue;
        sends.push_back(Xfer{p, (void*)(send + soff[p]), scnt[p] * sizeof(T)});
        recvs.push_back(Xfer{p, (void*)(recv + roff[p]), rcnt[p] * sizeof(T)});
    }
    return c_group(c, sends, recvs, s);
}

// Local failures must not strand the other ranks inside the next collective:
// every rank reports its status with the data of a collective it would run
// anyway (a status column in the count matrix and the totals, a status word
// in the samples), or through agree() where no such collective comes first,
// and all ranks return an error together.
int peer_failed(const char* phase) {
    return set_error(DBI_E_STATE, std::string("another rank failed (") + phase + "); see that rank's error");
}

// Test hook (test builds only, -DDBI_TEST_HOOKS: libdbindex_hip_hooks.so):
// option test_fail = "<phase>@<rank>" makes that rank fail locally at that
// phase (digest, partition, buffers, merge, qroute, qbuffers), so the
// agreement paths run without a real failure.  The product library has no
// such option.
int injected_failure(const dbi_handle* h, const char* phase, int rank) {
#ifdef DBI_TEST_HOOKS
    if (h->opt_test_fail.empty() || h->opt_test_fail != std::string(phase) + "@" + std::to_string(rank)) return 0;
    return set_error(DBI_E_STATE, std::string("injected failure (option test_fail) in ") + phase);
#else
    (void)h, (void)phase, (void)rank;
    return 0;
#endif
}

// max over ranks of (rc != 0): 0 when every rank succeeded
int agree(dbi_comm* c, int rc, hipStream_t s, bool* any) {
    const unsigned long long mine = rc ? 1ull : 0ull;
    unsigned long long all = 0;
    DBI_HIP(hipMemcpyAsync(c->d_flag, &mine, sizeof(mine), hipMemcpyHostToDevice, s));
    int rc_c;
    if ((rc_c = c_allreduce(c, c->d_flag, c->d_flag + 1, 1, ncclUint64, ncclMax, s))) return rc_c;
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
    int rc;
    if ((rc = c_allgather(c, c->d_cnt + (size_t)me * w, c->d_cnt, 8ull * w, s))) return rc;
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

// Sample keys of every shard, sorted (the sort happens once per sampled
// build): key (int)(m * factor) of every valid sample and its weight (records
// per valid sample of its shard)
void sample_keys(const double* samples, int nshards, int32_t factor, SampleKeys& out) {
    std::vector<std::pair<int32_t, double>> ks;
    for (int r = 0; r < nshards; ++r) {
        const double* b = samples + (size_t)r * (NS + 1);
        const double w = b[NS];
        if (!(w > 0.0)) continue;
        for (uint32_t i = 0; i < NS; ++i)
            if (b[i] == b[i]) ks.emplace_back(java_d2i(b[i] * (double)factor), w);
    }
    std::sort(ks.begin(), ks.end());
    out.key.resize(ks.size());
    out.w.resize(ks.size());
    for (size_t i = 0; i < ks.size(); ++i) {
        out.key[i] = ks[i].first;
        out.w[i] = ks[i].second;
    }
}

// split[j-1] = the first key whose preceding weight reaches j/n of the total;
// a key's weight = its sample weight x the cost per record of its band (band
// b: the band_split entries <= key; nbands = 0: 1).  Linear in the samples.
void split_from_keys(const SampleKeys& sk, int nshards, int nbands, const int32_t* band_split,
                     const double* band_cost, int32_t* split) {
    const size_t m = sk.key.size();
    std::vector<double> wt(m);
    int b = 0;
    double total = 0.0;
    for (size_t i = 0; i < m; ++i) {
        double c = 1.0;
        if (nbands > 0) {
            while (b < nbands - 1 && band_split[b] <= sk.key[i]) ++b;  // keys ascend: the band only moves up
            c = band_cost[b];
        }
        wt[i] = sk.w[i] * c;
        total += wt[i];
    }
    size_t i = 0;
    double cum = 0.0;
    for (int j = 1; j < nshards; ++j) {
        const double target = total * (double)j / (double)nshards;
        int32_t sp = INT32_MAX;
        for (; i < m; ++i) {
            if (cum >= target && (i == 0 || sk.key[i] != sk.key[i - 1])) {
                sp = sk.key[i];
                break;
            }
            cum += wt[i];
        }
        split[j - 1] = sp;
    }
}

// FNV-1a 64 over bytes
uint64_t fnv64(const void* p, size_t n, uint64_t h = 0xcbf29ce484222325ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
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
    DBI_HIP(launch_off_rebase(d_poff, 0, n_res, h->poff_g.p, n_prot + 1, s));
    DBI_HIP(launch_off_rebase(d_poff + p_begin, ends[0], ends[1] - ends[0], h->poff.p, np + 1, s));
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
    // the next build of this shard may digest device-sized when this one
    // was a bounded digest (its slots fit: a cold count + emit digest sizes
    // the buffer by records, which the slots outgrow)
    auto& dv = h->shard_dev;
    dv.valid = sparse;
    dv.d_res = d_res;
    dv.d_poff = d_poff;
    dv.n_res = n_res;
    dv.n_prot = n_prot;
    dv.p_begin = p_begin;
    dv.p_end = p_end;
    dv.e0 = ends[0];
    dv.e1 = ends[1];
    dv.width = sh.width;
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
    SampleKeys sk;
    sample_keys(samples, nshards, factor, sk);
    split_from_keys(sk, nshards, band_cost ? nbands : 0, band_split, band_cost, split);
    return 0;
}

namespace dbi {
void forget_best_split(dbi_handle* h);
}
namespace {
constexpr int CB = DBI_COST_BANDS;
constexpr double SPLIT_HOLD = 1.10;  // owners this balanced (slowest / mean merge time) keep their split
constexpr int SPLIT_TRIES = 3;       // re-splits without a faster slowest owner: back to the best split, kept
constexpr double SPLIT_BETTER = 0.98;  // (a split beats the best by 2 %)
constexpr double SPLIT_WORSE = 2.0;    // the best split re-measured this much slower: the search resumes
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
    // the best split so far (by its slowest owner): the same numbers on every rank
    double mx = 0.0;
    uint64_t total = 0;
    for (int r = 0; r < nshards; ++r) {
        mx = std::max(mx, merge_ms[r]);
        total += records[r];
    }
    // the best split belongs to the proteome it was measured on: a build of
    // another size (> 5 % more or fewer records) forgets it, and so does a
    // re-measurement of it SPLIT_WORSE slower (the data under the split
    // changed) -- the search runs again instead of staying frozen
    const uint64_t br = pf.best_records;
    if (pf.has_best && (total > br + br / 20 || total + br / 20 < br)) forget_best_split(h);
    const bool same = pf.has_best && pf.best_n == nshards && std::equal(split, split + nshards - 1, pf.best_split);
    if (same && mx > SPLIT_WORSE * pf.best_max) {
        forget_best_split(h);
    } else if (same) {
        pf.best_max = 0.5 * pf.best_max + 0.5 * mx;  // the best split re-measured (kept when frozen)
        return 0;
    }
    if (!pf.has_best || pf.best_n != nshards || mx < SPLIT_BETTER * pf.best_max) {
        pf.has_best = true;
        pf.best_n = nshards;
        pf.best_max = mx;
        pf.best_records = total;
        std::copy(split, split + nshards - 1, pf.best_split);
        pf.since_best = 0;
    } else {
        ++pf.since_best;
    }
    return 0;
}

namespace dbi {
void forget_best_split(dbi_handle* h) {
    auto& pf = h->shard_prof;
    pf.has_best = false;
    pf.since_best = 0;
    pf.best_records = 0;
}

// the profile's split search has stopped: the best split is kept
bool shard_split_frozen(const dbi_handle* h, int nshards) {
    const auto& pf = h->shard_prof;
    return pf.valid && pf.has_best && pf.best_n == nshards && pf.since_best >= SPLIT_TRIES;
}
}  // namespace dbi

int dbi_shard_splitters_profiled(dbi_handle* h, const double* samples, int nshards, int32_t* split) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    const auto& pf = h->shard_prof;
    if (split && nshards > 1 && dbi::shard_split_frozen(h, nshards)) {
        std::copy(pf.best_split, pf.best_split + nshards - 1, split);
        return 0;
    }
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
    const unsigned long long* dn = sh.dev ? &h->ctr.p->tail_in : nullptr;  // slots written (0: overflowed)
    if (n_in > 0) {
        STAGE(h, "owner_hist", by(0, 0, 0, 0, 0),
              launch_owner_hist(h->recA.p, n_in, om, sh.sparse, h->hist.p, s, dn));
        h->stages[h->nstage - 1].c0 = 8.0 * (double)n_in;
        STAGE(h, "owner_scan", by(0, 0, 0, 0, 0),
              launch_scan_u32(h->hist.p, h->hist.p, g << bits, h->scan_tmp.p, h->scan_tmp.cap, nullptr, s));
        STAGE(h, "owner_scatter", by(0, 0, 0, 0, 0),
              launch_owner_scatter(h->recA.p, h->xsend.p, n_in, om, sh.sparse, h->hist.p, s, dn));
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

}  // extern "C"

namespace dbi {
namespace {
// The owner merge in three parts, so that the RCCL driver can fold its
// counters into the totals all-gather (one host sync for both):
// merge_begin -- the handle turns into the owner of its key range of the
// whole proteome, every buffer allocated (the merge's device time then holds
// no host allocation); merge_enqueue -- its kernels, no host sync;
// merge_done -- after the counters are on the host: stats, device time.
struct MergeRange {
    double lo = 0, hi = 0;
    bool first = false;  // the handle's first build (code objects load): not timed
    // depth bins (attempt 0 of a warm owner): the plan, the map sampled in this merge, the chunks
    DepthPlan dpl{};
    bool fresh = false;
    bool part_over = false;  // attempt 0's regions overflowed: the redo takes the radix tail
    BinMap sub{};
    uint32_t T = 0, nchunks = 0;
};

// The owner merge on depth bins: the single-device warm
// tail -- the records partitioned by the depth bins' high digit on their way
// in (k_expand_locs_part), one pass over the low digit, chunks of whole bins
// binned in LDS by the chunk sort -- instead of the radix tail's passes.  The
// map comes from this owner's previous slice of the index (its mass range
// [lo, hi] in 2^DEPTH_SUB_BITS sub-bins), or the map that slice gave last
// time; a merge with neither (the first, after a replica or a single-device
// build on the handle), or whose key range moved since that slice (the
// records outside the sampled range would crowd the end bins' regions), takes
// the radix tail.  Any monotone map gives the exact index: a stale one costs
// balance, never correctness.
void owner_depth_plan(dbi_handle* h, MergeRange& mr, uint64_t n_recv) {
    mr.dpl = DepthPlan{};
    mr.fresh = false;
    if (!h->opt_owner_depth || !h->use_depth || n_recv == 0) return;
    // measured per owner: a slice whose depth-bin merges ran slower per record
    // than its radix-tail ones keeps the radix tail (the lowest masses: few
    // distinct masses per depth bin, chunks for the big tier)
    if (h->owner_us_depth > 0.0 && h->owner_us_radix > 0.0 && h->owner_us_depth > h->owner_us_radix) return;
    const DepthPlan pl = depth_plan_n(h, n_recv, std::min<uint64_t>(h->recA.cap, 0xFFFFFFFEull));
    if (!pl.on) return;
    const BinMap sub = make_binmap(mr.lo, mr.hi, 1u << DEPTH_SUB_BITS);
    const bool reuse = depth_map_reusable(h, pl.nbins, sub);
    const bool own_index = h->owner_serial == h->build_serial && h->owner_umass == h->umass.p &&
                           h->owner_occ == h->occ_off.p && h->prev_unique > 0 && h->owner_lo == mr.lo &&
                           h->owner_hi == mr.hi;
    if (!reuse && !own_index) return;
    mr.dpl = pl;
    mr.fresh = !reuse;
    mr.sub = sub;
    mr.T = h->chunk_t ? h->chunk_t : (uint32_t)CHUNK_T_DEPTH;
    mr.nchunks = (uint32_t)std::max<uint64_t>((n_recv + mr.T - 1) / mr.T, 1);
}

int merge_begin(dbi_handle* h, MergeRange& mr) {
    ShardState& sh = h->shard;
    DBI_HIP(hipSetDevice(h->device));
    h->d_res = sh.d_res_global;
    h->d_poff = h->poff_g.p;
    h->n_res = sh.n_res_global;
    h->n_prot = sh.n_prot_global;
    h->n_total_extra = 0;
    int rc;
    if ((rc = h->recA.ensure(std::max<uint64_t>(sh.n_recv, 1)))) return rc;
    int32_t klo, khi;
    key_range(sh.split, sh.nshards, sh.rank, &klo, &khi);
    const double f = (double)h->params.mass_group_factor;
    mr.lo = klo == INT32_MIN ? h->params.min_mh : std::max(h->params.min_mh, (double)klo / f);
    const double hi = khi == INT32_MAX ? h->params.max_mh : std::min(h->params.max_mh, (double)khi / f);
    mr.hi = std::max(hi, mr.lo);
    for (int e = 0; e < 2; ++e)
        if (!h->ev_merge[e]) DBI_HIP(hipEventCreate(&h->ev_merge[e]));
    // an owner's tail buffers -- its index among them -- grow with 1/8 to spare:
    // its share moves a little from build to build (the splitters), and an
    // index left in place is what the next merge's depth map samples
    const uint64_t room = h->umass.cap < sh.n_recv ? sh.n_recv + sh.n_recv / 8 : sh.n_recv;
    // (and for the radix tail's plan over exactly n_recv: no allocation once its kernels are queued)
    if ((rc = tail_buffers(h, room, room, false)) || (rc = tail_buffers(h, sh.n_recv, sh.n_recv, false))) return rc;
    owner_depth_plan(h, mr, sh.n_recv);
    if (mr.dpl.on) {
        if ((rc = depth_buffers(h, mr.dpl, mr.nchunks))) return rc;
        owner_depth_plan(h, mr, sh.n_recv);  // (the map's buffer may have moved: sampled again)
    }
    mr.first = h->build_serial == 0;
    return 0;
}

// attempt 0: the chunk-list grids (and whether to run the giant pass) from
// this owner's previous merge; attempt 1 (lists outgrew them, ERR_GRID): full
// grids, from the received words again
int merge_body(dbi_handle* h, const MergeRange& mr, int attempt) {
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;
    if (attempt > 0) h->giants_seen = true;
    DBI_HIP(hipEventRecord(h->ev_merge[0], s));
    // counters back to zero (the layout word max_plen stays), n_kept = records received
    DBI_HIP(hipMemsetAsync(h->ctr.p, 0, offsetof(Counters, max_plen), s));
    hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(64), 0, s, &h->ctr.p->n_kept, (unsigned long long)sh.n_recv);
    DBI_HIP(hipGetLastError());
    // depth bins; a redo (chunk lists longer than their grids) keeps attempt
    // 0's map (its finalize may have overwritten the index the map sampled),
    // after a region overflow the radix tail
    if (mr.dpl.on && !mr.part_over) {
        int rc;
        DBI_HIP(hipMemsetAsync(h->rcur.p, 0, sizeof(uint32_t) * DEPTH_XCDS * 256, s));
        const uint64_t U = std::min<uint64_t>({h->prev_unique, h->umass.cap, h->occ_off.cap ? h->occ_off.cap - 1 : 0});
        if (attempt == 0 && mr.fresh && (rc = depth_map_enqueue(h, mr.dpl, mr.sub, U))) return rc;
        PartOut po{};
        po.recs = h->recR.p;
        po.dig = h->rdig.p;
        po.cur = h->rcur.p;
        po.dm = DepthMap{h->dmap.p, mr.sub, mr.dpl.b2, mr.dpl.nbins - 1};
        po.cap = mr.dpl.cap;
        po.b1 = mr.dpl.b1;
        STAGE(h, "owner_expand", by(0, 0, 0, 0, 0),
              launch_expand_locs_part(h->xrecv.p, (uint32_t)sh.n_recv, h->d_res, h->d_poff, h->mass_tab.p, h->dp.m0,
                                      sh.width, po, h->ctr.p, s));
        h->stages[h->nstage - 1].c0 = 25.0 * (double)sh.n_recv;  // 8 B in, 16 B + the digit out (+ the residues)
        if ((rc = depth_tail(h, mr.dpl, mr.sub, sh.n_recv, mr.T, mr.nchunks, attempt == 0))) return rc;
        DBI_HIP(hipEventRecord(h->ev_merge[1], s));
        return 0;
    }
    // the received location words -> records (mass + tag from the residues);
    // recA is free (the partition read it before the exchange was enqueued).
    // The expansion also counts the tail's first radix histogram (the same
    // bins build_tail plans from n_recv and [lo, hi]): one kernel fewer
    const uint32_t nbins = choose_nbins(sh.n_recv, h->bin_bits_max);
    int width[8] = {};
    const int passes = radix_plan(nbins, false, width);
    h->h1_on = passes >= 1 && width[0] >= 1 && sh.n_recv > 0;
    if (h->h1_on)
        STAGE(h, "owner_expand", by(0, 0, 0, 0, 0),
              launch_expand_locs_hist(h->xrecv.p, (uint32_t)sh.n_recv, h->d_res, h->d_poff, h->mass_tab.p, h->dp.m0,
                                      sh.width, h->recA.p, make_binmap(mr.lo, mr.hi, nbins), width[0], h->hist.p, s));
    else
        STAGE(h, "owner_expand", by(0, 0, 0, 0, 0),
              launch_expand_locs(h->xrecv.p, sh.n_recv, h->d_res, h->d_poff, h->mass_tab.p, h->dp.m0, sh.width,
                                 h->recA.p, s));
    h->stages[h->nstage - 1].c0 = 24.0 * (double)sh.n_recv;  // 8 B in, 16 B out (+ the residues)
    const int rc = build_tail(h, sh.n_recv, mr.lo, mr.hi, sh.n_recv, false, nullptr, nullptr, 0, attempt == 0);
    h->h1_on = false;
    if (rc) return rc;
    DBI_HIP(hipEventRecord(h->ev_merge[1], s));
    return 0;
}

// The merge's kernels, enqueued -- or, for a warm merge identical to the
// previous one (a repeated build of the same proteome: the same records
// received, the same buffers, grids and key range), replayed as a hipGraph
// captured on the second such merge (~30 launches: their gaps), as the
// single-device warm build does (build_digest).  Not with every stage timed
// (events in the dispatch packets) and not for a redo (attempt 1).
int merge_enqueue(dbi_handle* h, const MergeRange& mr, int attempt) {
    const bool graphable = attempt == 0 && h->use_graph && !(h->timing && h->timing_only.empty());
    if (!graphable) return merge_body(h, mr, attempt);
    dbi_handle::MergeKey k;
    k.g = graph_key(h);
    k.n_recv = h->shard.n_recv;
    k.lo = mr.lo;
    k.hi = mr.hi;
    k.xrecv = h->xrecv.p;
    k.width = h->shard.width;
    k.nstage0 = h->nstage;
    k.depth_cap = mr.dpl.on ? mr.dpl.cap : 0u;
    k.depth_fresh = mr.dpl.on && mr.fresh;
    auto& mg = h->mgraph;
    if (mg.exec && mg.key == k) {
        DBI_HIP(hipGraphLaunch(mg.exec, h->stream));
        std::copy(mg.stages, mg.stages + mg.nstage, h->stages + k.nstage0);
        h->nstage = k.nstage0 + mg.nstage;
        h->stats.n_bins = mg.n_bins;
        h->skip_mid = h->grid_mid == GRID_NONE;  // as when it was captured (the grids are in the key)
        h->skip_big = h->grid_big == GRID_NONE;
        return 0;
    }
    if (!(h->prev_mkey_valid && h->prev_mkey == k)) {
        const int rc = merge_body(h, mr, attempt);
        h->prev_mkey = k;
        h->prev_mkey_valid = rc == 0;
        return rc;
    }
    // the same merge as last time: capture it, then run the graph
    if (mg.exec) (void)hipGraphExecDestroy(mg.exec);
    if (mg.graph) (void)hipGraphDestroy(mg.graph);
    mg.exec = nullptr;
    mg.graph = nullptr;
    DBI_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
    h->capturing = true;
    const int rc = merge_body(h, mr, attempt);
    h->capturing = false;
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(h->stream, &g);
    if (rc || ec != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        h->prev_mkey_valid = false;
        return rc ? rc : hip_fail(ec, "hipStreamEndCapture (owner merge)");
    }
    hipGraphExec_t ex = nullptr;
    const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
        (void)hipGraphDestroy(g);
        h->prev_mkey_valid = false;
        return hip_fail(ei, "hipGraphInstantiate (owner merge)");
    }
    DBI_HIP(hipGraphLaunch(ex, h->stream));
    mg.graph = g;
    mg.exec = ex;
    mg.key = k;
    mg.nstage = h->nstage - k.nstage0;
    std::copy(h->stages + k.nstage0, h->stages + h->nstage, mg.stages);
    mg.n_bins = h->stats.n_bins;
    if (graph_key(h).alloc_gen != k.g.alloc_gen) {  // buffers moved while capturing: once only
        (void)hipGraphExecDestroy(mg.exec);
        (void)hipGraphDestroy(mg.graph);
        mg.exec = nullptr;
        mg.graph = nullptr;
        h->prev_mkey_valid = false;
    }
    return 0;
}

// h->hc holds the merge's counters (read_counters, or the totals round)
int merge_done(dbi_handle* h, const MergeRange& mr) {
    int rc;
    if ((rc = finish_build(h))) return rc;
    // the index is this owner's slice: the next merge's depth map samples it
    h->owner_serial = h->build_serial;
    h->owner_umass = h->umass.p;
    h->owner_occ = h->occ_off.p;
    h->owner_lo = mr.lo;
    h->owner_hi = mr.hi;
    if (h->hc.err & ERR_PART) {  // a region overflowed (redone by the radix tail): more room, a fresh map
        h->depth_slack = std::min(8.0, 2.0 * h->depth_slack);
        h->depth_map_unique = 0;
    }
    float mg = 0.f;
    h->shard.ms_merge_gpu =
        !mr.first && hipEventElapsedTime(&mg, h->ev_merge[0], h->ev_merge[1]) == hipSuccess ? (double)mg : 0.0;
    // (a depth merge that sampled its map is not counted: the map, and its
    // first chunk lists against the radix tail's grids, are one-off costs)
    const bool depth = mr.dpl.on && !mr.part_over;
    if (h->shard.ms_merge_gpu > 0.0 && h->shard.n_recv > 0 && !(h->hc.err & ERR_PART) && !(depth && mr.fresh)) {
        double& us = depth ? h->owner_us_depth : h->owner_us_radix;
        const double v = 1e6 * h->shard.ms_merge_gpu / (double)h->shard.n_recv;
        us = us > 0.0 ? 0.5 * us + 0.5 * v : v;
    }
    return 0;
}

// the totals row's device columns: unique peptides, mass keys, and the
// merge's flags (bit 0: chunk lists outgrew their grids -- merge again;
// bits 8+: device error bits)
__global__ void k_totals_row(const Counters* __restrict__ ctr, unsigned long long* __restrict__ row, int skip_mid,
                             int skip_big) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned long long keys = ctr->n_keys;
    for (int i = 0; i < 8; ++i) keys += ctr->n_keys_shard[i];
    row[3] = ctr->n_unique;
    row[4] = keys;
    // (a depth-bin region that overflowed: the merge again, by the radix tail)
    const bool redo = (ctr->err & (ERR_GRID | ERR_PART)) || (skip_mid && ctr->n_mid) || (skip_big && ctr->n_big);
    row[7] = (redo ? 1ull : 0ull) | ((unsigned long long)(ctr->err & ~(ERR_GRID | ERR_PART)) << 8);
}
}  // namespace
}  // namespace dbi

extern "C" {

int dbi_shard_merge(dbi_handle* h) {
    if (!h) return set_error(DBI_E_INVALID, "NULL handle");
    int rc;
    if ((rc = need_phase(h, 3, "dbi_shard_merge"))) return rc;
    ShardState& sh = h->shard;
    const double t0 = now_ms();
    MergeRange mr;
    if ((rc = merge_begin(h, mr))) return rc;
    for (int attempt = 0;; ++attempt) {
        const int nstage0 = h->nstage;
        if ((rc = merge_enqueue(h, mr, attempt))) return rc;
        if ((rc = merge_done(h, mr))) return rc;  // (synchronises)
        if (h->hc.err & ERR_PART) mr.part_over = true;
        if (!h->lists_short && !(h->hc.err & ERR_PART)) break;
        if (attempt > 0) return set_error(DBI_E_STATE, "internal: chunk lists outgrew full grids");
        h->nstage = nstage0;
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
    st.split_sampled = sh.split_sampled;
    st.split_rounds = sh.split_rounds;
    st.split_held = sh.split_held ? 1 : 0;
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
    if (!rc_route) rc_route = injected_failure(h, "qroute", me);
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
    if (!rc_local) rc_local = injected_failure(h, "qbuffers", me);
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
    std::vector<Xfer> sends, recvs;
    for (const Arr& a : arrs)
        for (int p = 0; p < n; ++p) {
            if (p == me) continue;
            const uint64_t mc = a.occ ? z.k[me] : z.u[me];
            const uint64_t pc = a.occ ? z.k[p] : z.u[p], pb = a.occ ? z.kb[p] : z.ub[p];
            sends.push_back(Xfer{p, a.src, mc * a.esz});
            recvs.push_back(Xfer{p, a.dst + pb * a.esz, pc * a.esz});
        }
    if ((rc = c_group(c, sends, recvs, s))) return rc;
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

namespace {
// the communicator's device staging (status word, reduction buffer, sample
// blocks, count matrix / totals rows) and its stream
int comm_staging(dbi_comm* c) {
    if (hipMalloc((void**)&c->d_flag, 2 * sizeof(unsigned long long)) != hipSuccess)
        return set_error(DBI_E_OOM, "hipMalloc (communicator status word)");
    c->cnt_row = std::max(c->nranks + 4, TOTALS_W);  // count matrix row | the totals row
    if (hipMalloc((void**)&c->d_red, COMM_RED_MAX * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&c->d_samp, sizeof(double) * (size_t)c->nranks * (NS + 3)) != hipSuccess ||
        hipMalloc((void**)&c->d_cnt, sizeof(unsigned long long) * (size_t)c->nranks * c->cnt_row) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return set_error(DBI_E_HIP, "communicator stream / staging buffer");
    return 0;
}
}  // namespace

int dbi_comm_init_host(const char* name, int nranks, int rank, int device, uint64_t slot_bytes, dbi_comm** out) {
    if (!name || !out || name[0] != '/') return set_error(DBI_E_INVALID, "host transport: a '/name' is needed");
    *out = nullptr;
    if (nranks < 1 || nranks > MAX_SHARDS || rank < 0 || rank >= nranks)
        return set_error(DBI_E_INVALID, "rank / nranks out of range (1..64 ranks)");
    if (slot_bytes < 4096) return set_error(DBI_E_INVALID, "host transport: slots of at least 4096 bytes");
    DBI_HIP(hipSetDevice(device));
    dbi_comm* c = new dbi_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->host = new HostXport();
    HostXport& x = *c->host;
    x.name = name;
    x.slot = (slot_bytes + 63) & ~63ull;
    x.bytes = 4096 + (size_t)nranks * x.slot + (size_t)nranks * nranks * x.slot;
    auto fail = [&](int code, const std::string& msg) {
        if (rank != 0) x.name.clear();  // only rank 0 unlinks
        dbi_comm_destroy(c);
        return set_error(code, "host transport: " + msg);
    };
    if (rank == 0) {
        (void)shm_unlink(name);  // a segment a crashed run left behind
        x.fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (x.fd < 0 || ftruncate(x.fd, (off_t)x.bytes) != 0) return fail(DBI_E_OOM, "shm_open / ftruncate");
        void* m = mmap(nullptr, x.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, x.fd, 0);
        if (m == MAP_FAILED) return fail(DBI_E_OOM, "mmap");
        x.base = static_cast<uint8_t*>(m);
        ShmHeader* h = new (x.base) ShmHeader();
        h->count.store(0);
        h->gen.store(0);
        h->nranks = (uint32_t)nranks;
        h->slot = x.slot;
        h->ready.store(1, std::memory_order_release);
    } else {
        const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(60);
        for (;;) {
            x.fd = shm_open(name, O_RDWR, 0600);
            struct stat stt;
            if (x.fd >= 0 && fstat(x.fd, &stt) == 0 && (size_t)stt.st_size == x.bytes) {
                void* m = mmap(nullptr, x.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, x.fd, 0);
                if (m != MAP_FAILED) {
                    x.base = static_cast<uint8_t*>(m);
                    if (x.hdr()->ready.load(std::memory_order_acquire) == 1) break;
                    (void)munmap(x.base, x.bytes);
                    x.base = nullptr;
                }
            }
            if (x.fd >= 0) (void)close(x.fd);
            x.fd = -1;
            if (std::chrono::steady_clock::now() > t_end) return fail(DBI_E_RCCL, "rank 0's segment never appeared");
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
    }
    int rc;
    if ((rc = comm_staging(c)) || (rc = shm_barrier(c))) {
        const std::string msg = dbi_last_error();
        return fail(rc, msg);
    }
    *out = c;
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
    int rc;
    if ((rc = comm_staging(c))) {
        dbi_comm_destroy(c);
        return rc;
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
    if (c->host) {
        if (c->host->base) (void)munmap(c->host->base, c->host->bytes);
        if (c->host->fd >= 0) (void)close(c->host->fd);
        if (c->rank == 0 && !c->host->name.empty()) (void)shm_unlink(c->host->name.c_str());
        delete c->host;
    }
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
    int rc;
    if ((rc = c_allreduce(c, c->d_red, c->d_red, m, ncclFloat64, rop, c->stream))) return rc;
    if (n) DBI_HIP(hipMemcpyAsync(out, c->d_red, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    DBI_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int dbi_comm_allreduce_u64(dbi_comm* c, const uint64_t* d_in, uint64_t* d_out, uint64_t n, void* stream) {
    if (!c || (n && (!d_in || !d_out))) return set_error(DBI_E_INVALID, "NULL argument");
    DBI_HIP(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int rc;
    if (n && (rc = c_allreduce(c, d_in, d_out, n, ncclUint64, ncclSum, s))) return rc;
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
    std::vector<Xfer> sends, recvs;
    for (int p = 0; p < c->nranks; ++p) {
        if (p == c->rank) continue;
        sends.push_back(Xfer{p, mine, my_bytes});
        recvs.push_back(Xfer{p, recv + off[p], rank_bytes[p]});
    }
    int rc;
    if ((rc = c_group(c, sends, recvs, s))) return rc;
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

// Can this build digest its shard device-sized (shard_digest_dev)?  A warm
// handle (bounded digest into the previous capacity) digesting the same
// shard of the same inputs as its last sharded build.
bool shard_dev_ok(const dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_poff, uint64_t n_prot,
                  uint64_t p_begin, uint64_t p_end) {
    const auto& dv = h->shard_dev;
    return dv.valid && h->opt_shard_dev_digest && dv.d_res == d_res && dv.d_poff == d_poff && dv.n_res == n_res &&
           dv.n_prot == n_prot && dv.p_begin == p_begin && dv.p_end == p_end && dv.e1 > dv.e0 &&
           h->recA.cap >= 1024 && bounded_digest(h);
}

// dbi_shard_digest without its two host round trips (dbi_build_sharded, warm):
// the residue range and record width of the last build (k_shard_flags checks
// them on the device), the bounded digest into the previous capacity, and the
// partition reading the slot count on the device (k_tail_counts: 0 when the
// slots overflowed).  Host-side numbers (records, drops, errors) arrive with
// the count matrix (shard_digest_dev_done); a flagged rank digests again
// with dbi_shard_digest.
int shard_digest_dev(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_poff, uint64_t n_prot,
                     uint64_t p_begin, uint64_t p_end, int rank, int nshards) {
    int rc;
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    const double t0 = now_ms();
    hipStream_t s = h->stream;
    const auto& dv = h->shard_dev;
    const uint64_t np = p_end - p_begin;
    if ((rc = h->poff_g.ensure(n_prot + 1)) || (rc = h->poff.ensure(np + 1))) return rc;
    DBI_HIP(launch_off_rebase(d_poff, 0, n_res, h->poff_g.p, n_prot + 1, s));
    DBI_HIP(launch_off_rebase(d_poff + p_begin, dv.e0, dv.e1 - dv.e0, h->poff.p, np + 1, s));
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
    h->d_res = d_res + dv.e0;
    h->d_poff = h->poff.p;
    h->n_res = dv.e1 - dv.e0;
    h->n_prot = np;
    uint64_t n = 0, n_in = 0;
    bool sparse = false, dev = false;
    if ((rc = run_digest(h, &n, &n_in, &sparse, &dev))) return rc;
    if (!dev || !sparse) return set_error(DBI_E_STATE, "internal: device-sized shard digest without bounded slots");
    DBI_HIP(launch_tail_counts(h->ctr.p, n_in, true, s));
    sh.width = dv.width;
    sh.n_digest = n;  // the capacity until the count matrix arrives
    sh.n_in = n_in;
    sh.sparse = true;
    sh.dev = true;
    sh.ms_digest = now_ms() - t0;
    sh.phase = 1;
    return 0;
}

// after the count-matrix sync (h->hc holds the digest's counters): the
// numbers dbi_shard_digest reads at once
int shard_digest_dev_done(dbi_handle* h) {
    ShardState& sh = h->shard;
    if (h->hc.err & ERR_LAYOUT) return set_error(DBI_E_INVALID, "record layout overflow in the shard digest");
    if (h->hc.err & ERR_PTM) return set_error(DBI_E_INVALID, ptm_device_msg());
    for (int i = 0; i < h->nstage; ++i) {  // the digest stages' bytes are this shard's
        auto& st = h->stages[i];
        st.c0 += st.cR * (double)h->n_res + st.cN * (double)h->hc.n_kept + st.cP * (double)(h->n_prot + 1);
        st.cR = st.cN = st.cU = st.cP = st.cB = 0;
    }
    sh.n_digest = h->hc.n_kept;
    sh.n_in = h->hc.n_slots;
    sh.n_total = h->hc.n_kept + h->hc.n_dropped;
    sh.n_dropped = h->hc.n_dropped;
    sh.dev = false;
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
    // option shard_full_path: one rank takes the general path too (tests of
    // the partition / exchange / agreement code at N=1)
    if (n == 1 && p_begin == 0 && p_end == n_prot && !h->opt_shard_full_path)
        return build_single_owner(h, d_res, n_res, d_poff, n_prot);
    int rc;
    // a rank that fails locally still takes part in the next collective, with
    // its status, so that every rank returns an error (never a hang)
    const double t_digest = now_ms();
    auto& wm = h->shard_warm;
    auto& pf = h->shard_prof;
    h->shard.split_held = false;
    // a warm build of the same shard with a reusable split digests
    // device-sized: no host round trip before the count matrix
    const bool dev_digest = wm.valid && wm.n == n && !h->opt_shard_resample &&
                            shard_dev_ok(h, d_res, n_res, d_poff, n_prot, p_begin, p_end);
    int rc_digest = dev_digest ? shard_digest_dev(h, d_res, n_res, d_poff, n_prot, p_begin, p_end, me, n)
                               : dbi_shard_digest(h, d_res, n_res, d_poff, n_prot, p_begin, p_end, me, n);
    if (!rc_digest) rc_digest = injected_failure(h, "digest", me);
    ShardState& sh = h->shard;
    hipStream_t s = h->stream;

    // Owner splitters.  A warm build reuses the split the previous build left
    // (computed from the sorted samples of the last sampled build and the
    // updated cost profile -- the same inputs, hence the same split, on every
    // rank); the count matrix carries a hash of each rank's split.  A rank
    // without one (a new handle, another communicator size, option shard_resample)
    // or ranks that disagree: every rank samples (the samples all-gather, with
    // a fingerprint of each rank's cost profile: profiles that differ are not
    // used), and partitions again.  The decision is taken from the gathered
    // matrix, so every rank takes the same collectives.
    bool have_split = wm.valid && wm.n == n && !h->opt_shard_resample;
    int32_t split[MAX_SHARDS - 1] = {};
    if (have_split) std::copy(wm.split, wm.split + (n - 1), split);
    bool sampled = false;
    auto sample_split = [&]() -> int {
        // block of rank r: NS record masses (written on the device), its record
        // count, its status, its cost-profile fingerprint
        const size_t blk = NS + 3;
        int rc_s = rc_digest;
        double* my_blk = c->d_samp + (size_t)me * blk;
        if (!rc_s) {
            const hipError_t e = launch_sample_masses(h->recA.p, sh.n_in, NS, my_blk, s);
            if (e != hipSuccess) rc_s = hip_fail(e, "launch_sample_masses");
        }
        std::vector<double> samples((size_t)n * blk, 0.0);
        double* mine = samples.data() + (size_t)me * blk;
        mine[NS] = rc_s ? 0.0 : (double)sh.n_digest;
        mine[NS + 1] = rc_s ? 1.0 : 0.0;
        uint64_t fp = pf.valid ? fnv64(pf.cost, sizeof(pf.cost), fnv64(pf.split, sizeof(pf.split))) : 0ull;
        std::memcpy(&mine[NS + 2], &fp, 8);
        DBI_HIP(hipMemcpyAsync(my_blk + NS, mine + NS, 3 * sizeof(double), hipMemcpyHostToDevice, s));
        int rc_c;
        if ((rc_c = c_allgather(c, my_blk, c->d_samp, 8ull * blk, s))) return rc_c;
        DBI_HIP(hipMemcpyAsync(samples.data(), c->d_samp, sizeof(double) * n * blk, hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
        if (rc_s) return rc_s;
        std::vector<double> packed((size_t)n * (NS + 1));
        bool same_profile = true;
        for (int r = 0; r < n; ++r) {
            const double* b = samples.data() + (size_t)r * blk;
            if (b[NS + 1] != 0.0) return peer_failed("shard digest");
            uint64_t fr;
            std::memcpy(&fr, &b[NS + 2], 8);
            same_profile &= fr == fp;
            uint64_t valid = 0;
            for (uint32_t i = 0; i < NS; ++i) valid += b[i] == b[i];
            std::copy(b, b + NS, packed.begin() + (size_t)r * (NS + 1));
            packed[(size_t)r * (NS + 1) + NS] = valid ? b[NS] / (double)valid : 0.0;  // as dbi_shard_samples
        }
        sample_keys(packed.data(), n, h->params.mass_group_factor, wm.keys);
        // the profile only where every rank holds the same one (a
        // reopened handle or another build history must not split differently);
        // ranks whose profiles differ all drop theirs, so the next cost update
        // (the same gathered merge times on every rank) makes them equal again
        // at once (one rank's fresh profile beside the others'
        // averaged ones disagreed on every later build's split hash)
        if (!same_profile) pf = {};
        const bool prof = pf.valid;
        split_from_keys(wm.keys, n, prof ? CB : 0, prof ? pf.split : nullptr, prof ? pf.cost : nullptr, split);
        sampled = true;
        have_split = true;
        return 0;
    };

    // count matrix: row r = records shard r sends each owner (from its owner
    // histogram, on the device) | its status | its receive capacity | its
    // split's hash | its device flags (a device-sized digest to redo, k_shard_flags)
    const int w = n + 4;
    std::vector<unsigned long long> full((size_t)n * w, 0);
    std::vector<uint64_t> counts((size_t)n * n);
    bool failed = false, grow = false, sample_next = false;
    double t_part = now_ms();
    for (int round = 0;; ++round) {
        if (sample_next) {
            if ((rc = sample_split())) return rc;
            t_part = now_ms();
        }
        int rc_part = rc_digest;
        if (round == 0 && have_split) {
            // test hook (option test_split_skew = this rank): its reused split
            // differs from its peers' (another build history): the count
            // matrix's hashes disagree and every rank samples again
#ifdef DBI_TEST_HOOKS
            if (h->opt_test_split_skew == me && n > 1) split[0] += 1;
#endif
        }
        if (!rc_part && have_split) rc_part = partition_launch(h, split);
        if (!rc_part) rc_part = injected_failure(h, "partition", me);
        unsigned long long* my_row = c->d_cnt + (size_t)me * w;
        if (!rc_part && have_split && sh.n_in > 0) {
            hipLaunchKernelGGL(k_owner_counts, dim3(1), dim3(64), 0, s, h->hist.p, sh.part_blocks, (uint32_t)n,
                               sh.n_digest, sh.dev ? &h->ctr.p->tail_n : nullptr, my_row);
            if ((rc = hipGetLastError()) != hipSuccess) rc_part = hip_fail((hipError_t)rc, "k_owner_counts");
        } else if ((rc = hipMemsetAsync(my_row, 0, sizeof(unsigned long long) * n, s)) != hipSuccess && !rc_part) {
            rc_part = hip_fail((hipError_t)rc, "hipMemsetAsync");
        }
        unsigned long long* mine = &full[(size_t)me * w];
        mine[n] = rc_part ? 1u : 0u;
        mine[n + 1] = h->xrecv.cap;
        mine[n + 2] = have_split ? (fnv64(split, sizeof(int32_t) * (n - 1)) | 1ull) : 0ull;
        mine[n + 3] = 0;
        DBI_HIP(hipMemcpyAsync(my_row + n, mine + n, 4 * sizeof(unsigned long long), hipMemcpyHostToDevice, s));
        if (!rc_part && sh.dev) {
            const auto& dv = h->shard_dev;
            hipLaunchKernelGGL(k_shard_flags, dim3(1), dim3(64), 0, s, d_poff, p_begin, p_end, dv.e0, dv.e1, dv.width,
                               h->ctr.p, sh.n_in, my_row + n + 3);
            if ((rc = hipGetLastError()) != hipSuccess) rc_part = hip_fail((hipError_t)rc, "k_shard_flags");
        }
        if ((rc = c_allgather(c, my_row, c->d_cnt, 8ull * w, s))) return rc;
        DBI_HIP(hipMemcpyAsync(full.data(), c->d_cnt, sizeof(unsigned long long) * n * w, hipMemcpyDeviceToHost, s));
        if (sh.dev) DBI_HIP(hipMemcpyAsync(&h->hc, h->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
        if (rc_part) return rc_part;
        bool agree_split = true, redo = false;
        for (int i = 0; i < n; ++i) {
            failed |= full[(size_t)i * w + n] != 0;
            agree_split &= full[(size_t)i * w + n + 2] != 0 && full[(size_t)i * w + n + 2] == mine[n + 2];
            redo |= full[(size_t)i * w + n + 3] != 0;
        }
        if (failed) return peer_failed(round == 0 ? "owner partition" : "owner partition (sampled split)");
        if (redo) {
            // a device-sized digest did not fit its slots, or the offsets moved:
            // that rank digests again with dbi_shard_digest (grows the buffer,
            // reads the range), every rank partitions and gathers again (the
            // same verdict everywhere: the same matrix)
            if (round >= 2) return set_error(DBI_E_STATE, "internal: shard digest redone twice");
            if (full[(size_t)me * w + n + 3] != 0) {
                rc_digest = dbi_shard_digest(h, d_res, n_res, d_poff, n_prot, p_begin, p_end, me, n);
                t_part = now_ms();
            }
            continue;
        }
        if (sh.dev && (rc = shard_digest_dev_done(h))) return rc;  // (a device error is a flag: never here)
        sh.split_rounds = round + 1;
        if (agree_split) break;
        if (sample_next) return set_error(DBI_E_STATE, "internal: ranks computed different owner splits from the "
                                                       "same samples");
        sample_next = true;  // every rank samples: the same verdict from the same matrix
        have_split = false;
    }
    sh.ms_digest = t_part - t_digest;
    sh.split_sampled = sampled ? 1 : 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) counts[(size_t)i * n + j] = full[(size_t)i * w + j];
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
    const double t0 = now_ms();
    // an owner that must grow its receive buffer may fail to: then every rank
    // learns it before the exchange (a collective only when someone grows)
    if (grow) {
        int rc_local = h->xrecv.ensure(std::max<uint64_t>(roff[n], 1));
        if (!rc_local) rc_local = injected_failure(h, "buffers", me);
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

    // owner merge, then the whole-index totals: the merge's counters reach the
    // host with the totals all-gather (one host sync for both).  Row: n_total,
    // n_dropped, n_recv, n_unique, n_keys, status, the previous build's merge
    // device time (ns) and records received (the cost profile), merge flags
    // (bit 0: this owner's chunk lists outgrew their grids -- it merges again
    // and every rank gathers the totals again; bits 8+: device errors)
    const double t_merge = now_ms();
    MergeRange mr;
    int rc_merge = merge_begin(h, mr);
    std::vector<unsigned long long> rows((size_t)n * TOTALS_W);
    std::vector<uint64_t> tot(5, 0);
    bool redo_me = true;
    const int nstage0 = h->nstage;
    for (int attempt = 0;; ++attempt) {
        if (!rc_merge && redo_me) {
            if (attempt > 0) h->nstage = nstage0;
            rc_merge = merge_enqueue(h, mr, attempt);
        }
        if (!rc_merge && attempt == 0) rc_merge = injected_failure(h, "merge", me);
        unsigned long long row[TOTALS_W] = {};
        row[0] = sh.n_total;
        row[1] = sh.n_dropped;
        row[2] = sh.n_recv;
        row[5] = rc_merge ? 1u : 0u;
        row[6] = (unsigned long long)(wm.prev_merge_ms * 1e6);  // ns
        row[8] = wm.prev_recv;
        unsigned long long* my_row = c->d_cnt + (size_t)me * TOTALS_W;
        DBI_HIP(hipMemcpyAsync(my_row, row, sizeof(row), hipMemcpyHostToDevice, s));
        if (!rc_merge) {
            hipLaunchKernelGGL(k_totals_row, dim3(1), dim3(64), 0, s, h->ctr.p, my_row, h->skip_mid ? 1 : 0,
                               h->skip_big ? 1 : 0);
            if ((rc = hipGetLastError()) != hipSuccess) rc_merge = hip_fail((hipError_t)rc, "k_totals_row");
        }
        if ((rc = c_allgather(c, my_row, c->d_cnt, 8ull * TOTALS_W, s))) return rc;
        DBI_HIP(hipMemcpyAsync(rows.data(), c->d_cnt, sizeof(unsigned long long) * n * TOTALS_W,
                               hipMemcpyDeviceToHost, s));
        DBI_HIP(hipMemcpyAsync(&h->hc, h->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
        if (rc_merge) return rc_merge;
        if (h->hc.err & ERR_PART) {  // this owner's depth-bin region overflowed: more room, a fresh map next time
            h->depth_slack = std::min(8.0, 2.0 * h->depth_slack);
            h->depth_map_unique = 0;
            mr.part_over = true;
        }
        bool any_redo = false;
        for (int i = 0; i < n; ++i) {
            const unsigned long long* r = rows.data() + (size_t)i * TOTALS_W;
            if (r[5] || (r[7] >> 8)) {
                if (i == me) {  // this owner's device error: finish_build names it
                    h->hc_final = true;
                    if ((rc = finish_build(h))) return rc;
                }
                return peer_failed("owner merge");
            }
            any_redo |= (r[7] & 1u) != 0;
        }
        redo_me = (rows[(size_t)me * TOTALS_W + 7] & 1u) != 0;
        if (!any_redo) break;
        if (attempt > 0) return set_error(DBI_E_STATE, "internal: chunk lists outgrew full grids");
    }
    h->hc_final = true;  // the counters came with the totals
    if ((rc = merge_done(h, mr))) return rc;
    sh.ms_merge = now_ms() - t_merge;
    sh.phase = 4;
    sh.u_base = 0;
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < 5; ++k) tot[k] += rows[(size_t)i * TOTALS_W + k];
        if (i < me) sh.u_base += rows[(size_t)i * TOTALS_W + 3];
    }
    sh.u_base_known = true;
    // the cost profile from the PREVIOUS build's owners (merge device time and
    // records, the same numbers on every rank; this build's merge time is
    // known only after the totals round), then the split the next build uses
    std::vector<double> mms(n);
    std::vector<uint64_t> recs(n);
    for (int i = 0; i < n; ++i) {
        mms[i] = (double)rows[(size_t)i * TOTALS_W + 6] * 1e-6;
        recs[i] = rows[(size_t)i * TOTALS_W + 8];
    }
    if (wm.valid && wm.n == n && (rc = dbi_shard_cost_update(h, n, wm.prev_split, mms.data(), recs.data())))
        return rc;
    // hysteresis: the previous build ran this build's split and
    // its owners' merge times were within SPLIT_HOLD of their mean -- keep the
    // split instead of chasing the profile (every re-split moves the spiky
    // low-mass key bands between owners and the slowest owner with them)
    bool hold = wm.valid && wm.n == n && std::equal(sh.split, sh.split + (n - 1), wm.prev_split);
    if (hold) {
        double mx = 0.0, sum = 0.0;
        for (int i = 0; i < n; ++i) {
            hold = hold && mms[i] > 0.0;
            mx = std::max(mx, mms[i]);
            sum += mms[i];
        }
        hold = hold && mx <= SPLIT_HOLD * sum / n;
    }
    std::copy(sh.split, sh.split + (n - 1), wm.prev_split);
    wm.prev_merge_ms = sh.ms_merge_gpu;
    wm.prev_recv = sh.n_recv;
    if (sampled) wm.sampled_kept = tot[2];
    // a proteome of another size than the sampled one: sample again next time
    const bool stale = wm.sampled_kept == 0 || tot[2] > wm.sampled_kept + wm.sampled_kept / 20 ||
                       tot[2] + wm.sampled_kept / 20 < wm.sampled_kept;
    if (stale) {
        wm.valid = false;
        forget_best_split(h);  // (measured on another proteome)
    } else {
        if (hold)
            std::copy(sh.split, sh.split + (n - 1), wm.split);
        else if (shard_split_frozen(h, n))  // the search stopped: the best split, kept
            std::copy(pf.best_split, pf.best_split + (n - 1), wm.split);
        else
            split_from_keys(wm.keys, n, pf.valid ? CB : 0, pf.valid ? pf.split : nullptr, pf.valid ? pf.cost : nullptr,
                            wm.split);
        wm.valid = true;
        wm.n = n;
    }
    sh.split_held = hold && !stale;
    sh.global.g_total = tot[0];
    sh.global.g_dropped = tot[1];
    sh.global.g_kept = tot[2];
    sh.global.g_unique = tot[3];
    sh.global.g_keys = tot[4];
    return 0;
}

}  // extern "C"
