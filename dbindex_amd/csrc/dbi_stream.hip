// dbi_stream.hip — count-only streaming over proteomes too large to index
// (BASELINE.json configs[4]: TrEMBL-scale, 50M proteins, non-specific 6-50:
// ~7e11 peptide occurrences, ~12 TB of records — cannot be materialised).
//
// A proteome chunk is generated on the device from a counter-based hash
// (dbi_synth_proteome: no host data, any protein range of the proteome on any
// GPU, identical to the numpy twin in dbindex_amd/fasta.py), then digested in
// COUNT mode (the cutSeq loop, DBIndexer.java:237-405, without records:
// dbi_count).  The sums equal the reference's totalSeqCount
// (DBIndexStoreSQLiteMult.java:277) over the same proteins.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "dbi_engine.h"

using namespace dbi;

namespace dbi {
namespace {

constexpr int SYNTH_LEN_BITS = 12;  // 4096-entry protein length quantile table
constexpr int SYNTH_RES_BITS = 16;  // 65536-entry residue table (CDF of the residue frequencies)
constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;
constexpr uint64_t RES_SALT = 0xD1B54A32D192ED03ull;

__host__ __device__ inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

__global__ void k_synth_len(uint64_t seed, uint64_t p_begin, uint32_t n, const uint16_t* __restrict__ lentab,
                            uint32_t* __restrict__ len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    len[i] = lentab[fmix64(seed * GOLDEN + p_begin + i + 1) >> (64 - SYNTH_LEN_BITS)];
}

// 16 residues per thread, one 16-B store
__global__ void k_synth_res(uint64_t seed, uint64_t res_base, uint64_t n, const uint8_t* __restrict__ restab,
                            uint8_t* __restrict__ out) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i0 >= n) return;
    const uint64_t key = (seed ^ RES_SALT) * GOLDEN + res_base;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t g = i0 + 4 * q + b;
            v |= (uint32_t)restab[fmix64(key + g) >> (64 - SYNTH_RES_BITS)] << (8 * b);
        }
        w[q] = v;
    }
    if (i0 + 16 <= n) {
        *reinterpret_cast<uint4*>(out + i0) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (uint64_t g = i0; g < n; ++g) out[g] = (uint8_t)(w[(g - i0) / 4] >> (8 * ((g - i0) % 4)));
    }
}

__global__ void k_widen_offsets(const uint32_t* __restrict__ excl, uint32_t n, uint32_t total,
                                uint64_t* __restrict__ off) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) off[i] = excl[i];
    if (i == n) off[n] = total;
}

}  // namespace
}  // namespace dbi

extern "C" {

int dbi_synth_proteome(dbi_handle* h, uint64_t seed, uint64_t p_begin, uint64_t n_prot, uint64_t res_base,
                       const uint16_t* len_table, const uint8_t* res_table, const uint8_t** d_residues,
                       const uint64_t** d_prot_off, uint64_t* n_res) {
    if (!h || !len_table || !res_table || !d_residues || !d_prot_off || !n_res)
        return set_error(DBI_E_INVALID, "NULL argument");
    if (n_prot >= (1ull << 31)) return set_error(DBI_E_INVALID, "at most 2^31-1 proteins per chunk");
    DBI_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    int rc;
    if ((rc = h->synth_len.ensure(1u << SYNTH_LEN_BITS)) || (rc = h->synth_res.ensure(1u << SYNTH_RES_BITS)) ||
        (rc = h->thr.ensure(n_prot + 1)) || (rc = h->synth_off.ensure(n_prot + 1)) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(n_prot + 1), h->scan_tmp.cap))) ||
        (rc = h->xcount.ensure(std::max<size_t>(h->xcount.cap, 8))))
        return rc;
    DBI_HIP(hipMemcpyAsync(h->synth_len.p, len_table, sizeof(uint16_t) << SYNTH_LEN_BITS, hipMemcpyHostToDevice, s));
    DBI_HIP(hipMemcpyAsync(h->synth_res.p, res_table, (size_t)1 << SYNTH_RES_BITS, hipMemcpyHostToDevice, s));
    const uint32_t n = (uint32_t)n_prot;
    unsigned long long total = 0;
    if (n) {
        DBI_LAUNCH(k_synth_len, dim3((n + 255) / 256), dim3(256), 0, s, seed, p_begin, n, h->synth_len.p, h->thr.p);
        DBI_HIP(hipGetLastError());
        DBI_HIP(launch_scan_u32(h->thr.p, h->thr.p, n, h->scan_tmp.p, h->scan_tmp.cap, h->xcount.p, s));
        DBI_HIP(hipMemcpyAsync(&total, h->xcount.p, sizeof(total), hipMemcpyDeviceToHost, s));
        DBI_HIP(hipStreamSynchronize(s));
    }
    if (total >= (1ull << 32) - 16) return set_error(DBI_E_INVALID, "chunk above 2^32 residues: use smaller chunks");
    // the generator's own buffers: never the residues / offsets an index was built from
    if ((rc = h->synth_out.ensure(total + 16))) return rc;
    DBI_LAUNCH(k_widen_offsets, dim3((n + 1 + 255) / 256), dim3(256), 0, s, h->thr.p, n, (uint32_t)total,
               h->synth_off.p);
    DBI_HIP(hipGetLastError());
    if (total) {
        const uint64_t nt = (total + 15) / 16;
        DBI_LAUNCH(k_synth_res, dim3((uint32_t)((nt + 255) / 256)), dim3(256), 0, s, seed, res_base, total,
                   h->synth_res.p, h->synth_out.p);
        DBI_HIP(hipGetLastError());
    }
    DBI_HIP(hipStreamSynchronize(s));
    *d_residues = h->synth_out.p;
    *d_prot_off = h->synth_off.p;
    *n_res = total;
    return 0;
}

namespace {
// dbi_count / dbi_count_buckets (d_hist: accumulate bucket counts there)
int count_impl(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_prot_off, uint64_t n_prot,
               uint64_t* d_hist, uint64_t* n_total, uint64_t* n_dropped) {
    if (!h || (!d_res && n_res) || !d_prot_off || !n_total) return set_error(DBI_E_INVALID, "NULL argument");
    int rc;
    if ((rc = begin_build(h, n_res, n_prot))) return rc;
    hipStream_t s = h->stream;
    const uint32_t nblk = (uint32_t)((n_res + DIGEST_TILE - 1) / DIGEST_TILE);
    if ((rc = h->poff.ensure(n_prot + 1)) || (rc = h->blk.ensure(std::max<uint32_t>(nblk, 1))) ||
        (rc = h->thr.ensure((size_t)nblk * DIGEST_THREADS + 1)) ||
        (rc = h->scan_tmp.ensure(std::max<size_t>(scan_u32_tmp_elems(nblk), h->scan_tmp.cap))))
        return rc;
    DBI_HIP(launch_off64_to_32(d_prot_off, h->poff.p, n_prot + 1, s));
    h->d_res = d_res;
    h->d_poff = h->poff.p;
    if (n_res) {
        if ((rc = prepare_tiles(h))) return rc;
        if (d_hist)
            STAGE(h, "digest_count", by(1, 0, 0, 4, 0),
                  launch_digest_count_hist(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff,
                                           (uint32_t)n_prot, (uint32_t)n_res, h->tile_pf.p, h->blk.p, h->thr.p,
                                           h->ctr.p, reinterpret_cast<unsigned long long*>(d_hist), s));
        else
            STAGE(h, "digest_count", by(1, 0, 0, 4, 0),
                  launch_digest_count(h->dp, h->mass_tab.p, h->flags_tab.p, h->d_res, h->d_poff, (uint32_t)n_prot,
                                      (uint32_t)n_res, h->tile_pf.p, h->blk.p, h->thr.p, h->ctr.p, s));
        DBI_HIP(launch_scan_u32(h->blk.p, h->blk.p, nblk, h->scan_tmp.p, h->scan_tmp.cap, &h->ctr.p->n_kept, s));
    }
    if ((rc = read_counters(h))) return rc;
    if (h->hc.err & ERR_PTM) return set_error(DBI_E_INVALID, ptm_device_msg());
    *n_total = h->hc.n_kept + h->hc.n_dropped;
    if (n_dropped) *n_dropped = h->hc.n_dropped;
    return 0;
}
}  // namespace

int dbi_count(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_prot_off, uint64_t n_prot,
              uint64_t* n_total, uint64_t* n_dropped) {
    return count_impl(h, d_res, n_res, d_prot_off, n_prot, nullptr, n_total, n_dropped);
}

int dbi_count_buckets(dbi_handle* h, const uint8_t* d_res, uint64_t n_res, const uint64_t* d_prot_off,
                      uint64_t n_prot, uint64_t* d_bucket_counts, uint64_t* n_total, uint64_t* n_dropped) {
    if (!h || !d_bucket_counts) return set_error(DBI_E_INVALID, "NULL argument");
    if (h->dp.nb < 1 || h->dp.nb > HIST_MAX_BUCKETS)
        return set_error(DBI_E_INVALID, "dbi_count_buckets: index_factor (NUM_BUCKETS) must be 1..64");
    return count_impl(h, d_res, n_res, d_prot_off, n_prot, d_bucket_counts, n_total, n_dropped);
}

}  // extern "C"
