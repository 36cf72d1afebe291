// dedup.hip -- K7 `dedup_scan`: Chromaprint content-duplicate search on the GPU
// (SURVEY.md 8f row 4). Replaces the per-upload Python loop of the reference
// (audio-ident-service/app/audio/dedup.py:127-166 `_fingerprint_similarity`, :169-222
// `check_content_duplicate`): every catalog track within +-10 % of the query's duration is
// scored by bitwise Hamming agreement over the overlapping words, times the length ratio,
// and the best one (earliest on ties, strict >) wins.
//
// Exactness: the score is computed in binary64 with the reference's operation order,
// (matching / (min_len*32)) * (min_len / max_len), each op correctly rounded, so it equals
// the Python float bit for bit (tests/test_gpu_dedup.py vs tests/golden/ref_dedup.json).
//
// Layout: catalog words u32 concatenated (offsets i64[n+1]) + durations f64[n]; queries the
// same. Grid (query, chunk of 64 entries) with the query index fastest, so the workgroups in
// flight score the SAME catalog chunk for different queries and share it through L2; one wave
// per entry (coalesced 256-B reads, popcount, wave reduction).
#include "aidfp_device.h"

namespace aid {

constexpr int kDedupChunk = 64;

__device__ __forceinline__ double dedup_score(uint64_t matching, int64_t mn, int64_t mx) {
    return ((double)matching / (double)(mn * 32)) * ((double)mn / (double)mx);
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Hamming agreement of one (query, entry) pair by one wave
__device__ __forceinline__ double dedup_pair(const uint32_t *__restrict__ a, int64_t la, const uint32_t *__restrict__ b,
                                             int64_t lb, int lane) {
    const int64_t mn = min(la, lb), mx = max(la, lb);
    if (mn == 0) return 0.0;
    uint64_t diff = 0;
    for (int64_t i = lane; i < mn; i += 64) diff += __popc(a[i] ^ b[i]);
    diff = wave_sum(diff);
    return dedup_score((uint64_t)mn * 32 - diff, mn, mx);
}

__global__ __launch_bounds__(256) void k_dedup_scan(const uint32_t *__restrict__ cw, const int64_t *__restrict__ coff,
                                                    const double *__restrict__ cdur, int64_t n_cat,
                                                    const uint32_t *__restrict__ qw, const int64_t *__restrict__ qoff,
                                                    const double *__restrict__ qlo, const double *__restrict__ qhi,
                                                    int nq, double *__restrict__ part_sim, int64_t *__restrict__ part_idx,
                                                    int n_chunks) {
    __shared__ double s_sim[4];
    __shared__ int64_t s_idx[4];
    const int q = blockIdx.x, chunk = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double lo = qlo[q], hi = qhi[q];
    const uint32_t *a = qw + qoff[q];
    const int64_t la = qoff[q + 1] - qoff[q];
    double best = 0.0;
    int64_t bidx = -1;
    const int64_t e0 = (int64_t)chunk * kDedupChunk;
    for (int k = wave; k < kDedupChunk; k += 4) {  // entries in increasing order per wave
        const int64_t e = e0 + k;
        if (e >= n_cat) break;
        const double d = cdur[e];
        if (!(lo <= d && d <= hi)) continue;  // wave-uniform
        const double s = dedup_pair(a, la, cw + coff[e], coff[e + 1] - coff[e], lane);
        if (s > best) {
            best = s;
            bidx = e;
        }
    }
    if (lane == 0) {
        s_sim[wave] = best;
        s_idx[wave] = bidx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0;
        int64_t bi = -1;
        for (int w = 0; w < 4; ++w)  // max score, earliest entry on ties (a wave only keeps scores > 0)
            if (s_idx[w] >= 0 && (s_sim[w] > b || (s_sim[w] == b && s_idx[w] < bi))) {
                b = s_sim[w];
                bi = s_idx[w];
            }
        part_sim[(int64_t)q * n_chunks + chunk] = b;
        part_idx[(int64_t)q * n_chunks + chunk] = bi;
    }
}

__global__ __launch_bounds__(64) void k_dedup_final(const double *__restrict__ part_sim,
                                                    const int64_t *__restrict__ part_idx, int n_chunks,
                                                    double *__restrict__ best_sim, int64_t *__restrict__ best_idx) {
    const int q = blockIdx.x;
    if (threadIdx.x != 0) return;
    double b = 0.0;
    int64_t bi = -1;
    for (int c = 0; c < n_chunks; ++c) {  // chunks in catalog order: strict > keeps the earliest
        const double s = part_sim[(int64_t)q * n_chunks + c];
        if (part_idx[(int64_t)q * n_chunks + c] >= 0 && s > b) {
            b = s;
            bi = part_idx[(int64_t)q * n_chunks + c];
        }
    }
    best_sim[q] = b;
    best_idx[q] = bi;
}

__global__ __launch_bounds__(256) void k_dedup_pairs(const uint32_t *__restrict__ aw, const int64_t *__restrict__ aoff,
                                                     const uint32_t *__restrict__ bw, const int64_t *__restrict__ boff,
                                                     int n, double *__restrict__ sim) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (p >= n) return;
    const double s = dedup_pair(aw + aoff[p], aoff[p + 1] - aoff[p], bw + boff[p], boff[p + 1] - boff[p], lane);
    if (lane == 0) sim[p] = s;
}

int dedup_chunks(int64_t n_cat) { return (int)((n_cat + kDedupChunk - 1) / kDedupChunk); }

void launch_dedup_scan(const uint32_t *cw, const int64_t *coff, const double *cdur, int64_t n_cat, const uint32_t *qw,
                       const int64_t *qoff, const double *qlo, const double *qhi, int nq, double *part_sim,
                       int64_t *part_idx, double *best_sim, int64_t *best_idx, hipStream_t s) {
    if (nq <= 0) return;
    const int nc = dedup_chunks(n_cat);
    if (nc > 0)
        hipLaunchKernelGGL(k_dedup_scan, dim3((unsigned)nq, (unsigned)nc), dim3(256), 0, s, cw, coff, cdur, n_cat, qw,
                           qoff, qlo, qhi, nq, part_sim, part_idx, nc);
    hipLaunchKernelGGL(k_dedup_final, dim3((unsigned)nq), dim3(64), 0, s, part_sim, part_idx, nc, best_sim, best_idx);
}

void launch_dedup_pairs(const uint32_t *aw, const int64_t *aoff, const uint32_t *bw, const int64_t *boff, int n,
                        double *sim, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_dedup_pairs, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, aw, aoff, bw, boff, n, sim);
}

}  // namespace aid
