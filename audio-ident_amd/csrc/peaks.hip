// peaks.hip -- K2 `peak_pick`: 2-D local-maximum constellation (FPSPEC 5) with
// the tie rule "earliest (t,k) wins", emitted as a per-frame 1024-bit mask.
//
// Replaces the spectral-peak stage inside the external `olaf_c` binary
// (reference call sites fingerprint.py:117-125, 185-193).
//
// One workgroup streams one strip of kPeakStrip output frames of one clip and
// reads every power row of the strip (+7 halo rows each side) exactly once:
//   * thread j owns bins 4j..4j+3 (one float4 load per row, prefetched one row
//     ahead);
//   * the row is staged in LDS (double-buffered, one barrier per row) and each
//     thread reads its +-15-bin neighbours with 9 ds_read_b128;
//   * the vertical +-7-frame part is register-resident: `before` is complete when a
//     row arrives (the previous 7 rows' row-max live in an 8-slot register ring),
//     `after` is an accumulator that the next 7 rows max into; ring slots are
//     compile-time because the row loop is unrolled by 8;
//   * a decided row's 4-bit nibbles are OR-reduced over 16 lanes into one
//     natural-order 64-bit mask word (word w = bins 64w..64w+63).
// Strips are dealt to workgroups XCD-aware so neighbouring strips (which share
// halo rows) run on the same XCD's L2.
#include "aidfp_device.h"

namespace aid {

__device__ __forceinline__ uint64_t or16(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
        lo |= __shfl_xor(lo, m);
        hi |= __shfl_xor(hi, m);
    }
    return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void k_peak_pick(const float *__restrict__ power, const ClipDesc *__restrict__ clips,
                                                  int n_clips, int64_t total_strips, float thr,
                                                  uint64_t *__restrict__ mask) {
    __shared__ __attribute__((aligned(16))) float row[2][kBins + 32];
    const int tid = threadIdx.x;

    // XCD-aware deal: consecutive strips -> blocks b, b+8, b+16 ... (one XCD's L2)
    int64_t strip;
    {
        const int64_t nb = gridDim.x, b = blockIdx.x;
        const int64_t per = nb / 8, rem = nb % 8, x = b % 8, y = b / 8;
        strip = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + y;
    }
    if (strip >= total_strips) return;
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].strip_base <= strip) lo = mid; else hi = mid - 1;
    }
    const int64_t F = clips[lo].frames;
    const int64_t fb = clips[lo].frame_base;
    const int64_t t0 = (strip - clips[lo].strip_base) * kPeakStrip;
    const int64_t t1 = min(t0 + (int64_t)kPeakStrip, F);
    const float *P = power + fb * kBins;
    uint64_t *M = mask + fb * kMaskWords;

    if (tid < 16) {
        row[0][tid] = 0.f; row[0][kBins + 16 + tid] = 0.f;
        row[1][tid] = 0.f; row[1][kBins + 16 + tid] = 0.f;
    }

    float fh[8][4];    // row-max (Full) of recent rows, slot = iteration & 7
    float pend[8][4];  // candidate power of pending rows (-1 = not a candidate)
    float acc[8][4];   // running `after` max of pending rows
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) { fh[s][i] = 0.f; pend[s][i] = -1.f; acc[s][i] = 0.f; }

    // iteration it processes row r = t0 - 7 + it and decides row r - 7
    const int64_t rbeg = t0 - kPeakDT;
    const int iters = (int)(t1 - t0) + 2 * kPeakDT;
    float4 nxt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rbeg >= 0 && rbeg < F) nxt = reinterpret_cast<const float4 *>(P + rbeg * kBins)[tid];

    for (int base = 0; base < iters; base += 8) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int it = base + s;
            if (it < iters) {  // workgroup-uniform
                const int64_t r = rbeg + it;
                const float4 cur = nxt;
                {
                    const int64_t rn = r + 1;
                    nxt = (it + 1 < iters && rn >= 0 && rn < F) ? reinterpret_cast<const float4 *>(P + rn * kBins)[tid]
                                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                float *rb = row[it & 1];
                reinterpret_cast<float4 *>(rb + 16)[tid] = cur;
                __syncthreads();
                float q[36];  // bins 4j-16 .. 4j+19 (zero outside the frame)
#pragma unroll
                for (int v = 0; v < 9; ++v) {
                    const float4 w = reinterpret_cast<const float4 *>(rb)[tid + v];
                    q[4 * v + 0] = w.x; q[4 * v + 1] = w.y; q[4 * v + 2] = w.z; q[4 * v + 3] = w.w;
                }
                // own bin i is q[16+i]; left window q[1+i..15+i], right window q[17+i..31+i]
                float midL = q[4], midR = q[20];
#pragma unroll
                for (int u = 5; u <= 15; ++u) midL = fmaxf(midL, q[u]);
#pragma unroll
                for (int u = 21; u <= 31; ++u) midR = fmaxf(midR, q[u]);
                float L[4], R[4];
                L[0] = fmaxf(fmaxf(q[1], q[2]), fmaxf(q[3], midL));
                L[1] = fmaxf(fmaxf(q[2], q[3]), fmaxf(midL, q[16]));
                L[2] = fmaxf(fmaxf(q[3], midL), fmaxf(q[16], q[17]));
                L[3] = fmaxf(fmaxf(midL, q[16]), fmaxf(q[17], q[18]));
                R[0] = fmaxf(fmaxf(q[17], q[18]), fmaxf(q[19], midR));
                R[1] = fmaxf(fmaxf(q[18], q[19]), fmaxf(midR, q[32]));
                R[2] = fmaxf(fmaxf(q[19], midR), fmaxf(q[32], q[33]));
                R[3] = fmaxf(fmaxf(midR, q[32]), fmaxf(q[33], q[34]));

                const bool in_out = (r >= t0) && (r < t1);
                uint32_t nib = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = q[16 + i];
                    const float fm = fmaxf(fmaxf(L[i], p), R[i]);
                    float bf = L[i];
#pragma unroll
                    for (int d = 1; d <= 7; ++d) bf = fmaxf(bf, fh[(s - d) & 7][i]);
                    const bool cand = in_out && (4 * tid + i) >= 1 && p > thr && p > bf;
#pragma unroll
                    for (int d = 1; d <= 7; ++d) acc[(s - d) & 7][i] = fmaxf(acc[(s - d) & 7][i], fm);
                    // row r-7 (slot s-7 == s+1) now has its complete `after`
                    if (pend[(s + 1) & 7][i] >= acc[(s + 1) & 7][i]) nib |= 1u << i;
                    fh[s][i] = fm;
                    pend[s][i] = cand ? p : -1.f;
                    acc[s][i] = R[i];
                }
                const int64_t rd = r - kPeakDT;
                const uint64_t word = or16((uint64_t)nib << (4 * (tid & 15)));
                if (rd >= t0 && rd < t1 && (tid & 15) == 0) M[rd * kMaskWords + (tid >> 4)] = word;
            }
        }
    }
}

void launch_peak_pick(const float *power, const ClipDesc *clips, int n_clips, int64_t total_strips, float thr,
                      uint64_t *mask, hipStream_t s) {
    if (total_strips <= 0) return;
    hipLaunchKernelGGL(k_peak_pick, dim3((unsigned)total_strips), dim3(256), 0, s, power, clips, n_clips, total_strips,
                       thr, mask);
}

}  // namespace aid
