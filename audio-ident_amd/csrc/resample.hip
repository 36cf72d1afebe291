// resample.hip -- K6 `resample`: stereo downmix + rational polyphase resampling (FPSPEC 8),
// the GPU replacement of ffmpeg's `-ac 1 -ar <rate>` in the reference
// (audio-ident-service/app/audio/decode.py:41-60).
//
// A workgroup produces kResBlock consecutive outputs (4 per thread, strided by 256 so each
// store instruction writes 1 KB contiguous). It stages the input window those outputs touch
// ONCE into LDS, downmixed to mono at staging time (float2 loads for stereo), zero outside the
// clip; every output then runs its J-tap dot product from LDS with the phase row of the
// [up][J] tap table, itself staged in LDS when it fits 48 KB (else read from L1/L2). HBM traffic is the algorithmic
// minimum: input once (+ the J-sample window overlap per block) and output once.
#include "aidfp_device.h"

namespace aid {

constexpr int kResThreads = 256;
constexpr int kResPerThread = 4;
constexpr int kResBlock = kResThreads * kResPerThread;

constexpr int kResMaxLdsTaps = 12288;  // floats (48 KB): larger tables are read from L1/L2

// Stage input samples lo .. lo + cnt - 1 (stream indices; src[0] is stream sample in_base, 0 outside [0, n)) into
// sx[0 .. cnt), downmixed at load time. The loads go out kStageBatch at a time before their LDS stores: a plain
// strided loop waits for each load before the next (its trip count is not known at compile time), so a block
// staging ~12 samples per thread paid ~12 serial memory latencies (K6 at ~2.5 TB/s on the 256-stream push)
constexpr int kStageBatch = 8;
template <bool STEREO>
__device__ __forceinline__ void stage_window(const float *__restrict__ src, int64_t lo, int64_t in_base, int64_t n,
                                             int cnt, float *sx, int tid, int nthreads) {
    for (int i0 = tid; i0 < cnt; i0 += kStageBatch * nthreads) {
        float v[kStageBatch];
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) {
            const int i = i0 + u * nthreads;
            const int64_t g = lo + i - in_base;
            v[u] = 0.0f;
            if (i < cnt && g >= 0 && g < n) {
                if constexpr (STEREO) {
                    const float2 s = reinterpret_cast<const float2 *>(src)[g];
                    v[u] = (s.x + s.y) * 0.5f;
                } else {
                    v[u] = src[g];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u)
            if (i0 + u * nthreads < cnt) sx[i0 + u * nthreads] = v[u];
    }
}

// MODE 0: taps from L1/L2, 1: taps staged in LDS, 2: integer decimation (up == 1): one phase,
// the taps are wave-uniform and read as scalar loads (no LDS traffic for them)
template <bool STEREO, int MODE>
__global__ __launch_bounds__(kResThreads) void k_resample(const float *__restrict__ src, int64_t in_base, int64_t n,
                                                         int up, int down, int hl, int J,
                                                         const float *__restrict__ taps, float *__restrict__ dst,
                                                         int64_t m_first, int64_t m_end, int64_t src_stride,
                                                         int64_t dst_stride) {
    // src[0] is stream sample in_base; samples outside [in_base, in_base + n) read as 0.
    // Outputs m_first .. m_end-1 (stream indices) go to dst[m - m_first].
    // blockIdx.y = stream of a batch: its input at src + y * src_stride, its output at dst + y * dst_stride (floats)
    src += (int64_t)blockIdx.y * src_stride;
    dst += (int64_t)blockIdx.y * dst_stride;
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    // [up][J] tap table first (when it fits), then the input window
    constexpr bool LDS_TAPS = MODE == 1;
    float *sx = LDS_TAPS ? smem + ((up * J + 3) & ~3) : smem;
    if constexpr (LDS_TAPS) {
        for (int i = tid; i < up * J; i += kResThreads) smem[i] = taps[i];
    }
    const int64_t m0 = m_first + (int64_t)blockIdx.x * kResBlock;
    const int64_t mlast = min(m0 + kResBlock - 1, m_end - 1);
    const int64_t lo = (m0 * down + hl) / up - (J - 1);
    const int64_t hi = (mlast * down + hl) / up;  // inclusive
    const int cnt = (int)(hi - lo + 1);
    stage_window<STEREO>(src, lo, in_base, n, cnt, sx, tid, kResThreads);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kResPerThread; ++r) {
        const int64_t m = m0 + tid + r * kResThreads;
        if (m >= m_end) break;
        const int64_t c = m * down + hl;
        float acc = 0.0f;
        if constexpr (MODE == 2) {
            const float *xp = sx + (c - lo);
            for (int j = 0; j < J; ++j) acc = __builtin_fmaf(taps[j], xp[-j], acc);  // taps[j]: uniform
        } else {
            const int p = (int)(c % up);
            const float *tp = (LDS_TAPS ? smem : taps) + (int64_t)p * J;
            const float *xp = sx + (c / up - lo);
            for (int j = 0; j < J; ++j) acc = __builtin_fmaf(tp[j], xp[-j], acc);
        }
        dst[m - m_first] = acc;
    }
}

// MODE 3 (up > 1, the default): phase-major. Outputs m and m + up share a phase, so a thread
// owns one phase of the block and kResR outputs up apart: it loads its phase's taps once per
// 8-tap chunk (L1-resident table) and runs kResR dot products with them. Per output that is
// J input reads from LDS (+ J / kResR tap loads) instead of 2J LDS reads with per-lane phase
// rows (which also bank-conflicted). Same fma chain per output (taps j = 0..J-1 in order).
constexpr int kResR = 16;  // outputs per thread (one phase)

template <bool STEREO>
__global__ __launch_bounds__(256) void k_resample_phase(const float *__restrict__ src, int64_t in_base, int64_t n,
                                                       int up, int down, int hl, int J,
                                                       const float *__restrict__ taps, float *__restrict__ dst,
                                                       int64_t m_first, int64_t m_end, int64_t src_stride,
                                                       int64_t dst_stride) {
    src += (int64_t)blockIdx.y * src_stride;  // stream of a batch (k_resample)
    dst += (int64_t)blockIdx.y * dst_stride;
    extern __shared__ float sx[];
    const int tid = threadIdx.x;
    const int64_t m0 = m_first + (int64_t)blockIdx.x * up * kResR;
    const int64_t mlast = min(m0 + (int64_t)up * kResR - 1, m_end - 1);
    const int64_t lo = (m0 * down + hl) / up - (J - 1);
    const int64_t hi = (mlast * down + hl) / up;  // inclusive
    const int cnt = (int)(hi - lo + 1);
    stage_window<STEREO>(src, lo, in_base, n, cnt, sx, tid, (int)blockDim.x);
    __syncthreads();
    for (int t = tid; t < up; t += blockDim.x) {
        const int64_t c0 = (m0 + t) * down + hl;  // output r: c = c0 + r * up * down
        const int p = (int)(c0 % up);
        const int b0 = (int)(c0 / up - lo);       // its input index: b0 + r * down - j
        const float *tp = taps + (int64_t)p * J;
        float acc[kResR];
#pragma unroll
        for (int r = 0; r < kResR; ++r) acc[r] = 0.0f;
        for (int jb = 0; jb < J; jb += 8) {
            float tv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) tv[u] = jb + u < J ? tp[jb + u] : 0.0f;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (jb + u >= J) break;  // uniform
#pragma unroll
                for (int r = 0; r < kResR; ++r) acc[r] = __builtin_fmaf(tv[u], sx[b0 + r * down - (jb + u)], acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < kResR; ++r) {
            const int64_t m = m0 + t + (int64_t)r * up;
            if (m < m_end) dst[m - m_first] = acc[r];
        }
    }
}

// phase-major blocks hold up * kResR outputs: used while that window stays small (common rate
// pairs: up = 147, 160, 441); very large up (near-coprime rates) keep the 1024-output blocks
static bool use_phase(int up, int down, int J) {
    return up > 1 && up <= 1024 && ((int64_t)up * kResR - 1) * down / up + J + 2 <= 12288;
}

static int64_t window_floats(int up, int down, int J) {
    if (use_phase(up, down, J)) return ((int64_t)up * kResR - 1) * down / up + J + 2;
    return (int64_t)(kResBlock - 1) * down / up + J + 2;
}

static bool taps_in_lds(int up, int J) { return up > 1 && (int64_t)up * J <= kResMaxLdsTaps; }

int64_t resample_lds_floats(int up, int down, int J) {
    if (use_phase(up, down, J)) return window_floats(up, down, J);
    return window_floats(up, down, J) + (taps_in_lds(up, J) ? (((int64_t)up * J + 3) & ~3) : 0);
}

// n_streams > 1: the same output range of n_streams streams in one launch (grid.y = stream), each stream's input
// src_stride floats after the previous one's and its output dst_stride floats after; bit for bit the outputs of
// n_streams single launches (same staging, same fma chain per output)
void launch_resample(const float *src, int64_t in_base, int64_t n, int channels, int up, int down, int hl, int J,
                     const float *taps, float *dst, int64_t m_first, int64_t count, hipStream_t s, int n_streams,
                     int64_t src_stride, int64_t dst_stride) {
    if (count <= 0 || n_streams <= 0) return;
    if (use_phase(up, down, J)) {
        const int64_t per = (int64_t)up * kResR;
        const dim3 g((unsigned)((count + per - 1) / per), (unsigned)n_streams), b((unsigned)std::min(256, (up + 63) / 64 * 64));
        const size_t lds = (size_t)resample_lds_floats(up, down, J) * sizeof(float);
        if (channels == 2)
            hipLaunchKernelGGL((k_resample_phase<true>), g, b, lds, s, src, in_base, n, up, down, hl, J, taps, dst,
                               m_first, m_first + count, src_stride, dst_stride);
        else
            hipLaunchKernelGGL((k_resample_phase<false>), g, b, lds, s, src, in_base, n, up, down, hl, J, taps, dst,
                               m_first, m_first + count, src_stride, dst_stride);
        return;
    }
    const dim3 g((unsigned)((count + kResBlock - 1) / kResBlock), (unsigned)n_streams), b(kResThreads);
    const size_t lds = (size_t)resample_lds_floats(up, down, J) * sizeof(float);
    const int64_t m_end = m_first + count;
    const int mode = up == 1 ? 2 : taps_in_lds(up, J) ? 1 : 0;
#define AID_RS_LAUNCH(ST, MD) \
    hipLaunchKernelGGL((k_resample<ST, MD>), g, b, lds, s, src, in_base, n, up, down, hl, J, taps, dst, m_first, m_end, \
                       src_stride, dst_stride)
    if (channels == 2) {
        if (mode == 2) AID_RS_LAUNCH(true, 2); else if (mode == 1) AID_RS_LAUNCH(true, 1); else AID_RS_LAUNCH(true, 0);
    } else {
        if (mode == 2) AID_RS_LAUNCH(false, 2); else if (mode == 1) AID_RS_LAUNCH(false, 1); else AID_RS_LAUNCH(false, 0);
    }
#undef AID_RS_LAUNCH
}

}  // namespace aid
