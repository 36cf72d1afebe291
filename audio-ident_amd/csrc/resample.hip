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

// The input of one launch: stream frames [b_base, b_base + b_n) at b + y * b_stride and, optionally, the frames
// [a_base, a_base + a_n) just before them at a + y * a_stride (y = stream of a batch), so a live stream's chunk is read
// where its caller left it and only the last few frames of the previous chunk are kept (StreamBank); 0 elsewhere
struct ResIn {
    const float *a;
    int64_t a_base, a_n, a_stride;
    const float *b;
    int64_t b_base, b_n, b_stride;
};

// Stage input samples lo .. lo + cnt - 1 (stream indices) into sx[0 .. cnt), downmixed at load time. The loads go out
// kStageBatch at a time before their LDS stores: a plain strided loop waits for each load before the next (its trip
// count is not known at compile time), so a block staging ~12 samples per thread paid ~12 serial memory latencies
#ifndef AID_K6_STAGE_BATCH
#define AID_K6_STAGE_BATCH 8
#endif
constexpr int kStageBatch = AID_K6_STAGE_BATCH;
template <bool STEREO>
__device__ __forceinline__ void stage_window(const ResIn &in, int64_t lo, int cnt, float *sx, int tid, int nthreads) {
    const int64_t y = blockIdx.y;
    const float *A = in.a + y * in.a_stride, *B = in.b + y * in.b_stride;
    // a window wholly inside part B whose 16-B words are all in it (B 16-B aligned): 16-B loads, two stereo frames or
    // four mono samples each. The hardware moved ~3.3 TB/s on 8-B lane loads of the 256-stream push (77 % of K6's
    // wave cycles waiting, every fetched byte needed) and 22 % more on 16-B ones (profiles/r06yz_k6_v4_ab.txt)
    constexpr int kPer = STEREO ? 2 : 4;  // stream samples per 16-B word
    const int64_t k0 = lo - in.b_base;
#if defined(AID_K6_NO_V4)  // diagnostic A/B build: 8-B / 4-B loads only
    if (false) {
#else
    if (k0 >= 0 && (k0 + cnt + kPer - 1) / kPer * kPer <= in.b_n && (reinterpret_cast<uintptr_t>(B) & 15) == 0) {
#endif
        const int64_t p0 = k0 / kPer;
        const int np = (int)((k0 + cnt - 1) / kPer - p0 + 1);
        const float4 *B4 = reinterpret_cast<const float4 *>(B);
        for (int i0 = tid; i0 < np; i0 += kStageBatch * nthreads) {
            float4 v[kStageBatch];
#pragma unroll
            for (int u = 0; u < kStageBatch; ++u) {
                const int i = i0 + u * nthreads;
                v[u] = i < np ? B4[p0 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < kStageBatch; ++u) {
                const int i = i0 + u * nthreads;
                if (i >= np) continue;
                const int f = (int)(kPer * (p0 + i) - k0);  // window index of the word's first sample
                if constexpr (STEREO) {
                    if (f >= 0) sx[f] = (v[u].x + v[u].y) * 0.5f;
                    if (f + 1 < cnt) sx[f + 1] = (v[u].z + v[u].w) * 0.5f;
                } else {
                    if (f >= 0) sx[f] = v[u].x;
                    if (f + 1 >= 0 && f + 1 < cnt) sx[f + 1] = v[u].y;
                    if (f + 2 >= 0 && f + 2 < cnt) sx[f + 2] = v[u].z;
                    if (f + 3 < cnt) sx[f + 3] = v[u].w;
                }
            }
        }
        return;
    }
    for (int i0 = tid; i0 < cnt; i0 += kStageBatch * nthreads) {
        float v[kStageBatch];
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) {
            const int i = i0 + u * nthreads;
            const int64_t g = lo + i;
            const float *p = nullptr;
            int64_t k = 0;
            if (i < cnt) {
                if (g >= in.b_base && g - in.b_base < in.b_n) {
                    p = B;
                    k = g - in.b_base;
                } else if (g >= in.a_base && g - in.a_base < in.a_n) {
                    p = A;
                    k = g - in.a_base;
                }
            }
            v[u] = 0.0f;
            if (p) {
                if constexpr (STEREO) {
                    const float2 s = reinterpret_cast<const float2 *>(p)[k];
                    v[u] = (s.x + s.y) * 0.5f;
                } else {
                    v[u] = p[k];
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
__global__ __launch_bounds__(kResThreads) void k_resample(ResIn in, int up, int down, int hl, int J,
                                                         const float *__restrict__ taps, float *__restrict__ dst,
                                                         int64_t m_first, int64_t m_end, int64_t dst_stride) {
    // Outputs m_first .. m_end-1 (stream indices) go to dst[m - m_first].
    // blockIdx.y = stream of a batch: its input as ResIn says, its output at dst + y * dst_stride (floats)
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
    stage_window<STEREO>(in, lo, cnt, sx, tid, kResThreads);
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

// Integer decimation (up == 1) with compile-time DOWN and J (48 kHz -> 16 kHz: 3, 61), register-blocked: a thread
// owns kDecR consecutive outputs, whose windows are one run of (kDecR - 1) * DOWN + J staged inputs; it reads that run
// from LDS once with 16-B loads into registers and runs the kDecR dot products from there: ~19 LDS dwords per output
// instead of J single-dword reads (MODE 2). Same fma chain per output (taps j = 0..J-1 in order), so the outputs are
// MODE 2's bit for bit. kDecR 4 (80 VGPRs, 6 waves per SIMD): 98 us per 256-stream push against MODE 2's 105 and
// kDecR 8's 155 (164 VGPRs, 3 waves per SIMD; profiles/r06p_k6_decimate_ab.txt): K6 is not bound by its LDS reads.
#ifndef AID_K6_DECR
#define AID_K6_DECR 4
#endif
constexpr int kDecR = AID_K6_DECR;
constexpr int kDecThreads = 256;

template <int DOWN, int J>
constexpr int dec_window() { return (kDecThreads * kDecR - 1) * DOWN + J; }

template <bool STEREO, int DOWN, int J>
__global__ __launch_bounds__(kDecThreads) void k_decimate(ResIn in, int hl, const float *__restrict__ taps,
                                                          float *__restrict__ dst, int64_t m_first, int64_t m_end,
                                                          int64_t dst_stride) {
    static_assert((kDecR * DOWN) % 4 == 0, "a thread's run must start 16-B aligned in LDS");
    constexpr int NX = (kDecR - 1) * DOWN + J;  // inputs of one thread's outputs
    constexpr int NX4 = (NX + 3) / 4;
    dst += (int64_t)blockIdx.y * dst_stride;
    extern __shared__ float sx[];  // dec_window() + 4 floats (the last run's 16-B over-read)
    const int tid = threadIdx.x;
    const int64_t m0 = m_first + (int64_t)blockIdx.x * (kDecThreads * kDecR);
    const int64_t mlast = min(m0 + kDecThreads * kDecR - 1, m_end - 1);
    const int64_t lo = m0 * DOWN + hl - (J - 1);
    const int cnt = (int)(mlast * DOWN + hl - lo + 1);
    stage_window<STEREO>(in, lo, cnt, sx, tid, kDecThreads);
    __syncthreads();
    const int64_t mb = m0 + (int64_t)tid * kDecR;
    if (mb >= m_end) return;
    // output mb + r reads sx[tid * kDecR * DOWN + r * DOWN + J - 1 - j]; words past cnt only feed outputs >= m_end
    float x[NX4 * 4];
    const float4 *p = reinterpret_cast<const float4 *>(sx + tid * kDecR * DOWN);
#pragma unroll
    for (int i = 0; i < NX4; ++i) {
        const float4 v = p[i];
        x[4 * i] = v.x;
        x[4 * i + 1] = v.y;
        x[4 * i + 2] = v.z;
        x[4 * i + 3] = v.w;
    }
    float acc[kDecR];
#pragma unroll
    for (int r = 0; r < kDecR; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const float t = taps[j];  // uniform
#pragma unroll
        for (int r = 0; r < kDecR; ++r) acc[r] = __builtin_fmaf(t, x[r * DOWN + J - 1 - j], acc[r]);
    }
    float *o = dst + (mb - m_first);
    if (mb + kDecR <= m_end && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
#pragma unroll
        for (int r = 0; r < kDecR; r += 4)
            *reinterpret_cast<float4 *>(o + r) = make_float4(acc[r], acc[r + 1], acc[r + 2], acc[r + 3]);
    } else {
#pragma unroll
        for (int r = 0; r < kDecR; ++r)
            if (mb + r < m_end) o[r] = acc[r];
    }
}

// MODE 3 (up > 1, the default): phase-major. Outputs m and m + up share a phase, so a thread
// owns one phase of the block and kResR outputs up apart: it loads its phase's taps once per
// 8-tap chunk (L1-resident table) and runs kResR dot products with them. Per output that is
// J input reads from LDS (+ J / kResR tap loads) instead of 2J LDS reads with per-lane phase
// rows (which also bank-conflicted). Same fma chain per output (taps j = 0..J-1 in order).
constexpr int kResR = 16;  // outputs per thread (one phase)

template <bool STEREO>
__global__ __launch_bounds__(256) void k_resample_phase(ResIn in, int up, int down, int hl, int J,
                                                       const float *__restrict__ taps, float *__restrict__ dst,
                                                       int64_t m_first, int64_t m_end, int64_t dst_stride) {
    dst += (int64_t)blockIdx.y * dst_stride;  // stream of a batch (k_resample)
    extern __shared__ float sx[];
    const int tid = threadIdx.x;
    const int64_t m0 = m_first + (int64_t)blockIdx.x * up * kResR;
    const int64_t mlast = min(m0 + (int64_t)up * kResR - 1, m_end - 1);
    const int64_t lo = (m0 * down + hl) / up - (J - 1);
    const int64_t hi = (mlast * down + hl) / up;  // inclusive
    const int cnt = (int)(hi - lo + 1);
    stage_window<STEREO>(in, lo, cnt, sx, tid, (int)blockDim.x);
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
// n_streams single launches (same staging, same fma chain per output). With hist_n > 0 the input is two parts:
// stream frames [in_base - hist_n, in_base) from hist (hist_stride per stream), then [in_base, in_base + n) from src.
void launch_resample(const float *src, int64_t in_base, int64_t n, int channels, int up, int down, int hl, int J,
                     const float *taps, float *dst, int64_t m_first, int64_t count, hipStream_t s, int n_streams,
                     int64_t src_stride, int64_t dst_stride, const float *hist, int64_t hist_n, int64_t hist_stride) {
    if (count <= 0 || n_streams <= 0) return;
    const ResIn in{hist_n > 0 ? hist : src, in_base - hist_n, hist_n, hist_stride, src, in_base, n, src_stride};
    if (use_phase(up, down, J)) {
        const int64_t per = (int64_t)up * kResR;
        const dim3 g((unsigned)((count + per - 1) / per), (unsigned)n_streams), b((unsigned)std::min(256, (up + 63) / 64 * 64));
        const size_t lds = (size_t)resample_lds_floats(up, down, J) * sizeof(float);
        if (channels == 2)
            hipLaunchKernelGGL((k_resample_phase<true>), g, b, lds, s, in, up, down, hl, J, taps, dst, m_first,
                               m_first + count, dst_stride);
        else
            hipLaunchKernelGGL((k_resample_phase<false>), g, b, lds, s, in, up, down, hl, J, taps, dst, m_first,
                               m_first + count, dst_stride);
        return;
    }
    const int64_t m_end = m_first + count;
#ifndef AID_K6_NO_DEC  // diagnostic builds: MODE 2 for every decimation (A/B)
    if (up == 1 && down == 3 && J == 61) {  // 48 kHz -> 16 kHz (browser capture -> the index rate)
        const dim3 g((unsigned)((count + kDecThreads * kDecR - 1) / (kDecThreads * kDecR)), (unsigned)n_streams);
        const size_t lds = (size_t)(dec_window<3, 61>() + 4) * sizeof(float);
        if (channels == 2)
            hipLaunchKernelGGL((k_decimate<true, 3, 61>), g, dim3(kDecThreads), lds, s, in, hl, taps, dst, m_first,
                               m_end, dst_stride);
        else
            hipLaunchKernelGGL((k_decimate<false, 3, 61>), g, dim3(kDecThreads), lds, s, in, hl, taps, dst, m_first,
                               m_end, dst_stride);
        return;
    }
#endif
    const dim3 g((unsigned)((count + kResBlock - 1) / kResBlock), (unsigned)n_streams), b(kResThreads);
    const size_t lds = (size_t)resample_lds_floats(up, down, J) * sizeof(float);
    const int mode = up == 1 ? 2 : taps_in_lds(up, J) ? 1 : 0;
#define AID_RS_LAUNCH(ST, MD) \
    hipLaunchKernelGGL((k_resample<ST, MD>), g, b, lds, s, in, up, down, hl, J, taps, dst, m_first, m_end, dst_stride)
    if (channels == 2) {
        if (mode == 2) AID_RS_LAUNCH(true, 2); else if (mode == 1) AID_RS_LAUNCH(true, 1); else AID_RS_LAUNCH(true, 0);
    } else {
        if (mode == 2) AID_RS_LAUNCH(false, 2); else if (mode == 1) AID_RS_LAUNCH(false, 1); else AID_RS_LAUNCH(false, 0);
    }
#undef AID_RS_LAUNCH
}

}  // namespace aid
