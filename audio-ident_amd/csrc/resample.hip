// resample.hip -- K6 `resample`: stereo downmix + rational polyphase resampling (FPSPEC 8),
// the GPU replacement of ffmpeg's `-ac 1 -ar <rate>` in the reference
// (audio-ident-service/app/audio/decode.py:41-60).
//
// A workgroup produces kResBlock consecutive outputs (4 per thread, strided by 256 so each
// store instruction writes 1 KB contiguous). It stages the input window those outputs touch
// ONCE into LDS, downmixed to mono at staging time (float2 loads for stereo), zero outside the
// clip; every output then runs its J-tap dot product from LDS with the phase row of the
// [up][J] tap table (L1/L2-resident, a few KB to 54 KB). HBM traffic is the algorithmic
// minimum: input once (+ the J-sample window overlap per block) and output once.
#include "aidfp_device.h"

namespace aid {

constexpr int kResThreads = 256;
constexpr int kResPerThread = 4;
constexpr int kResBlock = kResThreads * kResPerThread;

template <bool STEREO>
__global__ __launch_bounds__(kResThreads) void k_resample(const float *__restrict__ src, int64_t in_base, int64_t n,
                                                         int up, int down, int hl, int J,
                                                         const float *__restrict__ taps, float *__restrict__ dst,
                                                         int64_t m_first, int64_t m_end) {
    // src[0] is stream sample in_base; samples outside [in_base, in_base + n) read as 0.
    // Outputs m_first .. m_end-1 (stream indices) go to dst[m - m_first].
    extern __shared__ float sx[];
    const int tid = threadIdx.x;
    const int64_t m0 = m_first + (int64_t)blockIdx.x * kResBlock;
    const int64_t mlast = min(m0 + kResBlock - 1, m_end - 1);
    const int64_t lo = (m0 * down + hl) / up - (J - 1);
    const int64_t hi = (mlast * down + hl) / up;  // inclusive
    const int cnt = (int)(hi - lo + 1);
    for (int i = tid; i < cnt; i += kResThreads) {
        const int64_t g = lo + i - in_base;
        float v = 0.0f;
        if (g >= 0 && g < n) {
            if constexpr (STEREO) {
                const float2 s = reinterpret_cast<const float2 *>(src)[g];
                v = (s.x + s.y) * 0.5f;
            } else {
                v = src[g];
            }
        }
        sx[i] = v;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kResPerThread; ++r) {
        const int64_t m = m0 + tid + r * kResThreads;
        if (m >= m_end) break;
        const int64_t c = m * down + hl;
        const int p = (int)(c % up);
        const float *tp = taps + (int64_t)p * J;
        const float *xp = sx + (c / up - lo);
        float acc = 0.0f;
        for (int j = 0; j < J; ++j) acc = __builtin_fmaf(tp[j], xp[-j], acc);
        dst[m - m_first] = acc;
    }
}

int64_t resample_lds_floats(int up, int down, int J) {
    return (int64_t)(kResBlock - 1) * down / up + J + 2;
}

void launch_resample(const float *src, int64_t in_base, int64_t n, int channels, int up, int down, int hl, int J,
                     const float *taps, float *dst, int64_t m_first, int64_t count, hipStream_t s) {
    if (count <= 0) return;
    const dim3 g((unsigned)((count + kResBlock - 1) / kResBlock)), b(kResThreads);
    const size_t lds = (size_t)resample_lds_floats(up, down, J) * sizeof(float);
    const int64_t m_end = m_first + count;
    if (channels == 2)
        hipLaunchKernelGGL(k_resample<true>, g, b, lds, s, src, in_base, n, up, down, hl, J, taps, dst, m_first, m_end);
    else
        hipLaunchKernelGGL(k_resample<false>, g, b, lds, s, src, in_base, n, up, down, hl, J, taps, dst, m_first,
                           m_end);
}

}  // namespace aid
