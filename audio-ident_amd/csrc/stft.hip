// stft.hip -- K1 `stft_power`: framing + Hann window + 1024-point complex FFT +
// real split + |X|^2 (spec/FPSPEC.md 4), one wavefront per frame.
//
// Replaces the FFT stage inside the external `olaf_c` binary that the reference
// runs per call (audio-ident-service/app/audio/fingerprint.py:117-125 store,
// :185-193 query).
//
// Work mapping (gfx950, wave64):
//   * a workgroup = 4 waves; the 4 waves take 4 consecutive frames at a time so
//     their 75 %-overlapping PCM loads share the CU's L1 (HBM reads PCM ~once);
//   * lane l loads z[64*n1 + l] (n1 < 16) as float2: 512 contiguous bytes per
//     wave-instruction;
//   * stage A = 16-point DFT in registers, twiddle, LDS transpose (E1, row stride
//     68 float2: conflict-free for both the write and the strided read);
//   * stage B = 16-point DFT in registers, twiddle, quad exchange through LDS
//     (E2, lane stride 17 float2);
//   * stage C = radix-4 in registers, natural-order spill to LDS (E3, +1 pad per
//     32), then the real split reads Z[k] and Z[1024-k] (both conflict-free) and
//     stores 64 consecutive bins per wave-instruction.
// The exchanges are wave-private, so there is no workgroup barrier in the loop.
#include "aidfp_device.h"

namespace aid {

__device__ __forceinline__ int find_clip_by_frame(const ClipDesc *__restrict__ clips, int n_clips, int64_t g) {
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {  // last clip with frame_base <= g (wave-uniform: scalar loads)
        int mid = (lo + hi + 1) >> 1;
        if (clips[mid].frame_base <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <bool LOGMAG>
__global__ __launch_bounds__(256, 3) void k_stft_power(const float *__restrict__ pcm, const ClipDesc *__restrict__ clips,
                                                   int n_clips, int64_t total_frames, int hop,
                                                   const Tables *__restrict__ tab, float *__restrict__ out) {
    __shared__ float2 lds[kStftWaves][kStftLdsPerWave];
    __shared__ float2 s_win[1024], s_t2k[1024], s_t64[64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float2 *buf = lds[wave];
    const int kq = lane >> 2;  // stage B/C: k1
    const int mq = lane & 3;   // stage B: m2 ; stage C: s

    // window, T2K, T64 staged once per workgroup (LDS reads are 4x cheaper than L1 here)
    for (int i = threadIdx.x; i < 1024; i += 256) {
        s_win[i] = tab->win2[i];
        s_t2k[i] = tab->t2k[i];
    }
    if (threadIdx.x < 64) s_t64[threadIdx.x] = tab->t64[threadIdx.x];
    float2 twA[16], t16[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t16[i] = tab->t16[i];
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) twA[k1] = tab->t1k[lane * k1];
    __syncthreads();

    for (int f = 0; f < kStftFramesPerWave; ++f) {
        const int64_t g = (int64_t)blockIdx.x * kStftFramesPerBlock + f * kStftWaves + wave;
        if (g >= total_frames) break;  // wave-uniform
        const int c = find_clip_by_frame(clips, n_clips, g);
        const int64_t t = g - clips[c].frame_base;
        const float2 *src = reinterpret_cast<const float2 *>(pcm + clips[c].pcm_off + t * hop);

        float2 v[16];
#pragma unroll
        for (int n1 = 0; n1 < 16; ++n1) {
            const float2 x = src[64 * n1 + lane];
            const float2 w = s_win[64 * n1 + lane];
            v[n1] = make_float2(x.x * w.x, x.y * w.y);
        }
        // stage A: lane = n2
        dft16(v, t16);
        // T1K[n2*k1]; lane 0 multiplies by T1K[0] = (1,-0): value-identical (FPSPEC 4 note)
#pragma unroll
        for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], twA[k1]);
        // E1: A[k1][n2] -> lane (k1 = kq, m2 = mq) gets A[kq][4*m1 + mq]
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) buf[k1 * 68 + lane] = v[k1];
        wave_lds_sync();
#pragma unroll
        for (int m1 = 0; m1 < 16; ++m1) v[m1] = buf[kq * 68 + 4 * m1 + mq];
        wave_lds_sync();
        // stage B
        dft16(v, t16);
#pragma unroll
        for (int j1 = 1; j1 < 16; ++j1) v[j1] = cmul(v[j1], s_t64[mq * j1]);
        // E2: lane (kq, m2) writes B[kq][m2][j1]; reader lane (kq, s = mq) takes j1 = s + 4r
#pragma unroll
        for (int j1 = 0; j1 < 16; ++j1) buf[lane * 17 + j1] = v[j1];
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int m2 = 0; m2 < 4; ++m2) v[4 * r + m2] = buf[(4 * kq + m2) * 17 + mq + 4 * r];
        wave_lds_sync();
        // stage C: DFT4 over m2 -> Z[kq + 16*(mq + 4r) + 256*j2]; E3 natural order, pad 1 per 32
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            dft4(v[4 * r + 0], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
#pragma unroll
            for (int j2 = 0; j2 < 4; ++j2) {
                const int k = kq + 16 * (mq + 4 * r) + 256 * j2;
                buf[k + (k >> 5)] = v[4 * r + j2];
            }
        }
        wave_lds_sync();
        float *dst = out + g * kBins;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int k = lane + 64 * i;
            const int kk = (1024 - k) & 1023;
            const float2 p = buf[k + (k >> 5)];
            const float2 q = buf[kk + (kk >> 5)];
            const float2 o = make_float2(p.y + q.y, q.x - p.x);
            const float er = p.x + q.x, ei = p.y - q.y;
            const float2 tw = cmul(o, s_t2k[k]);
            const float xr = er + tw.x, xi = ei + tw.y;
            const float P = __builtin_fmaf(xr, xr, xi * xi) * 0.25f;
            if constexpr (LOGMAG) dst[k] = 10.0f * log10f(P + 1e-10f);
            else dst[k] = P;
        }
        wave_lds_sync();
    }
}

void launch_stft_power(const float *pcm, const ClipDesc *clips, int n_clips, int64_t total_frames, int hop,
                       const Tables *tab, float *out, bool logmag, hipStream_t s) {
    if (total_frames <= 0) return;
    const unsigned blocks = (unsigned)((total_frames + kStftFramesPerBlock - 1) / kStftFramesPerBlock);
    if (logmag)
        hipLaunchKernelGGL(k_stft_power<true>, dim3(blocks), dim3(256), 0, s, pcm, clips, n_clips, total_frames, hop, tab, out);
    else
        hipLaunchKernelGGL(k_stft_power<false>, dim3(blocks), dim3(256), 0, s, pcm, clips, n_clips, total_frames, hop, tab, out);
}

}  // namespace aid
