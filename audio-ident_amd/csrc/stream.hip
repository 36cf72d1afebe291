// stream.hip -- stereo -> mono downmix for the streaming path (BASELINE config 5).
// Replaces the ffmpeg `-ac 1` downmix of the reference's decode step
// (audio-ident-service/app/audio/decode.py:50-51) for interleaved f32 stereo:
// m[i] = (L[i] + R[i]) * 0.5f (two correctly rounded binary32 ops; the *0.5 is exact).
// HBM-bound: 8 B in + 4 B out per sample frame, float4 loads / float2 stores.
#include "aidfp_device.h"

namespace aid {

__global__ __launch_bounds__(256) void k_downmix(const float4 *__restrict__ in, int64_t n_pairs2, float2 *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pairs2; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];  // L0 R0 L1 R1
        out[i] = make_float2((v.x + v.y) * 0.5f, (v.z + v.w) * 0.5f);
    }
}

__global__ void k_downmix_tail(const float *__restrict__ in, int64_t first, int64_t n, float *__restrict__ out) {
    const int64_t i = first + threadIdx.x;
    if (i < n) out[i] = (in[2 * i] + in[2 * i + 1]) * 0.5f;
}

void launch_downmix(const float *in, int64_t n, float *out, hipStream_t s) {
    if (n <= 0) return;
    const int64_t n2 = n / 2;
    if (n2 > 0) {
        const int64_t blocks = std::min<int64_t>((n2 + 255) / 256, 4096);
        hipLaunchKernelGGL(k_downmix, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<const float4 *>(in), n2,
                           reinterpret_cast<float2 *>(out));
    }
    if (n & 1) hipLaunchKernelGGL(k_downmix_tail, dim3(1), dim3(64), 0, s, in, 2 * n2, n, out);
}

}  // namespace aid
