// fetch_calib.hip -- FETCH_SIZE calibration for the access widths the K5 match kernels use.
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it reports half the bytes);
// K5 reads 8-B postings, 64 lanes per wave (512 contiguous bytes per load instruction, from a bucket start that
// is 8-B but not line aligned). Each kernel below reads a known number of bytes once; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and divide the known bytes by FETCH_SIZE x 1 KiB: that is the factor for that width.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, size_t n, size_t shift, float *__restrict__ out) {
    // n elements from p + shift (shift in elements: a misaligned start), grid-stride, one pass
    float acc = 0.0f;
    const T *q = p + shift;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = q[i];
        acc += reinterpret_cast<const float *>(&v)[0];
    }
    if (acc == 123.456f) out[0] = acc;  // keeps the loads
}

// K5-like: each wave reads runs of 64 x 8 B starting at pseudo-random 8-B aligned positions
__global__ __launch_bounds__(256) void k_runs8(const uint2 *__restrict__ p, size_t n_words, int runs_per_wave,
                                               float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    float acc = 0.0f;
    uint32_t h = (uint32_t)wave * 2654435761u + 12345u;
    for (int r = 0; r < runs_per_wave; ++r) {
        h = h * 1664525u + 1013904223u;
        const size_t start = (size_t)(h % (uint32_t)(n_words - 64));
        const uint2 v = p[start + lane];
        acc += __uint_as_float(v.x);
    }
    if (acc == 123.456f) out[0] = acc;
}

int main() {
    const size_t bytes = (size_t)2 << 30;  // 2 GiB: far past the 256 MiB Infinity Cache
    void *buf = nullptr;
    float *out = nullptr;
    if (hipMalloc(&buf, bytes + 4096) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes + 4096);
    const dim3 g(8192), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<uint32_t>, g, b, 0, 0, (const uint32_t *)buf, bytes / 4, 0, out);
        hipLaunchKernelGGL(k_read<uint2>, g, b, 0, 0, (const uint2 *)buf, bytes / 8, 0, out);
        hipLaunchKernelGGL(k_read<uint4>, g, b, 0, 0, (const uint4 *)buf, bytes / 16, 0, out);
        hipLaunchKernelGGL(k_read<uint2>, g, b, 0, 0, (const uint2 *)buf, bytes / 8 - 8, 3, out);  // 24-B shifted
    }
    // runs: 8192 blocks x 4 waves x R runs x 512 B
    const int R = 128;
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(k_runs8, g, b, 0, 0, (const uint2 *)buf, bytes / 8, R, out);
    hipDeviceSynchronize();
    std::printf("{\"k_read_u32_bytes\": %zu, \"k_read_uint2_bytes\": %zu, \"k_read_uint4_bytes\": %zu, "
                "\"k_read_uint2_shifted_bytes\": %zu, \"k_runs8_bytes\": %zu}\n",
                bytes, bytes, bytes, bytes - 64, (size_t)8192 * 4 * R * 512);
    hipFree(buf);
    hipFree(out);
    return 0;
}
