// pk_probe.hip -- issue rate of packed vs scalar FP32 VALU ops on gfx950 (timing only).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
template <bool PK>
__global__ __launch_bounds__(256) void k(float *out, int iters) {
    f2v a[8];
    float s[16];
    for (int i = 0; i < 8; ++i) { a[i] = (f2v){(float)threadIdx.x + i, 1.f + i}; s[2 * i] = a[i].x; s[2 * i + 1] = a[i].y; }
    const f2v m = (f2v){0.999f, 1.001f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (PK) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(m));
            else {
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[2 * i]) : "v"(m.x));
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[2 * i + 1]) : "v"(m.y));
            }
        }
    }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += PK ? a[i].x + a[i].y : s[2 * i] + s[2 * i + 1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
int main() {
    float *o; hipMalloc(&o, 1024 * 256 * 16 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 4096, blocks = 256 * 16;  // 16 waves per CU... 4 per block -> 64 per CU total over time
    for (int pk = 0; pk < 2; ++pk)
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (pk) k<true><<<blocks, 256>>>(o, iters); else k<false><<<blocks, 256>>>(o, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const double fmas = (double)blocks * 256 * iters * 16;  // scalar FMA lanes
            printf("%s: %.3f ms  %.1f TFLOP/s fp32 (fma=2)\n", pk ? "v_pk_fma_f32" : "v_fma_f32   ", ms, fmas * 2 / ms / 1e9);
        }
    return 0;
}
