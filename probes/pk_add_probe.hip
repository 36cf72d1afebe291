// pk_add_probe.hip -- issue rate of v_pk_add_f32 / v_pk_mul_f32 (incl. op_sel/neg forms) vs two v_add_f32 on gfx950 (timing only).
// build: hipcc --offload-arch=gfx950 -O3 probes/pk_add_probe.hip -o probes/pk_add_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, int iters) {
    f2v a[8];
    float s[16];
    for (int i = 0; i < 8; ++i) { a[i] = (f2v){(float)threadIdx.x + i, 1.f + i}; s[2 * i] = a[i].x; s[2 * i + 1] = a[i].y; }
    const f2v m = (f2v){0.999f, 1.001f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            else if (MODE == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            else if (MODE == 3) asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "+v"(a[i]) : "v"(m));
            else {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[2 * i]) : "v"(m.x));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[2 * i + 1]) : "v"(m.y));
            }
        }
    }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += MODE ? a[i].x + a[i].y : s[2 * i] + s[2 * i + 1];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
int main() {
    float *o; hipMalloc(&o, 1024 * 256 * 16 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 4096, blocks = 256 * 16;
    const char *names[4] = {"v_add_f32 x2", "v_pk_add_f32", "v_pk_mul_f32", "v_pk_add_f32 opsel"};
    for (int mode = 0; mode < 4; ++mode)
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (mode == 0) k<0><<<blocks, 256>>>(o, iters);
            else if (mode == 1) k<1><<<blocks, 256>>>(o, iters);
            else if (mode == 2) k<2><<<blocks, 256>>>(o, iters);
            else k<3><<<blocks, 256>>>(o, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            const double ops = (double)blocks * 256 * iters * 16;
            printf("%s: %.3f ms  %.1f Gop/s fp32\n", names[mode], ms, ops / ms / 1e6);
        }
    return 0;
}
