// aidfp_device.h -- device-side arithmetic of spec/FPSPEC.md for gfx950.
//
// Every expression here is the binary32 op sequence FPSPEC 3-4 pins; the build
// uses -ffp-contract=off so hipcc emits exactly one v_mul/v_add/v_fma per op.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aidfp_layout.h"

namespace aid {

// Launch-attached timing (hipExtLaunchKernel): the engine's profiler hands the next launch on this
// thread a start/stop event pair, and the runtime stamps them from the dispatch packet itself. No
// marker packets go between the extraction kernels, so K1 -> K2 -> K3 run back to back while timed
// (hipEventRecord markers cost ~5 us each plus a cache release between every pair of kernels).
struct LaunchTiming {
    hipEvent_t start = nullptr, stop = nullptr;
};
inline LaunchTiming &launch_timing() {
    static thread_local LaunchTiming t;
    return t;
}
template <typename... Args, typename F = void (*)(Args...)>
inline void timed_launch(F kernel, dim3 g, dim3 b, uint32_t shm, hipStream_t s, Args... args) {
    LaunchTiming &t = launch_timing();
    hipExtLaunchKernelGGL(kernel, g, b, shm, s, t.start, t.stop, 0u, args...);
    t.start = t.stop = nullptr;
}

struct Tables {
    float2 win2[1024];  // (w[2m], w[2m+1])
    float2 t16[16];
    float2 t64[64];
    float2 t1k[1024];
    float2 t2k[1024];
};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 x, float2 w) {
    return make_float2(__builtin_fmaf(x.x, w.x, -(x.y * w.y)), __builtin_fmaf(x.x, w.y, x.y * w.x));
}

// FPSPEC cmul by the three DFT16 twiddles whose binary32 table values are structured (checked on the host
// in aid_engine_create: T16[2] = (c, -c), T16[6] = (-c, -c), T16[4] = (e, -1)). Each returns exactly
// cmul(x, w): x.im * w.im is -(x.im * c) (or x.im * e, -x.im) bit for bit, so one product serves both
// components -- 3 VALU instead of 4.
__device__ __forceinline__ float2 cmul_w2(float2 x, float c) {  // w = (c, -c)
    const float t = x.y * c;  // -(x.im * w.im) and x.im * w.re
    return make_float2(__builtin_fmaf(x.x, c, t), __builtin_fmaf(x.x, -c, t));
}
__device__ __forceinline__ float2 cmul_w6(float2 x, float mc) {  // w = (mc, mc), mc = -c
    const float t = x.y * mc;  // x.im * w.im = x.im * w.re
    return make_float2(__builtin_fmaf(x.x, mc, -t), __builtin_fmaf(x.x, mc, t));
}
__device__ __forceinline__ float2 cmul_w4(float2 x, float e) {  // w = (e, -1): -(x.im * -1) = x.im
    return make_float2(__builtin_fmaf(x.x, e, x.y), __builtin_fmaf(x.x, -1.0f, x.y * e));
}

// FPSPEC 3 DFT4, in place on (a,b,c,d) -> (y0,y1,y2,y3)
__device__ __forceinline__ void dft4(float2 &a, float2 &b, float2 &c, float2 &d) {
    float2 t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
    a = cadd(t0, t2);
    c = csub(t0, t2);
    b = make_float2(t1.x + t3.y, t1.y - t3.x);
    d = make_float2(t1.x - t3.y, t1.y + t3.x);
}

// FPSPEC 3 DFT16: v[16] in natural input order -> out[c + 4d] in v (natural output order).
// t16 holds W16^1, W16^2, W16^3, W16^4 (unused), W16^6, W16^9 at indices 1,2,3,4,6,9.
__device__ __forceinline__ void dft16(float2 (&v)[16], const float2 (&t16)[10]) {
    // s[b][c] lives in v[b + 4c] after the first DFT4 over (b, b+4, b+8, b+12)
#pragma unroll
    for (int b = 0; b < 4; ++b) dft4(v[b], v[b + 4], v[b + 8], v[b + 12]);
    // twiddles W16^{b*c}, b,c in 1..3
    v[1 + 4 * 1] = cmul(v[1 + 4 * 1], t16[1]);
    v[1 + 4 * 3] = cmul(v[1 + 4 * 3], t16[3]);
    v[3 + 4 * 1] = cmul(v[3 + 4 * 1], t16[3]);
    v[3 + 4 * 3] = cmul(v[3 + 4 * 3], t16[9]);
    v[1 + 4 * 2] = cmul_w2(v[1 + 4 * 2], t16[2].x);
    v[2 + 4 * 1] = cmul_w2(v[2 + 4 * 1], t16[2].x);
    v[2 + 4 * 2] = cmul_w4(v[2 + 4 * 2], t16[4].x);
    v[2 + 4 * 3] = cmul_w6(v[2 + 4 * 3], t16[6].x);
    v[3 + 4 * 2] = cmul_w6(v[3 + 4 * 2], t16[6].x);
    // second DFT4 over b for each c: inputs v[0+4c..3+4c], outputs out[c + 4d]
    float2 o[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float2 a0 = v[0 + 4 * c], a1 = v[1 + 4 * c], a2 = v[2 + 4 * c], a3 = v[3 + 4 * c];
        dft4(a0, a1, a2, a3);
        o[c + 0] = a0;
        o[c + 4] = a1;
        o[c + 8] = a2;
        o[c + 12] = a3;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = o[i];
}

// Orders a wave's own LDS exchange (write -> read by other lanes of the SAME wave). A wave's
// LDS instructions are executed in issue order (LLVM AMDGPU memory model: LDS accesses of one
// wavefront stay in order), so only the compiler must be kept from moving accesses across
// (an s_waitcnt here measured equal: the wait is not the cost).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("" ::: "memory");
}

}  // namespace aid
