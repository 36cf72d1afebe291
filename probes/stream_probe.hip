// stream_probe.hip -- read-pattern probe for K1/K2's streaming structure (timing only, not
// product code): what HBM read rate a given WG/row layout reaches on this box.
//   A: grid-stride float4 sweep (the chip reads one contiguous window at a time)
//   B: W workgroups, each streams its own contiguous range of 4 KB rows (K2's shape), PF rows in
//      flight in registers, no LDS
//   C: B + K2's LDS staging (4 rows, double buffer, one barrier per 4 rows)
//   D: like B but row r of every range is read by all WGs at the same time step (rows
//      interleaved: WG w reads rows w, w+W, w+2W ...)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned fold(float4 v) {
    return __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
}

__global__ void kA(const float4 *__restrict__ p, long n, unsigned *out) {
    unsigned acc = 0;
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        float4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= fold(a) ^ fold(b) ^ fold(c) ^ fold(d);
    }
    for (; i < n; i += stride) acc ^= fold(p[i]);
    if (acc == 0x12345678u) out[0] = acc;
}

template <int PF, bool LDS, bool INTERLEAVE>
__global__ __launch_bounds__(256) void kB(const float4 *__restrict__ p, long rows, int W, unsigned *out) {
    __shared__ float4 st[2][4][256];
    const int tid = threadIdx.x;
    const long per = (rows + W - 1) / W;
    const long r0 = INTERLEAVE ? blockIdx.x : blockIdx.x * per;
    const long rstep = INTERLEAVE ? W : 1;
    const long nr = INTERLEAVE ? (rows - blockIdx.x + W - 1) / W : (r0 + per <= rows ? per : (rows > r0 ? rows - r0 : 0));
    unsigned acc = 0;
    float4 pf[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) pf[j] = j < nr ? p[(r0 + j * rstep) * 256 + tid] : make_float4(0, 0, 0, 0);
    for (long base = 0; base < nr; base += 8) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const long it = base + s;
            if (it >= nr) break;
            if (s % 4 == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int slot = (s + j) % PF;
                    if (LDS) st[(it / 4) & 1][j][tid] = pf[slot]; else acc ^= fold(pf[slot]);
                    const long rn = it + j + PF;
                    pf[slot] = rn < nr ? p[(r0 + rn * rstep) * 256 + tid] : make_float4(0, 0, 0, 0);
                }
                if (LDS) __syncthreads();
            }
            if (LDS) acc ^= fold(st[(it / 4) & 1][s % 4][(tid + 4 * s) & 255]);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void kW(float4 *__restrict__ p, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ void kWnt(float4 *__restrict__ p, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    {
        typedef float v4 __attribute__((ext_vector_type(4)));
        v4 v = {1.f, 2.f, 3.f, (float)i};
        __builtin_nontemporal_store(v, reinterpret_cast<v4 *>(p + i));
    }
}

int main(int argc, char **argv) {
    const long rows = 219648;  // 256 clips x 858 frames, 4 KB each = 900 MB
    const long n = rows * 256;
    float4 *p; unsigned *o;
    CK(hipMalloc(&p, n * sizeof(float4)));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(p, 1, n * sizeof(float4)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best; sum += ms;
        }
        printf("%-34s best %.4f ms avg %.4f ms  %.2f TB/s (best)\n", name, best, sum / 10, n * 16.0 / best / 1e9);
    };
    // reads right after a kernel that wrote the same 900 MB (K1 -> K2), timed per read launch
    {
        float tot = 0, totw = 0;
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0)); kW<<<8192, 256>>>(p, n); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); totw += ms;
            CK(hipEventRecord(e0)); kB<4, true, false><<<768, 256>>>(p, rows, 768, o); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1)); tot += ms;
        }
        printf("W write 900 MB avg %.4f ms; C W=768 PF4 right after it avg %.4f ms (%.2f TB/s)\n", totw / 10, tot / 10, n * 16.0 / (tot / 10) / 1e9);
        tot = 0;
        for (int r = 0; r < 10; ++r) {
            kW<<<8192, 256>>>(p, n);
            CK(hipEventRecord(e0)); kB<4, true, false><<<768, 256>>>(p, rows, 768, o); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); tot += ms;
        }
        printf("C W=768 PF4 queued behind W avg %.4f ms (%.2f TB/s)\n", tot / 10, n * 16.0 / (tot / 10) / 1e9);
        tot = 0; totw = 0;
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0)); kWnt<<<8192, 256>>>(p, n); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); totw += ms;
            CK(hipEventRecord(e0)); kB<4, true, false><<<768, 256>>>(p, rows, 768, o); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1)); tot += ms;
        }
        printf("Wnt write 900 MB avg %.4f ms; C right after it avg %.4f ms (%.2f TB/s)\n", totw / 10, tot / 10, n * 16.0 / (tot / 10) / 1e9);
        return 0;
    }
    // chunked write -> read (K1 -> K2 per chunk of clips): reused scratch vs a fresh region per chunk
    for (long mb : {32L, 64L, 112L, 160L, 224L, 300L}) {
        const long cr = mb * 256;  // rows of 4 KB
        const long nch = rows / cr;
        for (int reuse = 1; reuse >= 0; --reuse) {
            float best = 1e9;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (long c = 0; c < nch; ++c) {
                    float4 *q = p + (reuse ? 0 : c * cr * 256);
                    kW<<<2048, 256>>>(q, cr * 256);
                    kB<4, true, false><<<768, 256>>>(q, cr, 768, o);
                }
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;
            }
            printf("chunk %4ld MB x %3ld %s: %.4f ms for %.0f MB written+read (%.2f TB/s of w+r)\n", mb, nch,
                   reuse ? "reused " : "fresh  ", best, nch * cr * 4096.0 / 1e6, 2.0 * nch * cr * 4096 / best / 1e9);
        }
    }
    for (int g : {1024, 2048, 4096, 8192})
        { char b[64]; snprintf(b, 64, "A grid-stride g=%d", g); run(b, [&] { kA<<<g, 256>>>(p, n, o); }); }
    for (int W : {768, 1024, 2048, 3072, 6144}) {
        char b[64];
        snprintf(b, 64, "B ranges W=%d PF4", W); run(b, [&] { kB<4, false, false><<<W, 256>>>(p, rows, W, o); });
        snprintf(b, 64, "B ranges W=%d PF8", W); run(b, [&] { kB<8, false, false><<<W, 256>>>(p, rows, W, o); });
        snprintf(b, 64, "C ranges+LDS W=%d PF4", W); run(b, [&] { kB<4, true, false><<<W, 256>>>(p, rows, W, o); });
        snprintf(b, 64, "C ranges+LDS W=%d PF8", W); run(b, [&] { kB<8, true, false><<<W, 256>>>(p, rows, W, o); });
        snprintf(b, 64, "D interleaved W=%d PF4", W); run(b, [&] { kB<4, false, true><<<W, 256>>>(p, rows, W, o); });
        snprintf(b, 64, "D interleaved+LDS W=%d PF4", W); run(b, [&] { kB<4, true, true><<<W, 256>>>(p, rows, W, o); });
    }
    return 0;
}
