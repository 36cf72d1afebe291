// lookback_probe.hip -- prices a decoupled look-back (the onesweep structure) for K4's radix passes on MI355X
// (fold the per-pass count into the scatter). Timing-only; nothing here is product code.
//
// A pass of the product scatter (index_sort.hip) is 141,553 tiles of 4,096 postings, two 4-wave workgroups per
// CU (512 tiles in flight), each reading 12 B and writing 12 B per posting. Onesweep would replace the count pass and
// the column scan (~0.65 ms of each ~4.2 ms pass) by a look-back: each tile publishes its 512 digit counts
// (AGGREGATE), then walks back over its predecessors' published words, summing aggregates until it meets an
// INCLUSIVE prefix, and publishes its own inclusive prefix. The status words must be coherent across the 8 XCDs'
// L2s, i.e. agent-scope atomic loads and stores (global_load/store ... sc1).
//
// This probe runs the same tile count and residency with the same HBM traffic per tile (a 48 KB read, then a
// 48 KB write: a copy of 6.8 GB), and between the two, per mode:
//   0  nothing (the copy alone: the traffic floor of a pass),
//   1  a look-back walking one predecessor per step (each thread owns 2 digits),
//   2  a look-back reading M = 8 predecessors per step (all loads of a step in flight together),
// and checks the exclusive prefixes the look-back produced for every tile against the host. Tiles are taken in
// ticket order (an atomic counter), so a tile only ever waits for tiles that are already resident: every wait ends.
// Every spin is bounded all the same (then an error flag is set, later tiles skip the look-back, the run reports it).
//
//   hipcc --offload-arch=gfx950 -O3 -o probes/lookback_probe probes/lookback_probe.hip
//   probes/lookback_probe [tiles=141553] [reps=3] [lds_kb=60]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int kThreads = 256, kDigits = 512, kTileItems = 4096, kWords = kTileItems * 3;  // 12 B per posting
constexpr int kSpinCap = 1 << 14;
constexpr uint64_t kAgg = 1ull << 32, kInc = 2ull << 32;

__host__ __device__ inline uint32_t tile_count(uint32_t t, uint32_t d) {  // synthetic digit counts, sum 4096-ish
    uint32_t x = t * 0x9E3779B1u ^ d * 0x85EBCA77u;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x & 15u;
}

__device__ inline uint64_t ld_status(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_status(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_pass(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                                   uint64_t *__restrict__ status, uint32_t *__restrict__ ticket,
                                                   uint32_t *__restrict__ excl_out, uint32_t *__restrict__ err,
                                                   int tiles) {
    extern __shared__ uint4 stage[];  // 48 KB of the tile (the product scatter stages its tile in LDS too)
    __shared__ uint32_t s_tile;
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const int t = (int)s_tile;
    if (t >= tiles) return;
    constexpr int kVec = kWords / 4 / kThreads;  // uint4 per thread: 12
    const uint4 *src = in + (size_t)t * (kWords / 4);
    uint4 v[kVec];
#pragma unroll
    for (int i = 0; i < kVec; ++i) v[i] = src[i * kThreads + tid];
#pragma unroll
    for (int i = 0; i < kVec; ++i) stage[i * kThreads + tid] = v[i];
    __syncthreads();
    if (MODE > 0) {
        const uint32_t d0 = 2 * tid, d1 = 2 * tid + 1;
        const uint32_t a0 = tile_count(t, d0), a1 = tile_count(t, d1);
        uint64_t *me = status + (size_t)t * kDigits;
        st_status(me + d0, (t == 0 ? kInc : kAgg) | a0);
        st_status(me + d1, (t == 0 ? kInc : kAgg) | a1);
        uint32_t e0 = 0, e1 = 0;
        bool done0 = t == 0, done1 = t == 0;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) done0 = done1 = true;
        int j = t - 1, spins = 0;
        while (!(done0 && done1)) {
            if (MODE == 1) {
                const uint64_t s0 = done0 ? kInc : ld_status(status + (size_t)j * kDigits + d0);
                const uint64_t s1 = done1 ? kInc : ld_status(status + (size_t)j * kDigits + d1);
                if ((s0 >> 32) == 0 || (s1 >> 32) == 0) {  // a predecessor has not published yet
                    if (++spins > kSpinCap) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if (!done0) { e0 += (uint32_t)s0; done0 = (s0 >> 32) == 2; }
                if (!done1) { e1 += (uint32_t)s1; done1 = (s1 >> 32) == 2; }
                --j;
            } else {
                constexpr int M = 8;
                uint64_t s0[M], s1[M];
#pragma unroll
                for (int m = 0; m < M; ++m) {  // every load of the step in flight together
                    const int jj = j - m;
                    s0[m] = (done0 || jj < 0) ? kInc : ld_status(status + (size_t)jj * kDigits + d0);
                    s1[m] = (done1 || jj < 0) ? kInc : ld_status(status + (size_t)jj * kDigits + d1);
                }
                int adv = 0;
                bool stall = false;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    if (stall || (done0 && done1)) break;
                    if ((s0[m] >> 32) == 0 || (s1[m] >> 32) == 0) {
                        stall = true;
                        break;
                    }
                    if (!done0) { e0 += (uint32_t)s0[m]; done0 = (s0[m] >> 32) == 2; }
                    if (!done1) { e1 += (uint32_t)s1[m]; done1 = (s1[m] >> 32) == 2; }
                    ++adv;
                }
                j -= adv;
                if (stall) {
                    if (++spins > kSpinCap) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
        st_status(me + d0, kInc | (e0 + a0));
        st_status(me + d1, kInc | (e1 + a1));
        excl_out[(size_t)t * kDigits + d0] = e0;
        excl_out[(size_t)t * kDigits + d1] = e1;
    }
    uint4 *dst = out + (size_t)t * (kWords / 4);
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
        uint4 w = stage[((i + 1) % kVec) * kThreads + tid];  // some reordering through the LDS, as a scatter
        dst[i * kThreads + tid] = w;
    }
}

int main(int argc, char **argv) {
    const int tiles = argc > 1 ? std::atoi(argv[1]) : 141553;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    const int lds_kb = argc > 3 ? std::atoi(argv[3]) : 60;  // 60: two workgroups per CU; 100: one
    const size_t words = (size_t)tiles * kWords;
    uint4 *in = nullptr, *out = nullptr;
    uint64_t *status = nullptr;
    uint32_t *ticket = nullptr, *excl = nullptr, *err = nullptr;
    CK(hipMalloc(&in, words * 4));
    CK(hipMalloc(&out, words * 4));
    CK(hipMalloc(&status, (size_t)tiles * kDigits * 8));
    CK(hipMalloc(&excl, (size_t)tiles * kDigits * 4));
    CK(hipMalloc(&ticket, 64));
    CK(hipMalloc(&err, 64));
    CK(hipMemset(in, 1, words * 4));
    // 48 KB used; 60 KB held by default: two workgroups per CU, as the product scatter (61 KB)
    const size_t lds = (size_t)(lds_kb < 48 ? 48 : lds_kb) * 1024;
    CK(hipFuncSetAttribute((const void *)k_pass<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void *)k_pass<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void *)k_pass<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::printf("{\"tiles\": %d, \"lds_kb\": %d, \"bytes_per_pass\": %zu, \"modes\": [", tiles, (int)(lds / 1024),
                2 * words * 4);
    for (int mode = 0; mode < 3; ++mode) {
        std::vector<float> ms;
        uint32_t h_err = 0;
        for (int r = 0; r < reps + 1; ++r) {
            CK(hipMemset(status, 0, (size_t)tiles * kDigits * 8));
            CK(hipMemset(ticket, 0, 64));
            CK(hipMemset(err, 0, 64));
            CK(hipEventRecord(a));
            if (mode == 0)
                hipLaunchKernelGGL(k_pass<0>, dim3(tiles), dim3(kThreads), lds, 0, in, out, status, ticket, excl, err, tiles);
            else if (mode == 1)
                hipLaunchKernelGGL(k_pass<1>, dim3(tiles), dim3(kThreads), lds, 0, in, out, status, ticket, excl, err, tiles);
            else
                hipLaunchKernelGGL(k_pass<2>, dim3(tiles), dim3(kThreads), lds, 0, in, out, status, ticket, excl, err, tiles);
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float t = 0;
            CK(hipEventElapsedTime(&t, a, b));
            CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
            if (r > 0) ms.push_back(t);  // the first is a warm-up
            if (h_err) break;
        }
        // the prefixes of a sample of tiles against the host
        bool ok = true;
        if (mode > 0 && !h_err) {
            std::vector<uint32_t> got((size_t)kDigits);
            std::vector<uint32_t> ref(kDigits, 0);
            int next = 0;
            const int samples[] = {0, 1, 2, 7, 513, tiles / 2, tiles - 1};
            for (int s : samples) {
                if (s < 0 || s >= tiles) continue;
                for (; next < s; ++next)
                    for (int d = 0; d < kDigits; ++d) ref[d] += tile_count(next, d);
                CK(hipMemcpy(got.data(), excl + (size_t)s * kDigits, kDigits * 4, hipMemcpyDeviceToHost));
                for (int d = 0; d < kDigits; ++d) ok = ok && got[d] == ref[d];
            }
        }
        float best = 1e30f, sum = 0;
        for (float x : ms) { best = x < best ? x : best; sum += x; }
        std::printf("%s{\"mode\": %d, \"ms\": [", mode ? ", " : "", mode);
        for (size_t i = 0; i < ms.size(); ++i) std::printf("%s%.4f", i ? ", " : "", ms[i]);
        std::printf("], \"best_ms\": %.4f, \"spin_capped\": %s, \"prefixes_ok\": %s}", ms.empty() ? -1.0f : best,
                    h_err ? "true" : "false", ok ? "true" : "false");
        std::fflush(stdout);
    }
    std::printf("]}\n");
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(status));
    CK(hipFree(excl));
    CK(hipFree(ticket));
    CK(hipFree(err));
    return 0;
}
