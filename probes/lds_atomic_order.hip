// lds_atomic_order.hip -- does one wave's ds_add_rtn_u32 return its old values in ascending lane order when
// several lanes hit the same LDS address? (K4's scatter ranks with one ballot-matched atomic per digit group; one
// plain atomic per lane would be a stable rank only if it does.) Timing-free; nothing here is product code.
//
// Every wave of a grid of 256-thread workgroups runs `rounds` slots; in each slot lane l adds 1 to counter
// c[w][digit(l, slot)] of its wave's private 512 counters (digit patterns: random 9-bit, 4 hot digits, all equal,
// and the K4 pattern of a bucket-key digit), then checks, through a second LDS array written with the returned
// values, that for every pair of lanes l < l' with the same digit the returned old value of l is below that of l'.
// Violations are counted per pattern.
//
//   hipcc --offload-arch=gfx950 -O3 -o probes/lds_atomic_order probes/lds_atomic_order.hip
//   probes/lds_atomic_order [blocks=4096] [rounds=256]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

__device__ inline uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_order(int rounds, unsigned long long *viol, unsigned long long *checked) {
    __shared__ uint32_t cnt[4][512];
    __shared__ uint32_t ret[4][64];
    __shared__ uint32_t dig[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4 * 512; i += 256) (&cnt[0][0])[i] = 0;
    __syncthreads();
    unsigned long long v[4] = {0, 0, 0, 0}, c[4] = {0, 0, 0, 0};
    for (int r = 0; r < rounds; ++r) {
        const uint32_t h = mix(blockIdx.x * 0x9E3779B9u + r * 0x85EBCA6Bu + w * 0xC2B2AE35u + lane);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            uint32_t d;
            if (p == 0) d = h & 511u;                          // random digits
            else if (p == 1) d = (h >> 9) & 3u;                // 4 hot digits
            else if (p == 2) d = 7u;                           // one digit
            else d = ((h >> 11) & 1u) ? (h >> 12) & 15u : 200u + ((h >> 20) & 63u);  // mixed
            const uint32_t old = atomicAdd(&cnt[w][d], 1u);
            ret[w][lane] = old;
            dig[w][lane] = d;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // lane l compares itself with every later lane of the same digit
            for (int l2 = lane + 1; l2 < 64; ++l2) {
                if (dig[w][l2] == d) {
                    ++c[p];
                    if (ret[w][l2] <= old) ++v[p];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        atomicAdd(&viol[p], v[p]);
        atomicAdd(&checked[p], c[p]);
    }
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 256;
    unsigned long long *viol = nullptr, *checked = nullptr;
    CK(hipMalloc(&viol, 64));
    CK(hipMalloc(&checked, 64));
    CK(hipMemset(viol, 0, 64));
    CK(hipMemset(checked, 0, 64));
    hipLaunchKernelGGL(k_order, dim3(blocks), dim3(256), 0, 0, rounds, viol, checked);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long hv[4], hc[4];
    CK(hipMemcpy(hv, viol, 32, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hc, checked, 32, hipMemcpyDeviceToHost));
    const char *names[4] = {"random512", "hot4", "one", "mixed"};
    std::printf("{\"blocks\": %d, \"rounds\": %d, \"patterns\": {", blocks, rounds);
    for (int p = 0; p < 4; ++p)
        std::printf("%s\"%s\": {\"same_digit_lane_pairs\": %llu, \"out_of_lane_order\": %llu}", p ? ", " : "", names[p],
                    hc[p], hv[p]);
    std::printf("}}\n");
    CK(hipFree(viol));
    CK(hipFree(checked));
    return 0;
}
