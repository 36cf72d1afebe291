// index_sort.hip -- K4 index build as a key sort (AIDFP_K4=sort, the default).
//
// Replaces the LMDB put of `olaf_c store` (audio-ident-service/app/audio/fingerprint.py:117-125;
// SURVEY.md 8a row a4). The atomic counting sort of index.hip (K4a count + scan + K4b scatter)
// spends two random-address atomics and one random 8-B store per posting: at the 100k-track catalog
// (912 M postings) 31 ms + 68 ms, ~2 % of the HBM peak, because the 256 MB cursor array and the 7.3 GB
// posting array miss every cache. Here the build streams instead:
//   K4s-a  one coalesced pass: key26 of every posting (2^26 for a removed track's, so it sorts past
//          the live ones) and its value track | t << 32;
//   K4s-b  a stable LSD radix sort of the (key, value) pairs over bits 0..26 (rocPRIM onesweep: per
//          pass a digit histogram, a decoupled look-back scan and LDS-ranked coalesced scatters), in
//          double buffers; the value buffer the sort ends in becomes the CSR's post array;
//   K4s-c  bucket lengths from the sorted keys: 2 atomics per distinct key (run start adds -i, run
//          end adds i + 1), then the same exclusive scan as the atomic path gives the offsets.
// Postings of one bucket stay in arrival order (the sort is stable); FPSPEC 7 results are order-
// independent anyway, so queries give the same rows on either build (tests/test_gpu_match.py).
#include <rocprim/device/device_radix_sort.hpp>

#include "aidfp_device.h"

namespace aid {

constexpr int kSortKeyBits = 27;  // key26 plus the removed-posting sentinel 2^26

__device__ __forceinline__ uint32_t sort_key26(uint32_t h) {
    return ((h >> 22) << 16) | (((h >> 12) & 0x3FFu) << 6) | (h & 0x3Fu);  // = index.hip key26
}

__global__ void k_sort_keys(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack,
                            const uint32_t *__restrict__ pt, int64_t n, const uint8_t *__restrict__ tomb,
                            uint32_t n_tracks, uint32_t *__restrict__ keys, uint64_t *__restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t tr = ptrack[i];
        const bool removed = tr < n_tracks && tomb[tr];
        keys[i] = removed ? (1u << 26) : sort_key26(ph[i]);
        vals[i] = (uint64_t)tr | ((uint64_t)pt[i] << 32);
    }
}

// cnt[k] (zeroed) += run length of key k < 2^26 in the sorted keys: -start at a run's first
// element, +end+1 at its last (u32 wrap-around; both land before the scan reads cnt)
__global__ void k_sort_runs(const uint32_t *__restrict__ keys, int64_t n, uint32_t *__restrict__ cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        if (k >= (1u << 26)) continue;
        if (i == 0 || keys[i - 1] != k) atomicAdd(&cnt[k], (uint32_t)(-(uint32_t)i));
        if (i == n - 1 || keys[i + 1] != k) atomicAdd(&cnt[k], (uint32_t)(i + 1));
    }
}

// temporary storage of the radix sort for n pairs
size_t index_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
    rocprim::double_buffer<uint64_t> v(nullptr, nullptr);
    if (rocprim::radix_sort_pairs(nullptr, bytes, k, v, (size_t)n, 0, kSortKeyBits) != hipSuccess) return 0;
    return bytes;
}

// keys0/keys1: n u32 each; vals0/vals1: n u64 each (the sorted values end in *vals_out, one of the two);
// cnt: 2^26 + 1 u32, zeroed by the caller
hipError_t launch_index_sort_build(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                                   const uint8_t *tomb, uint32_t n_tracks, uint32_t *keys0, uint32_t *keys1,
                                   uint64_t *vals0, uint64_t *vals1, void *temp, size_t temp_bytes,
                                   uint32_t *cnt, uint64_t **vals_out, hipStream_t s) {
    *vals_out = vals0;
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_sort_keys, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptrack, pt, n, tomb, n_tracks, keys0,
                       vals0);
    rocprim::double_buffer<uint32_t> k(keys0, keys1);
    rocprim::double_buffer<uint64_t> v(vals0, vals1);
    size_t bytes = temp_bytes;
    hipError_t err = rocprim::radix_sort_pairs(temp, bytes, k, v, (size_t)n, 0, kSortKeyBits, s);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_sort_runs, dim3((unsigned)blocks), dim3(256), 0, s, k.current(), n, cnt);
    *vals_out = v.current();
    return hipGetLastError();
}

}  // namespace aid
