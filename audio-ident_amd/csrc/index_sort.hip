// index_sort.hip -- K4 index build as a key sort: a hand-written LSD radix sort for gfx950 (default),
// rocPRIM's onesweep kept only as an A/B reference (aid_engine_force K4_BUILD).
//
// Replaces the LMDB put of `olaf_c store` (audio-ident-service/app/audio/fingerprint.py:117-125;
// SURVEY.md 8a row a4). The index is a direct-address CSR over key26 = k1 << 16 | k2 << 6 | dt
// (index.hip); the build sorts the postings by key27 = key26, or 2^26 for a removed track's posting
// (it sorts past every live key and is dropped), stably, so a bucket keeps arrival order.
//
// Hand-written sort (3 passes of 9-bit digits over bits 0..26, 512 digits per pass):
//   count    per tile of kTile = 8192 postings, the digit histogram (wave ballot-match, then one LDS
//            add per distinct digit per wave) -> counts[digit][tile];
//   scan     exclusive scan of counts in digit-major order: the global start of (digit, tile);
//   scatter  a workgroup of 8 waves loads its tile (wave w: items w*1024 .. +1023, 64 consecutive per
//            load), ranks every item stably inside the tile (ballot match per 64-item slot, wave-private
//            running digit counters, cross-wave offsets), stages the tile in LDS in sorted order (96 KB)
//            and writes it out in runs of consecutive positions per digit (coalesced).
// Pass 1 reads the SoA postings (hash, track, t) and the tombstones itself (key generation fused in);
// pass 3 writes the values straight into the CSR's post array. Bytes per posting: 8 (count 1) + 24
// (scatter 1) + 2 x (4 + 24) + 4 (runs) = 92, against ~125 for the rocPRIM build.
// After the sort, bucket lengths come from the sorted keys (2 atomics per distinct key, in key order),
// then index.hip's scan gives the offsets.
#include <rocprim/device/device_radix_sort.hpp>

#include "aidfp_device.h"

namespace aid {

constexpr int kSortKeyBits = 27;  // key26 plus the removed-posting sentinel 2^26
constexpr int kDigitBits = 9;
constexpr int kDigits = 1 << kDigitBits;
constexpr int kSortPasses = 3;
constexpr int kSortThreads = 512;  // 8 waves
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kSlots = 16;                      // 64-item slots per wave
constexpr int kTile = kSortThreads * kSlots;    // 8192 postings per tile
static_assert(kDigits == kSortThreads, "one digit per thread in the tile-level steps");
static_assert(kDigitBits * kSortPasses == kSortKeyBits, "passes cover the key");

__device__ __forceinline__ uint32_t sort_key26(uint32_t h) {
    return ((h >> 22) << 16) | (((h >> 12) & 0x3FFu) << 6) | (h & 0x3Fu);  // = index.hip key26
}

// tomb == nullptr: no track is removed (the engine passes none then, saving a dependent load per posting)
__device__ __forceinline__ uint32_t make_key(uint32_t h, uint32_t tr, const uint8_t *__restrict__ tomb,
                                             uint32_t n_tracks) {
    return (tomb && tr < n_tracks && tomb[tr]) ? (1u << 26) : sort_key26(h);
}

// lanes of the wave holding the same 9-bit digit (among the lanes in `valid`)
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t valid) {
    uint64_t m = valid;
#pragma unroll
    for (int b = 0; b < kDigitBits; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    return m;
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// counts[d * tiles + tile] = items of tile `tile` whose digit at `shift` is d
template <bool FIRST>
__global__ __launch_bounds__(kSortThreads) void k_radix_count(const uint32_t *__restrict__ keys,
                                                              const uint32_t *__restrict__ ptrack,
                                                              const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                              int64_t n, int shift, uint32_t *__restrict__ counts,
                                                              int64_t tiles) {
    __shared__ uint32_t c[kSortWaves][kDigits];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < kSortWaves * kDigits; i += kSortThreads) (&c[0][0])[i] = 0u;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)w * (kSlots * 64);
    uint32_t d[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {  // all loads first
        const int64_t i = base + s * 64 + lane;
        uint32_t k = 0;
        if (i < n) k = FIRST ? make_key(keys[i], ptrack[i], tomb, n_tracks) : keys[i];
        d[s] = (k >> shift) & (kDigits - 1);
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const int64_t i0 = base + s * 64;
        const uint64_t valid = i0 + 64 <= n ? ~0ull : (i0 >= n ? 0ull : (~0ull >> (64 - (int)(n - i0))));
        const uint64_t m = match_digit(d[s], valid);
        // one LDS add per distinct digit of the slot (no return value: the slots' adds issue back to back)
        if (((valid >> lane) & 1) && (m & lanemask_lt(lane)) == 0) atomicAdd(&c[w][d[s]], (uint32_t)__popcll(m));
    }
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int ww = 0; ww < kSortWaves; ++ww) t += c[ww][tid];
    counts[(int64_t)tid * tiles + blockIdx.x] = t;
}

// exclusive scan over the 512 threads of the block (wave shuffles + one exchange of the wave totals)
__device__ __forceinline__ uint32_t block_scan512(uint32_t v, uint32_t *tmp /*[kSortWaves]*/) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) tmp[w] = x;
    __syncthreads();
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < kSortWaves; ++i) b += i < w ? tmp[i] : 0u;
    return b + x - v;
}

template <bool FIRST, bool LAST>
__global__ __launch_bounds__(kSortThreads) void k_radix_scatter(const uint32_t *__restrict__ keys_in,
                                                                const uint64_t *__restrict__ vals_in,
                                                                const uint32_t *__restrict__ ptrack,
                                                                const uint32_t *__restrict__ pt,
                                                                const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                                int64_t n, int shift,
                                                                const uint32_t *__restrict__ offs, int64_t tiles,
                                                                uint32_t *__restrict__ keys_out,
                                                                uint64_t *__restrict__ vals_out) {
    __shared__ uint32_t s_key[kTile];
    __shared__ uint64_t s_val[kTile];
    __shared__ uint32_t cnt[kSortWaves][kDigits];  // running per-wave counters, then cross-wave offsets
    __shared__ uint32_t t_start[kDigits];          // first local position of each digit in the tile
    __shared__ uint32_t g_start[kDigits];          // global position of (digit, tile)
    __shared__ uint32_t tmp[kSortWaves];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t tile0 = (int64_t)blockIdx.x * kTile;
    const int64_t base = tile0 + (int64_t)w * (kSlots * 64);
    for (int i = tid; i < kSortWaves * kDigits; i += kSortThreads) (&cnt[0][0])[i] = 0u;
    g_start[tid] = offs[(int64_t)tid * tiles + blockIdx.x];
    uint32_t key[kSlots];
    uint64_t val[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {  // every load of the tile in flight at once
        const int64_t i = base + s * 64 + lane;
        if (i < n) {
            if (FIRST) {
                const uint32_t tr = ptrack[i];
                key[s] = make_key(keys_in[i], tr, tomb, n_tracks);
                val[s] = (uint64_t)tr | ((uint64_t)pt[i] << 32);
            } else {
                key[s] = keys_in[i];
                val[s] = vals_in[i];
            }
        } else {
            key[s] = 0xFFFFFFFFu;
            val[s] = 0;
        }
    }
    __syncthreads();  // counters zeroed
    // stable rank inside the wave: slot by slot in item order, lanes in lane order. The leader of each digit
    // group adds the group's size to the wave's running counter and gets the count before it (LDS atomics of
    // one wave are executed in order, so slot s sees slots 0..s-1); the 16 slots' atomics issue back to back,
    // then each lane takes its leader's value (a cross-lane read) and adds its place in the group
    uint32_t rank[kSlots], old[kSlots];
    int lead[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const int64_t i0 = base + s * 64;
        const uint64_t valid = i0 + 64 <= n ? ~0ull : (i0 >= n ? 0ull : (~0ull >> (64 - (int)(n - i0))));
        const uint32_t d = (key[s] >> shift) & (kDigits - 1);
        const uint64_t m = match_digit(d, valid);
        const uint64_t mine = m | (1ull << lane);  // an invalid lane leads its own (empty) group
        lead[s] = __ffsll((unsigned long long)mine) - 1;
        rank[s] = (uint32_t)__popcll(m & lanemask_lt(lane));
        old[s] = 0;
        if (((valid >> lane) & 1) && lead[s] == lane) old[s] = atomicAdd(&cnt[w][d], (uint32_t)__popcll(m));
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s) rank[s] += (uint32_t)__shfl((int)old[s], lead[s], 64);
    __syncthreads();
    // thread = digit: cross-wave exclusive offsets (in place) and the tile's digit total
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < kSortWaves; ++ww) {
        const uint32_t c = cnt[ww][tid];
        cnt[ww][tid] = tot;
        tot += c;
    }
    const uint32_t start = block_scan512(tot, tmp);
    t_start[tid] = start;
    __syncthreads();
    // stage the tile in LDS in sorted (digit, item) order
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        if (base + s * 64 + lane < n) {
            const uint32_t d = (key[s] >> shift) & (kDigits - 1);
            const uint32_t pos = t_start[d] + cnt[w][d] + rank[s];  // a permutation of [0, tile items)
            if (pos < kTile) {
                s_key[pos] = key[s];
                s_val[pos] = val[s];
            }
        }
    }
    __syncthreads();
    // write out: consecutive threads, consecutive positions of one digit run
    const int m = (int)min((int64_t)kTile, n - tile0);
#pragma unroll 4
    for (int i = tid; i < m; i += kSortThreads) {
        const uint32_t k = s_key[i];
        const uint32_t d = (k >> shift) & (kDigits - 1);
        const int64_t dst = (int64_t)g_start[d] + (i - (int)t_start[d]);
        if (dst >= n) continue;  // cannot happen for consistent counts; never write out of bounds
        keys_out[dst] = k;
        if (LAST) __builtin_nontemporal_store(s_val[i], &vals_out[dst]);
        else vals_out[dst] = s_val[i];
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

// ---- rocPRIM reference build (A/B only) ----
__global__ void k_sort_keys(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack,
                            const uint32_t *__restrict__ pt, int64_t n, const uint8_t *__restrict__ tomb,
                            uint32_t n_tracks, uint32_t *__restrict__ keys, uint64_t *__restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t tr = ptrack[i];
        keys[i] = make_key(ph[i], tr, tomb, n_tracks);
        vals[i] = (uint64_t)tr | ((uint64_t)pt[i] << 32);
    }
}

void launch_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t s);

int64_t radix_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

// scratch of the hand-written sort in u32 units: counts + offsets matrices and the scan's temporary
size_t radix_scratch_u32(int64_t n) {
    const int64_t c = (int64_t)kDigits * radix_tiles(n);
    return (size_t)(2 * c + 4 * (c / 1024 + 2) + 4096);
}

// temporary storage of the rocPRIM sort for n pairs
size_t index_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
    rocprim::double_buffer<uint64_t> v(nullptr, nullptr);
    if (rocprim::radix_sort_pairs(nullptr, bytes, k, v, (size_t)n, 0, kSortKeyBits) != hipSuccess) return 0;
    return bytes;
}

// keys0/keys1: n u32 each; vals0/vals1: n u64 each (the sorted values end in *vals_out, one of the two);
// cnt: 2^26 + 1 u32, zeroed by the caller. use_rocprim: the A/B reference (temp/temp_bytes its storage);
// otherwise `scratch` holds radix_scratch_u32(n) u32.
hipError_t launch_index_sort_build(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                                   const uint8_t *tomb, uint32_t n_tracks, uint32_t *keys0, uint32_t *keys1,
                                   uint64_t *vals0, uint64_t *vals1, void *temp, size_t temp_bytes, bool use_rocprim,
                                   uint32_t *scratch, uint32_t *cnt, uint64_t **vals_out, hipStream_t s) {
    *vals_out = vals0;
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
    const uint32_t *sorted_keys = nullptr;
    if (use_rocprim) {
        hipLaunchKernelGGL(k_sort_keys, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptrack, pt, n, tomb, n_tracks,
                           keys0, vals0);
        rocprim::double_buffer<uint32_t> k(keys0, keys1);
        rocprim::double_buffer<uint64_t> v(vals0, vals1);
        size_t bytes = temp_bytes;
        hipError_t err = rocprim::radix_sort_pairs(temp, bytes, k, v, (size_t)n, 0, kSortKeyBits, s);
        if (err != hipSuccess) return err;
        sorted_keys = k.current();
        *vals_out = v.current();
    } else {
        const int64_t tiles = radix_tiles(n);
        const int64_t c = (int64_t)kDigits * tiles;
        uint32_t *counts = scratch, *offs = scratch + c, *stmp = scratch + 2 * c;
        // pass 1: SoA postings -> (keys1, vals1); pass 2: -> (keys0, vals0); pass 3: -> (keys1, vals1)
        const dim3 g((unsigned)tiles), b(kSortThreads);
        timed_launch(k_radix_count<true>, g, b, 0, s, ph, ptrack, tomb, n_tracks, n, 0, counts, tiles);
        launch_scan(counts, offs, c, stmp, s);
        timed_launch(k_radix_scatter<true, false>, g, b, 0, s, ph, (const uint64_t *)nullptr, ptrack, pt, tomb,
                     n_tracks, n, 0, (const uint32_t *)offs, tiles, keys1, vals1);
        timed_launch(k_radix_count<false>, g, b, 0, s, (const uint32_t *)keys1, (const uint32_t *)nullptr,
                     (const uint8_t *)nullptr, 0u, n, kDigitBits, counts, tiles);
        launch_scan(counts, offs, c, stmp, s);
        timed_launch(k_radix_scatter<false, false>, g, b, 0, s, (const uint32_t *)keys1, (const uint64_t *)vals1,
                     (const uint32_t *)nullptr, (const uint32_t *)nullptr, (const uint8_t *)nullptr, 0u, n,
                     kDigitBits, (const uint32_t *)offs, tiles, keys0, vals0);
        timed_launch(k_radix_count<false>, g, b, 0, s, (const uint32_t *)keys0, (const uint32_t *)nullptr,
                     (const uint8_t *)nullptr, 0u, n, 2 * kDigitBits, counts, tiles);
        launch_scan(counts, offs, c, stmp, s);
        timed_launch(k_radix_scatter<false, true>, g, b, 0, s, (const uint32_t *)keys0, (const uint64_t *)vals0,
                     (const uint32_t *)nullptr, (const uint32_t *)nullptr, (const uint8_t *)nullptr, 0u, n,
                     2 * kDigitBits, (const uint32_t *)offs, tiles, keys1, vals1);
        sorted_keys = keys1;
        *vals_out = vals1;
    }
    hipLaunchKernelGGL(k_sort_runs, dim3((unsigned)blocks), dim3(256), 0, s, sorted_keys, n, cnt);
    return hipGetLastError();
}

}  // namespace aid
