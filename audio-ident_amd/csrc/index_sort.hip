// index_sort.hip -- K4 index build as a key sort: a hand-written LSD radix sort for gfx950 (default),
// rocPRIM's onesweep kept only as an A/B reference (aid_engine_force K4_BUILD 3), compiled only into the
// diagnostic variant build -DAID_K4_ROCPRIM_AB (build_ext.build(variant="k4rocprim")), never into libaidfp.so.
//
// Replaces the LMDB put of `olaf_c store` (audio-ident-service/app/audio/fingerprint.py:117-125;
// SURVEY.md 8a row a4). The index is a direct-address CSR over key26 = bucket_key(hash) (aidfp_layout.h, a bit
// permutation of k1 | k2 | dt that spreads the busy low bits over the three digit passes); the build sorts the
// postings by key27 = key26, or 2^26 for a removed track's posting (it sorts past every live key and is dropped),
// stably, so a bucket keeps arrival order.
//
// Hand-written sort (3 passes of 9-bit digits over bits 0..26, 512 digits per pass):
//   count    per tile of kTile = 4096 postings, the digit histogram (LDS atomics) -> counts[tile][digit], one
//            contiguous 2 KB row per tile (full lines; a digit-major matrix put each 4-B entry ~890 KB from its
//            neighbour, one partial line per entry: 3.8 GB written for a 0.46 GB matrix, 3.6 GB re-read by the
//            scatter);
//   scan     the global start of (digit, tile) in digit-major order, over the tile-major matrix: column sums per
//            group of kColTiles tiles, a column scan of those with the digit totals' exclusive scan, then
//            each group's running column prefix (every read and write a contiguous row);
//   scatter  a workgroup of 4 waves loads its tile (wave w: items w*1024 .. +1023, 64 consecutive per
//            load), ranks every item stably inside the tile (one LDS atomic per item on a wave-private
//            digit counter, slot by slot: the wave's atomics execute in issue order and, as checked on the
//            device before the first build, same-counter lanes of one atomic are served in lane order; where
//            that check fails, a ballot match per 64-item slot and one atomic per digit group), then
//            cross-wave offsets, stages the tile in LDS in sorted order (52 KB with the counters in the key
//            area: three workgroups per CU overlap loads with ranking) and writes it out in runs of
//            consecutive positions per digit.
// Pass 1 reads the SoA postings (hash, track, t) itself (key generation fused in; the tombstones and the track
// column for the count only when a track is removed); pass 3 writes the values straight into the CSR's post array
// and, instead of a sorted key array, the CSR's run ends: at the last posting i of each key's run,
// E[key + 1] = i + 1 (a key's postings in one tile's digit run are contiguous and in key order; a run that may
// continue in the next tile raises E by atomicMax). An inclusive max-scan of E over the 2^26 + 1 keys is
// offsets[] (an absent key inherits the end of the largest key below it); it also counts the live keys (nonzero
// E). No bucket-length atomics, no key array after the last pass.
// Tiles are dealt XCD-contiguously (xcd_tile): adjacent tiles' partial lines complete in one L2.
// Bytes per posting: 4 (count 1) + 24 (scatter 1) + 2 x 4 (counts 2, 3) + 24 (scatter 2) + 20 (scatter 3) = 80,
// plus ~4 per distinct key (E) and the 2 KB of counts per tile per pass.
#include <atomic>

#ifdef AID_K4_ROCPRIM_AB  // diagnostic variant build only (build_ext.build(variant="k4rocprim")); never in libaidfp.so
#include <rocprim/device/device_radix_sort.hpp>
#endif

#include "aidfp_device.h"

namespace aid {

constexpr int kSortKeyBits = 27;  // key26 plus the removed-posting sentinel 2^26
constexpr int kDigitBits = 9;
constexpr int kDigits = 1 << kDigitBits;
constexpr int kSortPasses = 3;
constexpr int kSortThreads = 256;  // 4 waves
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kSlots = 16;  // 64-item slots per wave
constexpr int kTile = kSortThreads * kSlots;    // 4096 postings per tile
constexpr int kDigitsPerThread = kDigits / kSortThreads;
static_assert(kDigitBits * kSortPasses == kSortKeyBits, "passes cover the key");


// tomb == nullptr: no track is removed (the engine passes none then, saving a dependent load per posting)
__device__ __forceinline__ uint32_t make_key(uint32_t h, uint32_t tr, const uint8_t *__restrict__ tomb,
                                             uint32_t n_tracks) {
    return (tomb && tr < n_tracks && tomb[tr]) ? (1u << 26) : bucket_key(h);
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

// the tile of workgroup b: consecutive tiles on one XCD (workgroups b and b + 8 share an XCD's L2), so the partial
// 128-B lines where adjacent tiles' runs of one digit meet -- in the scatter's output and in the digit-major count
// matrix -- are completed in that L2 instead of going to HBM as separate partial writes and reads
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
    const int64_t per = nb / 8, rem = nb % 8, x = b % 8, y = b / 8;
    return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + y;
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ uint64_t valid_lanes(int64_t i0, int64_t n) {
    return i0 + 64 <= n ? ~0ull : (i0 >= n ? 0ull : (~0ull >> (64 - (int)(n - i0))));
}

// counts[tile * kDigits + d] = items of tile `tile` whose digit at `shift` is d (order does not matter here:
// one LDS atomic per item)
// TOMB (first pass only): a track is removed, so the key needs the posting's track and its tombstone. Without it the
// instantiation has no dependent loads: a runtime `tomb ?` test had made hipcc wait for each slot's track load
// before issuing the next slot's loads (16 serialised round trips per tile in the first scatter: 6.2 against 3.4 ms
// for the other passes at 580 M postings)
template <bool FIRST, bool TOMB = false>
__global__ __launch_bounds__(kSortThreads) void k_radix_count(const uint32_t *__restrict__ keys,
                                                              const uint32_t *__restrict__ ptrack,
                                                              const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                              int64_t n, int shift, uint32_t *__restrict__ counts,
                                                              int64_t tiles) {
    __shared__ uint32_t c[kDigits];
    const int tid = threadIdx.x;
    for (int i = tid; i < kDigits; i += kSortThreads) c[i] = 0u;
    __syncthreads();
    const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const int64_t base = tile * kTile;
    uint32_t raw[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {  // all loads first; no arithmetic on a loaded value inside the branch (hipcc
                                        // would wait for each slot's load before issuing the next)
        const int64_t i = base + s * kSortThreads + tid;
        raw[s] = 0u;
        if (i < n) {
            // the track column only when a track is removed (TOMB)
            raw[s] = (FIRST && TOMB) ? make_key(keys[i], ptrack[i], tomb, n_tracks) : keys[i];
        }
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const int64_t i = base + s * kSortThreads + tid;
        const uint32_t k = (FIRST && !TOMB) ? bucket_key(raw[s]) : raw[s];
        if (i < n) atomicAdd(&c[(k >> shift) & (kDigits - 1)], 1u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        const int dd = tid + j * kSortThreads;
        counts[tile * kDigits + dd] = c[dd];
    }
}

// ---- (digit, tile) starts from the tile-major counts: offs[t][d] = sum_{d' < d} total[d'] + sum_{t' < t} counts[t'][d]
constexpr int kColTiles = 256;  // tiles per column-sum group
__global__ __launch_bounds__(kDigits) void k_col_sum(const uint32_t *__restrict__ counts, int64_t tiles,
                                                     uint32_t *__restrict__ gsum) {
    const int d = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * kColTiles, t1 = min(t0 + kColTiles, tiles);
    uint32_t acc = 0;
#pragma unroll 8
    for (int64_t t = t0; t < t1; ++t) acc += counts[t * kDigits + d];
    gsum[(int64_t)blockIdx.x * kDigits + d] = acc;
}

// one workgroup per digit: the exclusive prefix of the digit's group sums down its column (goff), and the
// column total (a single workgroup walking the ~570 groups for all digits took 0.15 ms per pass)
constexpr int kColScanThreads = 256;
__global__ __launch_bounds__(kColScanThreads) void k_col_scan(const uint32_t *__restrict__ gsum, int64_t groups,
                                                              uint32_t *__restrict__ goff, uint32_t *__restrict__ total) {
    __shared__ uint32_t ws[kColScanThreads / 64];
    const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t carry = 0;
    for (int64_t g0 = 0; g0 < groups; g0 += kColScanThreads) {
        const int64_t g = g0 + tid;
        const uint32_t v = g < groups ? gsum[g * kDigits + d] : 0u;
        uint32_t x = v;  // inclusive scan over the workgroup
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) ws[w] = x;
        __syncthreads();
        uint32_t pre = carry;
        for (int i = 0; i < w; ++i) pre += ws[i];
        if (g < groups) goff[g * kDigits + d] = pre + x - v;
        uint32_t blk = 0;
        for (int i = 0; i < kColScanThreads / 64; ++i) blk += ws[i];
        carry += blk;
        __syncthreads();
    }
    if (tid == 0) total[d] = carry;
}

// one workgroup: the digits' global bases, base[d] = sum of the totals of digits d' < d
__global__ __launch_bounds__(kDigits) void k_digit_base(const uint32_t *__restrict__ total, uint32_t *__restrict__ base) {
    __shared__ uint32_t ws[kDigits / 64];
    const int d = threadIdx.x, lane = d & 63, w = d >> 6;
    const uint32_t v = total[d];
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = x - v;
    for (int i = 0; i < w; ++i) pre += ws[i];
    base[d] = pre;
}

__global__ __launch_bounds__(kDigits) void k_col_apply(const uint32_t *__restrict__ counts, int64_t tiles,
                                                       const uint32_t *__restrict__ goff,
                                                       const uint32_t *__restrict__ base, uint32_t *__restrict__ offs) {
    const int d = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * kColTiles, t1 = min(t0 + kColTiles, tiles);
    uint32_t run = base[d] + goff[(int64_t)blockIdx.x * kDigits + d];
#pragma unroll 8
    for (int64_t t = t0; t < t1; ++t) {
        const uint32_t c = counts[t * kDigits + d];
        offs[t * kDigits + d] = run;
        run += c;
    }
}

static int64_t col_groups(int64_t tiles) { return (tiles + kColTiles - 1) / kColTiles; }

static void digit_starts(const uint32_t *counts, int64_t tiles, uint32_t *offs, uint32_t *tmp, hipStream_t s) {
    const int64_t groups = col_groups(tiles);
    uint32_t *gsum = tmp, *goff = tmp + groups * kDigits, *total = goff + groups * kDigits, *base = total + kDigits;
    hipLaunchKernelGGL(k_col_sum, dim3((unsigned)groups), dim3(kDigits), 0, s, counts, tiles, gsum);
    hipLaunchKernelGGL(k_col_scan, dim3(kDigits), dim3(kColScanThreads), 0, s, (const uint32_t *)gsum, groups, goff,
                       total);
    hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(kDigits), 0, s, (const uint32_t *)total, base);
    hipLaunchKernelGGL(k_col_apply, dim3((unsigned)groups), dim3(kDigits), 0, s, counts, tiles,
                       (const uint32_t *)goff, (const uint32_t *)base, offs);
}

// ARANK: the stable in-wave rank by one LDS atomic per posting (lds_lane_order_ok() must hold), else by ballots
template <bool FIRST, bool LAST, bool TOMB = false, bool ARANK = false>
__global__ __launch_bounds__(kSortThreads, 3) void k_radix_scatter(const uint32_t *__restrict__ keys_in,
                                                                const uint64_t *__restrict__ vals_in,
                                                                const uint32_t *__restrict__ ptrack,
                                                                const uint32_t *__restrict__ pt,
                                                                const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                                int64_t n, int shift,
                                                                const uint32_t *__restrict__ offs, int64_t tiles,
                                                                uint32_t *__restrict__ keys_out,
                                                                uint64_t *__restrict__ vals_out,
                                                                uint32_t *__restrict__ E,
                                                                uint16_t *__restrict__ sig_out) {
    // the per-wave counters (running counts, then cross-wave offsets) live in the front of the key staging area
    // (52 KB per workgroup: three per CU): every posting's staging position is taken from them before the barrier that
    // precedes the staging
    static_assert(kSortWaves * kDigits <= kTile, "counters fit the key staging area");
    __shared__ uint32_t s_key[kTile];
    uint32_t(*cnt)[kDigits] = reinterpret_cast<uint32_t(*)[kDigits]>(s_key);
    __shared__ uint64_t s_val[kTile];
    __shared__ uint32_t t_start[kDigits];          // first local position of each digit in the tile
    __shared__ uint32_t g_start[kDigits];          // global position of (digit, tile)
    __shared__ uint32_t wsum[kSortWaves];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const int64_t tile0 = tile * kTile;
    const int64_t base = tile0 + (int64_t)w * (kSlots * 64);
    for (int i = tid; i < kSortWaves * kDigits; i += kSortThreads) (&cnt[0][0])[i] = 0u;
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        const int dd = tid + j * kSortThreads;
        g_start[dd] = offs[tile * kDigits + dd];
    }
    uint32_t key[kSlots];
    uint64_t val[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {  // every load of the tile in flight at once
        const int64_t i = base + s * 64 + lane;
        if (i < n) {
            if (FIRST) {
                const uint32_t tr = ptrack[i];
                // without tombstones the raw hash is loaded here and permuted after the loop: any arithmetic on a
                // loaded value inside this per-slot branch makes hipcc wait for that load before the next slot's
                key[s] = TOMB ? make_key(keys_in[i], tr, tomb, n_tracks) : keys_in[i];
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
    if (FIRST && !TOMB) {  // past-the-end slots get some key too: they are never ranked or staged (valid_lanes)
#pragma unroll
        for (int s = 0; s < kSlots; ++s) key[s] = bucket_key(key[s]);
    }
    __syncthreads();  // counters zeroed
    // stable rank inside the wave: slot by slot in item order, lanes in lane order. The leader of each digit
    // group adds the group's size to the wave's running counter and gets the count before it (LDS atomics of
    // one wave are executed in order, so slot s sees slots 0..s-1); the 16 slots' atomics issue back to back,
    // then each lane takes its leader's value (a cross-lane read) and adds its place in the group
    uint32_t rank[kSlots];
    if constexpr (ARANK) {
        // one LDS atomic per posting: the old value is the number of earlier postings of the wave with the same
        // digit, given that a wave's LDS atomics execute in issue order (slot by slot) and that the lanes of one
        // ds_add_rtn that hit the same counter are served in ascending lane order (checked on the device before
        // this path is taken: lds_lane_order_ok)
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            const uint32_t d = (key[s] >> shift) & (kDigits - 1);
            rank[s] = base + s * 64 + lane < n ? atomicAdd(&cnt[w][d], 1u) : 0u;
        }
    } else {
        uint32_t old[kSlots];
        int lead[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            const uint64_t valid = valid_lanes(base + s * 64, n);
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
    }
    __syncthreads();
    // thread = 2 consecutive digits: cross-wave exclusive offsets (in place) and the tile's digit totals, then
    // the exclusive scan of the totals over the digits (the thread's pair, wave shuffles, wave totals)
    uint32_t tot[kDigitsPerThread];
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        const int dd = tid * kDigitsPerThread + j;
        uint32_t t = 0;
#pragma unroll
        for (int ww = 0; ww < kSortWaves; ++ww) {
            const uint32_t c = cnt[ww][dd];
            cnt[ww][dd] = t;
            t += c;
        }
        tot[j] = t;
    }
    uint32_t mysum = 0;
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) mysum += tot[j];
    uint32_t x = mysum;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t start = x - mysum;
#pragma unroll
    for (int i = 0; i < kSortWaves; ++i) start += i < w ? wsum[i] : 0u;
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        t_start[tid * kDigitsPerThread + j] = start;
        start += tot[j];
    }
    __syncthreads();
    // stage the tile in LDS in sorted (digit, item) order: every posting's position first (a permutation of [0, tile
    // items); kTile = not staged), then, once no wave reads the counters any more, the staging over them
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const uint32_t d = (key[s] >> shift) & (kDigits - 1);
        rank[s] = base + s * 64 + lane < n ? t_start[d] + cnt[w][d] + rank[s] : (uint32_t)kTile;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const uint32_t pos = rank[s];
        if (pos < kTile) {
            s_key[pos] = key[s];
            s_val[pos] = val[s];
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
        if (LAST) {
            // the run ends of the CSR, from the sorted tile itself (no key array is written): inside a digit run
            // the tile's items are in full key order (stable passes), so a key change there is the key's last
            // posting; the last item of a digit run may continue in a later tile, so it only raises E[k + 1]
            // (every end is an atomicMax, so the true end -- the largest -- wins whatever the order)
            if (k < (1u << 26)) {
                const bool run_end = i + 1 == m || ((s_key[i + 1] >> shift) & (kDigits - 1)) != d;
                if (run_end || s_key[i + 1] != k) atomicMax(&E[k + 1], (uint32_t)(dst + 1));
            }
            const uint64_t v = s_val[i];
            __builtin_nontemporal_store(v, &vals_out[dst]);
            sig_out[dst] = posting_sig((uint32_t)v, (uint32_t)(v >> 32));  // K5's 2-B vote signature
        } else {
            keys_out[dst] = k;
            vals_out[dst] = s_val[i];
        }
    }
}

// E[key + 1] = i + 1 at the last posting i of each live key's run (E zeroed by the caller); nz += number of
// live keys (one atomic per workgroup)
__global__ __launch_bounds__(256) void k_run_ends(const uint32_t *__restrict__ keys, int64_t n,
                                                  uint32_t *__restrict__ E, unsigned long long *__restrict__ nz) {
    __shared__ unsigned long long part[4];
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        if (k < (1u << 26) && (i == n - 1 || keys[i + 1] != k)) {
            E[k + 1] = (uint32_t)(i + 1);
            ++c;
        }
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(nz, part[0] + part[1] + part[2] + part[3]);
}

// ---- scans over u32 (8 items per thread, wave shuffles): exclusive sum (tile counts) and inclusive max
// (offsets from run ends). Level 1 per 8192-item block; the block totals are scanned recursively and folded
// back into every block.
constexpr int kScanThreads = 1024, kScanItems = 8, kScanBlock = kScanThreads * kScanItems;

template <bool MAX>
__device__ __forceinline__ uint32_t sop(uint32_t a, uint32_t b) { return MAX ? max(a, b) : a + b; }

// nzc (MAX only, or nullptr): += the number of nonzero inputs (the live keys, for the offsets scan over E)
template <bool MAX>
__global__ __launch_bounds__(kScanThreads) void k_scan8(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                       int64_t n, uint32_t *__restrict__ bsum,
                                                       unsigned long long *__restrict__ nzc) {
    __shared__ uint32_t ws[kScanThreads / 64];
    __shared__ uint32_t wnz[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t i0 = (int64_t)blockIdx.x * kScanBlock + (int64_t)tid * kScanItems;
    uint32_t v[kScanItems];
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) v[j] = i0 + j < n ? in[i0 + j] : 0u;
    if (MAX && nzc) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) c += v[j] != 0u;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (lane == 0) wnz[w] = c;
    }
    uint32_t incl[kScanItems];
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) incl[j] = acc = sop<MAX>(acc, v[j]);
    uint32_t x = acc;  // inclusive over the wave's threads
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x = sop<MAX>(x, y);
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = __shfl_up(x, 1, 64);  // over the threads before this one in the wave
    if (lane == 0) pre = 0;
    for (int i = 0; i < w; ++i) pre = sop<MAX>(pre, ws[i]);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j)
        if (i0 + j < n) out[i0 + j] = MAX ? sop<MAX>(pre, incl[j]) : pre + incl[j] - v[j];
    if (tid == kScanThreads - 1) {
        uint32_t t = 0;
        for (int i = 0; i < kScanThreads / 64; ++i) t = sop<MAX>(t, ws[i]);
        bsum[blockIdx.x] = t;
        if (MAX && nzc) {
            unsigned long long c = 0;
            for (int i = 0; i < kScanThreads / 64; ++i) c += wnz[i];
            atomicAdd(nzc, c);
        }
    }
}

// out[block b + 1] op= add[b] (the caller offsets `out` by one block when `add` is an inclusive scan)
template <bool MAX>
__global__ __launch_bounds__(kScanThreads) void k_scan8_add(uint32_t *__restrict__ out, int64_t n,
                                                           const uint32_t *__restrict__ add) {
    const uint32_t a = add[blockIdx.x];
    const int64_t i0 = (int64_t)blockIdx.x * kScanBlock;
    for (int j = threadIdx.x; j < kScanBlock; j += kScanThreads)
        if (i0 + j < n) out[i0 + j] = sop<MAX>(a, out[i0 + j]);
}

// scratch u32 a scan of n needs (its block totals and their scan, recursively)
static size_t scan8_tmp(int64_t n) {
    size_t t = 8;
    for (int64_t m = n; m > kScanBlock;) {
        m = (m + kScanBlock - 1) / kScanBlock;
        t += 2 * (size_t)m + 8;
    }
    return t;
}

// MAX = false: exclusive sum; MAX = true: inclusive max
template <bool MAX>
static void scan8(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t s,
                  unsigned long long *nzc = nullptr) {
    if (n <= 0) return;
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    uint32_t *bsum = tmp, *boff = tmp + nb;
    hipLaunchKernelGGL(k_scan8<MAX>, dim3((unsigned)nb), dim3(kScanThreads), 0, s, in, out, n, bsum, nzc);
    if (nb > 1) {
        scan8<MAX>(bsum, boff, nb, tmp + 2 * nb + 8, s);
        if (MAX)  // boff = inclusive max of the block maxima: block b + 1 takes boff[b]
            hipLaunchKernelGGL(k_scan8_add<MAX>, dim3((unsigned)(nb - 1)), dim3(kScanThreads), 0, s, out + kScanBlock,
                               n - kScanBlock, (const uint32_t *)boff);
        else      // boff = exclusive sum of the block totals: block b takes boff[b]
            hipLaunchKernelGGL(k_scan8_add<MAX>, dim3((unsigned)nb), dim3(kScanThreads), 0, s, out, n,
                               (const uint32_t *)boff);
    }
}

// ---- the device property ARANK relies on, checked once per device before the first build that would use it ----
// The probe issues the scatter's own pattern: every wave of three resident 256-thread workgroups per CU
// adds 1 to its own 512 LDS counters kSlots times back to back (one item per lane per slot, no barrier between the
// atomics), with digit patterns from all-distinct to all-equal mixed across the slots; then every item's old value
// must equal the number of earlier items (slot by slot, lanes in lane order) of the wave with the same digit -- the
// stable rank k_radix_scatter<ARANK> takes from it. *viol counts the items that do not (0 on gfx950:
// profiles/r05n_lds_atomic_order.json for the one-atomic form of this probe)
__global__ __launch_bounds__(kSortThreads, 3) void k_lds_lane_order(uint32_t *__restrict__ viol) {
    __shared__ uint32_t cnt[kSortWaves][kDigits];
    __shared__ uint16_t dig[kSortWaves][kSlots][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t v = 0;
    for (int r = 0; r < 4; ++r) {
        for (int i = threadIdx.x; i < kSortWaves * kDigits; i += kSortThreads) (&cnt[0][0])[i] = 0u;
        __syncthreads();
        uint32_t d[kSlots], old[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            uint32_t x = (blockIdx.x * 0x9E3779B9u) ^ ((r * kSlots + s) * 0x85EBCA6Bu) ^ (w * 0xC2B2AE35u) ^
                         (lane * 0x27D4EB2Fu);
            x ^= x >> 15;
            x *= 0x2C1B3C6Du;
            x ^= x >> 12;
            const int p = (s + r + (int)blockIdx.x) & 3;
            d[s] = p == 0 ? x & (kDigits - 1) : p == 1 ? x & 3u : p == 2 ? 5u : (x & 1u) ? (x >> 1) & 7u : 300u;
        }
#pragma unroll
        for (int s = 0; s < kSlots; ++s) old[s] = atomicAdd(&cnt[w][d[s]], 1u);  // back to back, as the scatter
#pragma unroll
        for (int s = 0; s < kSlots; ++s) dig[w][s][lane] = (uint16_t)d[s];
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            uint32_t want = 0;
            for (int s2 = 0; s2 <= s; ++s2)
                for (int l2 = 0; l2 < (s2 < s ? 64 : lane); ++l2) want += dig[w][s2][l2] == d[s] ? 1u : 0u;
            v += old[s] != want ? 1u : 0u;
        }
        __syncthreads();
    }
    if (v) atomicAdd(viol, v);
}

// 1 = ds_add_rtn serves same-address lanes in ascending lane order on this device, 0 = not, <0 = the check failed
static int lds_lane_order_ok(uint32_t *dev_word, hipStream_t s) {
    static std::atomic<int> state[64];  // per device: 0 unknown, 1 ok, 2 not ok
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    const int st = state[dev].load();
    if (st) return st == 1 ? 1 : 0;
    if (hipMemsetAsync(dev_word, 0, sizeof(uint32_t), s) != hipSuccess) return -1;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipLaunchKernelGGL(k_lds_lane_order, dim3((unsigned)(3 * std::max(cus, 1))), dim3(kSortThreads), 0, s, dev_word);
    uint32_t viol = 1;
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(&viol, dev_word, sizeof(viol), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    state[dev].store(viol == 0 ? 1 : 2);
    return viol == 0 ? 1 : 0;
}

// ---- rocPRIM reference build (A/B only, in the AID_K4_ROCPRIM_AB variant build) ----
#ifdef AID_K4_ROCPRIM_AB
__global__ void k_sort_keys(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack,
                            const uint32_t *__restrict__ pt, int64_t n, const uint8_t *__restrict__ tomb,
                            uint32_t n_tracks, uint32_t *__restrict__ keys, uint64_t *__restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t tr = ptrack[i];
        keys[i] = make_key(ph[i], tr, tomb, n_tracks);
        vals[i] = (uint64_t)tr | ((uint64_t)pt[i] << 32);
    }
}
#endif

void launch_make_sig(const uint64_t *post, int64_t n, uint16_t *sig, hipStream_t s);  // index.hip

int64_t radix_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

// scratch of the sort build in u32 units: the tile counts, their scan, and the scans' temporaries
size_t radix_scratch_u32(int64_t n) {
    const int64_t c = (int64_t)kDigits * radix_tiles(n);
    return (size_t)(2 * c) +
           std::max<size_t>(2 * (size_t)kDigits * (col_groups(radix_tiles(n)) + 1), scan8_tmp((int64_t)(1u << 26) + 1)) +
           64;
}

// temporary storage of the rocPRIM sort for n pairs
size_t index_sort_temp_bytes(int64_t n) {
#ifdef AID_K4_ROCPRIM_AB
    size_t bytes = 0;
    rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
    rocprim::double_buffer<uint64_t> v(nullptr, nullptr);
    if (rocprim::radix_sort_pairs(nullptr, bytes, k, v, (size_t)n, 0, kSortKeyBits) != hipSuccess) return 0;
    return bytes;
#else
    (void)n;
    return 0;
#endif
}

bool k4_ab_sort_built() {
#ifdef AID_K4_ROCPRIM_AB
    return true;
#else
    return false;
#endif
}

// the three passes of the hand-written sort: SoA postings -> (keys1, vals1) -> (keys0, vals0) -> the CSR's values in
// vals1, its run ends in E and the K5 signatures in sig
template <bool ARANK>
static void radix_passes(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n, const uint8_t *tomb,
                         uint32_t n_tracks, uint32_t *keys0, uint32_t *keys1, uint64_t *vals0, uint64_t *vals1,
                         uint32_t *counts, uint32_t *offs, uint32_t *stmp, uint32_t *E, uint16_t *sig, int64_t tiles,
                         hipStream_t s) {
    // pass 1: SoA postings -> (keys1, vals1); pass 2: -> (keys0, vals0); pass 3: -> (keys1, vals1)
    const dim3 g((unsigned)tiles), b(kSortThreads);
    if (tomb) {
        timed_launch(k_radix_count<true, true>, g, b, 0, s, ph, ptrack, tomb, n_tracks, n, 0, counts, tiles);
        digit_starts(counts, tiles, offs, stmp, s);
        timed_launch(k_radix_scatter<true, false, true, ARANK>, g, b, 0, s, ph, (const uint64_t *)nullptr, ptrack, pt,
                     tomb, n_tracks, n, 0, (const uint32_t *)offs, tiles, keys1, vals1, (uint32_t *)nullptr,
                     (uint16_t *)nullptr);
    } else {
        timed_launch(k_radix_count<true, false>, g, b, 0, s, ph, ptrack, tomb, n_tracks, n, 0, counts, tiles);
        digit_starts(counts, tiles, offs, stmp, s);
        timed_launch(k_radix_scatter<true, false, false, ARANK>, g, b, 0, s, ph, (const uint64_t *)nullptr, ptrack, pt,
                     tomb, n_tracks, n, 0, (const uint32_t *)offs, tiles, keys1, vals1, (uint32_t *)nullptr,
                     (uint16_t *)nullptr);
    }
    timed_launch(k_radix_count<false>, g, b, 0, s, (const uint32_t *)keys1, (const uint32_t *)nullptr,
                 (const uint8_t *)nullptr, 0u, n, kDigitBits, counts, tiles);
    digit_starts(counts, tiles, offs, stmp, s);
    timed_launch(k_radix_scatter<false, false, false, ARANK>, g, b, 0, s, (const uint32_t *)keys1,
                 (const uint64_t *)vals1, (const uint32_t *)nullptr, (const uint32_t *)nullptr,
                 (const uint8_t *)nullptr, 0u, n, kDigitBits, (const uint32_t *)offs, tiles, keys0, vals0,
                 (uint32_t *)nullptr, (uint16_t *)nullptr);
    timed_launch(k_radix_count<false>, g, b, 0, s, (const uint32_t *)keys0, (const uint32_t *)nullptr,
                 (const uint8_t *)nullptr, 0u, n, 2 * kDigitBits, counts, tiles);
    digit_starts(counts, tiles, offs, stmp, s);
    timed_launch(k_radix_scatter<false, true, false, ARANK>, g, b, 0, s, (const uint32_t *)keys0,
                 (const uint64_t *)vals0, (const uint32_t *)nullptr, (const uint32_t *)nullptr,
                 (const uint8_t *)nullptr, 0u, n, 2 * kDigitBits, (const uint32_t *)offs, tiles,
                 (uint32_t *)nullptr,
                 vals1, E, sig);
}

// keys0/keys1: n u32 each; vals0/vals1: n u64 each (the sorted values end in *vals_out, one of the two).
// E (2^26 + 1 u32, zeroed by the caller) receives the run ends, offsets the CSR offsets, *nz (zeroed) the
// number of live keys. use_rocprim: the A/B reference (temp/temp_bytes its storage); `scratch` holds
// radix_scratch_u32(n) u32 either way (the offsets scan uses it too).
hipError_t launch_index_sort_build(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                                   const uint8_t *tomb, uint32_t n_tracks, uint32_t *keys0, uint32_t *keys1,
                                   uint64_t *vals0, uint64_t *vals1, void *temp, size_t temp_bytes, bool use_rocprim,
                                   uint32_t *scratch, uint32_t *E, uint32_t *offsets, unsigned long long *nz,
                                   uint64_t **vals_out, uint16_t *sig, int rank_mode, hipStream_t s) {
    *vals_out = vals0;
    const int64_t K = (int64_t)(1u << 26) + 1;
    const int64_t tiles = radix_tiles(n);
    const int64_t c = (int64_t)kDigits * tiles;
    uint32_t *stmp = scratch + 2 * c;
    const uint32_t *sorted_keys = nullptr;
    if (n > 0 && use_rocprim) {
#ifndef AID_K4_ROCPRIM_AB
        return hipErrorNotSupported;
#else
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
        hipLaunchKernelGGL(k_sort_keys, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptrack, pt, n, tomb, n_tracks,
                           keys0, vals0);
        rocprim::double_buffer<uint32_t> k(keys0, keys1);
        rocprim::double_buffer<uint64_t> v(vals0, vals1);
        size_t bytes = temp_bytes;
        hipError_t err = rocprim::radix_sort_pairs(temp, bytes, k, v, (size_t)n, 0, kSortKeyBits, s);
        if (err != hipSuccess) return err;
        sorted_keys = k.current();
        *vals_out = v.current();
#endif
    } else if (n > 0) {
        uint32_t *counts = scratch, *offs = scratch + c;
        // rank_mode 0: the one-atomic rank where the device serves same-address LDS lanes in order, 1: ballots
        bool arank = false;
        if (rank_mode == 0) {
            const int ok = lds_lane_order_ok(scratch + radix_scratch_u32(n) - 1, s);
            if (ok < 0) return hipErrorUnknown;
            arank = ok == 1;
        }
        if (arank)
            radix_passes<true>(ph, ptrack, pt, n, tomb, n_tracks, keys0, keys1, vals0, vals1, counts, offs, stmp, E, sig,
                               tiles, s);
        else
            radix_passes<false>(ph, ptrack, pt, n, tomb, n_tracks, keys0, keys1, vals0, vals1, counts, offs, stmp, E, sig,
                                tiles, s);
        *vals_out = vals1;
    }
#ifdef AID_K4_ROCPRIM_AB
    if (n > 0 && sorted_keys) {  // rocPRIM: run ends from its sorted keys, the signatures from its values
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
        hipLaunchKernelGGL(k_run_ends, dim3((unsigned)blocks), dim3(256), 0, s, sorted_keys, n, E, nz);
        launch_make_sig(*vals_out, n, sig, s);
    }
#endif
    // the hand-written sort wrote E in its last pass; its live keys are the nonzero E entries
    scan8<true>(E, offsets, K, stmp, s, sorted_keys ? nullptr : nz);
    return hipGetLastError();
}

}  // namespace aid
