// aidfp_layout.h -- HBM layout constants shared by host (engine.cpp) and kernels.
#pragma once
#include <stdint.h>

namespace aid {

constexpr int kN = 2048;          // FFT length (FPSPEC 1)
constexpr int kBins = 1024;       // bins kept per frame
constexpr int kPeakDT = 7;        // peak neighbourhood, frames
constexpr int kPeakDF = 15;       // peak neighbourhood, bins
constexpr int kZoneDT = 63;       // target zone, frames
constexpr int kZoneDF = 127;      // target zone, bins
constexpr int kFan = 10;          // targets per anchor
constexpr int kMaskWords = kBins / 64;  // 16 x u64 peak bitmask per frame

// K1: kStftWaves waves per workgroup, one workgroup per CU: 16 waves (4 per SIMD at <= 128 VGPRs),
// each with a private exchange buffer, + 24.5 KB of tables fit the 160 KB LDS
constexpr int kStftWaves = 16;
constexpr int kStftStrip = 16;   // frames per wave at least, for large batches (one ring fill per range)
constexpr int kK1MinFrames = 2;  // frames per wave at least, for small batches
// float2 entries of a wave's exchange buffer: E1's 32 regions of 64 dwords at shifted bases (2108 dwords),
// then E3's 1024 values in 32-B groups + the copy of Z[768] at slot 1026 and the lanes' dummy slots
constexpr int kStftLdsPerWave = 1092;

// K2: output frames per workgroup strip, sized per call (peak_strip_len) between these bounds
constexpr int kPeakStripMin = 16;
// ... and at most this long: K2 reads a strip's rows through one buffer descriptor with a 32-bit byte range
// (peaks.hip), (kPeakStripMax + 2 x 7) rows x 4 KiB < 2^31
constexpr int kPeakStripMax = 65536;

// Smallest strip length L >= kPeakStripMin with sum_c ceil(F_c / L) <= slots (the resident K2
// workgroups of the device): every strip then runs in the first (only) round. When the clips
// alone outnumber the slots, L = max F (one strip per clip).
inline int peak_strip_len(const int64_t *frames, int n, int64_t slots) {
    int64_t fmax = 0;
    for (int c = 0; c < n; ++c) fmax = frames[c] > fmax ? frames[c] : fmax;
    auto count = [&](int64_t L) {
        int64_t k = 0;
        for (int c = 0; c < n; ++c) k += (frames[c] + L - 1) / L;
        return k;
    };
    int64_t lo = kPeakStripMin, hi = fmax > lo ? fmax : lo;
    if (hi > kPeakStripMax) hi = kPeakStripMax;  // longer clips take several strips (more than one round)
    if (count(lo) <= slots) return (int)lo;
    while (lo < hi) {  // count(L) is non-increasing in L
        const int64_t mid = (lo + hi) / 2;
        if (count(mid) <= slots) hi = mid; else lo = mid + 1;
    }
    return (int)lo;
}

// K1 -> K2 hot word of a power row (u64): bit hot_bit(c) is set when some bin of the 16-bin chunk c
// (bins 16c .. 16c+15) is > thr. Chunks below 32 map to bit c, the others to bit 95 - c: the order in
// which K1's lanes hold the mirror bins 1024 - k (stft.hip), so K1 builds the word with two s_quadmask
// per register and no bit shuffling.
constexpr int hot_bit(int c) { return c < 32 ? c : 95 - c; }

// K4/K5 CSR bucket of a landmark hash (FPSPEC 6: k1 = h >> 22, k2 = (h >> 12) & 1023, dt = h & 63, the 26 bits a
// hash can set). Any bijection of (k1, k2, dt) gives the same index; the bit order only places the buckets, and is
// chosen for the radix build (index_sort.hip, 3 passes of 9-bit digits): on band-limited audio the high bits of k1
// and k2 are nearly constant, so each digit takes a share of the low (busy) bits -- bits 0..5 dt, 6..8 k2[7..9],
// 9..15 k2[0..6], 16..17 k1[8..9], 18..25 k1[0..7]. Distinct digits (= output runs) per 4096-posting tile on the
// synthetic catalog: 189 / 213 / 171 per pass, against 493 / 187 / 89 for k1 << 16 | k2 << 6 | dt, whose first
// pass wrote ~8-posting runs (partial lines) and took twice the time of the others.
__host__ __device__ constexpr uint32_t bucket_key(uint32_t h) {
    return (((h >> 22) & 0xFFu) << 18) | ((h >> 30) << 16) | (((h >> 12) & 0x7Fu) << 9) | (((h >> 19) & 0x7u) << 6) |
           (h & 0x3Fu);
}

// K5 posting signature (2 B per posting, stored beside the CSR's 8-B posting by K4): sig = H(track) + t mod 2^16.
// A query's vote on that posting has d = t - tq, so (sig - tq) mod 2^16 = H(track) + d mod 2^16 is a hash of
// (track, d) that needs neither of them: the LDS match path counts its votes from the 2-B signatures alone and
// reads the 8-B posting only for votes whose bucket turns out hot (any hash keeps the filter an exact superset).
__host__ __device__ constexpr uint16_t posting_sig(uint32_t track, uint32_t t) {
    return (uint16_t)(((track * 0x9E3779B1u) >> 16) + t);
}

// K5: the heaviest query (exact votes, k_query_votes) the LDS match path takes; heavier ones go straight to the
// global-histogram path (engine.cpp run_queries routes them, k_match_lds hands any back at once). 4 votes per
// counter of its 2^16-bucket filter (2^15 8-bit counters before round 6, 8 per counter): on config 4 (~84.5 k votes per window, a few up to ~2^18) every query stays in
// LDS, where the 132 of 36,864 heaviest ones had cost 0.3 ms per 4096-clip call on the global path at 2^17.
constexpr int64_t kLdsMaxVotes = (int64_t)1 << 18;

// K3: anchor frames per chunk; peaks in (chunk + zone) frames fit LDS
constexpr int kHashChunk = 1024;
constexpr int kHashChunkPeakCap = 64 * ((kHashChunk + kZoneDT + 7) / 8);

inline int64_t num_frames(int64_t n, int hop) { return (hop <= 0 || n < kN) ? 0 : 1 + (n - kN) / hop; }
inline int64_t peak_capacity(int64_t F) { return 64 * ((F + 7) / 8); }
inline int64_t hash_capacity(int64_t F) { return kFan * peak_capacity(F); }

// Per-clip descriptor uploaded with each extraction call (struct of 8 x int64).
struct ClipDesc {
    int64_t pcm_off;     // first sample of the clip in the PCM buffer (odd: 4-byte aligned float2 loads)
    int64_t frames;      // F
    int64_t frame_base;  // first row of the clip in the power plane / mask plane
    int64_t strip_base;  // first K2 strip of the clip
    int64_t chunk_base;  // first K3 chunk of the clip
    int64_t hash_base;   // first record slot of the clip in the output buffer
    int64_t hash_cap;    // record capacity of the clip
    int64_t stft_base;   // first K1 wave-strip of the clip
};

}  // namespace aid
