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

// K1: kStftWaves waves per workgroup, one workgroup per CU. With stage C on DPP (no E2) the
// exchange buffer is an unpadded, XOR-swizzled 8 KB per wave, so 16 waves (4 per SIMD at
// <= 128 VGPRs) + 24.5 KB of tables fit the 160 KB LDS: K1 0.383 -> 0.366 ms over 14 padded waves
#ifndef AID_STFT_WAVES
#define AID_STFT_WAVES 16
#endif
constexpr int kStftWaves = AID_STFT_WAVES;
constexpr int kStftStrip = 16;
#ifndef AID_K1_MIN_FRAMES
#define AID_K1_MIN_FRAMES 2  // frames per K1 wave when the batch has fewer than 16 per resident wave
#endif
constexpr int kK1MinFrames = AID_K1_MIN_FRAMES;
constexpr int kK1DummyRows = 256;
constexpr int kK2SinkBlocks = 1024;  // K2 mask-store sinks: 256 u64 per workgroup index mod 1024 (2 MB)  // K1 cold-block store sinks (one 8 KB row per workgroup index mod 256)
#ifndef AID_K1_COMPACT
#define AID_K1_COMPACT 1
#endif
#ifndef AID_K1_E1ADDTID
#define AID_K1_E1ADDTID 1  // K1 0.2644 -> 0.2577 ms, 6.10 -> 6.21 M audio-s/s same-box (r02)
#endif
// float2 entries (E1: 16x68, E2: 64x17, E3: 1024; E1 by ds_write_addtid: 32 regions of 64 dwords at
// shifted bases, 2160 dwords -- see stft.hip)
#ifndef AID_K1_E3Q
#define AID_K1_E3Q 1  // K1 -0.5 % / -0.3 % in two same-box A/Bs (r02). stft.hip: E3 slots in 32-B groups of Z[k + 256 j2] (+64 dummy slots for one copy store)
#endif
constexpr int kStftLdsPerWave = AID_K1_E3Q ? 1092 : AID_K1_E1ADDTID ? 1080 : AID_K1_COMPACT ? 1024 : 1088;

// K2: output frames per workgroup strip, sized per call (peak_strip_len) between these bounds
#ifndef AID_PEAK_STRIP_MIN
#define AID_PEAK_STRIP_MIN 16  // shorter strips re-read more halo (14 rows per strip); only batches with fewer
                               // than ~64 frames per resident K2 slot get them (a streaming window: 465 frames)
#endif
constexpr int kPeakStripMin = AID_PEAK_STRIP_MIN;

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
    if (count(lo) <= slots) return (int)lo;
    while (lo < hi) {  // count(L) is non-increasing in L
        const int64_t mid = (lo + hi) / 2;
        if (count(mid) <= slots) hi = mid; else lo = mid + 1;
    }
    return (int)lo;
}

// K3: anchor frames per chunk; peaks in (chunk + zone) frames fit LDS
#ifndef AID_HASH_CHUNK
#define AID_HASH_CHUNK 1024
#endif
constexpr int kHashChunk = AID_HASH_CHUNK;
constexpr int kHashChunkPeakCap = 64 * ((kHashChunk + kZoneDT + 7) / 8);

inline int64_t num_frames(int64_t n, int hop) { return (hop <= 0 || n < kN) ? 0 : 1 + (n - kN) / hop; }
inline int64_t peak_capacity(int64_t F) { return 64 * ((F + 7) / 8); }
inline int64_t hash_capacity(int64_t F) { return kFan * peak_capacity(F); }

// Per-clip descriptor uploaded with each extraction call (struct of 8 x int64).
struct ClipDesc {
    int64_t pcm_off;     // first sample of the clip in the PCM buffer (even)
    int64_t frames;      // F
    int64_t frame_base;  // first row of the clip in the power plane / mask plane
    int64_t strip_base;  // first K2 strip of the clip
    int64_t chunk_base;  // first K3 chunk of the clip
    int64_t hash_base;   // first record slot of the clip in the output buffer
    int64_t hash_cap;    // record capacity of the clip
    int64_t stft_base;   // first K1 wave-strip of the clip
};

}  // namespace aid
