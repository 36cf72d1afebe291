// synth.hip -- device generator of the deterministic synthetic PCM that
// audio-ident_amd/aidfp/synth.py defines (integer-exact, so both agree bit for
// bit). Used to put the benchmark and ingest catalogs straight into HBM
// ("generated on device").
#include "aidfp_device.h"

namespace aid {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t rnd(uint32_t track_key /* mix(track + seed*phi) */, uint32_t stream, uint32_t idx) {
    return mix32(mix32(track_key + stream * 0x85EBCA6Bu) + idx);
}

struct SynthParams {
    int64_t n;          // samples per clip
    int32_t note_len;   // sr / 4
    uint32_t inc_min, inc_rng;
    int32_t noise_a;    // query noise half-width (0 = none)
    uint32_t salt;
    uint32_t seed_mul;  // (SEED * 0x9E3779B9) mod 2^32
    int32_t envelope;   // 1: generator v2 (per-track tempo, per-partial onsets, decaying notes); 0: v0 (stationary,
                        // one 250 ms grid)
};

__global__ __launch_bounds__(256) void k_synth(float *__restrict__ out, const uint32_t *__restrict__ tracks,
                                              const int64_t *__restrict__ starts, int n_clips, SynthParams sp,
                                              const int16_t *__restrict__ sin_tab) {
    const int64_t per_clip_blocks = (sp.n + 255) / 256;
    const int64_t c = blockIdx.x / per_clip_blocks;
    if (c >= n_clips) return;
    const int64_t i_local = (blockIdx.x % per_clip_blocks) * 256 + threadIdx.x;
    if (i_local >= sp.n) return;
    const uint32_t tr = tracks[c];
    const int64_t i = starts[c] + i_local;
    const uint32_t key = mix32(tr + sp.seed_mul);
    // generator v2 (aidfp/synth.py): the track's tempo and each partial's onset phase; v0: one 250 ms grid
    const uint32_t nl = sp.envelope ? ((uint32_t)sp.note_len * (12u + rnd(key, 40, 0) % 9u)) / 16u : (uint32_t)sp.note_len;
    // sample indices below 2^31 take 32-bit divisions (a 64-bit one is a long software sequence)
    const bool narrow = i + (int64_t)nl < 0x80000000ll;
    int32_t acc = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const uint32_t off = sp.envelope ? (uint32_t)(((uint64_t)nl * (rnd(key, p + 32, 0) % 1024u)) >> 10) : 0u;
        const int64_t ip = i + off;
        const int64_t j = narrow ? (int64_t)((uint32_t)ip / nl) : ip / (int64_t)nl;
        const uint32_t rel = (uint32_t)(ip - j * (int64_t)nl);
        const uint32_t r = rnd(key, p, (uint32_t)j);
        const uint32_t inc = sp.inc_min + (uint32_t)(((uint64_t)r * sp.inc_rng) >> 32);
        int32_t amp = 983 + (int32_t)(rnd(key, p + 8, (uint32_t)j) % 2949u);
        // note envelope (Q16): 65536 at the onset down to ~32768 at the note's end
        if (sp.envelope) amp = (amp * (65536 - (int32_t)((rel * 32768u) / nl))) >> 16;  // rel < nl < 2^17
        const uint32_t ph = rnd(key, p + 16, (uint32_t)j) + inc * rel;
        acc += (amp * (int32_t)sin_tab[ph >> 20]) >> 15;
    }
    acc += (int32_t)(rnd(key, 24, (uint32_t)i) % 1137u) - 568;
    if (sp.noise_a > 0) {
        const uint32_t key2 = mix32((tr ^ sp.salt) + sp.seed_mul);
        acc += (int32_t)(rnd(key2, 25, (uint32_t)i) % (uint32_t)(2 * sp.noise_a + 1)) - sp.noise_a;
    }
    acc = acc < -32768 ? -32768 : (acc > 32767 ? 32767 : acc);
    out[c * sp.n + i_local] = (float)acc / 32768.0f;
}

void launch_synth(float *out, const uint32_t *tracks, const int64_t *starts, int n_clips, int64_t n, int sr,
                  int noise_a, uint32_t salt, int fmax_hz, bool envelope, const int16_t *sin_tab, hipStream_t s) {
    if (n <= 0 || n_clips <= 0) return;
    SynthParams sp;
    sp.n = n;
    sp.note_len = sr / 4;
    sp.inc_min = (uint32_t)floor(100.0 / sr * 4294967296.0);
    sp.inc_rng = (uint32_t)floor((double)(fmax_hz - 100) / sr * 4294967296.0);  // partials in [100, fmax_hz) Hz
    sp.noise_a = noise_a;
    sp.salt = salt;
    sp.seed_mul = (uint32_t)((42ull * 0x9E3779B9ull) & 0xFFFFFFFFull);
    sp.envelope = envelope ? 1 : 0;
    const int64_t blocks = (int64_t)n_clips * ((n + 255) / 256);
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(256), 0, s, out, tracks, starts, n_clips, sp, sin_tab);
}

}  // namespace aid
