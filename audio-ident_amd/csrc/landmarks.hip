// landmarks.hip -- K3 `landmark_hash`: peak compaction + anchor->target pairing +
// 32-bit hash pack (FPSPEC 5 ordering, FPSPEC 6 hashing).
//
// Replaces the hash stage inside the external `olaf_c` binary (SURVEY.md 8a row
// a3; reference call sites fingerprint.py:117-125, 185-193).
//
// Unit = (clip, chunk of kHashChunk anchor frames). A workgroup:
//   1. popcounts the 16 mask words of every frame in [c0, min(c1+63, F)) and
//      block-scans the counts (frame -> first peak index);
//   2. expands the masks into an LDS peak list packed (frame << 10 | bin), which
//      is already in (t, k) order -- exactly the target order of FPSPEC 6;
//   3. gives each thread a contiguous run of anchors; a thread walks forward from
//      each anchor while t2 - t1 <= 63 and keeps the first 10 targets with
//      |k2 - k1| <= 127.
// Pass COUNT writes the chunk's record total (only clips with more than one chunk
// need it; the host skips the launch when none has); pass WRITE re-derives its base
// from the totals of the clip's earlier chunks, block-scans per-thread totals and
// stores records {hash, t1} in canonical order. Chunk 0 of a clip also writes the
// clip's record count.
#include "aidfp_device.h"

namespace aid {

constexpr int kK3 = 512;  // threads per K3 workgroup (256: 0.055 ms, 512: 0.040, 1024: 0.040 at 256 x 10 s)

// exclusive scan of one int64 per thread: wave scans (shuffles) + one LDS exchange of the wave totals
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t *tmp /*[kK3]*/, int64_t *total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int64_t x = v;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) tmp[w] = x;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kK3 / 64; ++i) {
        const int64_t t = tmp[i];
        base += i < w ? t : 0;
        tot += t;
    }
    if (total) *total = tot;
    __syncthreads();  // every wave has read tmp before the next scan writes it
    return base + x - v;
}

__device__ __forceinline__ uint32_t make_hash(int k1, int k2, int dt) {
    return ((uint32_t)(k1 & 0x3FF) << 22) | ((uint32_t)(k2 & 0x3FF) << 12) | ((uint32_t)dt & 0xFFF);
}

template <bool WRITE>
__global__ __launch_bounds__(kK3) void k_landmarks(const uint64_t *__restrict__ mask, const ClipDesc *__restrict__ clips,
                                                  int n_clips, int64_t total_chunks, int64_t *__restrict__ chunk_counts,
                                                  uint64_t *__restrict__ records, int64_t *__restrict__ clip_counts,
                                                  uint32_t *__restrict__ k2_cold, uint64_t *__restrict__ k2_cold_host,
                                                  uint32_t k2_waves, int one_chunk_each) {
    __shared__ uint32_t plist[kHashChunkPeakCap];
    __shared__ uint32_t foff[kHashChunk + kZoneDT + 2];
    __shared__ int64_t scan_tmp[kK3];
    const int tid = threadIdx.x;
    const int64_t chunk = blockIdx.x;
    if (WRITE && k2_cold && blockIdx.x == 0 && tid < 64) {
        // K2's strip-cold wave count (peaks.hip) and the wave count of that same launch, stored together as
        // one 8-byte word in host-mapped memory for the next call's strip sizing (no sync: a stale pair only
        // delays the adaptation), then the counters are reset for the next K2
        uint32_t c = k2_cold[tid];
        k2_cold[tid] = 0u;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (tid == 0) *reinterpret_cast<volatile uint64_t *>(k2_cold_host) = (uint64_t)c | ((uint64_t)k2_waves << 32);
    }
    if (chunk >= total_chunks) return;
    int lo = 0, hi = n_clips - 1;
    if (one_chunk_each) lo = (int)chunk;  // every clip is exactly one chunk (host-checked): no search
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].chunk_base <= chunk) lo = mid; else hi = mid - 1;
    }
    const ClipDesc cd = clips[lo];
    const int64_t F = cd.frames;
    const int64_t q = chunk - cd.chunk_base;
    const int64_t c0 = q * kHashChunk;
    const int64_t c1 = min(c0 + (int64_t)kHashChunk, F);
    const int64_t g1 = min(c1 + (int64_t)kZoneDT, F);
    const int nf = (int)(g1 - c0);
    const uint64_t *Mc = mask + (cd.frame_base + c0) * kMaskWords;
    const int64_t nck = (F + kHashChunk - 1) / kHashChunk;
    if (!WRITE && nck == 1) return;  // single-chunk clips: the WRITE pass needs no base

    // 1. per-frame counts over a contiguous run of frames per thread, block scan
    const int per = (nf + kK3 - 1) / kK3;
    const int fa = min(tid * per, nf), fz = min(fa + per, nf);
    int64_t mine = 0;
    for (int f = fa; f < fz; ++f) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kMaskWords; ++w) c += __popcll(Mc[f * kMaskWords + w]);
        foff[f] = c;
        mine += c;
    }
    int64_t npk = 0;
    int64_t run = block_excl_scan(mine, scan_tmp, &npk);
    // 2. expand to the (t,k)-ordered peak list
    for (int f = fa; f < fz; ++f) {
        const uint32_t c = foff[f];
        foff[f] = (uint32_t)run;
        // most frames hold no peak (~0.35 per frame at the bench config): skip their mask reload
        if (c == 0) continue;
        int64_t idx = run;
        uint64_t W[kMaskWords];
#pragma unroll
        for (int w = 0; w < kMaskWords; ++w) W[w] = Mc[f * kMaskWords + w];
        // no unshuffle: a 4-bin group holds at most one peak (FPSPEC 5: no two peaks within +-15 bins), so the
        // OR of a 256-bin block's 4 ballot words has one bit per peak, in ascending bin order; the word
        // holding that bit gives the bin's offset i in the group (bin = 256 b + 4 l + i)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t w1 = W[4 * b + 1], w2 = W[4 * b + 2], w3 = W[4 * b + 3];
            for (uint64_t m = W[4 * b] | w1 | w2 | w3; m; m &= m - 1) {
                const int l = __ffsll((unsigned long long)m) - 1;
                const int i = (int)((w1 >> l) & 1) + 2 * (int)((w2 >> l) & 1) + 3 * (int)((w3 >> l) & 1);
                plist[idx++] = ((uint32_t)f << 10) | (uint32_t)(256 * b + 4 * l + i);
            }
        }
        run += c;
    }
    if (tid == 0) foff[nf] = (uint32_t)npk;
    __syncthreads();
    const int n_anchor = (int)foff[c1 - c0];

    // 3. anchors: contiguous run per thread
    const int pa_per = (n_anchor + kK3 - 1) / kK3;
    const int aa = min(tid * pa_per, n_anchor), az = min(aa + pa_per, n_anchor);
    int64_t my = 0;
    // the thread's first anchor keeps its accepted targets as a bitmask of walk positions j - i - 1 < 64,
    // so the write pass emits them without walking the zone again
    uint64_t tmask = 0;
    bool tmask_ok = false;
    for (int i = aa; i < az; ++i) {
        const uint32_t a = plist[i];
        const int ta = (int)(a >> 10), ka = (int)(a & 1023);
        int got = 0;
        uint64_t mk = 0;
        bool ok = true;
        for (int j = i + 1; j < (int)npk && got < kFan; ++j) {
            const uint32_t b = plist[j];
            const int dt = (int)(b >> 10) - ta;
            if (dt > kZoneDT) break;
            if (dt <= 0) continue;
            const int df = (int)(b & 1023) - ka;
            if (df < -kZoneDF || df > kZoneDF) continue;
            if (j - i - 1 < 64) mk |= 1ull << (j - i - 1);
            else ok = false;
            ++got;
        }
        if (i == aa) {
            tmask = mk;
            tmask_ok = ok;
        }
        my += got;
    }
    int64_t chunk_total = 0;
    const int64_t excl = block_excl_scan(my, scan_tmp, &chunk_total);
    if constexpr (!WRITE) {
        if (tid == 0) chunk_counts[chunk] = chunk_total;
    } else {
        int64_t before = 0;
        if (nck == 1) {
            if (tid == 0) clip_counts[lo] = chunk_total;
        } else {
            // base of this chunk inside the clip = sum of the clip's earlier chunks
            int64_t pre = 0;
            for (int64_t c = cd.chunk_base + tid; c < chunk; c += kK3) pre += chunk_counts[c];
            block_excl_scan(pre, scan_tmp, &before);
            if (q == 0) {
                int64_t all = 0;
                for (int64_t c = cd.chunk_base + tid; c < cd.chunk_base + nck; c += kK3) all += chunk_counts[c];
                int64_t tot = 0;
                block_excl_scan(all, scan_tmp, &tot);
                if (tid == 0) clip_counts[lo] = tot;
            }
        }
        uint64_t *out = records + cd.hash_base + before + excl;
        int64_t o = 0;
        for (int i = aa; i < az; ++i) {
            const uint32_t a = plist[i];
            const int ta = (int)(a >> 10), ka = (int)(a & 1023);
            const uint64_t t1 = (uint64_t)(c0 + ta) << 32;
            if (i == aa && tmask_ok) {
                for (uint64_t m = tmask; m; m &= m - 1) {
                    const uint32_t b = plist[i + 1 + (__ffsll((unsigned long long)m) - 1)];
                    out[o++] = t1 | make_hash(ka, (int)(b & 1023), (int)(b >> 10) - ta);
                }
                continue;
            }
            int got = 0;
            for (int j = i + 1; j < (int)npk && got < kFan; ++j) {
                const uint32_t b = plist[j];
                const int dt = (int)(b >> 10) - ta;
                if (dt > kZoneDT) break;
                if (dt <= 0) continue;
                const int kb = (int)(b & 1023);
                const int df = kb - ka;
                if (df < -kZoneDF || df > kZoneDF) continue;
                out[o++] = t1 | make_hash(ka, kb, dt);
                ++got;
            }
        }
    }
}

void launch_landmarks(const uint64_t *mask, const ClipDesc *clips, int n_clips, int64_t total_chunks,
                      int64_t *chunk_counts, uint64_t *records, int64_t *clip_counts, bool write, uint32_t *k2_cold,
                      uint64_t *k2_cold_host, uint32_t k2_waves, bool one_chunk_each, hipStream_t s) {
    if (total_chunks <= 0) return;
    if (write)
        timed_launch(k_landmarks<true>, dim3((unsigned)total_chunks), dim3(kK3), 0, s, mask, clips, n_clips,
                           total_chunks, chunk_counts, records, clip_counts, k2_cold, k2_cold_host, k2_waves,
                     one_chunk_each ? 1 : 0);
    else
        timed_launch(k_landmarks<false>, dim3((unsigned)total_chunks), dim3(kK3), 0, s, mask, clips, n_clips,
                           total_chunks, chunk_counts, records, clip_counts, (uint32_t *)nullptr, (uint64_t *)nullptr, 0u,
                     one_chunk_each ? 1 : 0);
}

}  // namespace aid
