// index.hip -- K4 index build and K5 match_vote (FPSPEC 7).
//
// Replaces the LMDB inverted index of the external `olaf_c` binary: `store`
// (audio-ident-service/app/audio/fingerprint.py:117-125, single writer :7-8) and
// `query` + offset voting (:185-202), whose per-track best bin becomes
// OlafMatch.match_count (:44-50). SURVEY.md 8a rows a4, a5.
//
// Index (HBM): postings grouped by key26(hash) = bucket_key(hash) (aidfp_layout.h: a bit
// permutation of the 26 bits FPSPEC 6 can set, k1 | k2 | dt), as a direct-address CSR:
//   offsets u32[2^26 + 1]  (256 MB, one counting-sort pass, no comparison sort)
//   post    u64[n]         (track | t_ref << 32)
// Build = K4a count (one atomic per posting) -> exclusive scan -> K4b scatter.
// Within a bucket the posting order is arrival order; FPSPEC 7 results are
// order-independent sums/min/max, so queries are deterministic regardless.
//
// Query (one workgroup per query clip):
//   K5a  every vote (track, d = t_ref - t_q) increments a hashed per-query
//        histogram of 2^b u32 (exact superset filter: a (track, d) with
//        >= min_match votes has a bucket with >= min_match); b is sized by the
//        host from the index's mean bucket length and widened on overflow;
//   K5b  re-enumerates only votes whose bucket passed into an exact LDS hash
//        table {(track,d) -> count, tq_min, tq_max}, reduces best d per track
//        (max count, then smallest d) with 64-bit LDS atomics, ranks the rows
//        (count desc, track asc) and writes at most max_rows; it re-zeroes its
//        histogram row for the next batch.
#include "aidfp_device.h"

namespace aid {

constexpr int kKeyBits = 26;
constexpr uint32_t kKeys = 1u << kKeyBits;
constexpr int kVoteCap = 4096;   // LDS (track, d) entries per query
constexpr int kTrackCap = 1024;  // LDS per-track best entries per query
// linear-probe bound of the exact (track, d) tables: past it the table counts as overflowed and
// the query is re-run on more buckets (still exact). Probing a full 4096-slot table per vote had
// made an overflowing query cost ~100x a normal one.
constexpr int kProbeMax = 512;
constexpr int kDistinctBits = 13;  // k_vote_final's (slot, t_q) set in LDS (32 KB, shared with its row staging)
constexpr int kDistinctCap = 1 << kDistinctBits;
constexpr int kHotLdsBits = 17;  // K5b stages hot bitmap rows of up to 2^17 bits (16 KB) in LDS

__device__ __forceinline__ uint32_t key26(uint32_t h) { return bucket_key(h); }  // aidfp_layout.h

__device__ __forceinline__ uint32_t mix_td(uint32_t track, int32_t d) {
    uint32_t x = track * 0x9E3779B1u ^ ((uint32_t)d * 0x85EBCA77u);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return x;
}

// FPSPEC v1 7: a (track, d) scores the DISTINCT query anchor frames among its votes. The exact tables count a vote
// only when its (table slot, t_q) pair is new: an open-addressed LDS set of (slot << 20 | t_q) keys (t_q < 2^20 - 1,
// host-checked), whose first insert of a key returns true. A full set (more probes than entries) reports overflow:
// the query is answered again on a larger table, as for the (track, d) tables themselves.
constexpr uint32_t kDistinctEmpty = 0xFFFFFFFFu;
__device__ __forceinline__ bool distinct_first(uint32_t *set, int bits, uint32_t slot, uint32_t tq, int32_t *overflow) {
    const uint32_t key = (slot << 20) | tq, mask = (1u << bits) - 1;
    uint32_t i = (key * 0x9E3779B1u) >> (32 - bits);
    for (uint32_t probes = 0; probes <= mask; ++probes) {
        const uint32_t old = atomicCAS(&set[i], kDistinctEmpty, key);
        if (old == kDistinctEmpty) return true;
        if (old == key) return false;
        i = (i + 1) & mask;
    }
    atomicMax(overflow, 3);  // K5 fallback reason 3: the distinct set is full
    return false;
}

// ---- K4: build ----
__global__ void k_index_count(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack, int64_t n,
                              const uint8_t *__restrict__ tomb, uint32_t n_tracks, uint32_t *__restrict__ cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t tr = ptrack[i];
        if (tr < n_tracks && tomb[tr]) continue;
        atomicAdd(&cnt[key26(ph[i])], 1u);
    }
}

__global__ void k_index_scatter(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack,
                                const uint32_t *__restrict__ pt, int64_t n, const uint8_t *__restrict__ tomb,
                                uint32_t n_tracks, uint32_t *__restrict__ cursor, uint64_t *__restrict__ post) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t tr = ptrack[i];
        if (tr < n_tracks && tomb[tr]) continue;
        const uint32_t pos = atomicAdd(&cursor[key26(ph[i])], 1u);
        post[pos] = (uint64_t)tr | ((uint64_t)pt[i] << 32);
    }
}

// exclusive scan of n u32 counts (n = k * 1024) -> out; block sums -> bsum
__global__ __launch_bounds__(1024) void k_scan_blocks(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                     uint32_t *__restrict__ bsum, int64_t n) {
    __shared__ uint32_t s[1024];
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint32_t v = i < n ? in[i] : 0u;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t a = threadIdx.x >= off ? s[threadIdx.x - off] : 0u;
        __syncthreads();
        s[threadIdx.x] += a;
        __syncthreads();
    }
    if (i < n) out[i] = s[threadIdx.x] - v;
    if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}

__global__ __launch_bounds__(1024) void k_scan_add(uint32_t *__restrict__ out, const uint32_t *__restrict__ boff,
                                                  int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    if (i < n) out[i] += boff[blockIdx.x];
}

void launch_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t s);

// K5's 2-B vote signatures of the CSR's postings (aidfp_layout.h posting_sig), for the builds that do not write
// them in their last pass (the atomic build and the rocPRIM A/B; the radix build fuses it)
__global__ __launch_bounds__(256) void k_make_sig(const uint64_t *__restrict__ post, int64_t n, uint16_t *__restrict__ sig) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = post[i];
        sig[i] = posting_sig((uint32_t)v, (uint32_t)(v >> 32));
    }
}

void launch_make_sig(const uint64_t *post, int64_t n, uint16_t *sig, hipStream_t s) {
    if (n <= 0) return;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_make_sig, dim3((unsigned)blocks), dim3(256), 0, s, post, n, sig);
}

// ---- posting compaction (aid_index_compact): drop the postings of removed tracks, order kept ----
// The store's LMDB delete (`olaf_c del`, fingerprint.py:239-246) frees the track's entries; here a
// removal only tombstones the track, and compaction reclaims its postings. 1024 postings per block.
__device__ __forceinline__ bool posting_live(const uint32_t *ptrack, int64_t i, int64_t n, const uint8_t *tomb,
                                             uint32_t n_tracks) {
    if (i >= n) return false;
    const uint32_t tr = ptrack[i];
    return !(tr < n_tracks && tomb[tr]);
}

__global__ __launch_bounds__(1024) void k_compact_count(const uint32_t *__restrict__ ptrack, int64_t n,
                                                        const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                        uint32_t *__restrict__ cnt) {
    __shared__ uint32_t s_w[16];
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t b = __ballot(posting_live(ptrack, i, n, tomb, n_tracks));
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = (uint32_t)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < 16; ++w) t += s_w[w];
        cnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void k_compact_scatter(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptrack,
                                                          const uint32_t *__restrict__ pt, int64_t n,
                                                          const uint8_t *__restrict__ tomb, uint32_t n_tracks,
                                                          const uint32_t *__restrict__ off, uint32_t *__restrict__ oh,
                                                          uint32_t *__restrict__ otrack, uint32_t *__restrict__ ot) {
    __shared__ uint32_t s_w[16];
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    const bool live = posting_live(ptrack, i, n, tomb, n_tracks);
    const uint64_t b = __ballot(live);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) s_w[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t base = off[blockIdx.x];
    for (int q = 0; q < w; ++q) base += s_w[q];
    if (live) {
        const uint32_t o = base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        oh[o] = ph[i];
        otrack[o] = ptrack[i];
        ot[o] = pt[i];
    }
}

void launch_compact(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n, const uint8_t *tomb,
                    uint32_t n_tracks, uint32_t *cnt, uint32_t *off, uint32_t *tmp, uint32_t *oh, uint32_t *otrack,
                    uint32_t *ot, hipStream_t s) {
    const int64_t nb = (n + 1023) / 1024;
    if (nb <= 0) return;
    hipLaunchKernelGGL(k_compact_count, dim3((unsigned)nb), dim3(1024), 0, s, ptrack, n, tomb, n_tracks, cnt);
    launch_scan(cnt, off, nb, tmp, s);
    hipLaunchKernelGGL(k_compact_scatter, dim3((unsigned)nb), dim3(1024), 0, s, ph, ptrack, pt, n, tomb, n_tracks, off,
                       oh, otrack, ot);
}

// extracted records of clip c -> postings (hash, track_ids[c], t) at dst_off[c]
__global__ void k_records_to_postings(const uint64_t *__restrict__ recs, const int64_t *__restrict__ src_off,
                                      const int64_t *__restrict__ counts, const int64_t *__restrict__ dst_off,
                                      const uint32_t *__restrict__ track_ids, int n_clips, uint32_t *__restrict__ ph,
                                      uint32_t *__restrict__ ptrack, uint32_t *__restrict__ pt) {
    const int c = blockIdx.y;
    if (c >= n_clips) return;
    const int64_t n = counts[c];
    const uint64_t *src = recs + src_off[c];
    const int64_t o = dst_off[c];
    const uint32_t tr = track_ids[c];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t r = src[i];
        ph[o + i] = (uint32_t)r;
        ptrack[o + i] = tr;
        pt[o + i] = (uint32_t)(r >> 32);
    }
}

// clips' posting counts -> their append offsets base + exclusive prefix, and the new posting total, in one
// workgroup (a batch is at most a few thousand clips): the append needs no host round trip for the counts
__global__ __launch_bounds__(1024) void k_append_offsets(const int64_t *__restrict__ counts, int n_clips, int64_t base,
                                                         int64_t *__restrict__ dst_off, int64_t *__restrict__ total) {
    __shared__ int64_t s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int64_t run = base;
    for (int c0 = 0; c0 < n_clips; c0 += 1024) {
        const int c = c0 + tid;
        const int64_t v = c < n_clips ? counts[c] : 0;
        int64_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        int64_t t = 0;  // wave 0: inclusive scan of the 16 wave sums
        if (w == 0) {
            t = lane < 16 ? s_w[lane] : 0;
            for (int d = 1; d < 16; d <<= 1) {
                const int64_t y = __shfl_up(t, d);
                if (lane >= d) t += y;
            }
        }
        __syncthreads();
        if (w == 0 && lane < 16) s_w[lane] = t;
        __syncthreads();
        if (c < n_clips) dst_off[c] = run + (w ? s_w[w - 1] : 0) + x - v;
        run += s_w[15];
        __syncthreads();
    }
    if (tid == 0) *total = run;
}

void launch_append_offsets(const int64_t *counts, int n_clips, int64_t base, int64_t *dst_off, int64_t *total,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_append_offsets, dim3(1), dim3(1024), 0, s, counts, n_clips, base, dst_off, total);
}

void launch_records_to_postings(const uint64_t *recs, const int64_t *src_off, const int64_t *counts,
                                const int64_t *dst_off, const uint32_t *track_ids, int n_clips, uint32_t *ph,
                                uint32_t *ptrack, uint32_t *pt, hipStream_t s) {
    if (n_clips <= 0) return;
    hipLaunchKernelGGL(k_records_to_postings, dim3(16, n_clips), dim3(256), 0, s, recs, src_off, counts, dst_off,
                       track_ids, n_clips, ph, ptrack, pt);
}

// ---- K5: query ----
struct QueryParams {
    const uint64_t *recs;      // query records (hash | tq << 32)
    const int64_t *qstart;     // [nq] first record of query q (device)
    const int64_t *qcount;     // [nq] records of query q (device)
    int32_t nq;
    const uint32_t *offsets;   // [2^26 + 1]
    const uint64_t *post;
    const uint8_t *tomb;
    uint32_t n_tracks;
    int32_t min_match;
    int32_t max_rows;
    uint32_t *hist;            // [nq][2^hist_bits], zero on entry, re-zeroed on exit
    int32_t hist_bits;
    int32_t *rows;             // [nq][max_rows][5]
    int32_t *nrows;            // [nq]; -1 = LDS table overflow (query not answered)
    int32_t tomb_live;         // 0: the CSR holds no posting of a removed track (skip tomb[] loads)
    uint32_t *hot;             // [nq][2^hist_bits / 32] bit per histogram bucket >= min_match (K5h)
    int32_t parts;             // K5a workgroups (key partitions) per query
    const int64_t *votes;      // [nq] exact votes per query (k_query_votes, earlier on the stream); LDS path only
    const uint16_t *sig;       // [n] 2-B vote signature per posting (aidfp_layout.h posting_sig); LDS path only
    const uint64_t *ranges;    // LDS path: per record (same index as recs) its CSR range p0 | p1 << 32, written by
                               // k_query_votes earlier on the stream (nullptr: read offsets[] instead)
    uint32_t *dset;            // K5b: [nq][2^dset_bits] distinct (slot, t_q) sets in HBM, all kDistinctEmpty on entry
                               // (a retry of queries whose LDS set overflowed); nullptr = the LDS set
    int32_t dset_bits;
};

// Every vote (track, d = t_ref - t_q, t_q) of query records [a, a + n), for the calling wave's
// share of the records, with all 64 lanes on postings: the wave takes 64 records (one per
// lane: key, bucket start and length), scans the lengths, then walks the concatenated postings
// 64 at a time -- a lane finds its record among the few whose ranges meet the 64-posting window
// (ballot + readlane, scalar loop) -- with U windows' posting loads in flight before use. (One
// record per wave with lanes over its ~10-200 postings left most lanes idle and serialised
// recs -> offsets -> post -> tomb round trips per record.)
// The batch form hands the callback U windows at once (e[u]: posting, tq[u]: query time,
// ok[u]: a live vote), so K5a can issue its LDS filter tests for all U windows before any of its
// global atomics: a global atomic counts in vmcnt, and a wait for the next window's posting load
// would otherwise wait for it too (one L2 round trip per window). The loads are unconditional
// (invalid lanes read post[0]) so the waits before the windows can count precisely; the record
// of a window is found with readlane (the record index is wave-uniform), not ds_bpermute.
// A wave takes ceil(n / (waves x rounds)) <= 64 records at a time, rounds = ceil(n / (64 waves)),
// so the records spread evenly over every wave (config 4's windows: ~650 records, which 64-record
// groups had left on 11 of 16 waves).
template <int U, typename G>
__device__ __forceinline__ void for_each_window(const QueryParams &qp, int64_t a, int64_t n, int wave, int nw, int lane,
                                                G &&g) {
    const int64_t rounds = (n + (int64_t)nw * 64 - 1) / ((int64_t)nw * 64);
    const int64_t chunk = rounds ? (n + nw * rounds - 1) / (nw * rounds) : 64;
    for (int64_t base = (int64_t)wave * chunk; base < n; base += (int64_t)nw * chunk) {
        const int64_t i = base + lane;
        uint32_t p0 = 0, len = 0;
        int32_t tq = 0;
        if (lane < chunk && i < n) {
            const uint64_t r = qp.recs[a + i];
            const uint32_t k = key26((uint32_t)r);
            tq = (int32_t)(r >> 32);
            p0 = qp.offsets[k];
            len = qp.offsets[k + 1] - p0;
        }
        uint32_t incl = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        const uint32_t excl = incl - len;
        const uint32_t total = __shfl(incl, 63);
        // the window's record(s) come from a scalar cursor over the 64 records (records average
        // hundreds of postings, so most windows lie inside one record: one VALU op for the lane's
        // posting index instead of a ballot + per-record compare/select)
        int r = 0;
        uint32_t r_excl = __builtin_amdgcn_readlane(excl, 0), r_incl = __builtin_amdgcn_readlane(incl, 0);
        uint32_t r_p0 = __builtin_amdgcn_readlane(p0, 0);
        int32_t r_tq = __builtin_amdgcn_readlane(tq, 0);
        auto next_rec = [&]() {
            ++r;
            r_excl = __builtin_amdgcn_readlane(excl, r);
            r_incl = __builtin_amdgcn_readlane(incl, r);
            r_p0 = __builtin_amdgcn_readlane(p0, r);
            r_tq = __builtin_amdgcn_readlane(tq, r);
        };
        for (uint32_t w0 = 0; w0 < total; w0 += 64u * U) {
            uint32_t pos[U];
            int32_t tqs[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t lo = w0 + 64u * u, j = lo + lane;
                pos[u] = 0;
                tqs[u] = 0;
                ok[u] = false;
                if (lo >= total) continue;  // uniform
                while (r_incl <= lo) next_rec();  // r < 63 here: incl of lane 63 is total > lo
                if (r_incl >= lo + 64u) {  // the whole window inside record r (uniform)
                    pos[u] = r_p0 + (j - r_excl);
                    tqs[u] = r_tq;
                    ok[u] = true;
                } else {
                    for (;;) {  // records r, r+1, ... up to the one holding lo + 63 (or the last)
                        if (j >= r_excl && j < r_incl) {
                            pos[u] = r_p0 + (j - r_excl);
                            tqs[u] = r_tq;
                            ok[u] = true;
                        }
                        if (r_incl >= lo + 64u || r == 63) break;
                        next_rec();
                    }
                }
            }
            g(pos, tqs, ok);
        }
    }
}

// for_each_window with each window's postings loaded (and removed tracks' votes dropped while tombstones are newer
// than the CSR): g(e, tq, ok) for U windows at once
template <int U, typename G>
__device__ __forceinline__ void for_each_vote_batch(const QueryParams &qp, int64_t a, int64_t n, int wave, int nw,
                                                    int lane, G &&g) {
    for_each_window<U>(qp, a, n, wave, nw, lane, [&](const uint32_t *pos, const int32_t *tqs, bool *ok) {
        uint64_t e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = qp.post[pos[u]];
        if (qp.tomb_live) {  // uniform
            uint8_t tb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) tb[u] = qp.tomb[(uint32_t)e[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) ok[u] = ok[u] && !tb[u];
        }
        g(e, tqs, ok);
    });
}

template <int U, typename F>
__device__ __forceinline__ void for_each_vote(const QueryParams &qp, int64_t a, int64_t n, int wave, int nw, int lane,
                                              F &&f) {
    for_each_vote_batch<U>(qp, a, n, wave, nw, lane, [&](const uint64_t *e, const int32_t *tqs, const bool *ok) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) f((uint32_t)e[u], (int32_t)(e[u] >> 32) - tqs[u], tqs[u]);
    });
}

constexpr int kVoteWindows = 16;  // windows of 64 posting loads a wave keeps in flight

// one wave per query record; its lanes stride over the record's posting list (coalesced)
// K5a. A vote first sets its key's bits in a 2^20-bit LDS "seen" filter (128 KB)
// and reaches the global histogram only if they were all set already: of a key's c votes at most
// the first is held back, so a bucket holding a key with c >= min_match votes still counts
// >= min_match - 1 (K5h tests that). Config 4's windows have ~540k votes each (popular hashes:
// the vote count is size-biased, ~3x the mean bucket length times the records), and the filter
// keeps the random global atomics -- the kernel's cost -- to the chance collisions.
__global__ __launch_bounds__(1024) void k_vote_hist(QueryParams qp) {
    // qp.parts workgroups per query, each with its own seen filter for one hash partition of the
    // keys: on config 4 (~540k votes) the 2^20-bit filter saturates and lets ~20 % of the votes
    // through to the global histogram; two partitions read every posting twice but forward far
    // fewer (46.6k -> 60.2k clips/s; four 44.5k)
    const int q = blockIdx.x / qp.parts;
    const uint32_t part = blockIdx.x & (qp.parts - 1);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int64_t a = qp.qstart[q], n = qp.qcount[q];
    const uint32_t hmask = (1u << qp.hist_bits) - 1;
    uint32_t *H = qp.hist + ((int64_t)q << qp.hist_bits);
    __shared__ uint32_t seen[1 << 15];
    for (int i = threadIdx.x; i < (1 << 15); i += blockDim.x) seen[i] = 0u;
    __syncthreads();
    // The key's 2 bits (a blocked Bloom filter) sit in ONE word, so a single
    // atomicOr tests and sets them together: of racing votes of one key exactly one sees a bit
    // clear, so at most the key's first vote is held back, as with one bit. Two bits let fewer
    // chance "seen" collisions through to the global histogram (config 4: 36.9k -> 39.9k clips/s;
    // three bits 38.5k).
    for_each_vote_batch<kVoteWindows>(qp, a, n, wave, nw, lane, [&](const uint64_t *e, const int32_t *tqs, const bool *ok) {
        uint32_t fw[kVoteWindows];
#pragma unroll
        for (int u = 0; u < kVoteWindows; ++u) {  // all filter tests first (LDS only)
            const uint32_t x = mix_td((uint32_t)e[u], (int32_t)(e[u] >> 32) - tqs[u]);
            uint32_t m = (1u << (x & 31)) | (1u << ((x >> 5) & 31));
            // a partition's keys (from bits the filter does not use) get the whole filter
            m = ok[u] && ((x >> 10) & (uint32_t)(qp.parts - 1)) == part ? m : 0u;  // parts: 1, 2 or 4
            fw[u] = ((atomicOr(&seen[x >> 17], m) & m) == m && m) ? x & hmask : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kVoteWindows; ++u)  // then the global histogram
            if (fw[u] != 0xFFFFFFFFu) atomicAdd(&H[fw[u]], 1u);
    });
}

// K5h: one coalesced pass over each query's histogram row: bucket >= min_match -> a bit of the
// row's hot bitmap (64 counters per wave ballot), and the row is zeroed for the next batch.
// K5b then tests 4-byte words of a 64 KB bitmap (L2-resident) instead of gathering its votes'
// counters from the 2 MB row (a 64-128 B line per 4-byte read: ~46 GB of fetch per 2048 queries).
__global__ __launch_bounds__(256) void k_hot_scan(QueryParams qp) {
    const int64_t per_q = 1ll << qp.hist_bits;
    const uint32_t mm = (uint32_t)qp.min_match - 1u;  // the seen filter holds back a key's first vote (k_vote_hist)
    for (int q = blockIdx.y; q < qp.nq; q += gridDim.y) {
        uint32_t *H = qp.hist + ((int64_t)q << qp.hist_bits);
        uint64_t *B = reinterpret_cast<uint64_t *>(qp.hot + ((int64_t)q << (qp.hist_bits - 5)));
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < per_q; i += (int64_t)gridDim.x * 256) {
            const uint32_t c = H[i];
            const uint64_t m = __ballot(c >= mm);
            if ((threadIdx.x & 63) == 0) B[i >> 6] = m;  // i of lane 0 is a multiple of 64
            H[i] = 0u;
        }
    }
}

__global__ __launch_bounds__(1024) void k_vote_final(QueryParams qp) {
    __shared__ unsigned long long vkey[kVoteCap];  // (track << 32) | (uint32)d ; ~0 = empty
    __shared__ uint32_t vcnt[kVoteCap], vmin[kVoteCap], vmax[kVoteCap];
    __shared__ uint32_t tkey[kTrackCap];               // track ; ~0 = empty
    __shared__ unsigned long long tbest[kTrackCap];    // count << 32 | ~(d + 2^31)
    __shared__ int32_t out_n;
    __shared__ int32_t overflow;
    // the distinct-frame set of the insert phase and the row staging of the output phase share their LDS
    __shared__ union {
        uint32_t dset[kDistinctCap];
        int32_t rowbuf[kTrackCap][5];
    } ur;
    int32_t(*rowbuf)[5] = ur.rowbuf;
    __shared__ uint32_t hotl[1 << (kHotLdsBits - 5)];
    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    for (int i = tid; i < kVoteCap; i += blockDim.x) {
        vkey[i] = ~0ull;
        vcnt[i] = 0;
        vmin[i] = 0xFFFFFFFFu;
        vmax[i] = 0;
    }
    for (int i = tid; i < kTrackCap; i += blockDim.x) {
        tkey[i] = 0xFFFFFFFFu;
        tbest[i] = 0ull;
    }
    // the set of distinct (slot, t_q): in LDS, or (a retry of a query whose LDS set overflowed: long queries with
    // strong matches) a larger one in HBM that the host filled with kDistinctEmpty
    uint32_t *dset = qp.dset ? qp.dset + ((int64_t)blockIdx.x << qp.dset_bits) : ur.dset;
    const int dbits = qp.dset ? qp.dset_bits : kDistinctBits;
    if (!qp.dset)
        for (int i = tid; i < kDistinctCap; i += blockDim.x) ur.dset[i] = kDistinctEmpty;
    if (tid == 0) { out_n = 0; overflow = 0; }
    __syncthreads();
    const int64_t a = qp.qstart[q], z = a + qp.qcount[q];
    const uint32_t hmask = (1u << qp.hist_bits) - 1;
    const uint32_t *hot = qp.hot + ((int64_t)q << (qp.hist_bits - 5));
    const uint32_t mm = (uint32_t)qp.min_match;
    const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    // 1. exact table of candidate votes. The query's hot bitmap row (2^bits / 32 words) is staged
    // in LDS while it fits 16 KB (bits <= 17, every first attempt on config 4); all U windows'
    // bitmap tests run before any table insert
    const bool hot_in_lds = qp.hist_bits <= kHotLdsBits;
    if (hot_in_lds)
        for (int i = tid; i < (1 << (qp.hist_bits - 5)); i += blockDim.x) hotl[i] = hot[i];
    __syncthreads();
    auto insert = [&](uint32_t tr, int32_t d, int32_t tq, uint32_t h) {
        if (*(volatile int32_t *)&overflow) return;  // the query is re-run on a bigger histogram anyway
        const unsigned long long key = ((unsigned long long)tr << 32) | (uint32_t)d;
        uint32_t s = (h >> 20) & (kVoteCap - 1);
        int probes = 0;
        for (;;) {
            const unsigned long long old = atomicCAS(&vkey[s], ~0ull, key);
            if (old == ~0ull || old == key) {
                if (distinct_first(dset, dbits, s, (uint32_t)tq, &overflow)) atomicAdd(&vcnt[s], 1u);
                atomicMin(&vmin[s], (uint32_t)tq);
                atomicMax(&vmax[s], (uint32_t)tq);
                break;
            }
            if (++probes >= kProbeMax) { overflow = 1; break; }
            s = (s + 1) & (kVoteCap - 1);
        }
    };
    auto phase1 = [&](auto word) {
        for_each_vote_batch<kVoteWindows>(qp, a, z - a, wave, nw, lane, [&](const uint64_t *e, const int32_t *tqs, const bool *ok) {
            uint32_t h[kVoteWindows];
            bool hit[kVoteWindows];
#pragma unroll
            for (int u = 0; u < kVoteWindows; ++u) {
                h[u] = mix_td((uint32_t)e[u], (int32_t)(e[u] >> 32) - tqs[u]);
                const uint32_t hb = h[u] & hmask;
                hit[u] = ok[u] && ((word(hb >> 5) >> (hb & 31)) & 1u);
            }
#pragma unroll
            for (int u = 0; u < kVoteWindows; ++u)
                if (hit[u]) insert((uint32_t)e[u], (int32_t)(e[u] >> 32) - tqs[u], tqs[u], h[u]);
        });
    };
    if (hot_in_lds) phase1([&](uint32_t w) { return hotl[w]; });
    else phase1([&](uint32_t w) { return hot[w]; });
    __syncthreads();
    // 2. best d per track: max count, then smallest d
    for (int s = tid; s < kVoteCap; s += blockDim.x) {
        if (vkey[s] == ~0ull || vcnt[s] < mm) continue;
        const uint32_t tr = (uint32_t)(vkey[s] >> 32);
        const int32_t d = (int32_t)(uint32_t)vkey[s];
        const unsigned long long packed = ((unsigned long long)vcnt[s] << 32) | (uint32_t)~((uint32_t)d + 0x80000000u);
        uint32_t t = (tr * 0x9E3779B1u >> 22) & (kTrackCap - 1);
        int probes = 0;
        for (;;) {
            const uint32_t old = atomicCAS(&tkey[t], 0xFFFFFFFFu, tr);
            if (old == 0xFFFFFFFFu || old == tr) {
                atomicMax(&tbest[t], packed);
                break;
            }
            if (++probes >= kTrackCap) { overflow = 1; break; }
            t = (t + 1) & (kTrackCap - 1);
        }
    }
    __syncthreads();
    // 3. emit one row per track from the winning (track, d) entry
    for (int s = tid; s < kVoteCap; s += blockDim.x) {
        if (vkey[s] == ~0ull || vcnt[s] < mm) continue;
        const uint32_t tr = (uint32_t)(vkey[s] >> 32);
        const int32_t d = (int32_t)(uint32_t)vkey[s];
        const unsigned long long packed = ((unsigned long long)vcnt[s] << 32) | (uint32_t)~((uint32_t)d + 0x80000000u);
        uint32_t t = (tr * 0x9E3779B1u >> 22) & (kTrackCap - 1);
        for (int probes = 0; probes < kTrackCap && tkey[t] != tr; ++probes) t = (t + 1) & (kTrackCap - 1);
        if (tkey[t] == tr && tbest[t] == packed) {
            const int o = atomicAdd(&out_n, 1);
            if (o < kTrackCap) {
                rowbuf[o][0] = (int32_t)vcnt[s];
                rowbuf[o][1] = (int32_t)tr;
                rowbuf[o][2] = d;
                rowbuf[o][3] = (int32_t)vmin[s];
                rowbuf[o][4] = (int32_t)vmax[s];
            }
        }
    }
    __syncthreads();
    // 4. rank (count desc, track asc) by counting rank, write the first max_rows
    const int n = min(out_n, kTrackCap);
    for (int i = tid; i < n; i += blockDim.x) {
        int rank = 0;
        for (int j = 0; j < n; ++j) {
            const bool before = rowbuf[j][0] > rowbuf[i][0] ||
                                (rowbuf[j][0] == rowbuf[i][0] && (uint32_t)rowbuf[j][1] < (uint32_t)rowbuf[i][1]);
            rank += before ? 1 : 0;
        }
        if (rank < qp.max_rows) {
            int32_t *o = qp.rows + ((int64_t)q * qp.max_rows + rank) * 5;
#pragma unroll
            for (int c = 0; c < 5; ++c) o[c] = rowbuf[i][c];
        }
    }
    if (tid == 0) qp.nrows[q] = (overflow || out_n > kTrackCap) ? -1 : min(n, qp.max_rows);
}

// ---- K5 (fast path): the whole vote filter in LDS, one 512-thread workgroup per query, four per CU ----
// Phase 1: every vote counted in 2^15 8-bit hashed counters (32 KB of LDS) from its posting's 2-B signature alone
//          (bucket = sig - tq = H(track) + d: aidfp_layout.h posting_sig); the waves walk their records' signatures
//          in 8-posting chunks (one 16-B load per lane, for_each_chunk).
// Phase 2: counters >= min_match -> a 2^15-bit "hot" bitmap (4 KB).
// Phase 3: the counter region is reused as the exact (track, d) table; the signatures are walked again and only a
//          vote whose bucket is hot is queued (posting index, tq) in the LDS the table leaves free; after the walk
//          every thread reads its queued votes' 8-B postings at once and inserts them (exact superset filter, as in
//          K5a/K5b).
// Phase 4: best d per track, rank, write rows (same as K5b). Any table overflow reports nrows = -1 and the host
//          re-runs the query on the global-histogram path; a query above kLdsMaxVotes is handed back at once.
// A counter that wraps past 255 marks its bucket hot at once (>= 256 votes), as does any full counter its carry
// runs through, so the filter stays an exact superset. Round 5 (config 4, per 4096-clip lane call, same-box A/Bs
// r05d-r05i): 8-B postings walked one per lane, 2^16 counters, two 1024-thread workgroups per CU 3.60-3.73 ms ->
// 2-B signatures one per lane 3.64-3.74 (bytes were not the bound: the walk's ~95 instructions per 64 votes were)
// -> 4-posting chunks 2.71-2.76 -> hot-vote queue 2.68 -> 8-posting chunks, four 512-thread workgroups per CU, the
// LDS path up to 2^18 votes per query 1.80-1.86.
constexpr int kLdsSigWindows = 3;  // windows of 64 two-byte signature loads a wave keeps in flight
// The filter: 2^16 4-bit counters in 32 KB (round 6; 2^15 8-bit counters before). FPSPEC v1's min_match 10 had made
// the 8-bit filter's chance-hot buckets ~20x more frequent than at 12 (a Poisson tail at ~2.6 votes per bucket on
// config 4), and 11 % of config-4 windows overflowed the exact table; twice the buckets halve the load per counter.
// A counter that wraps (>= 16 votes) marks its bucket hot, so the filter stays an exact superset for any min_match.
// The hot bitmap holds one bit per PAIR of buckets (2^15 bits, 4 KB as before): a hot bucket makes its pair
// neighbour a candidate too (still a superset).
constexpr int kLdsHistBits = 16;
constexpr int kLdsCtrBits = 4;
constexpr int kLdsCtrPerWord = 32 / kLdsCtrBits;
constexpr uint32_t kLdsCtrMax = (1u << kLdsCtrBits) - 1;
constexpr int kHotShift = 1;                              // buckets per hot bit = 2^kHotShift
constexpr int kHotWords = (1 << (kLdsHistBits - kHotShift)) / 32;
constexpr int kFastVoteCap = 1024;     // (track, d) entries of the exact table
constexpr int kFastDistinctBits = 11;  // FPSPEC v1: the (slot, t_q) set of the inserted votes, 2,048 keys
constexpr int kFastTrackCap = 256;  // tracks with a candidate (track, d); the row staging holds 204 anyway
constexpr int kFastDistinctCap = 1 << kFastDistinctBits;
constexpr int kFastThreads = 512;

static_assert(kLdsHistBits <= 16, "the LDS filter's buckets come from 16-bit posting signatures");
// kLdsMaxVotes (aidfp_layout.h): a heavier query reports nrows = -1 at once and the host runs it on the global path

// The LDS path walks the records' postings in CHUNKS of kSigChunk (8 or 16 B of 2-B signatures, one load per lane):
// a wave takes its share of the records (as for_each_window), scans their chunk counts -- a record at CSR positions
// [p0, p1) covers the aligned chunks p0 / C .. (p1 + C - 1) / C -- and walks the concatenated chunks 64 at a time
// (64 C postings per window) with U windows of loads in flight; a lane's C-bit mask says which of its chunk's
// postings belong to the record (the first and last chunk of a record are partial). The per-window bookkeeping
// (record cursor, positions) is paid once per 64 C votes instead of once per 64: with one posting per lane the walk
// issued ~63 VALU + 32 SALU per 64 votes and was the LDS path's cost (r05e: without its second enumeration K5 took
// 1.76 of 3.63 ms, without the first pass's LDS atomics 3.24).
constexpr int kSigChunk = 8;
static_assert(kSigChunk == 4 || kSigChunk == 8, "signature chunks of 4 or 8 postings");
typedef uint32_t sig_chunk_t __attribute__((ext_vector_type(kSigChunk / 2)));

// one wave's group of <= 64 records: lane = record (CSR range [p0, p1), query time tq), chunk-count scan
struct ChunkGroup {
    uint32_t p0, p1, incl, excl, total;
    int32_t tq;
};

__device__ __forceinline__ ChunkGroup load_group(const QueryParams &qp, int64_t a, int64_t n, int64_t base,
                                                 int64_t chunk, int lane) {
    ChunkGroup gr{0u, 0u, 0u, 0u, 0u, 0};
    const int64_t i = base + lane;
    uint32_t clen = 0;
    if (lane < chunk && i < n) {
        const uint64_t r = qp.recs[a + i];
        gr.tq = (int32_t)(r >> 32);
        if (qp.ranges) {  // coalesced, and independent of the record load (no recs -> offsets chain)
            const uint64_t rg = qp.ranges[a + i];
            gr.p0 = (uint32_t)rg;
            gr.p1 = (uint32_t)(rg >> 32);
        } else {
            const uint32_t k = key26((uint32_t)r);
            gr.p0 = qp.offsets[k];
            gr.p1 = qp.offsets[k + 1];
        }
        clen = gr.p1 > gr.p0 ? (gr.p1 + (kSigChunk - 1)) / kSigChunk - gr.p0 / kSigChunk : 0u;
    }
    uint32_t incl = clen;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    gr.incl = incl;
    gr.excl = incl - clen;
    gr.total = __shfl(incl, 63);
    return gr;
}

// g(cid[U], tq[U], vm[U]) for every window of the group: chunk index, query time and posting mask per lane
template <int U, typename G>
__device__ __forceinline__ void walk_group(const ChunkGroup &gr, int lane, G &&g) {
    int r = 0;
    uint32_t r_excl = __builtin_amdgcn_readlane(gr.excl, 0), r_incl = __builtin_amdgcn_readlane(gr.incl, 0);
    uint32_t r_p0 = __builtin_amdgcn_readlane(gr.p0, 0), r_p1 = __builtin_amdgcn_readlane(gr.p1, 0);
    int32_t r_tq = __builtin_amdgcn_readlane(gr.tq, 0);
    auto next_rec = [&]() {
        ++r;
        r_excl = __builtin_amdgcn_readlane(gr.excl, r);
        r_incl = __builtin_amdgcn_readlane(gr.incl, r);
        r_p0 = __builtin_amdgcn_readlane(gr.p0, r);
        r_p1 = __builtin_amdgcn_readlane(gr.p1, r);
        r_tq = __builtin_amdgcn_readlane(gr.tq, r);
    };
    // chunk c of the record [rp0, rp1): mask of its postings C c + e inside the record
    constexpr uint32_t kAll = (1u << kSigChunk) - 1;
    auto maskc = [](uint32_t c, uint32_t rp0, uint32_t rp1) -> uint32_t {
        const int s0 = (int)rp0 - (int)(kSigChunk * c), s1 = (int)rp1 - (int)(kSigChunk * c);
        const int lo = min(max(s0, 0), kSigChunk), hi = min(max(s1, 0), kSigChunk);
        return (kAll << lo) & ~(kAll << hi) & kAll;
    };
    const uint32_t total = gr.total;
    for (uint32_t w0 = 0; w0 < total; w0 += 64u * U) {
        uint32_t cid[U], vm[U];
        int32_t tqs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t lo = w0 + 64u * u, j = lo + lane;
            cid[u] = 0;
            vm[u] = 0;
            tqs[u] = 0;
            if (lo >= total) continue;  // uniform
            while (r_incl <= lo) next_rec();  // r < 63 here: incl of lane 63 is total > lo
            if (r_incl >= lo + 64u) {  // the whole window inside record r (uniform)
                cid[u] = r_p0 / kSigChunk + (j - r_excl);
                tqs[u] = r_tq;
                vm[u] = maskc(cid[u], r_p0, r_p1);
            } else {
                for (;;) {  // records r, r+1, ... up to the one holding chunk lo + 63 (or the last)
                    if (j >= r_excl && j < r_incl) {
                        cid[u] = r_p0 / kSigChunk + (j - r_excl);
                        tqs[u] = r_tq;
                        vm[u] = maskc(cid[u], r_p0, r_p1);
                    }
                    if (r_incl >= lo + 64u || r == 63) break;
                    next_rec();
                }
            }
        }
        g(cid, tqs, vm);
    }
}

// records per wave group: ceil(n / (waves x rounds)) <= 64, rounds = ceil(n / (64 waves)) (as for_each_window)
__device__ __forceinline__ int64_t group_records(int64_t n, int nw) {
    const int64_t rounds = (n + (int64_t)nw * 64 - 1) / ((int64_t)nw * 64);
    return rounds ? (n + nw * rounds - 1) / (nw * rounds) : 64;
}

template <int U, typename G>
__device__ __forceinline__ void for_each_chunk(const QueryParams &qp, int64_t a, int64_t n, int wave, int nw, int lane,
                                               G &&g) {
    const int64_t chunk = group_records(n, nw);
    for (int64_t base = (int64_t)wave * chunk; base < n; base += (int64_t)nw * chunk)
        walk_group<U>(load_group(qp, a, n, base, chunk, lane), lane, g);
}

// the signatures of one window's chunks, element e of the lane's chunk: (sig_e - tq) mod 2^bits = the LDS bucket
__device__ __forceinline__ sig_chunk_t load_sigs(const QueryParams &qp, uint32_t cid) {
    return reinterpret_cast<const sig_chunk_t *>(qp.sig)[cid];
}
__device__ __forceinline__ uint32_t sig_bucket(const sig_chunk_t &v, int e, int32_t tq) {
    return ((uint32_t)(v[e >> 1] >> (16 * (e & 1))) - (uint32_t)tq) & ((1u << kLdsHistBits) - 1);
}

// every live vote's LDS filter bucket for the calling wave's records: f(bucket), U windows in flight; with `one`
// (the wave's records are ONE group, `grp`, loaded once for both passes) the group's record loads are not repeated
template <typename F>
__device__ __forceinline__ void sig_votes(const QueryParams &qp, int64_t a, int64_t n, int wave, int nw, int lane,
                                          bool one, const ChunkGroup &grp, F &&f) {
    auto g = [&](const uint32_t *cid, const int32_t *tqs, const uint32_t *vm) {
        sig_chunk_t sw[kLdsSigWindows];
#pragma unroll
        for (int u = 0; u < kLdsSigWindows; ++u) sw[u] = load_sigs(qp, cid[u]);
#pragma unroll
        for (int u = 0; u < kLdsSigWindows; ++u)
#pragma unroll
            for (int e = 0; e < kSigChunk; ++e)
                if ((vm[u] >> e) & 1u) f(sig_bucket(sw[u], e, tqs[u]));
    };
    if (one) walk_group<kLdsSigWindows>(grp, lane, g);
    else for_each_chunk<kLdsSigWindows>(qp, a, n, wave, nw, lane, g);
}

// hot votes queued by the insert pass (posting index, tq): the LDS the counters leave beside the exact table
// The union holds the 32 KB of filter counters, then the exact tables, the distinct set, the phase-3..5 counters and
// the hot-vote queue in 36 KB: with the 4 KB hot bitmap a workgroup takes 40 KB, four per CU in the 160 KB LDS
constexpr int kUnionBytes = 36864;
constexpr int kTableBytes = kFastVoteCap * (8 + 3 * 4) + kFastTrackCap * (4 + 8) + kFastDistinctCap * 4 + 16;
constexpr int kHotQueue = (kUnionBytes - kTableBytes) / 8;

struct FastLds {
    union {
        uint32_t hist[(1 << kLdsHistBits) / kLdsCtrPerWord];  // packed vote counters
        struct {
            unsigned long long vkey[kFastVoteCap];
            uint32_t vcnt[kFastVoteCap], vmin[kFastVoteCap], vmax[kFastVoteCap];
            uint32_t tkey[kFastTrackCap];
            unsigned long long tbest[kFastTrackCap];
            uint32_t dset[kFastDistinctCap];  // distinct (slot, t_q) of the inserted votes
            int32_t out_n, overflow, hq_n, pad;  // phases 3-5 (the counters' LDS is free by then)
            uint2 hq[kHotQueue > 0 ? kHotQueue : 1];  // the insert pass's hot votes (posting index, tq)
        } t;
        uint32_t bytes[kUnionBytes / 4];
    } u;
    uint32_t hot[kHotWords];
};
static_assert(kHotQueue >= 512 && sizeof(FastLds::u) == kUnionBytes && sizeof(FastLds) == 40960,
              "the hot-vote queue lives in the counters' LDS beside the exact table; 40 KB = four workgroups per CU");

__global__ __launch_bounds__(kFastThreads)
__attribute__((amdgpu_waves_per_eu(8)))
void k_match_lds(QueryParams qp) {
    __shared__ FastLds L;  // 2^16 4-bit counters, then the exact tables / hot-vote queue; 40 KB, four workgroups per CU
    const int q = blockIdx.x;
    // a query heavier than the LDS filter suits goes to the global path at once, by its own vote count (a heavy
    // query here would wrap many 8-bit counters, mark their buckets hot and likely overflow the exact table after a
    // slow run); uniform, before any barrier
    if (qp.votes[q] > kLdsMaxVotes) {
        if (threadIdx.x == 0) qp.nrows[q] = -1;
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = kFastThreads / 64;
    const int64_t a = qp.qstart[q], n = qp.qcount[q];
    const uint32_t mm = (uint32_t)qp.min_match;
    for (int i = tid; i < (1 << kLdsHistBits) / kLdsCtrPerWord; i += kFastThreads) L.u.hist[i] = 0u;
    for (int i = tid; i < kHotWords; i += kFastThreads) L.hot[i] = 0u;
    __syncthreads();
    // the query's exact vote total (k_query_votes): below the counter maximum no counter can wrap, so only
    // heavier queries pay for returning atomics (the carry check below)
    const bool check_wrap = qp.votes[q] >= (int64_t)kLdsCtrMax;
    // a query whose records fit one group per wave (<= 64 x waves: config 4's ~650) loads them once for both passes
    ChunkGroup grp_one{0u, 0u, 0u, 0u, 0u, 0};
    const bool one_group = n <= (int64_t)nw * 64;
    if (one_group) {
        const int64_t chunk = group_records(n, nw);
        grp_one = load_group(qp, a, n, (int64_t)wave * chunk, chunk, lane);
    }

    // phase 1: every vote counted from its posting's 2-B signature alone (bucket = sig - tq = H(track) + d)
    auto mark_hot = [&](uint32_t b) {
        const uint32_t hb = b >> kHotShift;
        atomicOr(&L.hot[hb >> 5], 1u << (hb & 31));
    };
    sig_votes(qp, a, n, wave, nw, lane, one_group, grp_one, [&](uint32_t h) {
        const uint32_t sh = kLdsCtrBits * (h % kLdsCtrPerWord);
        uint32_t *w = &L.u.hist[h / kLdsCtrPerWord];
        if (check_wrap) {
            const uint32_t old = atomicAdd(w, 1u << sh);
            if (((old >> sh) & kLdsCtrMax) == kLdsCtrMax) {
                // wrapped: the bucket holds > kLdsCtrMax votes, so it is hot whatever its counter ends at;
                // the carry went on into the next counters of the word, and through each full one
                mark_hot(h);
                for (uint32_t j = h % kLdsCtrPerWord + 1;
                     j < kLdsCtrPerWord && ((old >> (kLdsCtrBits * j)) & kLdsCtrMax) == kLdsCtrMax; ++j)
                    mark_hot((h & ~(uint32_t)(kLdsCtrPerWord - 1)) + j);
            }
        } else {
            atomicAdd(w, 1u << sh);
        }
    });
    __syncthreads();
    // phase 2
    // phase 2: hot bit of a bucket pair = either counter >= min_match (a hot word covers 32 pairs = 8 counter words)
    constexpr int kPairsPerWord = kLdsCtrPerWord >> kHotShift;
    for (int w = tid; w < kHotWords; w += kFastThreads) {
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 32 / kPairsPerWord; ++j) {
            const uint32_t v = L.u.hist[w * (32 / kPairsPerWord) + j];
#pragma unroll
            for (int b = 0; b < kLdsCtrPerWord; ++b)
                bits |= (uint32_t)(((v >> (kLdsCtrBits * b)) & kLdsCtrMax) >= mm) << (kPairsPerWord * j + (b >> kHotShift));
        }
        L.hot[w] |= bits;  // with the buckets phase 1 found wrapped
    }
    __syncthreads();
    for (int i = tid; i < kFastVoteCap; i += kFastThreads) {
        L.u.t.vkey[i] = ~0ull;
        L.u.t.vcnt[i] = 0;
        L.u.t.vmin[i] = 0xFFFFFFFFu;
        L.u.t.vmax[i] = 0;
    }
    for (int i = tid; i < kFastTrackCap; i += kFastThreads) {
        L.u.t.tkey[i] = 0xFFFFFFFFu;
        L.u.t.tbest[i] = 0ull;
    }
    for (int i = tid; i < kFastDistinctCap; i += kFastThreads) L.u.t.dset[i] = kDistinctEmpty;
    if (tid == 0) { L.u.t.out_n = 0; L.u.t.overflow = 0; L.u.t.hq_n = 0; }
    __syncthreads();
    // the exact (track, d) table insert of one hot vote (slot from the full mix of (track, d))
    auto insert = [&](uint32_t tr, int32_t d, int32_t tq) {
        // once some table is full the query goes to the global path anyway: later inserts would each probe a full
        // table (512 slots, or the whole 2,048-key distinct set) for nothing
        if (*(volatile int32_t *)&L.u.t.overflow) return;
        const unsigned long long key = ((unsigned long long)tr << 32) | (uint32_t)d;
        uint32_t s = (mix_td(tr, d) >> 20) & (kFastVoteCap - 1);
        int probes = 0;
        for (;;) {
            const unsigned long long old = atomicCAS(&L.u.t.vkey[s], ~0ull, key);
            if (old == ~0ull || old == key) {
                if (distinct_first(L.u.t.dset, kFastDistinctBits, s, (uint32_t)tq, &L.u.t.overflow))
                    atomicAdd(&L.u.t.vcnt[s], 1u);
                atomicMin(&L.u.t.vmin[s], (uint32_t)tq);
                atomicMax(&L.u.t.vmax[s], (uint32_t)tq);
                break;
            }
            if (++probes >= kProbeMax) { atomicMax(&L.u.t.overflow, 2); break; }  // reason 2: (track, d) table
            s = (s + 1) & (kFastVoteCap - 1);
        }
    };
    // phase 3: the signatures again; only a vote whose bucket is hot reads its 8-B posting and enters the table
    auto insert_pass = [&](const uint32_t *cid, const int32_t *tqs, const uint32_t *vm) {
        sig_chunk_t sw[kLdsSigWindows];
#pragma unroll
        for (int u = 0; u < kLdsSigWindows; ++u) sw[u] = load_sigs(qp, cid[u]);
        uint32_t hm[kLdsSigWindows];  // the chunk's postings whose bucket is hot
#pragma unroll
        for (int u = 0; u < kLdsSigWindows; ++u) {
            hm[u] = 0;
#pragma unroll
            for (int e = 0; e < kSigChunk; ++e) {
                const uint32_t h = sig_bucket(sw[u], e, tqs[u]);
                const uint32_t hb = h >> kHotShift;
                hm[u] |= ((vm[u] >> e) & (L.hot[hb >> 5] >> (hb & 31)) & 1u) << e;
            }
        }
#pragma unroll
        for (int u = 0; u < kLdsSigWindows; ++u)
            while (hm[u]) {  // rare: each hot vote is queued in LDS; its posting is read after the walk
                const int e = __builtin_ctz(hm[u]);
                hm[u] &= hm[u] - 1;
                const uint32_t pi = (uint32_t)kSigChunk * cid[u] + (uint32_t)e;
                const int slot = atomicAdd(&L.u.t.hq_n, 1);
                if (slot < kHotQueue) {
                    L.u.t.hq[slot] = make_uint2(pi, (uint32_t)tqs[u]);
                } else {  // queue full: this vote's posting now (a dependent load: one memory latency)
                    const uint64_t pv = qp.post[pi];
                    const uint32_t tr = (uint32_t)pv;
                    if (!(qp.tomb_live && qp.tomb[tr])) insert(tr, (int32_t)(pv >> 32) - tqs[u], tqs[u]);
                }
            }
    };
    if (one_group) walk_group<kLdsSigWindows>(grp_one, lane, insert_pass);
    else for_each_chunk<kLdsSigWindows>(qp, a, n, wave, nw, lane, insert_pass);
    __syncthreads();
    // the queued hot votes: every thread loads its entries' postings at once (one memory latency for the whole
    // queue instead of one per hot vote inside the walk), then inserts them
    {
        const int nh = min(L.u.t.hq_n, kHotQueue);
        for (int i = tid; i < nh; i += kFastThreads) {
            const uint2 h = L.u.t.hq[i];
            const uint64_t pv = qp.post[h.x];
            const uint32_t tr = (uint32_t)pv;
            if (qp.tomb_live && qp.tomb[tr]) continue;  // a removed track's vote (the filter counted it: superset)
            insert(tr, (int32_t)(pv >> 32) - (int32_t)h.y, (int32_t)h.y);
        }
    }
    __syncthreads();
    // phase 4: best d per track
    for (int s = tid; s < kFastVoteCap; s += kFastThreads) {
        if (L.u.t.vkey[s] == ~0ull || L.u.t.vcnt[s] < mm) continue;
        const uint32_t tr = (uint32_t)(L.u.t.vkey[s] >> 32);
        const int32_t d = (int32_t)(uint32_t)L.u.t.vkey[s];
        const unsigned long long packed = ((unsigned long long)L.u.t.vcnt[s] << 32) | (uint32_t)~((uint32_t)d + 0x80000000u);
        uint32_t t = (tr * 0x9E3779B1u >> 22) & (kFastTrackCap - 1);
        int probes = 0;
        for (;;) {
            const uint32_t old = atomicCAS(&L.u.t.tkey[t], 0xFFFFFFFFu, tr);
            if (old == 0xFFFFFFFFu || old == tr) {
                atomicMax(&L.u.t.tbest[t], packed);
                break;
            }
            if (++probes >= kFastTrackCap) { atomicMax(&L.u.t.overflow, 4); break; }  // reason 4: track table
            t = (t + 1) & (kFastTrackCap - 1);
        }
    }
    __syncthreads();
    // phase 5: winning (track, d) rows -> rank -> output (rows staged in the hot bitmap area)
    int32_t(*rowbuf)[5] = reinterpret_cast<int32_t(*)[5]>(L.hot);  // 8 KB = 409 rows
    constexpr int kRowCap = (int)(sizeof(L.hot) / (5 * sizeof(int32_t)));
    for (int s = tid; s < kFastVoteCap; s += kFastThreads) {
        if (L.u.t.vkey[s] == ~0ull || L.u.t.vcnt[s] < mm) continue;
        const uint32_t tr = (uint32_t)(L.u.t.vkey[s] >> 32);
        const int32_t d = (int32_t)(uint32_t)L.u.t.vkey[s];
        const unsigned long long packed = ((unsigned long long)L.u.t.vcnt[s] << 32) | (uint32_t)~((uint32_t)d + 0x80000000u);
        uint32_t t = (tr * 0x9E3779B1u >> 22) & (kFastTrackCap - 1);
        for (int probes = 0; probes < kFastTrackCap && L.u.t.tkey[t] != tr; ++probes) t = (t + 1) & (kFastTrackCap - 1);
        if (L.u.t.tkey[t] == tr && L.u.t.tbest[t] == packed) {
            const int o = atomicAdd(&L.u.t.out_n, 1);
            if (o < kRowCap) {
                rowbuf[o][0] = (int32_t)L.u.t.vcnt[s];
                rowbuf[o][1] = (int32_t)tr;
                rowbuf[o][2] = d;
                rowbuf[o][3] = (int32_t)L.u.t.vmin[s];
                rowbuf[o][4] = (int32_t)L.u.t.vmax[s];
            }
        }
    }
    __syncthreads();
    const int nr = min(L.u.t.out_n, kRowCap);
    for (int i = tid; i < nr; i += kFastThreads) {
        int rank = 0;
        for (int j = 0; j < nr; ++j) {
            const bool before = rowbuf[j][0] > rowbuf[i][0] ||
                                (rowbuf[j][0] == rowbuf[i][0] && (uint32_t)rowbuf[j][1] < (uint32_t)rowbuf[i][1]);
            rank += before ? 1 : 0;
        }
        if (rank < qp.max_rows) {
            int32_t *o = qp.rows + ((int64_t)q * qp.max_rows + rank) * 5;
#pragma unroll
            for (int c = 0; c < 5; ++c) o[c] = rowbuf[i][c];
        }
    }
    // a query the LDS path cannot answer reports -(reason): 1 above kLdsMaxVotes, 2 (track, d) table, 3 distinct set,
    // 4 track table, 5 more rows than the staging holds (the engine re-runs it on the global path and counts reasons)
    if (tid == 0)
        qp.nrows[q] = L.u.t.overflow ? -L.u.t.overflow : L.u.t.out_n > kRowCap ? -5 : min(nr, qp.max_rows);
}

void launch_match_lds(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq,
                      const uint32_t *offsets, const uint64_t *post, const uint8_t *tomb, uint32_t n_tracks,
                      int min_match, int max_rows, int32_t *rows, int32_t *nrows, int tomb_live, const int64_t *votes,
                      const uint16_t *sig, const uint64_t *ranges, hipStream_t s) {
    if (nq <= 0) return;
    QueryParams qp{recs, qstart, qcount, nq, offsets, post, tomb, n_tracks, min_match, max_rows, nullptr, 0, rows, nrows,
                   tomb_live, nullptr, 1, votes, sig, ranges};
    timed_launch(k_match_lds, dim3(nq), dim3(kFastThreads), 0, s, qp);
}

// resident k_match_lds workgroups per CU (LDS- and register-limited; 4 by design), for the match statistics
int match_lds_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_match_lds, kFastThreads, 0) != hipSuccess) n = -1;
    return n;
}

void launch_index_count(const uint32_t *ph, const uint32_t *ptrack, int64_t n, const uint8_t *tomb, uint32_t n_tracks,
                        uint32_t *cnt, hipStream_t s) {
    if (n <= 0) return;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_index_count, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptrack, n, tomb, n_tracks, cnt);
}

void launch_index_scatter(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                          const uint8_t *tomb, uint32_t n_tracks, uint32_t *cursor, uint64_t *post, hipStream_t s) {
    if (n <= 0) return;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_index_scatter, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptrack, pt, n, tomb, n_tracks,
                       cursor, post);
}

// exclusive scan of n counts (n multiple of 1024); tmp holds >= 2 * ceil(n/1024) + 1024 u32
void launch_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t s) {
    const int64_t nb = (n + 1023) / 1024;
    uint32_t *bsum = tmp, *boff = tmp + nb, *b2 = tmp + 2 * nb;
    hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nb), dim3(1024), 0, s, in, out, bsum, n);
    if (nb > 1) {
        // recursive on block sums (nb <= 2^16 for 2^26 keys -> at most two levels)
        launch_scan(bsum, boff, nb, b2, s);
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(1024), 0, s, out, boff, n);
    }
}

void launch_query(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq, const uint32_t *offsets,
                  const uint64_t *post, const uint8_t *tomb, uint32_t n_tracks, int min_match, int max_rows,
                  uint32_t *hist, int hist_bits, uint32_t *hot, int32_t *rows, int32_t *nrows, int tomb_live,
                  int parts, int stage, uint32_t *dset, int dset_bits, hipStream_t s) {
    if (nq <= 0) return;
    QueryParams qp{recs, qstart, qcount, nq, offsets, post, tomb, n_tracks, min_match, max_rows, hist, hist_bits, rows,
                   nrows, tomb_live, hot, parts, nullptr, nullptr, nullptr, dset, dset_bits};
    // stage = 0: all three kernels; 1, 2, 3: K5a, K5h, K5b alone (the engine times them one by one)
    if (stage == 0 || stage == 1) timed_launch(k_vote_hist, dim3(nq * parts), dim3(1024), 0, s, qp);
    if (stage == 0 || stage == 2)
        timed_launch(k_hot_scan, dim3(16, (unsigned)(nq < 65535 ? nq : 65535)), dim3(256), 0, s, qp);
    if (stage == 0 || stage == 3) timed_launch(k_vote_final, dim3(nq), dim3(1024), 0, s, qp);
}

// exact vote count of each query: the sum of its records' bucket lengths (one block per query)
// and (ranges != nullptr) every record's CSR range p0 | p1 << 32 at its record index, so the LDS match path reads the
// ranges coalesced in both of its passes instead of two dependent random offset loads per record and pass (config 4's
// ~650-record windows take more than one record group per wave, so the groups are loaded once per pass)
__global__ __launch_bounds__(256) void k_query_votes(const uint64_t *__restrict__ recs, const int64_t *__restrict__ qstart,
                                                     const int64_t *__restrict__ qcount,
                                                     const uint32_t *__restrict__ offsets, int64_t *__restrict__ votes,
                                                     uint64_t *__restrict__ ranges) {
    __shared__ unsigned long long part[4];
    const int q = blockIdx.x;
    const int64_t a = qstart[q], n = qcount[q];
    unsigned long long v = 0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const uint32_t k = key26((uint32_t)recs[a + i]);
        const uint32_t p0 = offsets[k], p1 = offsets[k + 1];
        v += p1 - p0;
        if (ranges) ranges[a + i] = (uint64_t)p0 | ((uint64_t)p1 << 32);
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) votes[q] = (int64_t)(part[0] + part[1] + part[2] + part[3]);
}

void launch_query_votes(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq,
                        const uint32_t *offsets, int64_t *votes, uint64_t *ranges, hipStream_t s) {
    if (nq > 0)
        hipLaunchKernelGGL(k_query_votes, dim3(nq), dim3(256), 0, s, recs, qstart, qcount, offsets, votes, ranges);
}

// number of non-empty buckets (for the query histogram sizing)
__global__ void k_count_nonzero(const uint32_t *__restrict__ cnt, int64_t n, unsigned long long *__restrict__ out) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += cnt[i] != 0u;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, c);
}

void launch_count_nonzero(const uint32_t *cnt, int64_t n, unsigned long long *out, hipStream_t s) {
    hipLaunchKernelGGL(k_count_nonzero, dim3(2048), dim3(256), 0, s, cnt, n, out);
}

// Order-sensitive checksum of postings [first, first + n) of the SoA planes: the sum mod 2^64 of
// mix64((hash << 32 | t) ^ track * C1 ^ i * C2) over positions i relative to `first` (aidfp.catalog.checksum_np is
// its host mirror). Replicas with equal checksums hold the same postings in the same order (a collision has
// probability ~2^-64): the catalog ingest compares them across ranks after the exchange.
__device__ __forceinline__ uint64_t splitmix64_fin(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_index_checksum(const uint32_t *__restrict__ ph, const uint32_t *__restrict__ ptr,
                                                        const uint32_t *__restrict__ pt, int64_t first, int64_t n,
                                                        unsigned long long *__restrict__ out) {
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = first + i;
        const uint64_t key = (((uint64_t)ph[j] << 32) | pt[j]) ^ ((uint64_t)ptr[j] * 0x9E3779B97F4A7C15ull) ^
                             ((uint64_t)i * 0xD6E8FEB86659FD93ull);
        acc += splitmix64_fin(key);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

void launch_index_checksum(const uint32_t *ph, const uint32_t *ptr, const uint32_t *pt, int64_t first, int64_t n,
                           unsigned long long *out, hipStream_t s) {
    if (n <= 0) return;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_index_checksum, dim3((unsigned)blocks), dim3(256), 0, s, ph, ptr, pt, first, n, out);
}

uint32_t index_keys() { return kKeys; }

}  // namespace aid
