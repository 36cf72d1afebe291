// peaks.hip -- K2 `peak_pick`: 2-D local-maximum constellation (FPSPEC 5) with
// the tie rule "earliest (t,k) wins", emitted as a per-frame 1024-bit mask.
//
// Replaces the spectral-peak stage inside the external `olaf_c` binary
// (reference call sites fingerprint.py:117-125, 185-193).
//
// One workgroup streams one strip of `strip_len` output frames of one clip and
// reads every power row of the strip (+7 halo rows each side) once. The host sizes
// strip_len per call so the strips fill the resident workgroup slots in one round
// (peak_strip_len); a fixed 128-frame strip left a third round 1/3 full at 256 x 10 s:
//
//   * thread j owns bins 4j..4j+3 (one float4 load per row); the next batch of 4
//     rows is in flight in registers while the current one is processed;
//   * rows are staged in LDS as int32 keys 4 at a time (one buffer, a barrier before and
//     after each staging: 21 KB per workgroup, 4+ workgroups per CU), with the maxima of
//     every 4-bin block; each thread reads its +-15-bin neighbours from LDS;
//   * the vertical +-7-frame part is register-resident: one sliding maximum M7 of the
//     row-max over the last 7 rows (from an 8-slot ring of pair maxima, 4 VALU/bin)
//     gives both `before` of the arriving row (the previous M7, strict) and `after` of
//     the row 7 back (the current M7, non-strict), whose candidate power waits in an
//     8-slot ring; ring slots are compile-time because the row loop is unrolled by 8;
//   * a decided row is emitted with 4 wave ballots (one per bin offset i < 4): mask
//     word 4*w + i of a frame holds, at bit l, the peak flag of bin 256*w + 4*l + i
//     ("ballot layout"; K3 and aidfp.engine.peaks_from_mask unshuffle it).
// Only hot 16-bin chunks (K1's per-row hot word, aidfp_layout.h hot_bit) are loaded; a wave whose
// window chunks are cold in every row of its strip exits at once (it only writes zero mask words).
// Strips are dealt to workgroups XCD-aware so neighbouring strips (which share
// halo rows) run on the same XCD's L2. The variants measured against this layout
//  live in the git history (commit c236449, the AID_K2_* switches).
#include "aidfp_device.h"

namespace aid {

constexpr int kRowsPerStep = 4;

#if defined(AID_K2_STAMPS)
// Diagnostic build only (build_ext.build(variant=..., defines=("AID_K2_STAMPS",)), probes/k2_stamps_probe.py): each
// surviving wave sums s_memtime cycles spent at the step's first barrier (waiting for the other waves of its
// workgroup to finish the previous 4 rows) and adds them here at its end. Two s_memtime per step, their
// difference taken a step later (no extra wait in the row logic). [0] barrier wait, [5] surviving waves,
// [6] their whole lives (entry to end), [7] strip-cold (exiting) waves; [1..4] unused
__device__ unsigned long long g_k2_stamps[8];
#define AID_K2_T() ((unsigned long long)__builtin_amdgcn_s_memtime())
#endif

// Peak decisions compare powers as int32 keys: a power is >= +0 (never -0: FPSPEC 4's
// fma(Xr, Xr, Xi*Xi), stored unscaled as 4P by K1), and non-negative binary32 values order exactly like their bit
// patterns. NaN maps to key 0, which reproduces the oracle's `row > l ? row : l` maxima (a NaN
// neighbour never raises a maximum) and `!(p > thr)` (a NaN is never a peak); +inf keeps its
// bits. Integer max needs no NaN canonicalisation: hipcc put a `v_max_f32 x, x, x` in front of
// ~19 of the ~65 fmaxf operands of every row.
template <int LANE>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t s_val) {  // v[LANE] = s_val (uniform)
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s_val), "i"(LANE));
    return v;
}

__device__ __forceinline__ int pkey(float x) {
    // one VALU instead of v_cmp + v_cndmask (+ the VCC hazard's s_nop). Same keys: the plane holds K1's
    // fma results (quiet NaNs, no sNaN, no negative non-NaN values), and maxNum(qNaN, 0) = 0
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
    return __float_as_int(r);
}

// occupancy 4 forced by the launch bounds (<= 128 VGPRs, no spills)
#if defined(AID_K2_PF2) && defined(AID_K2_OCC3)
__global__ __launch_bounds__(256, 3) void k_peak_pick(
#else
__global__ __launch_bounds__(256, 4) void k_peak_pick(
#endif
                                                  const float *__restrict__ power, const ClipDesc *__restrict__ clips,
                                                  int n_clips, int64_t f0, int64_t total_strips, int strip_len, float thr,
                                                  const uint64_t *__restrict__ hot, uint64_t *__restrict__ mask,
                                                  uint32_t *__restrict__ cold_cnt) {
    __shared__ __attribute__((aligned(16))) int rows[kRowsPerStep][kBins + 32];  // keys, 16 pads each side
    __shared__ __attribute__((aligned(16))) int bms[kRowsPerStep][256 + 8];  // block maxima, 4 pads each side
    // wave = the 256-bin quarter of the row this wave owns, rotated by the workgroup index: the
    // waves of a workgroup go to the CU's 4 SIMDs in order, so without rotation every workgroup's
    // low-frequency (hot) quarter lands on SIMD 0 and its cold top quarter on SIMD 3
#if defined(AID_K2_STAMPS)
    const unsigned long long st_birth = AID_K2_T();
    unsigned long long st_bar = 0, st_b0 = 0, st_b1 = 0;
#endif
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(((int)(threadIdx.x >> 6) + (int)blockIdx.x) & 3);
    const int tid = wave * 64 + lane;  // owner of bins 4 tid .. 4 tid + 3
    constexpr int kInf = 0x7F800000;  // key of +inf

    // XCD-aware deal: consecutive strips -> blocks b, b+8, b+16 ... (one XCD's L2)
    int64_t strip;
    {
        const int64_t nb = gridDim.x, b = blockIdx.x;
        const int64_t per = nb / 8, rem = nb % 8, x = b % 8, y = b / 8;
        strip = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + y;
        strip = nb - 1 - strip;  // last-written power rows (still in the MALL after K1) first
    }
    if (strip >= total_strips) return;
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].strip_base <= strip) lo = mid; else hi = mid - 1;
    }
    // row indices of one clip fit 32 bits (scalar compares; 64-bit ones went to the VALU)
    const int F = (int)clips[lo].frames;
    const int64_t fb = clips[lo].frame_base;
    const int t0 = (int)(strip - clips[lo].strip_base) * strip_len;
    const int t1 = min(t0 + strip_len, F);
    const float *P = power + (fb - f0) * kBins;  // the plane holds rows from absolute frame f0 on
    uint64_t *M = mask + fb * kMaskWords + 4 * wave + lane;  // lanes 0..3 store ballot words
    // K1's plane holds Q = 4P (stft.hip, real split): compare against 4 thr (exact: thr <= 2^100)
    const int kthr = __float_as_int(4.0f * thr);            // thr > 0 (engine config check)

    if (tid < 16) {
#pragma unroll
        for (int r = 0; r < kRowsPerStep; ++r) {
            rows[r][tid] = 0;
            rows[r][kBins + 16 + tid] = 0;
            if (tid < 4) {
                bms[r][tid] = 0;
                bms[r][260 + tid] = 0;
            }
        }
    }

    // vertical +-7 as one sliding max: M7(s) = max row-max (fm) over rows s-6..s, built from
    // pair maxima m2[s] = max(fm[s], fm[s-1]) as max(m2[s], m2[s-2], m2[s-4], m2[s-5]).
    // `before` of row s is M7(s-1) (strict), `after` of row s-7 is M7(s) (non-strict).
    int m2r[8][4];   // pair maxima, slot = iteration & 7
    int pend[8][4];  // key of this row's candidates (-1 = none), decided 7 rows later
    int fprev[4], m7p[4];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) { m2r[s][i] = 0; pend[s][i] = -1; }
#pragma unroll
    for (int i = 0; i < 4; ++i) { fprev[i] = 0; m7p[i] = 0; }
    // bin 0 is never a peak: a uniform lane mask applied in the candidate test (SALU) instead of a per-lane +inf
    // `before` bound (one VALU per row): K2 -0.7 % same-box (profiles/r03ai_k2_b0mask_ab.txt)
    const uint64_t b0ok = __ballot(tid != 0);

    // iteration it processes row r = t0 - 7 + it and decides row r - 7
    const int rbeg = t0 - kPeakDT;
    const int iters = (t1 - t0) + 2 * kPeakDT;
    // K1's hot word of each row: a thread loads its 4 bins only if their 16-bin chunk has a value
    // > thr; others stay 0 (a value <= thr neither is a peak nor suppresses one: exact).
    // Words are fetched one step ahead of the row loads they gate (scalar loads)
    const uint64_t *HW = hot + fb;
    const int myb = hot_bit(tid >> 2);
    auto hotword = [&](int r) -> uint64_t { return (r >= 0 && r < F) ? HW[r] : 0ull; };
    // The loop's words come in through ONE vector load per step (lane l & 3 holds the word of row rb + (l & 3))
    // and are read out with v_readlane: a scalar load shares lgkmcnt with the LDS, so the barrier after the
    // staging (s_waitcnt lgkmcnt(0)) waited for the words just fetched, an L2/MALL round trip every 4 rows; the
    // vector load is waited together with the row loads issued beside it (vmcnt, one step later)
    auto hotwords = [&](int rb) -> uint64_t {
        const int r = rb + (lane & 3);
        return (r >= 0 && r < F) ? HW[r] : 0ull;
    };
    auto word_of = [](uint64_t v, int j) -> uint64_t {  // lane j's word, uniform (j compile-time)
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), j) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)v, j);
    };
    // chunks 16w-1 .. 16w+16 hold the wave's bins and their +-15 neighbours
    uint64_t wmask = 0;
    for (int c = max(16 * wave - 1, 0); c <= min(16 * wave + 16, 63); ++c) wmask |= 1ull << hot_bit(c);
    {
        // strip-cold wave: if those blocks are cold in every row the strip reads, every key this wave
        // stages or compares is 0, so it has no candidate and its mask words are 0 (exact, as the
        // per-row cold skip). It writes those zeros, zeroes its staged bins once (the neighbouring
        // waves' windows read them), and only keeps the workgroup's barrier count (2 per 4 rows)
        uint64_t acc = 0;
        for (int r = rbeg + lane; r < rbeg + iters; r += 64) acc |= (r >= 0 && r < F) ? HW[r] : 0ull;
        if (__ballot((acc & wmask) != 0ull) == 0) {
#pragma unroll
            for (int j = 0; j < kRowsPerStep; ++j) {
                reinterpret_cast<int4 *>(&rows[j][16])[tid] = make_int4(0, 0, 0, 0);
                bms[j][4 + tid] = 0;
            }
            uint64_t *Mz = mask + fb * kMaskWords + 4 * wave + (lane & 3);
            for (int r = t0 + (lane >> 2); r < t1; r += 16) Mz[(int64_t)r * kMaskWords] = 0;
            // the wave terminates: s_barrier waits only for a workgroup's surviving waves, and its
            // registers go to waves of workgroups still waiting for a slot (host: extract_locked); its
            // zeroed LDS bins are written before it ends. The cold waves are counted (64 counters, read
            // and reset by K3) so the host can size the next call's strips (extract_locked)
            if (lane == 0 && cold_cnt) atomicAdd(&cold_cnt[blockIdx.x & 63], 1u);
#if defined(AID_K2_STAMPS)
            if (lane == 0) atomicAdd(&g_k2_stamps[7], 1ull);
#endif
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            return;
        }
    }
    // Row loads are range-checked buffer loads over the strip's rows (rlo .. rhi): a thread whose chunk is cold (or
    // whose row lies outside the clip: hot word 0) passes an offset past the range and gets zeros without a branch
    // (an exec-masked load with a zero-initialised phi made hipcc copy the loaded registers right after the load,
    // behind an s_waitcnt vmcnt(0))
    const int rlo = max(rbeg, 0), rhi = min(rbeg + iters, F);
    const __amdgpu_buffer_rsrc_t rows_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(P + (int64_t)rlo * kBins), (short)0, (rhi - rlo) * kBins * 4, 0x00020000);
    constexpr uint32_t kOOB = 0x80000000u;  // past any strip's byte count (< 2^31)
    auto load_row = [&](int r, uint64_t hwr) -> float4 {
        const uint32_t off = ((hwr >> myb) & 1ull) ? (uint32_t)(r - rlo) * (kBins * 4) + 16u * tid : kOOB;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rows_rsrc, off, 0, 0);
        return make_float4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
    };
#if defined(AID_K2_PF2)
    // diagnostic variant (timing A/B only, tools/variant_build.py ... -DAID_K2_PF2): rows fetched TWO steps ahead (8 rows
    // in flight per thread) from two register buffers that alternate with the 8-row unroll (buffer s / 4)
    float4 pfb[2][kRowsPerStep];
    uint64_t hs[2][kRowsPerStep], hcur[kRowsPerStep];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < kRowsPerStep; ++j) {
            const int r = rbeg + b * kRowsPerStep + j;
            hs[b][j] = hotword(r);
            pfb[b][j] = load_row(r, b * kRowsPerStep + j < iters ? hs[b][j] : 0ull);
            hcur[j] = 0ull;
        }
    uint64_t hwv = hotwords(rbeg + 2 * kRowsPerStep);  // hot words of the rows the next staging fetches (lane & 3)
#else
    float4 pf[kRowsPerStep];  // rows of the next step, in flight
#pragma unroll
    for (int j = 0; j < kRowsPerStep; ++j) pf[j] = load_row(rbeg + j, j < iters ? hotword(rbeg + j) : 0ull);
    uint64_t hwv = hotwords(rbeg + kRowsPerStep);  // hot words of the rows the next step fetches (lane & 3)
    // hot words of the rows in flight (hsave) and of the rows being processed (hcur)
    uint64_t hsave[kRowsPerStep], hcur[kRowsPerStep];
#pragma unroll
    for (int j = 0; j < kRowsPerStep; ++j) hsave[j] = hcur[j] = hotword(rbeg + j);
#endif

    for (int base = 0; base < iters; base += 8) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int it = base + s;
            if (it >= iters) break;  // workgroup-uniform
            if (s % kRowsPerStep == 0) {
#if defined(AID_K2_STAMPS)
                st_bar += st_b1 - st_b0;  // the previous step's barrier wait (its stamps have long arrived)
                st_b0 = AID_K2_T();
                if (it > 0) __syncthreads();
                st_b1 = AID_K2_T();
#else
                if (it > 0) __syncthreads();  // every wave is done with the previous 4 rows
#endif
                // stage rows it .. it+3 as keys, then fetch rows it+PF .. (register staging beats
                // LDS-DMA here: 0.299 vs 0.323 ms at the same occupancy)
#if defined(AID_K2_PF2)
                const int b = (s / kRowsPerStep) & 1;  // compile-time after the 8-row unroll
#pragma unroll
                for (int j = 0; j < kRowsPerStep; ++j) {
                    const float4 v = pfb[b][j];
                    const int4 kv = make_int4(pkey(v.x), pkey(v.y), pkey(v.z), pkey(v.w));
                    reinterpret_cast<int4 *>(&rows[j][16])[tid] = kv;
                    bms[j][4 + tid] = max(max(kv.x, kv.y), max(kv.z, kv.w));
                    const int rn = rbeg + it + j + 2 * kRowsPerStep;
                    hcur[j] = hs[b][j];
                    hs[b][j] = word_of(hwv, j);
                    pfb[b][j] = load_row(rn, it + j + 2 * kRowsPerStep < iters ? hs[b][j] : 0ull);
                }
                hwv = hotwords(rbeg + it + 3 * kRowsPerStep);
#else
#pragma unroll
                for (int j = 0; j < kRowsPerStep; ++j) {
                    const int slot = (s + j) % kRowsPerStep;  // compile-time: the loop is unrolled by 8
                    const float4 v = pf[slot];
                    const int4 kv = make_int4(pkey(v.x), pkey(v.y), pkey(v.z), pkey(v.w));
                    reinterpret_cast<int4 *>(&rows[j][16])[tid] = kv;
                    bms[j][4 + tid] = max(max(kv.x, kv.y), max(kv.z, kv.w));
                    const int rn = rbeg + it + j + kRowsPerStep;
                    hcur[j] = hsave[j];
                    hsave[j] = word_of(hwv, j);
                    pf[slot] = load_row(rn, it + j + kRowsPerStep < iters ? hsave[j] : 0ull);
                }
                hwv = hotwords(rbeg + it + 2 * kRowsPerStep);
#endif
                __syncthreads();
            }
            const int r = rbeg + it;
            bool pk[4];
            uint64_t bal[4];  // ballots of pk, taken where pk is computed (SGPR results, no 0/1 VGPRs)
            if (!(hcur[s % kRowsPerStep] & wmask)) {
                // every key the wave's windows see is 0: fm = 0, no candidate (p = 0 is never > the
                // threshold); only the vertical ring advances and row r-7 is decided
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m2 = fprev[i];
                    fprev[i] = 0;
                    m2r[s][i] = m2;
                    const int m7 = max(max(max(m2, m2r[(s - 2) & 7][i]), m2r[(s - 4) & 7][i]), m2r[(s - 5) & 7][i]);
                    m7p[i] = m7;
                    pk[i] = pend[(s + 1) & 7][i] >= m7;
                    bal[i] = __ballot(pk[i]);
                    pend[s][i] = -1;
                }
            } else {
            // thread j owns block j = bins 4j..4j+3. Its +-15 windows span blocks j-4..j+4: the
            // far blocks j-4 / j+4 contribute a suffix / prefix of their bins, blocks j+-1..3 whole
            // (their maxima, staged with the row), the own block a prefix / suffix -- 18 max ops
            // per thread and row instead of 46, and 2 x 16 B + 6 x 4 B of LDS reads instead of 9 x 16 B
            const int4 *rb4 = reinterpret_cast<const int4 *>(rows[s % kRowsPerStep]);
            const int *bm = bms[s % kRowsPerStep];
            const int4 lf = rb4[tid], me = rb4[tid + 4], rt = rb4[tid + 8];  // blocks j-4, j, j+4
            // keep lf.x / rt.w live so hipcc issues ds_read_b128, not ds_read_b96 (lf uses bins 1..3, rt 0..2)
            asm volatile("" ::"v"(lf.x), "v"(rt.w));
            const int M3L = max(max(bm[tid + 1], bm[tid + 2]), bm[tid + 3]);  // blocks j-3..j-1
            const int M3R = max(max(bm[tid + 5], bm[tid + 6]), bm[tid + 7]);  // blocks j+1..j+3
            const int lsuf2 = max(lf.z, lf.w), lsuf1 = max(lf.y, lsuf2);      // block j-4: bins 1..3, 2..3
            const int rpre1 = max(rt.x, rt.y), rpre2 = max(rpre1, rt.z);      // block j+4: bins 0..1, 0..2
            const int mpre1 = max(me.x, me.y), mpre2 = max(mpre1, me.z);      // own prefixes
            const int msuf2 = max(me.z, me.w), msuf1 = max(me.y, msuf2);      // own suffixes
            int L[4], R[4];
            L[0] = max(lsuf1, M3L);
            L[1] = max(max(lsuf2, M3L), me.x);
            L[2] = max(max(lf.w, M3L), mpre1);
            L[3] = max(M3L, mpre2);
            R[0] = max(msuf1, M3R);
            R[1] = max(max(msuf2, M3R), rt.x);
            R[2] = max(max(me.w, M3R), rpre1);
            R[3] = max(M3R, rpre2);
            const int mev[4] = {me.x, me.y, me.z, me.w};

            // candidates only inside the strip's output rows (uniform): other rows get +inf
            const int thr_row = (r >= t0 && r < t1) ? kthr : kInf;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p = mev[i];
                const int fm = max(max(L[i], p), R[i]);
                const int m2 = max(fm, fprev[i]);
                fprev[i] = fm;
                // `before` reads the previous M7 ahead of the ring update, so the new M7 can take its register (with
                // the update first, both were live together and every hot row ended in 4 phi copies)
                const int bf = max(max(L[i], thr_row), m7p[i]);
                m2r[s][i] = m2;
                const int m7 = max(max(max(m2, m2r[(s - 2) & 7][i]), m2r[(s - 4) & 7][i]), m2r[(s - 5) & 7][i]);
                m7p[i] = m7;
                // row r-7 (slot s+1) has now met all 7 later rows: p >= their row-max
                pk[i] = pend[(s + 1) & 7][i] >= m7;
                bal[i] = __ballot(pk[i]);
                // candidate: p > before (strict) and p >= right window; keys >= 0, so -1 = none
                // two compares into SGPR masks and one s_and (3 VALU + 1 SALU) instead of add, max and one compare
                // (4 VALU): K2 -2.5 % bench data, -3.5 % full-band (profiles/r03ah_k2_cmp2_ab.txt)
                bool cand = p > bf && p >= R[i];
                if (i == 0) cand = cand && ((b0ok >> lane) & 1ull);
                pend[s][i] = cand ? p : -1;
            }
            }
            const uint64_t b0 = bal[0], b1 = bal[1], b2 = bal[2], b3 = bal[3];
            const int rd = r - kPeakDT;
            if (rd >= t0 && rd < t1) {
                // lane i < 4 stores ballot word i: 8 v_writelane of the SGPR ballots
                uint32_t lo, hi;  // no zero init (2 VALU per row): only lanes 0..3 are stored
                asm volatile("" : "=v"(lo), "=v"(hi));
                lo = write_lane<0>(lo, (uint32_t)b0);
                hi = write_lane<0>(hi, (uint32_t)(b0 >> 32));
                lo = write_lane<1>(lo, (uint32_t)b1);
                hi = write_lane<1>(hi, (uint32_t)(b1 >> 32));
                lo = write_lane<2>(lo, (uint32_t)b2);
                hi = write_lane<2>(hi, (uint32_t)(b2 >> 32));
                lo = write_lane<3>(lo, (uint32_t)b3);
                hi = write_lane<3>(hi, (uint32_t)(b3 >> 32));
                if (lane < 4) M[(int64_t)rd * kMaskWords] = ((uint64_t)hi << 32) | lo;
            }
        }
    }
#if defined(AID_K2_STAMPS)
    {
        const unsigned long long t = AID_K2_T();
        st_bar += st_b1 - st_b0;
        if (lane == 0) {
            atomicAdd(&g_k2_stamps[0], st_bar);
            atomicAdd(&g_k2_stamps[5], 1ull);
            atomicAdd(&g_k2_stamps[6], t - st_birth);
        }
    }
#endif
}

#if defined(AID_K2_STAMPS)
int k2_stamps_read(unsigned long long *out, bool reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k2_stamps), sizeof(unsigned long long) * 8) != hipSuccess) return -2;
    if (reset) {
        const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_k2_stamps), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

// power holds the rows from absolute frame f0 on (a group of the call's clips, extract_locked); the clips' strip_base
// count from 0 within the group
void launch_peak_pick(const float *power, const ClipDesc *clips, int n_clips, int64_t f0, int64_t total_strips,
                      int strip_len, float thr, const uint64_t *hot, uint64_t *mask, uint32_t *cold_cnt, hipStream_t s) {
    if (total_strips <= 0) return;
    timed_launch(k_peak_pick, dim3((unsigned)total_strips), dim3(256), 0, s, power, clips, n_clips, f0, total_strips,
                 strip_len, thr, hot, mask, cold_cnt);
}

// resident K2 workgroups per CU (registers / LDS), for sizing strips to one round
int peak_pick_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_peak_pick, 256, 0) != hipSuccess || n <= 0) n = 1;
    return n;
}

}  // namespace aid
