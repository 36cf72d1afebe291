// stft.hip -- K1 `stft_power`: framing + Hann window + 1024-point complex FFT +
// real split + |X|^2 (spec/FPSPEC.md 4), one wavefront per frame.
//
// Replaces the FFT stage inside the external `olaf_c` binary that the reference
// runs per call (audio-ident-service/app/audio/fingerprint.py:117-125 store,
// :185-193 query).
//
// Work mapping (gfx950, wave64):
//   * each wave owns an equal range of the batch's frames. Lane l keeps the complex
//     samples z[64*n1 + l] (n1 < 16, "rows" of 128 PCM samples) in a 16-slot register
//     ring: frame t+1 reuses 16 - H/128 rows of frame t, so only the new hop is loaded
//     (H/128 float2 loads per lane, 512 contiguous bytes per wave-instruction) and every
//     PCM byte crosses HBM -> VGPR once per range (the ring restarts at clip edges only).
//     The next frame's rows are loaded right after the window multiply, so their latency
//     hides under the FFT;
//   * stage A = 16-point DFT in registers, twiddle by T1K, then the transpose E1 through
//     the wave's LDS buffer (written with ds_write_addtid_b32, read as ds_read_b128);
//   * stage B = 16-point DFT in registers, twiddle by T64;
//   * stage C = radix 4 across the lane quad on DPP (v_fmac_f32_dpp butterflies), spilled
//     to LDS (E3) in 32-byte groups, from which the real split reads each mirror pair
//     (Z[k], Z[1024-k]) once and produces both bins; stores are 64 consecutive bins per
//     wave-instruction (the mirror bins in descending order, same 256-B segment).
// A workgroup is kStftWaves = 16 waves (4 per SIMD) sharing the tables in LDS; the
// exchanges are wave-private, so there is no workgroup barrier in the frame loop.
// The variants measured against this layout live in the git history
// (commit c236449, the AID_K1_* switches).
#include "aidfp_device.h"

// The add-TID writes below set M0 inside their asm and name it as clobbered; clang warns that M0 is a reserved
// register whose value it will not preserve across the asm. Nothing else in this kernel may use M0:
// tests/test_isa_m0.py compiles this file and fails on any M0 access outside these asm blocks. The warning
// is silenced for the AID_TID8 statements only (push/pop around each use).

// E1 layout. Each (k1, component) register of stage A goes lane-linear to its own 64-dword
// region with ds_write_addtid_b32 (address = M0 + offset + 4 lane: no address VGPR, 2 LDS
// cycles per instruction). Stage-A lane p holds n2 = e1_perm(p) = 4 (p & 15) + (p >> 4), so a
// stage-B reader (kq, mq) finds n2 = 4 m1 + mq for m1 = 4t .. 4t+3 at positions 16 mq + 4t .. +3
// of region (kq, c): one ds_read_b128 per (t, c), 8 per frame. The region bases
// 128 k1 + 64 c + 4 (k1 & 3) + 16 (k1 >> 2) put the 16 lanes of every b128 lane group on 16
// distinct 4-bank quads (conflict-free writes and reads). The PCM loads of a stage-A lane stay
// inside the same 512-B segment; the window and T1K tables are staged in that lane order.
__host__ __device__ constexpr int e1_perm(int p) { return 4 * (p & 15) + (p >> 4); }
__host__ __device__ constexpr int e1_region(int k1, int c) { return 128 * k1 + 64 * c + 4 * (k1 & 3) + 16 * (k1 >> 2); }
static_assert(e1_region(15, 1) + 64 <= 2 * aid::kStftLdsPerWave, "E1 regions exceed the wave buffer");
// 8 registers' components -> their regions (M0 = the wave buffer's LDS byte address). s_nop 0: one wait
// state between an SALU write of M0 and an add-TID LDS instruction
#define AID_TID8(RG, K0)                                                                                     \
    _Pragma("clang diagnostic push") _Pragma("clang diagnostic ignored \"-Winline-asm\"")                      \
    asm volatile("s_mov_b32 m0, %[base]\n\ts_nop 0\n\t"                                                      \
                 "ds_write_addtid_b32 %0 offset:%8\n\tds_write_addtid_b32 %1 offset:%9\n\t"                  \
                 "ds_write_addtid_b32 %2 offset:%10\n\tds_write_addtid_b32 %3 offset:%11\n\t"                \
                 "ds_write_addtid_b32 %4 offset:%12\n\tds_write_addtid_b32 %5 offset:%13\n\t"                \
                 "ds_write_addtid_b32 %6 offset:%14\n\tds_write_addtid_b32 %7 offset:%15"                    \
                 :                                                                                           \
                 : "v"(v[K0].x), "v"(v[K0].y), "v"(v[K0 + 1].x), "v"(v[K0 + 1].y), "v"(v[K0 + 2].x),         \
                   "v"(v[K0 + 2].y), "v"(v[K0 + 3].x), "v"(v[K0 + 3].y), "i"(4 * RG(K0, 0)),                 \
                   "i"(4 * RG(K0, 1)), "i"(4 * RG(K0 + 1, 0)), "i"(4 * RG(K0 + 1, 1)),                       \
                   "i"(4 * RG(K0 + 2, 0)), "i"(4 * RG(K0 + 2, 1)), "i"(4 * RG(K0 + 3, 0)),                   \
                   "i"(4 * RG(K0 + 3, 1)), [base] "s"(m0base)                                                \
                 : "memory", "m0");                                                                          \
    _Pragma("clang diagnostic pop")

namespace aid {

// 16-lane groups of a wave-wide mask -> 4 bits: bit g = some lane of lanes 16g .. 16g+15 is set (two
// s_quadmask_b64: 64 lanes -> 16 quads -> 4 groups of 4 quads). s_quadmask writes SCC: without the clobber hipcc
// may compute a branch condition into SCC before these and branch on it after them
__device__ __forceinline__ uint64_t group16(uint64_t m) {
    uint64_t q, r;
    asm("s_quadmask_b64 %0, %1" : "=s"(q) : "s"(m) : "scc");
    asm("s_quadmask_b64 %0, %1" : "=s"(r) : "s"(q) : "scc");
    return r;
}

// power-row store, non-temporal (streaming): K1 0.268 -> 0.266 ms, K2 0.134 -> 0.130 ms same-box (r02)
__device__ __forceinline__ void pstore(float *p, float v) {
#if defined(AID_K1_NOSTORE)  // timing-only diagnostic build: what K1's power stores cost (results are wrong)
    asm volatile("" ::"v"(v), "v"(p));
#else
    __builtin_nontemporal_store(v, p);
#endif
}

// E3 slot of Z[k] = 4 (k & 255) + (j2 ^ 2 h), j2 = k >> 8, h = bit 3 of k: the four Z[k + 256 j2] sit in one
// 32-B group with the (j2 = 0, 1) and (2, 3) halves swapped by bit 3, so the real split reads (Z[k], Z[k + 256])
// and (Z[768 - k], Z[1024 - k]) as one ds_read_b128 each (8 per frame; stage-C writers and both readers
// conflict-free, checked exhaustively). Lane 0's unit-0 mirror read lands on a copy of Z[768] at slot 1026,
// written by lane 3 of stage C.
// PCM ring loads are non-temporal: K1 reads each sample once, and streaming it past the caches leaves the Infinity
// Cache to the hot power rows K2 reads next (K2 -2 %, step -0.8 %, K1 unchanged in a 3-round same-box A/B,
// profiles/r04q_k1_ntload_ab.txt)
// A clip may start at an odd sample (device clips, the exact lane's in-place sub-windows), so a frame's sample
// pairs are only 4-byte aligned: they are read through a 2-float vector type declared 4-byte aligned (the same
// global_load_dwordx2; a float2 pointer would promise the compiler 8 bytes)
typedef float aid_f2u __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ float2 pcm_ld(const aid_f2u &r) {
    const aid_f2u v = __builtin_nontemporal_load(&r);
    return make_float2(v.x, v.y);
}
#define AID_PCM(ref) pcm_ld(ref)

__device__ __forceinline__ int e3q_slot(int k) { return 4 * (k & 255) + ((k >> 8) ^ (2 * ((k >> 3) & 1))); }

template <bool LOGMAG, int ROWS>
__global__ __launch_bounds__(kStftWaves * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_stft_power(const float *__restrict__ pcm,
                                                                const ClipDesc *__restrict__ clips, int n_clips,
                                                                int64_t f0, int64_t total, int64_t n_waves,
                                                                const Tables *__restrict__ tab, float *__restrict__ out,
                                                                uint64_t *__restrict__ hot, float thr, int keep) {
    constexpr int PERIOD = 16 / ROWS;  // frames per full ring rotation
    constexpr int HOP2 = 64 * ROWS;    // hop in float2 units
    __shared__ __attribute__((aligned(16))) float2 lds[kStftWaves][kStftLdsPerWave];  // E1 regions, then E3
    // tables as float4 pairs [h][lane], one ds_read_b128 per pair (hipcc would otherwise merge the
    // stride-512-B float2 reads into ds_read2st64_b64, which costs the LDS twice the cycles):
    //   s_win4[h] = window of rows 2h, 2h+1 ; s_ta4[h] = T1K[lane*k1], k1 = 2h, 2h+1
    //   s_tb4[h] = T64[(lane&3)*j1], j1 = 2h, 2h+1 ; s_t24[j][lane] = T2K[k], T2K[k + 256], k = 64 j + lane < 256:
    //   the pair the real split uses together (T2K[1024-k] = (-re, im), checked in aid_engine_create; as float2
    //   reads hipcc merged them into ds_read2st64_b64, 8 LDS cycles per pair instead of 4)
    __shared__ float4 s_win4[512], s_ta4[512];
    __shared__ float4 s_t24[256];
    __shared__ float4 s_tb4[32];  // [h][lane & 3]: T64[m2*j1] depends on the lane only through m2
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar strip/segment math
    float2 *buf = lds[wave];
    const int kq = lane >> 2;  // stage B/C: k1
    const int mq = lane & 3;   // stage B: m2 ; stage C: s
    // LDS byte address of this wave's buffer (M0 of the add-TID writes) and of the lane's E1 reads
    const uint32_t m0base =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float2 *)buf);
    const uint32_t e1rd = m0base + 4u * (uint32_t)(e1_region(kq, 0) + 16 * mq);
    // stage-C lane (kq, mq) holds Z[kq + 16 j1 + 256 bitrev2(mq)] in register j1
    const int j2q = ((mq & 1) << 1) | (mq >> 1);
    const int e3wq = 4 * kq + (j2q ^ (2 * ((kq >> 3) & 1)));  // its E3 slot, + 64 j1
    // split reads (float4 units): (Z[k], Z[k + 256]) at 2 k + h(k), (Z[768 - k], Z[1024 - k]) at 2 m + 1 - h(m),
    // m = 256 - k, k = lane + 64 i (i < 4; the i terms are immediates)
    const int e3qa = 2 * lane + ((lane >> 3) & 1);
    const int e3qb = 513 - 2 * lane - (((256 - lane) >> 3) & 1);
    // lane 0's unit-0 mirror read (m = 256) takes slots 1026, 1027 as (Z[768 - 0], Z[1024 - 0]): Z[768] (stage-C lane 3,
    // register 0) is copied to 1026; slot 1027 (Z[0]) is not used (k = 0 pairs with Z[0] from its own read)
    const int e3dup = lane == 3 ? 1026 : 1028 + lane;  // < kStftLdsPerWave (1092)
    const float s1 = mq < 2 ? 1.0f : -1.0f;                     // butterfly over lanes (mq, mq ^ 2)
    const float s2 = (mq == 1 || mq == 2) ? -1.0f : 1.0f;       // butterfly over lanes (mq, mq ^ 1)
    const float s0 = lane == 0 ? 1.0f : -1.0f;  // sign of Z[0]'s mirror slot for i = 0 (Z[0] itself)

    for (int i = threadIdx.x; i < 512; i += kStftWaves * 64) {
        const int h = i >> 6, l = i & 63, a = 2 * h, b = 2 * h + 1;
        const int ln = e1_perm(l);  // the n2 stage-A lane l holds
        const float2 w0 = tab->win2[64 * a + ln], w1 = tab->win2[64 * b + ln];
        s_win4[i] = make_float4(w0.x, w0.y, w1.x, w1.y);
        const float2 ta0 = tab->t1k[ln * a], ta1 = tab->t1k[ln * b];
        s_ta4[i] = make_float4(ta0.x, ta0.y, ta1.x, ta1.y);
        if (l < 4) {
            const float2 tb0 = tab->t64[l * a], tb1 = tab->t64[l * b];
            s_tb4[4 * h + l] = make_float4(tb0.x, tb0.y, tb1.x, tb1.y);
        }
        if (i < 256) {
            const float2 ta = tab->t2k[i], tb = tab->t2k[i + 256];
            s_t24[i] = make_float4(ta.x, ta.y, tb.x, tb.y);
        }
    }
    const float2 t512 = tab->t2k[512];
    float2 t16[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t16[i] = tab->t16[i];
    __syncthreads();

    // wave g takes frames [g*T/W, (g+1)*T/W) of the batch's T frames (W waves): every wave has
    // the same work (no partial last round), and a segment restarts the ring only at a clip edge
    const int64_t g = (int64_t)blockIdx.x * kStftWaves + wave;
    if (g >= n_waves) return;  // wave-uniform, after the only barrier
    // frames [f0, f0 + total) of the call (a group of its clips, extract_locked); out holds rows from f0 on
    int64_t f = f0 + g * total / n_waves;
    const int64_t f_end = f0 + (g + 1) * total / n_waves;
    while (f < f_end) {
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {  // last clip with frame_base <= f (scalar loads): the clip holding frame f
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].frame_base <= f) lo = mid; else hi = mid - 1;
    }
    const int64_t t0 = f - clips[lo].frame_base;
    const int nfr = (int)min(f_end - f, clips[lo].frames - t0);
    const aid_f2u *src = reinterpret_cast<const aid_f2u *>(pcm + clips[lo].pcm_off) + t0 * HOP2 + e1_perm(lane);
    float *dst = out + (clips[lo].frame_base - f0 + t0) * kBins;
    uint64_t *dhot = LOGMAG ? nullptr : hot + clips[lo].frame_base + t0;

    float2 ring[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ring[r] = AID_PCM(src[64 * r]);
    // the segment's first frame needs the whole ring anyway: wait for it here, so the frame loop's
    // header does not inherit this path's pending loads (hipcc's wait at the header, merged over both
    // edges, was vmcnt(1): every 4 frames the wave also waited for the previous frame's 17 stores)
    // (an empty asm reading every ring register: hipcc must complete the loads before it)
#pragma unroll
    for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(ring[r].x), "v"(ring[r].y));

    for (int f0 = 0; f0 < nfr; f0 += PERIOD) {
#pragma unroll
        for (int p = 0; p < PERIOD; ++p) {
            const int f = f0 + p;
            if (f < nfr) {  // wave-uniform
                float2 v[16];
                // the 8 window reads issued together ahead of a sched_barrier (hipcc serialized them, each
                // behind its own lgkmcnt(0))
                float4 wpf[8];
#pragma unroll
                for (int h = 0; h < 8; ++h) wpf[h] = s_win4[64 * h + lane];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const float4 w = wpf[h];
                    const float2 x0 = ring[(2 * h + ROWS * p) & 15], x1 = ring[(2 * h + 1 + ROWS * p) & 15];
                    v[2 * h] = make_float2(x0.x * w.x, x0.y * w.y);
                    v[2 * h + 1] = make_float2(x1.x * w.z, x1.y * w.w);
                }
                // the rows just consumed (n1 < ROWS) are replaced by frame f+1's new rows (after the
                // last frame of the segment: a harmless re-load of its own rows, instead of a branch)
                {
                    const int fn = min(f + 1, nfr - 1);
#pragma unroll
                    for (int j = 0; j < ROWS; ++j)
                        ring[(ROWS * p + j) & 15] = AID_PCM(src[(int64_t)fn * HOP2 + 64 * (16 - ROWS + j)]);
                }
                // stage A: lane = n2
                dft16(v, t16);
                // T1K[n2*k1]; lane 0 multiplies by T1K[0] = (1,-0): value-identical (FPSPEC 4 note)
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const float4 t = s_ta4[64 * h + lane];
                    if (h) v[2 * h] = cmul(v[2 * h], make_float2(t.x, t.y));
                    v[2 * h + 1] = cmul(v[2 * h + 1], make_float2(t.z, t.w));
                }
                // E1: A[k1][n2] -> lane (k1 = kq, m2 = mq) gets A[kq][4*m1 + mq]
                {
                    AID_TID8(e1_region, 0);
                    AID_TID8(e1_region, 4);
                    AID_TID8(e1_region, 8);
                    AID_TID8(e1_region, 12);
                    {
                        float4 q[8];  // q[2 t + c] = component c of A[kq][4 m1 + mq], m1 = 4t .. 4t+3
                        asm volatile(
                            "ds_read_b128 %0, %8 offset:0\n\tds_read_b128 %1, %8 offset:256\n\t"
                            "ds_read_b128 %2, %8 offset:16\n\tds_read_b128 %3, %8 offset:272\n\t"
                            "ds_read_b128 %4, %8 offset:32\n\tds_read_b128 %5, %8 offset:288\n\t"
                            "ds_read_b128 %6, %8 offset:48\n\tds_read_b128 %7, %8 offset:304\n\t"
                            "s_waitcnt lgkmcnt(0)"
                            : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),
                              "=&v"(q[6]), "=&v"(q[7])
                            : "v"(e1rd)
                            : "memory");
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const float4 re = q[2 * t], im = q[2 * t + 1];
                            v[4 * t] = make_float2(re.x, im.x);
                            v[4 * t + 1] = make_float2(re.y, im.y);
                            v[4 * t + 2] = make_float2(re.z, im.z);
                            v[4 * t + 3] = make_float2(re.w, im.w);
                        }
                    }
                    wave_lds_sync();
                }
                // stage B
                float4 tpb[8];
#pragma unroll
                for (int h = 0; h < 8; ++h) tpb[h] = s_tb4[4 * h + mq];
                __builtin_amdgcn_sched_barrier(0);
                dft16(v, t16);
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const float4 t = tpb[h];
                    if (h) v[2 * h] = cmul(v[2 * h], make_float2(t.x, t.y));
                    v[2 * h + 1] = cmul(v[2 * h + 1], make_float2(t.z, t.w));
                }
                // stage C across the quad (FPSPEC 3 DFT4 over m2 = mq, for every j1), each butterfly
                // one in-place fma with the partner as DPP operand: x <- partner * s + x
                //   s1 = (+1, +1, -1, -1): lanes 0..3 -> t0, t2, -t1, -t3
                //   lane 3: u = -i t3 from -t3: (-T.im, T.re); lanes 0..2 keep their value
                //   s2 = (+1, -1, -1, +1): lanes 0..3 -> y0, -y2, -y1, -y3
                // fma(p, +-1, x) rounds x +- p once: FPSPEC's add/sub values; the signs are exact
                // and cancel in the real split (see there)
                // hand-placed: v_fmac_f32_dpp (partner * s + x, in place) keeps the DPP inside the
                // fma; the leading s_nop 1 covers the VALU-write -> DPP-read hazard of the block's
                // inputs, and every other DPP source was written >= 2 instructions earlier
#pragma unroll
                for (int j0 = 0; j0 < 16; j0 += 4) {
                    float u0, w0, u1, w1, u2, w2, u3, w3;
                    asm volatile(
                        "s_nop 1\n\t"
                        "v_fmac_f32_dpp %8, %8, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %9, %9, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %10, %10, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %11, %11, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %12, %12, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %13, %13, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %14, %14, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %15, %15, %16 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                        "v_cndmask_b32_e64 %0, %8, -%9, %18\n\t"
                        "v_cndmask_b32_e64 %1, %9, %8, %18\n\t"
                        "v_cndmask_b32_e64 %2, %10, -%11, %18\n\t"
                        "v_cndmask_b32_e64 %3, %11, %10, %18\n\t"
                        "v_cndmask_b32_e64 %4, %12, -%13, %18\n\t"
                        "v_cndmask_b32_e64 %5, %13, %12, %18\n\t"
                        "v_cndmask_b32_e64 %6, %14, -%15, %18\n\t"
                        "v_cndmask_b32_e64 %7, %15, %14, %18\n\t"
                        "v_fmac_f32_dpp %0, %0, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %1, %1, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %2, %2, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %3, %3, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %4, %4, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %5, %5, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %6, %6, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %7, %7, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                        : "=&v"(u0), "=&v"(w0), "=&v"(u1), "=&v"(w1), "=&v"(u2), "=&v"(w2), "=&v"(u3), "=&v"(w3),
                          "+v"(v[j0].x), "+v"(v[j0].y), "+v"(v[j0 + 1].x), "+v"(v[j0 + 1].y), "+v"(v[j0 + 2].x),
                          "+v"(v[j0 + 2].y), "+v"(v[j0 + 3].x), "+v"(v[j0 + 3].y)
                        : "v"(s1), "v"(s2), "s"(0x8888888888888888ull));
                    v[j0] = make_float2(u0, w0);
                    v[j0 + 1] = make_float2(u1, w1);
                    v[j0 + 2] = make_float2(u2, w2);
                    v[j0 + 3] = make_float2(u3, w3);
#pragma unroll
                    for (int j = 0; j < 4; ++j) buf[e3wq + 64 * (j0 + j)] = v[j0 + j];
                    // Z[768] (lane 3) copied to 1026, every other lane to its own dummy slot: one unconditional
                    // store (an exec-masked branch here made hipcc spill)
                    if (j0 == 0) buf[e3dup] = v[0];
                }
                wave_lds_sync();
                float *drow = dst + (int64_t)f * kBins;
                if constexpr (!LOGMAG) {
                    // straight-line real split: all 16 powers first, then the row's hot word, then the
                    // stores of the hot blocks (scalar branches after the arithmetic, so no branch splits it)
                    // the row's hot word (aidfp_layout.h hot_bit): bit of 16-bin chunk c = some bin of c is > thr
                    uint64_t hotw = 0;
                    float po[8], pm[8];
                    float4 qa, qb, t2p;  // the b128 reads that serve bins i and i + 4
#pragma unroll
                    for (int ii = 0; ii < 8; ++ii) {
                        // order i = 0, 4, 1, 5, ...: one set of reads serves two mirror pairs, then dies
                        const int i = (ii >> 1) + 4 * (ii & 1);
                        if ((ii & 1) == 0) {
                            const float4 *buf4 = reinterpret_cast<const float4 *>(buf);
                            qa = buf4[e3qa + 128 * (ii >> 1)];
                            qb = buf4[e3qb - 128 * (ii >> 1)];
                            t2p = s_t24[64 * (ii >> 1) + lane];
                        }
                        // i < 4: a = Z[k], bs = -Z[1024 - k] (stored); i >= 4: a = -Z[k], bs = -Z[1024 - k] (k >= 256)
                        const float2 a = i < 4 ? make_float2(qa.x, qa.y) : make_float2(qa.z, qa.w);
                        const float2 bs = i < 4 ? make_float2(qb.z, qb.w) : make_float2(qb.x, qb.y);
                        // k = 0 (lane 0, i = 0) pairs with Z[0] itself
                        const float2 b = i == 0 ? (lane == 0 ? a : make_float2(-bs.x, -bs.y)) : i < 4 ? make_float2(-bs.x, -bs.y) : bs;
                        const float er = a.x + b.x, ei = a.y - b.y;
                        const float orr = a.y + b.y, oi = b.x - a.x;
                        const float2 t2h = i < 4 ? make_float2(t2p.x, t2p.y) : make_float2(t2p.z, t2p.w);
                        const float2 tw = cmul(make_float2(orr, oi), t2h);
                        const float xr = er + tw.x, xi = ei + tw.y;
                        // FPSPEC 4: P = fma(..) * 0.25f. The plane stores Q = fma(..) = 4P instead (one VALU
                        // less per bin): the scaling by 4 is exact and order-preserving, so every decision
                        // against thr is the same against 4 thr (the caller passes 4 thr), and
                        // aid_result_power applies the spec's * 0.25f on readout (bit-identical P)
                        po[i] = __builtin_fmaf(xr, xr, xi * xi);
                        // the mirror bin's product cmul((orr, -oi), (-t2.re, t2.im)) is (-tw.x, tw.y) bit for bit:
                        // its re is fma(orr, -c, oi*s) = -fma(orr, c, -(oi*s)) (round-to-nearest is odd-symmetric)
                        // and its im is fma(orr, s, (-oi)*(-c)) = tw.y; so xr2 = er + (-tw.x), xi2 = -ei + tw.y
                        const float xr2 = er - tw.x, xi2 = tw.y - ei;
                        // k = 0 (lane 0, i = 0): the mirror is the dropped Nyquist bin
                        pm[i] = (i == 0 && lane == 0) ? 0.f : __builtin_fmaf(xr2, xr2, xi2 * xi2);
                        // direct bins 64i + l: lanes 16g..16g+15 = chunk 4i + g -> bit 4i + g
                        hotw |= group16(__ballot(po[i] > thr)) << (4 * i);
                        // mirror bins 1024 - 64i - l: lanes 16g+1 .. 16g+16 = chunk 63 - 4i - g -> bit 32 + 4i + g;
                        // lane 0 (bin 1024 - 64i, chunk 64 - 4i) -> bit 31 + 4i (lane 0 of register 0 is the
                        // dropped Nyquist bin, never hot)
                        const uint64_t hm = __ballot(pm[i] > thr);
                        hotw |= group16(hm >> 1) << (32 + 4 * i);
                        if (i > 0) hotw |= (hm & 1ull) << (31 + 4 * i);
                    }
                    // Wait here for the next frame's ring loads (issued after the window multiply, a frame's work
                    // ago: they have landed) and for the previous frame's stores. vmcnt counts loads and stores in
                    // issue order, and this frame's stores are conditional: without this wait hipcc waits at the next
                    // frame's window multiply with a count that only covers the unconditional stores, which also
                    // waits for the L2 acknowledgement of the hot stores issued just before
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
                    {  // bin 512 pairs with itself: every lane computes it (same address, same value),
                       // so its store and the hot word's need no lane-0 branch
                        const float2 a = buf[2];  // Z[512] (E3 slot 2)
                        const float er = a.x + a.x, ei = a.y - a.y, orr = a.y + a.y, oi = a.x - a.x;
                        const float2 tw = cmul(make_float2(orr, oi), t512);
                        const float xr = er + tw.x, xi = ei + tw.y;
                        const float p512 = __builtin_fmaf(xr, xr, xi * xi);
                        pstore(drow + 512, p512);
                        hotw |= p512 > thr ? 1ull << 63 : 0ull;  // chunk 32
                    }
                    dhot[f] = hotw;
                    // K2 reads only hot chunks (a value <= thr can neither be a peak nor suppress one, FPSPEC
                    // 5), so a store whose chunks are all cold is skipped unless the engine keeps the whole
                    // plane. Direct store i covers chunks 4i .. 4i+3 (bits 4i..4i+3); mirror store i covers
                    // chunks 60-4i .. 63-4i (bits 32+4i .. 35+4i) and, by lane 0, chunk 64-4i (bit 31+4i)
                    const uint64_t hsel = keep ? ~0ull : hotw;  // one select, not a branch per store
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if ((hsel >> (4 * i)) & 0xFull) pstore(drow + lane + 64 * i, po[i]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint64_t need = i > 0 ? (hsel >> (31 + 4 * i)) & 0x1Full : (hsel >> 32) & 0xFull;
                        if (need && (i > 0 || lane != 0)) pstore(drow + 1024 - (lane + 64 * i), pm[i]);
                    }
                } else {
                    // log-magnitude rows (aid_spectrogram: the 1e-4 check against float64 numpy), every bin.
                    // Real split in mirror pairs (k, 1024-k): one read of Z[k], Z[1024-k] serves both. For
                    // bin 1024-k the FPSPEC sums are the same exact values with signs flipped (a+c, c+a
                    // commute; b-d = -(d-b)), so both bins stay bit-exact.
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int k = lane + 64 * i;  // 0..511
                        const float2 a = buf[e3q_slot(k)];
                        // k = 0 mirrors onto itself (Z[0]: slot 0)
                        const int bi = (i == 0 && lane == 0) ? 0 : e3q_slot(1024 - k);
                        // stored Z[k] is -Z[k] for k >= 256 (lanes 1..3 of stage C): for i < 4, a is exact
                        // and b is stored negated (except Z[0] for lane 0, i = 0), so flip b; for i >= 4 both
                        // are negated, every sum below flips sign and the squares in P do not see it
                        const float2 bs = buf[bi];
                        const float2 b = i == 0 ? make_float2(bs.x * s0, bs.y * s0) : i < 4 ? make_float2(-bs.x, -bs.y) : bs;
                        const float er = a.x + b.x, ei = a.y - b.y;
                        const float orr = a.y + b.y, oi = b.x - a.x;
                        const float4 t2q = s_t24[64 * (i & 3) + lane];
                        const float2 t2h = i < 4 ? make_float2(t2q.x, t2q.y) : make_float2(t2q.z, t2q.w);
                        const float4 t2 = make_float4(t2h.x, t2h.y, -t2h.x, t2h.y);  // T2K[1024-k] = (-re, im)
                        {
                            const float2 tw = cmul(make_float2(orr, oi), make_float2(t2.x, t2.y));
                            const float xr = er + tw.x, xi = ei + tw.y;
                            const float P = __builtin_fmaf(xr, xr, xi * xi) * 0.25f;  // FPSPEC 4
                            drow[k] = 10.0f * log10f(P + 1e-10f);
                        }
                        if (k != 0) {  // bin 1024-k (513..1023); k = 0's mirror is the dropped Nyquist bin
                            const float2 tw = cmul(make_float2(orr, -oi), make_float2(t2.z, t2.w));
                            const float xr = er + tw.x, xi = -ei + tw.y;
                            const float P = __builtin_fmaf(xr, xr, xi * xi) * 0.25f;
                            drow[1024 - k] = 10.0f * log10f(P + 1e-10f);
                        }
                    }
                    if (lane == 0) {  // bin 512 pairs with itself
                        const float2 a = buf[2];  // Z[512] (E3 slot 2)
                        const float er = a.x + a.x, ei = a.y - a.y, orr = a.y + a.y, oi = a.x - a.x;
                        const float2 tw = cmul(make_float2(orr, oi), t512);
                        const float xr = er + tw.x, xi = ei + tw.y;
                        const float P = __builtin_fmaf(xr, xr, xi * xi) * 0.25f;
                        drow[512] = 10.0f * log10f(P + 1e-10f);
                    }
                }
                wave_lds_sync();
            }
        }
    }
    f += nfr;
    }
}

template <bool LOGMAG>
static void launch_rows(int rows, dim3 g, dim3 b, hipStream_t s, const float *pcm, const ClipDesc *clips, int n_clips,
                        int64_t f0, int64_t total, int64_t n_waves, const Tables *tab, float *out, uint64_t *hot, float thr,
                        int keep) {
    switch (rows) {
        case 1: timed_launch((k_stft_power<LOGMAG, 1>), g, b, 0, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, thr, keep); break;
        case 2: timed_launch((k_stft_power<LOGMAG, 2>), g, b, 0, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, thr, keep); break;
        case 4: timed_launch((k_stft_power<LOGMAG, 4>), g, b, 0, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, thr, keep); break;
        case 8: timed_launch((k_stft_power<LOGMAG, 8>), g, b, 0, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, thr, keep); break;
        default: timed_launch((k_stft_power<LOGMAG, 16>), g, b, 0, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, thr, keep); break;
    }
}

// total_frames = sum of the clips' frames, the first at absolute frame f0 (out = its power row),
// total_strips = sum of ceil(F / kStftStrip) (strip mode), slots = resident K1 waves on the device (CUs x kStftWaves)
void launch_stft_power(const float *pcm, const ClipDesc *clips, int n_clips, int64_t f0, int64_t total_frames,
                       int64_t total_strips, int64_t slots, int hop, const Tables *tab, float *out, bool logmag,
                       uint64_t *hot, float thr, bool keep_power, hipStream_t s) {
    if (total_frames <= 0) return;
    // one round of equal ranges. A wave reloads its 16-row ring once per segment, so large batches keep
    // >= kStftStrip frames per wave; a batch smaller than that spreads over >= kK1MinFrames-frame ranges
    // instead (a 5 s window, 465 frames: 29 waves x 16 frames ran 77 us of serial frames per wave)
    const int64_t n_waves = std::max<int64_t>(
        1, total_frames >= slots * kStftStrip ? slots : std::min<int64_t>(slots, total_frames / kK1MinFrames));
    const int64_t total = total_frames;
    const dim3 g((unsigned)((n_waves + kStftWaves - 1) / kStftWaves)), b(kStftWaves * 64);
    if (logmag) launch_rows<true>(hop / 128, g, b, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, nullptr, thr, 1);
    else  // the power plane holds 4P (see the real split): hot blocks are those with 4P > 4 thr
        launch_rows<false>(hop / 128, g, b, s, pcm, clips, n_clips, f0, total, n_waves, tab, out, hot, 4.0f * thr,
                           keep_power ? 1 : 0);
}

}  // namespace aid
