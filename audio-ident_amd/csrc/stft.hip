// stft.hip -- K1 `stft_power`: framing + Hann window + 1024-point complex FFT +
// real split + |X|^2 (spec/FPSPEC.md 4), one wavefront per frame.
//
// Replaces the FFT stage inside the external `olaf_c` binary that the reference
// runs per call (audio-ident-service/app/audio/fingerprint.py:117-125 store,
// :185-193 query).
//
// Work mapping (gfx950, wave64):
//   * each wave owns an equal range of the batch's frames (AID_K1_BALANCED). Lane l
//     keeps the complex samples z[64*n1 + l] (n1 < 16, "rows" of 128 PCM samples)
//     in a 16-slot register ring: frame t+1 reuses 16 - H/128 rows of frame t, so
//     only the new hop is loaded (H/128 float2 loads per lane, 512 contiguous bytes
//     per wave-instruction) and every PCM byte crosses HBM -> VGPR once per range (the ring
//     restarts at clip edges only);
//     the next frame's rows are loaded right after the window multiply so their
//     latency hides under the FFT;
//   * stage A = 16-point DFT in registers, twiddle (LDS table laid out [k1][lane]),
//     LDS transpose (E1, row stride 68 float2: conflict-free write and read);
//   * stage B = 16-point DFT in registers, twiddle;
//   * stage C = radix-4 across the lane quad with DPP (AID_K1_DPPC; formerly a quad exchange
//     E2 through LDS + radix-4 in registers), spill to LDS in XOR-swizzled natural order
//     (E3), then the real split reads each mirror pair (Z[k], Z[1024-k]) once
//     (conflict-free) and produces both bins; stores are 64 consecutive bins per
//     wave-instruction (the mirror bins in descending order, same 256-B segment).
// A workgroup is kStftWaves = 14 waves (3-4 per SIMD, <= 128 VGPRs) sharing 32 KB of tables in LDS (float4 pairs,
// read with ds_read_b128); the
// exchanges are wave-private, so there is no workgroup barrier in the loop.
#include "aidfp_device.h"

// AID_K1_DIAG selects a timing-only variant for LDS-conflict attribution (wrong results):
//   1 = E3 writes lane-contiguous, 2 = real-split mirror reads lane-contiguous,
//   4 = E1 read lane-contiguous, 5 = E2 read lane-contiguous,
//   6 = no E1 exchange, 7 = no E2 exchange, 8 = no E3 exchange (real split on registers),
//   9 = no stage A/B DFT16 arithmetic, 10 = one float stored per lane and frame (not 16 rows),
//   11 = the 16 rows stored as 4 dwordx4 per lane (same bytes, a quarter of the store instructions)
// Round-1 ablation of the DPP build (one box, K1 0.343 ms): no E1 0.306, no E3 0.306, no DFT16
// arithmetic 0.312, no power stores 0.310, dwordx4 stores 0.346 -- no single phase dominates.
#ifndef AID_K1_DIAG
#define AID_K1_DIAG 0
#endif
// AID_K1_WINREG=1: the lane's 32 window values live in registers for the whole strip
// (they do not change from frame to frame) instead of 8 ds_read_b128 per frame
#ifndef AID_K1_WINREG
#define AID_K1_WINREG 0
#endif
// AID_K1_BALANCED=1 (default): waves take equal frame ranges of the whole batch (ring restarts
// only at clip edges) instead of 16-frame strips; 0 = strips (A/B)
#ifndef AID_K1_PRIO
#define AID_K1_PRIO 0  // s_setprio level around the E1 exchange (experiment)
#endif
#ifndef AID_K1_BALANCED
#define AID_K1_BALANCED 1
#endif
// AID_K1_DPPC: stage C's DFT4 over m2 runs across the lane quad with DPP operands (two
// butterflies of fma(partner, +-1, self) and a -i rotation in lane 3) instead of the E2 quad
// exchange through LDS; the results then sit at Z[kq + 16*j1 + 256*bitrev2(mq)] and E3 uses the
// swizzle "bit 4 ^= bit 9". 2 (default) = hand-placed v_fmac_f32_dpp (K1 0.386 -> 0.377 ms in
// same-box A/Bs), 1 = the same arithmetic through intrinsics (hipcc keeps a separate
// v_mov_b32_dpp per operand: 0.393), 0 = E2 through LDS
#ifndef AID_K1_DPPC
#define AID_K1_DPPC 2
#endif
// AID_K1_E1V=1: E1 read side as 8 ds_read_b128 instead of 16 ds_read_b64. Row k1 holds writer
// lane n2 = 4 m1 + m2 at float2 slot 8 ((m1 >> 1) ^ (k1 & 7)) + 2 m2 + (m1 & 1), so the reader
// (kq, mq) finds A[kq][4 (2j) + mq] and A[kq][4 (2j+1) + mq] side by side at 8 (j ^ (kq & 7)) + 2 mq.
// Writes (4 x 16 contiguous lanes, bank = slot mod 16) and reads (4 x 16-lane groups of ds_read_b128,
// float4 slot mod 16 = 4 ((j ^ kq) & 3) + mq) are both conflict-free. Same bytes, same LDS cycles,
// half the read instructions.
// AID_K1_T2HALF=1: the real split's mirror twiddle T2K[1024-k] is taken as (-re, im) of T2K[k] (the
// host tables satisfy it exactly for every k, checked in aid_engine_create), so the split table is
// float2 [512] read with ds_read_b64 instead of float4 pairs with ds_read_b128 (half the LDS bytes)
#ifndef AID_K1_T2HALF
#define AID_K1_T2HALF 1
#endif
#ifndef AID_K1_E1V
#define AID_K1_E1V 1
#endif
// AID_K1_E1ADDTID=1 (aidfp_layout.h): E1's write side as 32 ds_write_addtid_b32 (address = M0 + offset +
// 4 lane: no address VGPR, 2 LDS cycles each) instead of 16 ds_write_b64 (6 cycles each: the address and
// two data dwords cross to the LDS at 2 cycles per dword, MI355X_MICROARCH LDS table) -- 64 instead of 96
// LDS cycles per frame. Each (k1, component) register goes to its own 64-dword region, lane-linear, so the
// permutation E1 needs moves to (a) which n2 a stage-A lane holds and (b) the region bases:
//   * stage-A lane p = 8 j + 2 m + b holds n2 = 8 j + 4 b + m (e1_perm; its PCM loads stay inside the
//     same 512-B segment, and the window / T1K tables are staged in that lane order), so the two values a
//     stage-B reader (kq, mq) needs for m1 = 2 j, 2 j + 1, n2 = 4 m1 + mq, sit side by side at 8 j + 2 mq;
//   * region (k1, c) starts at dword 128 k1 + 64 c + 8 s(k1), s = k1 (k1 < 8) or k1 - 1 (k1 >= 8): the 8
//     readers kq of one 32-lane group then hit 8 distinct 8-bank slots (ds_read_b64: 64 banks).
// Reads are 16 ds_read_b64 (2 cycles each, as the 8 ds_read_b128 before). 2160 dwords per wave: 16 waves
// + the tables take 159,232 of the 163,840 LDS bytes.
#ifndef AID_K1_E1STAGED
#define AID_K1_E1STAGED 0  // 1: E1 reads in two blocks; stage B's first two DFT4s run while the second lands
#endif
#ifndef AID_K1_E1Q
#define AID_K1_E1Q 1  // E1 read side as 8 ds_read_b128 (see below): K1 -0.6 % and -2.4 % in two same-box A/Bs (r02)
#endif
#if AID_K1_E1ADDTID && AID_K1_E1Q
// AID_K1_E1Q: stage-A lane p holds n2 = 4 (p & 15) + (p >> 4), so a stage-B reader (kq, mq) finds n2 = 4 m1 + mq for
// m1 = 4t .. 4t+3 at positions 16 mq + 4t .. +3 of region (kq, c): one ds_read_b128 per (t, c), 8 per frame instead
// of 16 ds_read_b64 (same LDS cycles). Region bases 128 k1 + 64 c + 4 (k1 & 3) + 16 (k1 >> 2) (2108 dwords) put the
// 16 lanes of every b128 lane group on 16 distinct 4-bank quads
__host__ __device__ constexpr int e1_perm(int p) { return 4 * (p & 15) + (p >> 4); }
__host__ __device__ constexpr int e1_region(int k1, int c) { return 128 * k1 + 64 * c + 4 * (k1 & 3) + 16 * (k1 >> 2); }
#elif AID_K1_E1ADDTID
__host__ __device__ constexpr int e1_perm(int p) { return (p & ~7) | ((p & 1) << 2) | ((p >> 1) & 3); }
__host__ __device__ constexpr int e1_region(int k1, int c) { return 128 * k1 + 64 * c + 8 * (k1 < 8 ? k1 : k1 - 1); }
#endif
#if AID_K1_E1ADDTID
static_assert(e1_region(15, 1) + 64 <= 2 * aid::kStftLdsPerWave, "E1 regions exceed the wave buffer");
#endif
// AID_K1_E3ADDTID=1 (needs AID_K1_E1ADDTID): E3 (the stage-C spill the real split reads) as 32
// ds_write_addtid_b32 too (64 instead of 96 LDS cycles per frame). Stage-C lane L = 4 kq + mq holds
// Z[kq + 16 j1 + 256 bitrev2(mq)] (negated for mq > 0) in register j1; component c of register j1 goes to
// region (j1, c) at dword 130 j1 + 64 c, position L. A pair of adjacent positions then holds
//   (4 kq, 4 kq + 1):     (Z[k], -Z[k + 512])            k = kq + 16 j1 < 256
//   (4 kq + 2, 4 kq + 3): (-Z[k + 256], -Z[k + 768])
// so one ds_read_b64 per component gives the real split two mirror pairs at once. Lane l, unit u < 4
// reads, for k = l + 64 u: (Z[k], Z[k + 512]) from region 4 u + l / 16 and (Z[512 - k], Z[1024 - k]) from
// region 4 (3 - u) + (64 - l) / 16, and computes the pairs (k, 1024 - k) and (512 - k, 512 + k): the same
// stores of 64 consecutive bins as the layout above. Region bases 130 j1 (= 2 j1 mod 4) put the two
// 16-lane halves of each 32-lane read group on the even / odd bank pairs: conflict-free except lane 0
// against lane 31 in the mirror reads of u = 1..3. Bins 256 and 768 (the pair k = 256, which no unit
// holds) are computed by every lane from one broadcast read, as bin 512 is in the layout above.
#ifndef AID_K1_E3ADDTID
#define AID_K1_E3ADDTID 0
#endif
#ifndef AID_K1_E3STAGED
#define AID_K1_E3STAGED 0  // 1: the split's reads waited for unit by unit (counted lgkmcnt) instead of all at once
#endif
#if AID_K1_E3ADDTID
static_assert(AID_K1_E1ADDTID, "AID_K1_E3ADDTID needs the add-TID E1 buffer layout");
__host__ __device__ constexpr int e3_region(int j1, int c) { return 130 * j1 + 64 * c; }
// highest dword read: lane 0's (unused) mirror read of unit 0, component 1
static_assert(e3_region(15, 1) + 64 <= 2 * aid::kStftLdsPerWave && 520 * 3 + 522 + 64 + 2 <= 2 * aid::kStftLdsPerWave,
              "E3 regions exceed the wave buffer");
#endif
#if AID_K1_E1ADDTID
__host__ __device__ constexpr int e2_region(int j1, int c) { return 128 * j1 + 64 * c; }  // AID_K1_DPPC 3
// 8 registers' components -> their regions (M0 = the wave buffer's LDS byte address). s_nop 0: one wait
// state between an SALU write of M0 and an add-TID LDS instruction
#define AID_TID8(RG, K0)                                                                                     \
    asm volatile("s_mov_b32 m0, %[base]\n\ts_nop 0\n\t"                                                      \
                 "ds_write_addtid_b32 %0 offset:%8\n\tds_write_addtid_b32 %1 offset:%9\n\t"                  \
                 "ds_write_addtid_b32 %2 offset:%10\n\tds_write_addtid_b32 %3 offset:%11\n\t"                \
                 "ds_write_addtid_b32 %4 offset:%12\n\tds_write_addtid_b32 %5 offset:%13\n\t"                \
                 "ds_write_addtid_b32 %6 offset:%14\n\tds_write_addtid_b32 %7 offset:%15"                    \
                 :                                                                                           \
                 : "v"(v[K0].x), "v"(v[K0].y), "v"(v[K0 + 1].x), "v"(v[K0 + 1].y), "v"(v[K0 + 2].x),         \
                   "v"(v[K0 + 2].y), "v"(v[K0 + 3].x), "v"(v[K0 + 3].y), "i"(4 * RG(K0, 0)),                 \
                   "i"(4 * RG(K0, 1)), "i"(4 * RG(K0 + 1, 0)), "i"(4 * RG(K0 + 1, 1)),   \
                   "i"(4 * RG(K0 + 2, 0)), "i"(4 * RG(K0 + 2, 1)), "i"(4 * RG(K0 + 3, 0)), \
                   "i"(4 * RG(K0 + 3, 1)), [base] "s"(m0base)                                         \
                 : "memory", "m0")
#endif
// AID_K1_BRANCHFREE=1: the real split computes the row's 16 powers per lane first, then the hot word,
// then stores all 16 unconditionally, a cold block's into a per-workgroup dummy row (scalar base
// select). The guarded stores of the earlier code put a scalar branch after every bin pair, which
// cut the split into 16 short blocks the compiler could not interleave.
#ifndef AID_K1_BRANCHFREE
#define AID_K1_BRANCHFREE 1  // K1 0.2935 -> 0.2863 ms same-box (r02)
#endif
// AID_K1_TPF_W / _A / _B: table prefetch. hipcc issued every window / twiddle ds_read_b128 right before
// its use behind its own s_waitcnt lgkmcnt(0) (24 serialized LDS round trips per frame). With these set,
// the first N float4 reads of the window (W), the stage-A twiddles (A, before stage A's DFT16) and the
// stage-B twiddles (B, before stage B's DFT16) are issued together ahead of a sched_barrier, the rest
// right after the DFT16.
#ifndef AID_K1_TPF_W
#define AID_K1_TPF_W 8  // K1 0.2804 -> 0.2778 ms same-box (r02; 0.2752 with AID_K1_PREWAIT)
#endif
#ifndef AID_K1_TPF_A
#define AID_K1_TPF_A 0
#endif
#ifndef AID_K1_TPF_B
#define AID_K1_TPF_B 8  // K1 0.2657 -> 0.2619 ms same-box on top of AID_K1_E1ADDTID (r02)
#endif
#ifndef AID_K1_TPF_S  // 1: the real split's 24 LDS reads (E3 pairs + split twiddles) issued up front
#define AID_K1_TPF_S 0
#endif
#ifndef AID_K1_HOTSUP
#define AID_K1_HOTSUP 1  // 1: a mirror ballot marks blocks 15-i and 16-i together (superset hot word)
#endif
#ifndef AID_K1_STBR
#define AID_K1_STBR 1  // 1: cold-block stores skipped by scalar branches instead of redirected to a sink row
#endif
#ifndef AID_K1_PK_WIN
#define AID_K1_PK_WIN 0  // 1: window multiply as 16 v_pk_mul_f32 per frame instead of 32 v_mul_f32
#endif
#ifndef AID_K1_MIRROR_ID
#define AID_K1_MIRROR_ID 1  // real split: the mirror bin reuses the direct bin's twiddle product (see there)
#endif
#ifndef AID_K1_PREWAIT
#define AID_K1_PREWAIT 1  // K1 0.2804 -> 0.2785 ms alone, 0.2752 with AID_K1_TPF_W (same-box, r02)
#endif
// AID_K1_COMPACT=1: E1/E2 through unpadded 1024-entry buffers with XOR column swizzles
// (8 KB per wave instead of 8.5 KB), so 16 waves + tables fit in 160 KB of LDS

namespace aid {

// power-row store: AID_K1_NTSTORE=1 marks it non-temporal (streaming): K1 0.268 -> 0.266 ms, K2 0.134 ->
// 0.130 ms, 5.88 -> 5.95 M audio-s/s same-box (r02). A second K2 over the same rows right after the first
// (AID_K2_TWICE diagnostic) takes as long as the first, so K2 is not bound by draining K1's dirty lines
#ifndef AID_K1_NTSTORE
#define AID_K1_NTSTORE 1
#endif
__device__ __forceinline__ void pstore(float *p, float v) {
#if AID_K1_NTSTORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// E3 slot of Z[k]: XOR-swizzle bits 2-3 by bits 4-5. The stage-C writers of one 16-lane
// group hold k = kq + 16*mq (+const): k ^ (mq << 2) puts them on 16 distinct 8-byte bank
// pairs; the readers (k = lane + 64i, and the mirror 1024-k) stay a permutation of one or two
// 16-entry blocks, so every access is conflict-free (the mirror read: one 2-way pair per wave).
#if AID_K1_DPPC
// E3 slot of Z[k] (DPP stage C): bit 2 ^= bit 9, bit 3 ^= bit 8. ds_write_b64 is serviced in
// 4 groups of 16 contiguous lanes on 32 banks (MI355X_MICROARCH LDS table): a group's writers
// (k = kq + 16 j1 + 256 j2, 4 consecutive kq x 4 j2, one j1 per instruction) then hit 16 distinct
// 8-byte bank pairs, and the real split's readers Z[lane + 64 i] (lane ^ const) and their
// mirrors stay conflict-free too (lane 0 aside). (Bit 4 ^= bit 9 alone left the writes 4-way:
// 34 % of K1's LDS cycles were conflicts; bits 3/4 from bits 8/9 still 2-way.)
__device__ __forceinline__ int e3(int k) { return k ^ (((k >> 9) & 1) << 2) ^ (((k >> 8) & 1) << 3); }
// AID_K1_E3Q=1: E3 slot of Z[k] = 4 (k & 255) + (j2 ^ 2 h), j2 = k >> 8, h = bit 3 of k: the four Z[k + 256 j2]
// sit in one 32-B group with the (j2 = 0, 1) and (2, 3) halves swapped by bit 3, so the real split reads
// (Z[k], Z[k + 256]) and (Z[768 - k], Z[1024 - k]) as one ds_read_b128 each (8 instead of 16 ds_read_b64 per frame;
// stage-C writers and both readers conflict-free, checked exhaustively). Lane 0's unit-0 mirror read lands on a
// copy of Z[768] at slot 1026, written by lane 3 of stage C.
#ifndef AID_K1_E3Q_DUP
#define AID_K1_E3Q_DUP 1  // diagnostic: 0 drops the copy (wrong results for bins 768 of lane 0)
#endif
__device__ __forceinline__ int e3q_slot(int k) { return 4 * (k & 255) + ((k >> 8) ^ (2 * ((k >> 3) & 1))); }
// partner value across the lane quad (DPP quad_perm; every lane of the quad is valid)
template <int CTRL>
__device__ __forceinline__ float quad_dpp(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
#else
__device__ __forceinline__ int e3(int k) { return k ^ (((k >> 4) & 3) << 2); }
#endif

// AID_K1_E1SWAP=1: E1 as an in-register transpose of (register k1) x (lane bits 2-5 = m1): register
// bit s is exchanged with lane bit 2+s, s = 3 and 2 by v_permlane32/16_swap (one instruction moves one
// float of two registers), s = 1 and 0 by DPP v_cndmask (row_shr/row_shl by 8 / 4 lanes inside a
// row, two instructions per float pair). No LDS, no wait; 96 VALU instead of 16 ds_write_b64 +
// 8 ds_read_b128. Pure data movement: the values are bit-identical to the LDS exchange.
#ifndef AID_K1_E1SWAP
#define AID_K1_E1SWAP 0
#endif
#if AID_K1_E1SWAP
__device__ __forceinline__ void lane_swap32(float &a, float &b) {  // a[32+i] <-> b[i]
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void lane_swap16(float &a, float &b) {  // a[odd row] <-> b[even row]
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// Exchange across lane bit log2(D) (D = 4 or 8, inside a row of 16) for two register pairs (a_i, b_i):
//   a'[l] = bit ? b[l - D] : a[l] ;  b'[l] = bit ? b[l] : a[l + D]
// v_cndmask_b32 (VOP2 + DPP on src0): D = vcc ? src1 : dpp(src0). bound_ctrl:0 zero-fills the source of
// the lanes whose partner is outside the row; those lanes select src1 anyway.
#define AID_XCHG_ASM(SHR, SHL)                                                            \
    "s_mov_b64 vcc, %[nm]\n\t"                                                            \
    "s_nop 1\n\t"                                                                         \
    "v_cndmask_b32_dpp %0, %12, %8, vcc " SHR " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"  \
    "v_cndmask_b32_dpp %1, %13, %9, vcc " SHR " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"  \
    "v_cndmask_b32_dpp %2, %14, %10, vcc " SHR " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t" \
    "v_cndmask_b32_dpp %3, %15, %11, vcc " SHR " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t" \
    "s_mov_b64 vcc, %[m]\n\t"                                                             \
    "v_cndmask_b32_dpp %4, %8, %12, vcc " SHL " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"  \
    "v_cndmask_b32_dpp %5, %9, %13, vcc " SHL " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"  \
    "v_cndmask_b32_dpp %6, %10, %14, vcc " SHL " row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t" \
    "v_cndmask_b32_dpp %7, %11, %15, vcc " SHL " row_mask:0xf bank_mask:0xf bound_ctrl:0"
template <int D>
__device__ __forceinline__ void lane_xchg(float2 &a0, float2 &b0, float2 &a1, float2 &b1) {
    // nm = lanes with the exchanged bit CLEAR (they keep a), m = lanes with it set (they keep b). Only
    // s_mov touches scalar state here: an s_not would write SCC, which the compiler may hold live
    // between the halves of a 64-bit s_add_u32/s_addc_u32 around this block (it did: a wrong address).
    constexpr unsigned long long nm = D == 4 ? 0x0F0F0F0F0F0F0F0Full : 0x00FF00FF00FF00FFull;
    constexpr unsigned long long m = ~nm;
    float o[8];
#define AID_XCHG_OPERANDS                                                                               \
    : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]) \
    : "v"(a0.x), "v"(a0.y), "v"(a1.x), "v"(a1.y), "v"(b0.x), "v"(b0.y), "v"(b1.x), "v"(b1.y), [nm] "s"(nm), [m] "s"(m) \
    : "vcc"
    if constexpr (D == 4) asm volatile(AID_XCHG_ASM("row_shr:4", "row_shl:4") AID_XCHG_OPERANDS);
    else asm volatile(AID_XCHG_ASM("row_shr:8", "row_shl:8") AID_XCHG_OPERANDS);
#undef AID_XCHG_OPERANDS
    a0 = make_float2(o[0], o[1]);
    a1 = make_float2(o[2], o[3]);
    b0 = make_float2(o[4], o[5]);
    b1 = make_float2(o[6], o[7]);
}
// E1 transpose: in lane n2 = 4 m1 + m2, v[k1] = A[k1][n2]; out in lane 4 k1 + m2, v[m1] = A[k1][4 m1 + m2]
__device__ __forceinline__ void e1_transpose(float2 (&v)[16]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {  // register bit 3 <-> lane bit 5
        lane_swap32(v[r].x, v[r + 8].x);
        lane_swap32(v[r].y, v[r + 8].y);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r)  // register bit 2 <-> lane bit 4
        if (!(r & 4)) {
            lane_swap16(v[r].x, v[r + 4].x);
            lane_swap16(v[r].y, v[r + 4].y);
        }
#pragma unroll
    for (int r = 0; r < 16; r += 4) lane_xchg<8>(v[r], v[r + 2], v[r + 1], v[r + 3]);  // bit 1 <-> lane bit 3
#pragma unroll
    for (int r = 0; r < 16; r += 4) lane_xchg<4>(v[r], v[r + 1], v[r + 2], v[r + 3]);  // bit 0 <-> lane bit 2
}
#endif

template <bool LOGMAG, int ROWS>
__global__ __launch_bounds__(kStftWaves * 64) void k_stft_power(const float *__restrict__ pcm,
                                                                const ClipDesc *__restrict__ clips, int n_clips,
                                                                int64_t total, int64_t n_waves,
                                                                const Tables *__restrict__ tab, float *__restrict__ out,
                                                                uint32_t *__restrict__ hot, float thr, int keep,
                                                                float *__restrict__ dummy_rows) {
    constexpr int PERIOD = 16 / ROWS;  // frames per full ring rotation
    constexpr int HOP2 = 64 * ROWS;    // hop in float2 units
    __shared__ __attribute__((aligned(16))) float2 lds[kStftWaves][kStftLdsPerWave];  // E1: 16 x 68 (compact: 16 x 64), E2: 64 x 17 (16 x 64), E3: 1024
    // tables as float4 pairs [h][lane], one ds_read_b128 per pair (hipcc would otherwise merge the
    // stride-512-B float2 reads into ds_read2st64_b64, which costs the LDS twice the cycles):
    //   s_win4[h] = window of rows 2h, 2h+1 ; s_ta4[h] = T1K[lane*k1], k1 = 2h, 2h+1
    //   s_tb4[h] = T64[(lane&3)*j1], j1 = 2h, 2h+1 ; s_t2p[i] = (T2K[k], T2K[1024-k]), k = lane + 64i
    __shared__ float4 s_win4[512], s_ta4[512];
#if AID_K1_T2HALF
    __shared__ float2 s_t2[512 + AID_K1_E3ADDTID];  // T2K[k], k < 512 (E3ADDTID: k <= 512)
#else
    __shared__ float4 s_t2p[512];
#endif
    __shared__ float4 s_tb4[32];  // [h][lane & 3]: T64[m2*j1] depends on the lane only through m2
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar strip/segment math
    float2 *buf = lds[wave];
    const int kq = lane >> 2;  // stage B/C: k1
    const int mq = lane & 3;   // stage B: m2 ; stage C: s
#if AID_K1_E1ADDTID
    // LDS byte address of this wave's buffer (M0 of the add-TID writes) and of the lane's E1 reads
    const uint32_t m0base =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float2 *)buf);
#if AID_K1_E1Q
    const uint32_t e1rd = m0base + 4u * (uint32_t)(e1_region(kq, 0) + 16 * mq);
#else
    const uint32_t e1rd = m0base + 4u * (uint32_t)(e1_region(kq, 0) + 2 * mq);
#endif
#endif
#if AID_K1_DPPC == 3
    // E2 reader lane: kq2 = lane & 15, s = lane >> 4 (regions j1 = 4 s + r); its E3 slots e3(kq2 + 16 (4 s + r) +
    // 256 j2) = e3c[j2] + 16 r + 256 j2 (the E3 swizzle flips bits 2-3 of kq2 by bits 8-9 = j2)
    static_assert(AID_K1_E1ADDTID, "AID_K1_DPPC 3 writes E2 by add-TID");
    const uint32_t e2rd = m0base + 4u * (uint32_t)(512 * (lane >> 4) + 4 * (lane & 15));
    int e3c[4];
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) e3c[j2] = e3((lane & 15) + 64 * (lane >> 4) + 256 * j2) - 256 * j2;
#endif
#if AID_K1_E3ADDTID
    // real-split read addresses (unit u, component c add 2080 u + 256 c, resp. 2080 (3 - u) + 256 c bytes):
    // (Z[k], Z[k + 512]) at region 4 u + lane / 16, position 4 (lane & 15); (Z[512 - k], Z[1024 - k]) at region
    // 4 (3 - u) + (64 - lane) / 16, position 4 ((64 - lane) & 15) + 2; (Z[256], Z[768]) at region 0, position 2
    const uint32_t e3d = m0base + 4u * (uint32_t)(130 * (lane >> 4) + 4 * (lane & 15));
    const uint32_t e3m = m0base + 4u * (uint32_t)(130 * ((64 - lane) >> 4) + 4 * ((64 - lane) & 15) + 2);
    const uint32_t e3x = m0base + 8u;
#endif
    // E3 addresses as one per-lane base + compile-time offsets (the XOR only touches bits 2-3):
    //   stage-C slot of Z[kq + 16(mq+4r) + 256 j2]: bits 4-5 of k are mq      -> e3w + 64r + 256 j2
    //   Z[lane + 64i]: bits 4-5 are those of lane                              -> e3a + 64i
    //   Z[1024 - lane - 64i] = Z[64(15-i) + m], m = 64 - lane in 1..64         -> e3b + 64(15-i)
    //   (except k = 0, whose mirror is Z[0] itself)
#if AID_K1_DPPC
    // writer slots: e3(kq + 16 j1 + 256 j2) = kq + 256 j2 + 16 (j1 ^ (j2 >> 1)) = base[j1 & 1] + 16 j1
    const int j2q = ((mq & 1) << 1) | (mq >> 1);  // lane mq holds output j2 = bitrev2(mq)
    // writer slots: e3(kq + 16 j1 + 256 j2) = (kq ^ 4 (j2 >> 1) ^ 8 (j2 & 1)) + 256 j2 + 16 j1
    const int e3w = (kq ^ (((j2q >> 1) << 2) | ((j2q & 1) << 3))) + 256 * j2q;
#if AID_K1_E3Q
    static_assert(AID_K1_DPPC == 2, "AID_K1_E3Q is laid out for the DPP stage C");
    const int e3wq = 4 * kq + (j2q ^ (2 * ((kq >> 3) & 1)));  // + 64 j1
    // split reads (float4 units): (Z[k], Z[k + 256]) at 2 k + h(k), (Z[768 - k], Z[1024 - k]) at 2 m + 1 - h(m),
    // m = 256 - k, k = lane + 64 i (i < 4; the i terms are immediates)
    const int e3qa = 2 * lane + ((lane >> 3) & 1);
    const int e3qb = 513 - 2 * lane - (((256 - lane) >> 3) & 1);
    // lane 0's unit-0 mirror read (m = 256) takes slots 1026, 1027 as (Z[768 - 0], Z[1024 - 0]): Z[768] (stage-C lane 3,
    // register 0) is copied to 1026; slot 1027 (Z[0]) is not used (k = 0 pairs with Z[0] from its own read)
    const int e3dup = lane == 3 ? 1026 : 1028 + lane;  // < kStftLdsPerWave (1092)
#endif
    // readers: Z[lane + 64 i] (i < 8: bit 9 clear, bit 8 = i >> 2) -> e3a[i >> 2] + 64 i;
    // Z[1024 - lane - 64 i] = Z[64 (15 - i) + m], m = 64 - lane (bit 9 set, bit 8 = i < 4)
    //   -> e3b[i < 4] + 64 (15 - i); lane 0 (m = 64, Z[64 (16 - i)]) matches that except at i = 4
    const int e3a0 = lane, e3a1 = lane ^ 8;
    const int e3b1 = (64 - lane) ^ 12, e3b0 = (64 - lane) ^ 4;
    const int e3b4 = (lane == 0) ? 76 : e3b0;  // i = 4: Z[768] for lane 0
#define AID_E3A(i) ((i) < 4 ? e3a0 : e3a1)
#define AID_E3B(i) ((i) < 4 ? e3b1 : (i) == 4 ? e3b4 : e3b0)
    const float s1 = mq < 2 ? 1.0f : -1.0f;                     // butterfly over lanes (mq, mq ^ 2)
    const float s2 = (mq == 1 || mq == 2) ? -1.0f : 1.0f;       // butterfly over lanes (mq, mq ^ 1)
    const float s0 = lane == 0 ? 1.0f : -1.0f;  // sign of Z[0]'s mirror slot for i = 0 (Z[0] itself)
#else
    const int e3w = (kq ^ (mq << 2)) + 16 * mq;
    const int e3a = e3(lane);
    const int e3b = e3(64 - lane);
#endif

    for (int i = threadIdx.x; i < 512; i += kStftWaves * 64) {
        const int h = i >> 6, l = i & 63, a = 2 * h, b = 2 * h + 1;
#if AID_K1_E1ADDTID
        const int ln = e1_perm(l);  // the n2 stage-A lane l holds
#else
        const int ln = l;
#endif
        const float2 w0 = tab->win2[64 * a + ln], w1 = tab->win2[64 * b + ln];
        s_win4[i] = make_float4(w0.x, w0.y, w1.x, w1.y);
        const float2 ta0 = tab->t1k[ln * a], ta1 = tab->t1k[ln * b];
        s_ta4[i] = make_float4(ta0.x, ta0.y, ta1.x, ta1.y);
        if (l < 4) {
            const float2 tb0 = tab->t64[l * a], tb1 = tab->t64[l * b];
            s_tb4[4 * h + l] = make_float4(tb0.x, tb0.y, tb1.x, tb1.y);
        }
        const int k = l + 64 * h;
#if AID_K1_T2HALF
        s_t2[i] = tab->t2k[k];
#else
        const float2 c0 = tab->t2k[k], c1 = tab->t2k[(1024 - k) & 1023];  // k = 0: mirror unused
        s_t2p[i] = make_float4(c0.x, c0.y, c1.x, c1.y);
#endif
    }
    const float2 t512 = tab->t2k[512];
#if AID_K1_E3ADDTID
    if (threadIdx.x == 0) s_t2[512] = t512;
#endif
    float2 t16[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t16[i] = tab->t16[i];
    __syncthreads();

#if AID_K1_BALANCED
    // wave g takes frames [g*T/W, (g+1)*T/W) of the batch's T frames (W waves): every wave has
    // the same work (no partial last round), and a segment restarts the ring only at a clip edge
    const int64_t g = (int64_t)blockIdx.x * kStftWaves + wave;
    if (g >= n_waves) return;  // wave-uniform, after the only barrier
    int64_t f = g * total / n_waves;
    const int64_t f_end = (g + 1) * total / n_waves;
    while (f < f_end) {
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {  // last clip with frame_base <= f (scalar loads): the clip holding frame f
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].frame_base <= f) lo = mid; else hi = mid - 1;
    }
    const int64_t t0 = f - clips[lo].frame_base;
    const int nfr = (int)min(f_end - f, clips[lo].frames - t0);
#else
    const int64_t strip = (int64_t)blockIdx.x * kStftWaves + wave;
    if (strip >= total) return;  // wave-uniform, after the only barrier
    int lo = 0, hi = n_clips - 1;
    while (lo < hi) {  // last clip with stft_base <= strip (scalar loads)
        const int mid = (lo + hi + 1) >> 1;
        if (clips[mid].stft_base <= strip) lo = mid; else hi = mid - 1;
    }
    const int64_t t0 = (strip - clips[lo].stft_base) * kStftStrip;
    const int nfr = (int)min((int64_t)kStftStrip, clips[lo].frames - t0);
#endif
#if AID_K1_E1ADDTID
    const float2 *src = reinterpret_cast<const float2 *>(pcm + clips[lo].pcm_off) + t0 * HOP2 + e1_perm(lane);
#else
    const float2 *src = reinterpret_cast<const float2 *>(pcm + clips[lo].pcm_off) + t0 * HOP2 + lane;
#endif
    float *dst = out + (clips[lo].frame_base + t0) * kBins;
    float *dummy = dummy_rows + (int64_t)(blockIdx.x & (kK1DummyRows - 1)) * 2048;  // cold-block store sink
    (void)dummy;  // unused with AID_K1_STBR
    uint32_t *dhot = LOGMAG ? nullptr : hot + clips[lo].frame_base + t0;

    float2 ring[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ring[r] = src[64 * r];
#if AID_K1_PREWAIT
    // the segment's first frame needs the whole ring anyway: wait for it here, so the frame loop's
    // header does not inherit this path's pending loads (hipcc's wait at the header, merged over both
    // edges, was vmcnt(1): every 4 frames the wave also waited for the previous frame's 17 stores)
    // (an empty asm reading every ring register: hipcc must complete the loads before it)
#pragma unroll
    for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(ring[r].x), "v"(ring[r].y));
#endif
#if AID_K1_WINREG
    float4 wreg[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) wreg[h] = s_win4[64 * h + lane];
#endif

    for (int f0 = 0; f0 < nfr; f0 += PERIOD) {
#pragma unroll
        for (int p = 0; p < PERIOD; ++p) {
            const int f = f0 + p;
            if (f < nfr) {  // wave-uniform
                float2 v[16];
#if AID_K1_TPF_W
                float4 wpf[8];
#pragma unroll
                for (int h = 0; h < AID_K1_TPF_W; ++h) wpf[h] = s_win4[64 * h + lane];
                __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
                for (int h = 0; h < 8; ++h) {
#if AID_K1_WINREG
                    const float4 w = wreg[h];
#elif AID_K1_TPF_W
                    const float4 w = h < AID_K1_TPF_W ? wpf[h] : s_win4[64 * h + lane];
#else
                    const float4 w = s_win4[64 * h + lane];
#endif
                    const float2 x0 = ring[(2 * h + ROWS * p) & 15], x1 = ring[(2 * h + 1 + ROWS * p) & 15];
#if AID_K1_PK_WIN
                    v[2 * h] = f2_of(pk_mul(pk_of(x0), (aid_pk2){w.x, w.y}));
                    v[2 * h + 1] = f2_of(pk_mul(pk_of(x1), (aid_pk2){w.z, w.w}));
#else
                    v[2 * h] = make_float2(x0.x * w.x, x0.y * w.y);
                    v[2 * h + 1] = make_float2(x1.x * w.z, x1.y * w.w);
#endif
                }
                // the rows just consumed (n1 < ROWS) are replaced by frame f+1's new rows (after the
                // last frame of the segment: a harmless re-load of its own rows, instead of a branch)
                {
                    const int fn = min(f + 1, nfr - 1);
#pragma unroll
                    for (int j = 0; j < ROWS; ++j)
                        ring[(ROWS * p + j) & 15] = src[(int64_t)fn * HOP2 + 64 * (16 - ROWS + j)];
                }
                // stage A: lane = n2
#if AID_K1_TPF_A
                float4 tpa[8];
#pragma unroll
                for (int h = 0; h < AID_K1_TPF_A; ++h) tpa[h] = s_ta4[64 * h + lane];
                __builtin_amdgcn_sched_barrier(0);
#endif
                if (AID_K1_DIAG != 9) dft16(v, t16);
#if AID_K1_TPF_A
#pragma unroll
                for (int h = AID_K1_TPF_A; h < 8; ++h) tpa[h] = s_ta4[64 * h + lane];
#endif
                // T1K[n2*k1]; lane 0 multiplies by T1K[0] = (1,-0): value-identical (FPSPEC 4 note)
#pragma unroll
                for (int h = 0; h < 8; ++h) {
#if AID_K1_TPF_A
                    const float4 t = tpa[h];
#else
                    const float4 t = s_ta4[64 * h + lane];
#endif
                    if (h) v[2 * h] = cmul(v[2 * h], make_float2(t.x, t.y));
                    v[2 * h + 1] = cmul(v[2 * h + 1], make_float2(t.z, t.w));
                }
#if AID_K1_PRIO
                __builtin_amdgcn_s_setprio(AID_K1_PRIO);  // exchange phase: keep the LDS queue fed
#endif
                // E1: A[k1][n2] -> lane (k1 = kq, m2 = mq) gets A[kq][4*m1 + mq]
                if (AID_K1_DIAG != 6) {
#if AID_K1_E1ADDTID
                    AID_TID8(e1_region, 0);
                    AID_TID8(e1_region, 4);
                    AID_TID8(e1_region, 8);
                    AID_TID8(e1_region, 12);
#if AID_K1_E1Q
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
#elif AID_K1_E1STAGED
                    {
                        // the reads of m1 = 0, 1, 4, 5, 8, 9, 12, 13 (j even) first: once they are in (8 later
                        // reads outstanding), stage B's first-round DFT4s over b = 0, 1 run while the rest land
                        float2 qa[8], qb[8];
                        asm volatile(
                            "ds_read_b64 %0, %8 offset:0\n\tds_read_b64 %1, %8 offset:256\n\t"
                            "ds_read_b64 %2, %8 offset:64\n\tds_read_b64 %3, %8 offset:320\n\t"
                            "ds_read_b64 %4, %8 offset:128\n\tds_read_b64 %5, %8 offset:384\n\t"
                            "ds_read_b64 %6, %8 offset:192\n\tds_read_b64 %7, %8 offset:448"
                            : "=&v"(qa[0]), "=&v"(qa[1]), "=&v"(qa[2]), "=&v"(qa[3]), "=&v"(qa[4]), "=&v"(qa[5]),
                              "=&v"(qa[6]), "=&v"(qa[7])
                            : "v"(e1rd)
                            : "memory");
                        asm volatile(
                            "ds_read_b64 %0, %8 offset:32\n\tds_read_b64 %1, %8 offset:288\n\t"
                            "ds_read_b64 %2, %8 offset:96\n\tds_read_b64 %3, %8 offset:352\n\t"
                            "ds_read_b64 %4, %8 offset:160\n\tds_read_b64 %5, %8 offset:416\n\t"
                            "ds_read_b64 %6, %8 offset:224\n\tds_read_b64 %7, %8 offset:480"
                            : "=&v"(qb[0]), "=&v"(qb[1]), "=&v"(qb[2]), "=&v"(qb[3]), "=&v"(qb[4]), "=&v"(qb[5]),
                              "=&v"(qb[6]), "=&v"(qb[7])
                            : "v"(e1rd)
                            : "memory");
                        // a wave's LDS reads complete in order: <= 8 outstanding = the first block is in
                        asm volatile("s_waitcnt lgkmcnt(8)"
                                     : "+v"(qa[0]), "+v"(qa[1]), "+v"(qa[2]), "+v"(qa[3]), "+v"(qa[4]), "+v"(qa[5]),
                                       "+v"(qa[6]), "+v"(qa[7])
                                     :
                                     : "memory");
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {  // j = 2 jj
                            v[4 * jj] = make_float2(qa[2 * jj].x, qa[2 * jj + 1].x);
                            v[4 * jj + 1] = make_float2(qa[2 * jj].y, qa[2 * jj + 1].y);
                        }
                        if (AID_K1_DIAG != 9) {
                            dft4(v[0], v[4], v[8], v[12]);
                            dft4(v[1], v[5], v[9], v[13]);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        asm volatile("s_waitcnt lgkmcnt(0)"
                                     : "+v"(qb[0]), "+v"(qb[1]), "+v"(qb[2]), "+v"(qb[3]), "+v"(qb[4]), "+v"(qb[5]),
                                       "+v"(qb[6]), "+v"(qb[7])
                                     :
                                     : "memory");
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {  // j = 2 jj + 1
                            v[4 * jj + 2] = make_float2(qb[2 * jj].x, qb[2 * jj + 1].x);
                            v[4 * jj + 3] = make_float2(qb[2 * jj].y, qb[2 * jj + 1].y);
                        }
                    }
#else
                    {
                        // 16 ds_read_b64 in one block (hipcc would pair them into ds_read2_b64 / read2st64,
                        // 8 LDS cycles per pair instead of 2 + 2); the block waits for its own results
                        float2 q[16];
                        asm volatile(
                            "ds_read_b64 %0, %16 offset:0\n\tds_read_b64 %1, %16 offset:256\n\t"
                            "ds_read_b64 %2, %16 offset:32\n\tds_read_b64 %3, %16 offset:288\n\t"
                            "ds_read_b64 %4, %16 offset:64\n\tds_read_b64 %5, %16 offset:320\n\t"
                            "ds_read_b64 %6, %16 offset:96\n\tds_read_b64 %7, %16 offset:352\n\t"
                            "ds_read_b64 %8, %16 offset:128\n\tds_read_b64 %9, %16 offset:384\n\t"
                            "ds_read_b64 %10, %16 offset:160\n\tds_read_b64 %11, %16 offset:416\n\t"
                            "ds_read_b64 %12, %16 offset:192\n\tds_read_b64 %13, %16 offset:448\n\t"
                            "ds_read_b64 %14, %16 offset:224\n\tds_read_b64 %15, %16 offset:480\n\t"
                            "s_waitcnt lgkmcnt(0)"
                            : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),
                              "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]),
                              "=&v"(q[12]), "=&v"(q[13]), "=&v"(q[14]), "=&v"(q[15])
                            : "v"(e1rd)
                            : "memory");
                        // q[2 j + c] = component c of (A[kq][8 j + mq], A[kq][8 j + 4 + mq]) = m1 = 2 j, 2 j + 1
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            v[2 * j] = make_float2(q[2 * j].x, q[2 * j + 1].x);
                            v[2 * j + 1] = make_float2(q[2 * j].y, q[2 * j + 1].y);
                        }
                    }
#endif  // AID_K1_E1STAGED
#elif AID_K1_E1SWAP
                    e1_transpose(v);
#elif AID_K1_E1V
#pragma unroll
                    for (int k1 = 0; k1 < 16; ++k1)
                        buf[k1 * 64 + 8 * ((kq >> 1) ^ (k1 & 7)) + 2 * mq + (kq & 1)] = v[k1];
                    wave_lds_sync();
                    const float4 *buf4 = reinterpret_cast<const float4 *>(buf);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float4 q = buf4[kq * 32 + 4 * (j ^ (kq & 7)) + mq];
                        v[2 * j] = make_float2(q.x, q.y);
                        v[2 * j + 1] = make_float2(q.z, q.w);
                    }
#else
#pragma unroll
                    for (int k1 = 0; k1 < 16; ++k1)
                        buf[AID_K1_COMPACT ? k1 * 64 + (lane ^ (4 * (k1 & 7))) : k1 * 68 + lane] = v[k1];
                    wave_lds_sync();
#pragma unroll
                    for (int m1 = 0; m1 < 16; ++m1)
                        v[m1] = buf[AID_K1_DIAG == 4    ? m1 * 68 + lane
                                    : AID_K1_COMPACT ? kq * 64 + 4 * ((m1 & 8) | ((m1 ^ kq) & 7)) + mq
                                                     : kq * 68 + 4 * m1 + mq];
#endif
                    if (!AID_K1_E1SWAP) wave_lds_sync();
                }
                // stage B
#if AID_K1_PRIO
                __builtin_amdgcn_s_setprio(0);
#endif
#if AID_K1_TPF_B
                float4 tpb[8];
#pragma unroll
                for (int h = 0; h < AID_K1_TPF_B; ++h) tpb[h] = s_tb4[4 * h + mq];
                __builtin_amdgcn_sched_barrier(0);
#endif
                if (AID_K1_DIAG != 9) dft16(v, t16, AID_K1_E1ADDTID && AID_K1_E1STAGED && !AID_K1_E1Q ? 2 : 0);
#if AID_K1_TPF_B
#pragma unroll
                for (int h = AID_K1_TPF_B; h < 8; ++h) tpb[h] = s_tb4[4 * h + mq];
#endif
#pragma unroll
                for (int h = 0; h < 8; ++h) {
#if AID_K1_TPF_B
                    const float4 t = tpb[h];
#else
                    const float4 t = s_tb4[4 * h + mq];
#endif
                    if (h) v[2 * h] = cmul(v[2 * h], make_float2(t.x, t.y));
                    v[2 * h + 1] = cmul(v[2 * h + 1], make_float2(t.z, t.w));
                }
#if AID_K1_DPPC
                // stage C across the quad (FPSPEC 3 DFT4 over m2 = mq, for every j1), each butterfly
                // one in-place fma with the partner as DPP operand: x <- partner * s + x
                //   s1 = (+1, +1, -1, -1): lanes 0..3 -> t0, t2, -t1, -t3
                //   lane 3: u = -i t3 from -t3: (-T.im, T.re); lanes 0..2 keep their value
                //   s2 = (+1, -1, -1, +1): lanes 0..3 -> y0, -y2, -y1, -y3
                // fma(p, +-1, x) rounds x +- p once: FPSPEC's add/sub values; the signs are exact
                // and cancel in the real split (see there)
#if AID_K1_DPPC == 3
                {
                    // E2 by add-TID: lane (kq, mq) puts component c of B[kq][mq][j1] at position 4 kq + mq of
                    // region (j1, c) = dword 128 j1 + 64 c; reader lane l (kq2 = l & 15, s = l >> 4) takes the
                    // 4 m2 values of B[kq2][.][4 s + r] as one ds_read_b128 per component (conflict-free: the 16
                    // lanes of each b128 group cover 16 distinct 4-bank quads), runs FPSPEC 3's DFT4 in
                    // registers and spills Z[kq2 + 16 (4 s + r) + 256 j2] (true signs) to E3
                    AID_TID8(e2_region, 0);
                    AID_TID8(e2_region, 4);
                    AID_TID8(e2_region, 8);
                    AID_TID8(e2_region, 12);
                    float4 q2[8];
                    asm volatile(
                        "ds_read_b128 %0, %8 offset:0\n\tds_read_b128 %1, %8 offset:256\n\t"
                        "ds_read_b128 %2, %8 offset:512\n\tds_read_b128 %3, %8 offset:768\n\t"
                        "ds_read_b128 %4, %8 offset:1024\n\tds_read_b128 %5, %8 offset:1280\n\t"
                        "ds_read_b128 %6, %8 offset:1536\n\tds_read_b128 %7, %8 offset:1792\n\t"
                        "s_waitcnt lgkmcnt(0)"
                        : "=&v"(q2[0]), "=&v"(q2[1]), "=&v"(q2[2]), "=&v"(q2[3]), "=&v"(q2[4]), "=&v"(q2[5]),
                          "=&v"(q2[6]), "=&v"(q2[7])
                        : "v"(e2rd)
                        : "memory");
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float4 re = q2[2 * r], im = q2[2 * r + 1];
                        float2 x0 = make_float2(re.x, im.x), x1 = make_float2(re.y, im.y);
                        float2 x2 = make_float2(re.z, im.z), x3 = make_float2(re.w, im.w);
                        dft4(x0, x1, x2, x3);
                        if (AID_K1_DIAG != 8) {
                            buf[e3c[0] + 16 * r] = x0;
                            buf[e3c[1] + 16 * r + 256] = x1;
                            buf[e3c[2] + 16 * r + 512] = x2;
                            buf[e3c[3] + 16 * r + 768] = x3;
                        }
                    }
                }
#elif AID_K1_DPPC == 2
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
#if AID_K1_E3ADDTID
                    if constexpr (!LOGMAG) {  // literal register groups for the asm's immediates
                        if (j0 == 0) AID_TID8(e3_region, 0);
                        else if (j0 == 4) AID_TID8(e3_region, 4);
                        else if (j0 == 8) AID_TID8(e3_region, 8);
                        else AID_TID8(e3_region, 12);
                    } else
#endif
                    {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (AID_K1_DIAG != 8) buf[
#if AID_K1_E3Q
                                    e3wq + 64 * (j0 + j)
#else
                                    e3w + 16 * (j0 + j)
#endif
                            ] = v[j0 + j];
#if AID_K1_E3Q
                        // Z[768] (lane 3) copied to 1026, every other lane to its own dummy slot: one unconditional
                        // store (an exec-masked branch here made hipcc spill)
                        if (AID_K1_E3Q_DUP && j0 == 0) buf[e3dup] = v[0];
#endif
                    }
                }
#else
#pragma unroll
                for (int j1 = 0; j1 < 16; ++j1) {
                    float2 x = v[j1];
                    x.x = __builtin_fmaf(quad_dpp<0x4E>(x.x), s1, x.x);
                    x.y = __builtin_fmaf(quad_dpp<0x4E>(x.y), s1, x.y);
                    const float ux = mq == 3 ? -x.y : x.x, uy = mq == 3 ? x.x : x.y;
                    v[j1] = make_float2(__builtin_fmaf(quad_dpp<0xB1>(ux), s2, ux), __builtin_fmaf(quad_dpp<0xB1>(uy), s2, uy));
                    buf[e3w + 16 * j1] = v[j1];
                }
#endif
#else
                // E2: lane (kq, m2) writes B[kq][m2][j1]; reader lane (kq, s = mq) takes j1 = s + 4r
                if (AID_K1_DIAG != 7) {
#pragma unroll
                    for (int j1 = 0; j1 < 16; ++j1)
                        buf[AID_K1_COMPACT ? j1 * 64 + (lane ^ (j1 & 3)) : lane * 17 + j1] = v[j1];
                    wave_lds_sync();
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int m2 = 0; m2 < 4; ++m2)
                            v[4 * r + m2] = buf[AID_K1_DIAG == 5    ? (4 * r + m2) * 68 + lane
                                                : AID_K1_COMPACT ? (mq + 4 * r) * 64 + 4 * kq + (m2 ^ mq)
                                                                 : (4 * kq + m2) * 17 + mq + 4 * r];
                    wave_lds_sync();
                }
                // stage C: DFT4 over m2 -> Z[kq + 16*(mq + 4r) + 256*j2]; E3 natural order, pad 1 per 32
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    dft4(v[4 * r + 0], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
#pragma unroll
                    for (int j2 = 0; j2 < 4; ++j2) {
                        const int a = AID_K1_DIAG == 1 ? lane + 64 * (r + 4 * j2) : e3w + 64 * r + 256 * j2;
                        if (AID_K1_DIAG != 8) buf[a] = v[4 * r + j2];
                    }
                }
#endif
                wave_lds_sync();
                float *drow = dst + (int64_t)f * kBins;
#if AID_K1_BRANCHFREE
                if constexpr (!LOGMAG && AID_K1_DIAG == 0) {
#if AID_K1_E3ADDTID
                    // real split over the add-TID E3 regions (see e3_region): 18 ds_read_b64 in one block
                    // (hipcc would pair them into 8-cycle ds_read2 forms); q[4u + 0/1] = (Z[k], -Z[k + 512])
                    // re / im, q[4u + 2/3] = (-Z[512 - k], -Z[1024 - k]) re / im, k = lane + 64 u; x = the
                    // broadcast (-Z[256], -Z[768])
                    uint32_t hotw = 0;
                    float2 q[16], qx0, qx1;
                    asm volatile(
                        "ds_read_b64 %0, %18 offset:0\n\tds_read_b64 %1, %18 offset:256\n\t"
                        "ds_read_b64 %2, %19 offset:6240\n\tds_read_b64 %3, %19 offset:6496\n\t"
                        "ds_read_b64 %4, %18 offset:2080\n\tds_read_b64 %5, %18 offset:2336\n\t"
                        "ds_read_b64 %6, %19 offset:4160\n\tds_read_b64 %7, %19 offset:4416\n\t"
                        "ds_read_b64 %8, %18 offset:4160\n\tds_read_b64 %9, %18 offset:4416\n\t"
                        "ds_read_b64 %10, %19 offset:2080\n\tds_read_b64 %11, %19 offset:2336\n\t"
                        "ds_read_b64 %12, %18 offset:6240\n\tds_read_b64 %13, %18 offset:6496\n\t"
                        "ds_read_b64 %14, %19 offset:0\n\tds_read_b64 %15, %19 offset:256\n\t"
                        "ds_read_b64 %16, %20 offset:0\n\tds_read_b64 %17, %20 offset:256"
#if !AID_K1_E3STAGED
                        "\n\ts_waitcnt lgkmcnt(0)"
#endif
                        : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]),
                          "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]), "=&v"(q[12]),
                          "=&v"(q[13]), "=&v"(q[14]), "=&v"(q[15]), "=&v"(qx0), "=&v"(qx1)
                        : "v"(e3d), "v"(e3m), "v"(e3x)
                        : "memory");
                    float pa[4], pb[4], pc[4], pd[4];  // bins k, 1024 - k, 512 + k, 512 - k
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
#if AID_K1_E3STAGED
                        // LDS reads of one wave complete in order: unit u's 4 are done once at most
                        // 14 - 4 u of the block's reads (or later LDS ops) are outstanding
                        if (u == 0) asm volatile("s_waitcnt lgkmcnt(14)" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
                        if (u == 1) asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(q[4]), "+v"(q[5]), "+v"(q[6]), "+v"(q[7]));
                        if (u == 2) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(q[8]), "+v"(q[9]), "+v"(q[10]), "+v"(q[11]));
                        if (u == 3) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(q[12]), "+v"(q[13]), "+v"(q[14]), "+v"(q[15]));
#endif
                        const float2 dre = q[4 * u], dim = q[4 * u + 1], mre = q[4 * u + 2], mim = q[4 * u + 3];
                        const bool l0 = u == 0 && lane == 0;  // k = 0
                        {   // pair (k, 1024 - k): Z[1024 - k] is stored negated; k = 0 pairs with Z[0] itself
                            const float2 a = make_float2(dre.x, dim.x);
                            const float2 b = l0 ? a : make_float2(-mre.y, -mim.y);
                            const float er = a.x + b.x, ei = a.y - b.y;
                            const float orr = a.y + b.y, oi = b.x - a.x;
                            const float2 tw = cmul(make_float2(orr, oi), s_t2[64 * u + lane]);
                            const float xr = er + tw.x, xi = ei + tw.y;
                            pa[u] = __builtin_fmaf(xr, xr, xi * xi);
                            const float xr2 = er - tw.x, xi2 = tw.y - ei;  // AID_K1_MIRROR_ID
                            pb[u] = l0 ? 0.f : __builtin_fmaf(xr2, xr2, xi2 * xi2);  // k = 0: Nyquist, dropped
                        }
                        {   // pair (K, 1024 - K), K = 512 - k: both stored negated (every sum flips sign, the
                            // squares do not see it); k = 0: K = 512 is its own mirror (lane 0's mirror read
                            // of unit 0 is not a bin)
                            const float2 b = make_float2(dre.y, dim.y);
                            const float2 a = l0 ? b : make_float2(mre.x, mim.x);
                            const float er = a.x + b.x, ei = a.y - b.y;
                            const float orr = a.y + b.y, oi = b.x - a.x;
                            const float2 tw = cmul(make_float2(orr, oi), s_t2[512 - 64 * u - lane]);
                            const float xr = er + tw.x, xi = ei + tw.y;
                            pd[u] = __builtin_fmaf(xr, xr, xi * xi);
                            const float xr2 = er - tw.x, xi2 = tw.y - ei;
                            pc[u] = l0 ? 0.f : __builtin_fmaf(xr2, xr2, xi2 * xi2);
                        }
                        hotw |= __ballot(pa[u] > thr) ? 1u << u : 0u;                            // block u
                        hotw |= __ballot(pb[u] > thr) ? (u == 0 ? 1u << 15 : 3u << (15 - u)) : 0u;  // 15-u, 16-u
                        hotw |= __ballot(pc[u] > thr) ? 1u << (8 + u) : 0u;                      // block 8+u
                        {  // exact bits: a superset here would mark block 8 - u hot above a hot block 7 - u
                            const uint64_t hb = __ballot(pd[u] > thr);
                            hotw |= (hb >> 1) ? 1u << (7 - u) : 0u;  // lanes 1..63: block 7 - u
                            hotw |= (hb & 1) ? 1u << (8 - u) : 0u;   // lane 0: block 8 - u
                        }
                    }
#if AID_K1_E3STAGED
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(qx0), "+v"(qx1));
#endif
                    {  // bins 256 and 768: every lane (same addresses, same values)
                        const float2 a = make_float2(qx0.x, qx1.x), b = make_float2(qx0.y, qx1.y);
                        const float er = a.x + b.x, ei = a.y - b.y;
                        const float orr = a.y + b.y, oi = b.x - a.x;
                        const float2 tw = cmul(make_float2(orr, oi), s_t2[256]);
                        const float xr = er + tw.x, xi = ei + tw.y;
                        const float p256 = __builtin_fmaf(xr, xr, xi * xi);
                        const float xr2 = er - tw.x, xi2 = tw.y - ei;
                        const float p768 = __builtin_fmaf(xr2, xr2, xi2 * xi2);
                        pstore(drow + 256, p256);
                        pstore(drow + 768, p768);
                        hotw |= p256 > thr ? 1u << 4 : 0u;
                        hotw |= p768 > thr ? 1u << 12 : 0u;
                    }
                    hotw = __builtin_amdgcn_readfirstlane(hotw);
                    dhot[f] = hotw;
                    const uint32_t hsel = keep ? 0x1FFFFu : hotw;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if ((hsel >> u) & 1u) pstore(drow + lane + 64 * u, pa[u]);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (((hsel >> (8 + u)) & 1u) && (u > 0 || lane != 0)) pstore(drow + 512 + lane + 64 * u, pc[u]);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (((hsel >> (7 - u)) | (hsel >> (8 - u))) & 1u) pstore(drow + 512 - (lane + 64 * u), pd[u]);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t need = (hsel >> (15 - u)) | (u > 0 ? hsel >> (16 - u) : 0u);
                        if ((need & 1u) && (u > 0 || lane != 0)) pstore(drow + 1024 - (lane + 64 * u), pb[u]);
                    }
#else
                    // straight-line real split: all 16 powers first, then the hot word, then 16
                    // unconditional stores whose base is the row or, for a cold block, this
                    // workgroup's dummy row (a scalar select: no branch splits the arithmetic)
                    uint32_t hotw = 0;
                    float po[8], pm[8];
#if AID_K1_TPF_S
                    // every read of the split issued up front (v is dead here: its 32 VGPRs hold them)
                    float2 sa[8], sb[8], st[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        sa[i] = buf[(i < 4 ? e3a0 : e3a1) + 64 * i];
                        sb[i] = buf[(i == 0 && lane == 0) ? 0 : (i < 4 ? e3b1 : i == 4 ? e3b4 : e3b0) + 64 * (15 - i)];
                        st[i] = s_t2[64 * i + lane];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#endif
#if AID_K1_E3Q
                    float4 qa, qb;  // the pair of b128 reads that serve bins i and i + 4
#endif
#pragma unroll
                    for (int ii = 0; ii < 8; ++ii) {
#if AID_K1_E3Q
                        // order i = 0, 4, 1, 5, ...: one pair of reads serves two mirror pairs, then dies
                        const int i = (ii >> 1) + 4 * (ii & 1);
                        if ((ii & 1) == 0) {
                            const float4 *buf4 = reinterpret_cast<const float4 *>(buf);
                            qa = buf4[e3qa + 128 * (ii >> 1)];
                            qb = buf4[e3qb - 128 * (ii >> 1)];
                        }
                        // i < 4: a = Z[k], bs = -Z[1024 - k] (stored); i >= 4: a = -Z[k], bs = -Z[1024 - k] (k >= 256)
                        const float2 a = i < 4 ? make_float2(qa.x, qa.y) : make_float2(qa.z, qa.w);
                        const float2 bs = i < 4 ? make_float2(qb.z, qb.w) : make_float2(qb.x, qb.y);
                        // k = 0 (lane 0, i = 0) pairs with Z[0] itself
                        const float2 b = i == 0 ? (lane == 0 ? a : make_float2(-bs.x, -bs.y)) : i < 4 ? make_float2(-bs.x, -bs.y) : bs;
#else
                        const int i = ii;
#if AID_K1_TPF_S
                        const float2 a = sa[i], bs = sb[i];
#else
                        const float2 a = buf[AID_E3A(i) + 64 * i];
                        const int bi = (i == 0 && lane == 0) ? 0 : AID_E3B(i) + 64 * (15 - i);
                        const float2 bs = buf[bi];
#endif
                        const float2 b = AID_K1_DPPC == 3 ? bs : i == 0 ? make_float2(bs.x * s0, bs.y * s0) : i < 4 ? make_float2(-bs.x, -bs.y) : bs;
#endif
                        const float er = a.x + b.x, ei = a.y - b.y;
                        const float orr = a.y + b.y, oi = b.x - a.x;
#if AID_K1_TPF_S
                        const float2 t2h = st[i];
#else
                        const float2 t2h = s_t2[64 * i + lane];
#endif
                        const float2 tw = cmul(make_float2(orr, oi), make_float2(t2h.x, t2h.y));
                        const float xr = er + tw.x, xi = ei + tw.y;
                        po[i] = __builtin_fmaf(xr, xr, xi * xi);  // Q = 4P (see below)
#if AID_K1_MIRROR_ID
                        // the mirror bin's product cmul((orr, -oi), (-t2.re, t2.im)) is (-tw.x, tw.y) bit for bit:
                        // its re is fma(orr, -c, oi*s) = -fma(orr, c, -(oi*s)) (round-to-nearest is odd-symmetric)
                        // and its im is fma(orr, s, (-oi)*(-c)) = tw.y; so xr2 = er + (-tw.x), xi2 = -ei + tw.y
                        const float xr2 = er - tw.x, xi2 = tw.y - ei;
#else
                        const float2 tw2 = cmul(make_float2(orr, -oi), make_float2(-t2h.x, t2h.y));
                        const float xr2 = er + tw2.x, xi2 = -ei + tw2.y;
#endif
                        // k = 0 (lane 0, i = 0): the mirror is the dropped Nyquist bin
                        pm[i] = (i == 0 && lane == 0) ? 0.f : __builtin_fmaf(xr2, xr2, xi2 * xi2);
                        hotw |= __ballot(po[i] > thr) ? 1u << i : 0u;  // bins 64i..64i+63
                        // lanes 1..63: bins of block 15 - i; lane 0 (i > 0): block 16 - i
                        const uint64_t hb = __ballot(pm[i] > thr);
#if AID_K1_HOTSUP
                        // one test marks both blocks: a superset of the hot blocks (exact for K2, which
                        // only skips blocks marked cold), 3 scalar ops instead of 6 + a 64-bit VALU compare
                        hotw |= hb ? (i == 0 ? 1u << 15 : 3u << (15 - i)) : 0u;
#else
                        hotw |= (hb >> 1) ? 1u << (15 - i) : 0u;
                        hotw |= (hb & 1) ? 1u << (16 - i) : 0u;
#endif
                    }
                    {  // bin 512 pairs with itself: every lane computes it (same address, same value),
                       // so its store and the hot word's need no lane-0 branch
                        const float2 a = buf[AID_K1_E3Q ? 2 : e3(512)];
                        const float er = a.x + a.x, ei = a.y - a.y, orr = a.y + a.y, oi = a.x - a.x;
                        const float2 tw = cmul(make_float2(orr, oi), t512);
                        const float xr = er + tw.x, xi = ei + tw.y;
                        const float p512 = __builtin_fmaf(xr, xr, xi * xi);
                        pstore(drow + 512, p512);
                        hotw |= p512 > thr ? 1u << 8 : 0u;
                    }
                    hotw = __builtin_amdgcn_readfirstlane(hotw);
                    dhot[f] = hotw;
                    const uint32_t hsel = keep ? 0x1FFFFu : hotw;  // one select, not a branch per store
#if AID_K1_STBR
                    // cold stores skipped by scalar branches (the powers are all computed above, so the
                    // branches no longer split the arithmetic)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if ((hsel >> i) & 1u) pstore(drow + lane + 64 * i, po[i]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t need = (hsel >> (15 - i)) | (i > 0 ? hsel >> (16 - i) : 0u);
                        if ((need & 1u) && (i > 0 || lane != 0)) pstore(drow + 1024 - (lane + 64 * i), pm[i]);
                    }
#else
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        float *b = ((hsel >> i) & 1u) ? drow : dummy;
                        b[lane + 64 * i] = po[i];
                    }
                    // mirror store i covers bins 1025-64(i+1) .. 1023-64i of block 15-i (lanes 1..63)
                    // and bin 1024-64i of block 16-i (lane 0): written when either block is hot. A
                    // skipped store leaves only bins of cold blocks stale, which K2 never reads.
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t need = (hsel >> (15 - i)) | (i > 0 ? hsel >> (16 - i) : 0u);
                        float *b = (need & 1u) ? drow : dummy;
                        if (i == 0) b = lane == 0 ? dummy : b;  // lane 0's mirror of k = 0 is not a bin
                        b[1024 - (lane + 64 * i)] = pm[i];
                    }
#endif
#endif  // AID_K1_E3ADDTID
                } else
#endif
                {
                // hot blocks of the row: bit b = some bin of 64-bin block b is > thr (K2 skips the
                // others: a value <= thr can neither be a peak nor suppress one, FPSPEC 5)
                uint32_t hotw = 0;
                float acc10 = 0.f;
                float pm[8];  // the mirror bins 1024-k, held until hotw is complete
                float pv11[16];  // AID_K1_DIAG 11: the lane's 16 powers, stored as 4 dwordx4 (timing only)
                // real split, bins in mirror pairs (k, 1024-k): one read of Z[k], Z[1024-k] serves
                // both. For bin 1024-k the FPSPEC sums are the same exact values with signs
                // flipped (a+c, c+a commute; b-d = -(d-b)), so both bins stay bit-exact.
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int k = lane + 64 * i;  // 0..511
#if AID_K1_DPPC
                    const float2 a = AID_K1_DIAG == 8 ? v[i] : buf[AID_K1_E3Q ? e3q_slot(k) : (i < 4 ? e3a0 : e3a1) + 64 * i];
                    // k = 0 mirrors onto itself (Z[0]: slot 0)
                    const int bi = (i == 0 && lane == 0) ? 0 : AID_K1_E3Q ? e3q_slot(1024 - k) : (i < 4 ? e3b1 : i == 4 ? e3b4 : e3b0) + 64 * (15 - i);
#else
                    const float2 a = AID_K1_DIAG == 8 ? v[i] : buf[e3a + 64 * i];
                    // k = 0 mirrors onto itself (Z[0]): lane 0's e3b + 960 would be slot 1024
                    const int bi = (i == 0 && lane == 0) ? 0 : e3b + 64 * (15 - i);
#endif
#if AID_K1_DPPC
                    // stored Z[k] is -Z[k] for k >= 256 (lanes 1..3 of stage C): for i < 4, a is exact
                    // and b is stored negated (except Z[0] for lane 0, i = 0), so flip b; for i >= 4 both
                    // are negated, every sum below flips sign and the squares in P do not see it
                    const float2 bs = AID_K1_DIAG == 8 ? v[15 - i] : buf[bi];
                    const float2 b = AID_K1_DPPC == 3 ? bs : i == 0 ? make_float2(bs.x * s0, bs.y * s0) : i < 4 ? make_float2(-bs.x, -bs.y) : bs;
#else
                    const float2 b = AID_K1_DIAG == 8 ? v[15 - i] : buf[AID_K1_DIAG == 2 ? e3(k ^ 512) : bi];
#endif
                    const float er = a.x + b.x, ei = a.y - b.y;
                    const float orr = a.y + b.y, oi = b.x - a.x;
#if AID_K1_T2HALF
                    const float2 t2h = s_t2[64 * i + lane];
                    const float4 t2 = make_float4(t2h.x, t2h.y, -t2h.x, t2h.y);  // T2K[1024-k] = (-re, im)
#else
                    const float4 t2 = s_t2p[64 * i + lane];
#endif
                    {
                        const float2 tw = cmul(make_float2(orr, oi), make_float2(t2.x, t2.y));
                        const float xr = er + tw.x, xi = ei + tw.y;
                        // FPSPEC 4: P = fma(..) * 0.25f. The plane stores Q = fma(..) = 4P instead (one
                        // VALU less per bin): the scaling by 4 is exact and order-preserving, so every
                        // decision against thr is the same against 4 thr (the caller passes 4 thr), and
                        // aid_result_power applies the spec's * 0.25f on readout (bit-identical P)
                        const float P = LOGMAG ? __builtin_fmaf(xr, xr, xi * xi) * 0.25f : __builtin_fmaf(xr, xr, xi * xi);
                        const uint64_t hd = LOGMAG ? 0 : __ballot(P > thr);
                        if constexpr (LOGMAG) drow[k] = 10.0f * log10f(P + 1e-10f);
                        else if (AID_K1_DIAG == 10) acc10 += P;
                        else if (AID_K1_DIAG == 11) pv11[2 * i] = P;
                        else if (keep || hd) drow[k] = P;  // block i exactly
                        if constexpr (!LOGMAG) hotw |= hd ? 1u << i : 0u;  // bins 64i..64i+63
                    }
                    bool hot2 = false;
                    if (k != 0) {  // bin 1024-k (513..1023); k = 0's mirror is the dropped Nyquist bin
                        const float2 tw = cmul(make_float2(orr, -oi), make_float2(t2.z, t2.w));
                        const float xr = er + tw.x, xi = -ei + tw.y;
                        const float P = LOGMAG ? __builtin_fmaf(xr, xr, xi * xi) * 0.25f : __builtin_fmaf(xr, xr, xi * xi);
                        if constexpr (LOGMAG) drow[1024 - k] = 10.0f * log10f(P + 1e-10f);
                        else if (AID_K1_DIAG == 10) acc10 += P;
                        else if (AID_K1_DIAG == 11) pv11[2 * i + 1] = P;
                        else if (!LOGMAG) pm[i] = P;  // stored once the row's hot word is known
                        else drow[1024 - k] = P;
                        hot2 = P > thr;
                    } else if (AID_K1_DIAG == 11) {
                        pv11[2 * i + 1] = 0.f;
                    }
                    if constexpr (!LOGMAG) {  // lanes 1..63: bins of block 15 - i; lane 0 (i > 0): block 16 - i
                        const uint64_t hb = __ballot(hot2);
                        hotw |= (hb >> 1) ? 1u << (15 - i) : 0u;
                        hotw |= (hb & 1) ? 1u << (16 - i) : 0u;
                    }
                }
                if (AID_K1_DIAG == 10) drow[lane] = acc10;
                if (AID_K1_DIAG == 11) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        reinterpret_cast<float4 *>(drow)[64 * q + lane] =
                            make_float4(pv11[4 * q], pv11[4 * q + 1], pv11[4 * q + 2], pv11[4 * q + 3]);
                }
                if (lane == 0) {  // bin 512 pairs with itself
                    const float2 a = buf[AID_K1_E3Q ? 2 : e3(512)];
                    const float er = a.x + a.x, ei = a.y - a.y, orr = a.y + a.y, oi = a.x - a.x;
                    const float2 tw = cmul(make_float2(orr, oi), t512);
                    const float xr = er + tw.x, xi = ei + tw.y;
                    const float P = LOGMAG ? __builtin_fmaf(xr, xr, xi * xi) * 0.25f : __builtin_fmaf(xr, xr, xi * xi);
                    if constexpr (LOGMAG) drow[512] = 10.0f * log10f(P + 1e-10f);
                    else drow[512] = P;
                    if (P > thr) hotw |= 1u << 8;
                }
                if constexpr (!LOGMAG) {
                    hotw = __builtin_amdgcn_readlane(hotw, 0);  // lane 0 also holds bin 512's bit
                    if (lane == 0) dhot[f] = hotw;
                    // mirror store i covers bins 1025-64(i+1) .. 1023-64i of block 15-i (lanes 1..63)
                    // and bin 1024-64i of block 16-i (lane 0): written when either block is hot. A
                    // skipped store leaves only bins of cold blocks stale, which K2 never reads.
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t need = (hotw >> (15 - i)) | (i > 0 ? hotw >> (16 - i) : 0u);
                        if ((keep || (need & 1u)) && (i > 0 || lane != 0)) drow[1024 - (lane + 64 * i)] = pm[i];
                    }
                }
                }
                wave_lds_sync();
            }
        }
    }
#if AID_K1_BALANCED
    f += nfr;
    }
#endif
}

template <bool LOGMAG>
static void launch_rows(int rows, dim3 g, dim3 b, hipStream_t s, float *dummy, const float *pcm, const ClipDesc *clips, int n_clips,
                        int64_t total, int64_t n_waves, const Tables *tab, float *out, uint32_t *hot, float thr, int keep) {
    switch (rows) {
        case 1: timed_launch((k_stft_power<LOGMAG, 1>), g, b, 0, s, pcm, clips, n_clips, total, n_waves, tab, out, hot, thr, keep, dummy); break;
        case 2: timed_launch((k_stft_power<LOGMAG, 2>), g, b, 0, s, pcm, clips, n_clips, total, n_waves, tab, out, hot, thr, keep, dummy); break;
        case 4: timed_launch((k_stft_power<LOGMAG, 4>), g, b, 0, s, pcm, clips, n_clips, total, n_waves, tab, out, hot, thr, keep, dummy); break;
        case 8: timed_launch((k_stft_power<LOGMAG, 8>), g, b, 0, s, pcm, clips, n_clips, total, n_waves, tab, out, hot, thr, keep, dummy); break;
        default: timed_launch((k_stft_power<LOGMAG, 16>), g, b, 0, s, pcm, clips, n_clips, total, n_waves, tab, out, hot, thr, keep, dummy); break;
    }
}

// total_frames = sum of the clips' frames, total_strips = sum of ceil(F / kStftStrip) (strip mode),
// slots = resident K1 waves on the device (CUs x kStftWaves)
void launch_stft_power(const float *pcm, const ClipDesc *clips, int n_clips, int64_t total_frames,
                       int64_t total_strips, int64_t slots, int hop, const Tables *tab, float *out, bool logmag,
                       uint32_t *hot, float thr, bool keep_power, float *dummy, hipStream_t s) {
    if (total_frames <= 0) return;
#if AID_K1_BALANCED
    // one round of equal ranges. A wave reloads its 16-row ring once per segment, so large batches keep
    // >= kStftStrip frames per wave; a batch smaller than that spreads over >= kK1MinFrames-frame ranges
    // instead (a 5 s window, 465 frames: 29 waves x 16 frames ran 77 us of serial frames per wave)
    const int64_t n_waves = std::max<int64_t>(
        1, total_frames >= slots * kStftStrip ? slots : std::min<int64_t>(slots, total_frames / kK1MinFrames));
    const int64_t total = total_frames;
#else
    const int64_t n_waves = total_strips, total = total_strips;
    (void)slots;
#endif
    const dim3 g((unsigned)((n_waves + kStftWaves - 1) / kStftWaves)), b(kStftWaves * 64);
    if (logmag) launch_rows<true>(hop / 128, g, b, s, dummy, pcm, clips, n_clips, total, n_waves, tab, out, nullptr, thr, 1);
    else  // the power plane holds 4P (see the real split): hot blocks are those with 4P > 4 thr
        launch_rows<false>(hop / 128, g, b, s, dummy, pcm, clips, n_clips, total, n_waves, tab, out, hot, 4.0f * thr,
                           keep_power ? 1 : 0);
}

}  // namespace aid
