// engine.cpp -- host side of libaidfp.so: the C ABI of include/aidfp.h.
//
// Owns one GPU's tables and workspaces, builds the per-call clip descriptors
// (one small H2D copy), launches K1..K3 on the caller's stream and exposes the
// results. Replaces the `olaf_c` process boundary of the reference
// (audio-ident-service/app/audio/fingerprint.py:87-270).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/aidfp.h"
#include "aidfp_device.h"
#include "aidfp_layout.h"
#include "resample_design.h"

namespace aid {
void launch_stft_power(const float *pcm, const ClipDesc *clips, int n_clips, int64_t f0, int64_t total_frames,
                       int64_t total_strips, int64_t slots, int hop, const Tables *tab, float *out, bool logmag,
                       uint64_t *hot, float thr, bool keep_power, hipStream_t s);
int peak_pick_blocks_per_cu();
void launch_peak_pick(const float *power, const ClipDesc *clips, int n_clips, int64_t f0, int64_t total_strips,
                      int strip_len, float thr, const uint64_t *hot, uint64_t *mask, uint32_t *cold_cnt, hipStream_t s);
void launch_landmarks(const uint64_t *mask, const ClipDesc *clips, int n_clips, int64_t total_chunks,
                      int64_t *chunk_counts, uint64_t *records, int64_t *clip_counts, bool write, uint32_t *k2_cold,
                      uint64_t *k2_cold_host, uint32_t k2_waves, bool one_chunk_each, hipStream_t s);
void launch_synth(float *out, const uint32_t *tracks, const int64_t *starts, int n_clips, int64_t n, int sr,
                  int noise_a, uint32_t salt, int fmax_hz, bool envelope, const int16_t *sin_tab, hipStream_t s);
int64_t resample_lds_floats(int up, int down, int J);
void launch_resample(const float *src, int64_t in_base, int64_t n, int channels, int up, int down, int hl, int J,
                     const float *taps, float *dst, int64_t m_first, int64_t count, hipStream_t s, int n_streams = 1,
                     int64_t src_stride = 0, int64_t dst_stride = 0, const float *hist = nullptr, int64_t hist_n = 0,
                     int64_t hist_stride = 0);
int dedup_chunks(int64_t n_cat);
void launch_dedup_scan(const uint32_t *cw, const int64_t *coff, const double *cdur, int64_t n_cat, const uint32_t *qw,
                       const int64_t *qoff, const double *qlo, const double *qhi, int nq, double *part_sim,
                       int64_t *part_idx, double *best_sim, int64_t *best_idx, hipStream_t s);
void launch_dedup_pairs(const uint32_t *aw, const int64_t *aoff, const uint32_t *bw, const int64_t *boff, int n,
                        double *sim, hipStream_t s);
void launch_index_count(const uint32_t *ph, const uint32_t *ptrack, int64_t n, const uint8_t *tomb, uint32_t n_tracks,
                        uint32_t *cnt, hipStream_t s);
void launch_index_scatter(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                          const uint8_t *tomb, uint32_t n_tracks, uint32_t *cursor, uint64_t *post, hipStream_t s);
void launch_scan(const uint32_t *in, uint32_t *out, int64_t n, uint32_t *tmp, hipStream_t s);
size_t index_sort_temp_bytes(int64_t n);
bool k4_ab_sort_built();
int match_lds_blocks_per_cu();
size_t radix_scratch_u32(int64_t n);
hipError_t launch_index_sort_build(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n,
                                   const uint8_t *tomb, uint32_t n_tracks, uint32_t *keys0, uint32_t *keys1,
                                   uint64_t *vals0, uint64_t *vals1, void *temp, size_t temp_bytes, bool use_rocprim,
                                   uint32_t *scratch, uint32_t *E, uint32_t *offsets, unsigned long long *nz,
                                   uint64_t **vals_out, uint16_t *sig, int rank_mode, hipStream_t s);
void launch_make_sig(const uint64_t *post, int64_t n, uint16_t *sig, hipStream_t s);
void launch_compact(const uint32_t *ph, const uint32_t *ptrack, const uint32_t *pt, int64_t n, const uint8_t *tomb,
                    uint32_t n_tracks, uint32_t *cnt, uint32_t *off, uint32_t *tmp, uint32_t *oh, uint32_t *otrack,
                    uint32_t *ot, hipStream_t s);
void launch_records_to_postings(const uint64_t *recs, const int64_t *src_off, const int64_t *counts,
                                const int64_t *dst_off, const uint32_t *track_ids, int n_clips, uint32_t *ph,
                                uint32_t *ptrack, uint32_t *pt, hipStream_t s);
void launch_append_offsets(const int64_t *counts, int n_clips, int64_t base, int64_t *dst_off, int64_t *total,
                           hipStream_t s);
void launch_query_votes(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq,
                        const uint32_t *offsets, int64_t *votes, uint64_t *ranges, hipStream_t s);
void launch_query(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq, const uint32_t *offsets,
                  const uint64_t *post, const uint8_t *tomb, uint32_t n_tracks, int min_match, int max_rows,
                  uint32_t *hist, int hist_bits, uint32_t *hot, int32_t *rows, int32_t *nrows, int tomb_live,
                  int parts, int stage, uint32_t *dset, int dset_bits, hipStream_t s);
void launch_count_nonzero(const uint32_t *cnt, int64_t n, unsigned long long *out, hipStream_t s);
void launch_index_checksum(const uint32_t *ph, const uint32_t *ptr, const uint32_t *pt, int64_t first, int64_t n,
                           unsigned long long *out, hipStream_t s);
void launch_match_lds(const uint64_t *recs, const int64_t *qstart, const int64_t *qcount, int nq,
                      const uint32_t *offsets, const uint64_t *post, const uint8_t *tomb, uint32_t n_tracks,
                      int min_match, int max_rows, int32_t *rows, int32_t *nrows, int tomb_live, const int64_t *votes,
                      const uint16_t *sig, const uint64_t *ranges, hipStream_t s);
uint32_t index_keys();
void launch_downmix(const float *in, int64_t n, float *out, hipStream_t s);
void launch_window_gather(const float *src, const int64_t *win, int n_win, int64_t max_len, float *dst, hipStream_t s);
void launch_exact_consensus(const int32_t *rows, const int32_t *nrows, int mr, const int32_t *clip_win, int n_clips,
                            double sec, int max_out, void *out, int32_t *n_out, hipStream_t s);
void launch_rows_scatter(const int32_t *src, const int32_t *order, int n, int mr, int32_t *dst, hipStream_t s);
}  // namespace aid

#if defined(AID_K2_STAMPS)
namespace aid {
int k2_stamps_read(unsigned long long *out, bool reset);
}
extern "C" int aid_diag_k2_stamps(unsigned long long *out, int reset) {  // diagnostic build only
    return aid::k2_stamps_read(out, reset != 0);
}
#endif

using namespace aid;

static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail(_e == hipErrorOutOfMemory ? AID_ERR_NOMEM : AID_ERR_DEVICE,                \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                        \
    } while (0)

namespace {

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;  // capacity in elements
    hipError_t reserve(size_t want) {
        if (want <= n) return hipSuccess;
        if (p) {  // growing: in-flight work of earlier calls may still use the old buffer
            (void)hipDeviceSynchronize();
            (void)hipFree(p);
        }
        p = nullptr;
        n = 0;
        size_t cap = std::max(want, (size_t)1);
        hipError_t e = hipMalloc(&p, cap * sizeof(T));
        if (e == hipSuccess) n = cap;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// page-locked host buffer (hipHostMalloc): device-to-host copies into it are asynchronous, so a call can queue its
// result copies behind its kernels and wait once
template <typename T>
struct HostBuf {
    T *p = nullptr;
    size_t n = 0;  // capacity in elements
    hipError_t reserve(size_t want) {  // callers have synchronised any copy still targeting the old buffer
        if (want <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        const size_t cap = std::max(want, (size_t)64);
        hipError_t e = hipHostMalloc((void **)&p, cap * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = cap;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

struct ProfEvent {
    int kernel;
    hipEvent_t a, b;
};

}  // namespace

struct aid_engine;
static void free_ticket_pool(aid_engine *e);

struct aid_engine {
    aid_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    Tables *d_tab = nullptr;
    int16_t *d_sin = nullptr;

    DevBuf<float> pcm_stage;
    DevBuf<float> power;
    DevBuf<uint64_t> mask;
    DevBuf<uint64_t> hotw;  // K1 -> K2: per power row, bit hot_bit(c) = 16-bin chunk c has a value > thr
    DevBuf<uint32_t> k2_cold;  // K2: strip-cold wave counters (64), summed and reset by K3
    uint64_t *h_cold = nullptr;      // pinned, host-mapped: K3 stores (cold waves | waves << 32) of the last K2 here
    uint64_t *h_cold_dev = nullptr;  // its device address
    double k2_slots_x = 0.0;         // aid_engine_force K2_STRIPS: fixed strips per slot; 0 = adaptive (extract_locked)
    DevBuf<ClipDesc> desc;
    DevBuf<int64_t> chunk_counts;
    DevBuf<uint64_t> records;
    DevBuf<int64_t> counts;
    DevBuf<uint32_t> synth_tracks;
    DevBuf<int64_t> synth_starts;
    uint8_t *h_synth = nullptr;  // pinned staging of aid_synth_rate's tracks + starts (AID_SYNTH_ASYNC returns early)
    size_t h_synth_cap = 0;
    hipEvent_t synth_ev = nullptr;
    bool synth_ev_live = false;

    // index (FPSPEC 7): all postings (SoA source of truth) + the CSR built from them
    DevBuf<uint32_t> p_hash, p_track, p_t;
    int64_t n_post = 0;  // exact unless post_pend: then the last aid_index_add_extracted's count is in flight
    // aid_index_add_extracted appends without waiting for its clips' counts: K_append scans them on the device and
    // the new total comes back to pinned h_npost behind add_ev; settle_postings() makes n_post exact again
    DevBuf<int64_t> d_npost;
    int64_t *h_npost = nullptr;
    hipEvent_t add_ev = nullptr;  // after the last append's staging copies (and, if post_pend, its count copy)
    bool add_live = false, post_pend = false;
    std::vector<uint8_t> h_tomb;  // per track id: 1 = removed
    DevBuf<uint8_t> tomb;
    uint32_t n_tracks = 0;        // max track id + 1
    DevBuf<uint32_t> idx_cnt, idx_off, scan_tmp;
    DevBuf<uint64_t> idx_post;
    DevBuf<uint16_t> idx_sig;  // K5's 2-B vote signature per CSR posting (aidfp_layout.h posting_sig)
    DevBuf<uint32_t> srt_k0, srt_k1;  // K4 sort build: key double buffer
    DevBuf<uint64_t> srt_v;           // K4 sort build: the value buffer idx_post pairs with
    DevBuf<uint8_t> srt_tmp;          // K4 rocPRIM build (A/B): its temporary storage
    DevBuf<uint32_t> srt_scratch;     // K4 radix build: per-tile digit counts, their scan, scan temporary
    int k4_mode = 2;                  // internal K4 build: 2 radix sort (the default; K4_BUILD force 0, 1 or 4),
                                      // 1 rocPRIM sort (force 3, variant build only), 0 atomic counting sort (force 2)
    int k4_rank = 0;                  // radix sort's in-wave rank: 0 one LDS atomic per posting where the device
                                      // serves same-address lanes in order (else ballots), 1 ballots (K4_BUILD 4)
    bool index_built = false, index_dirty = true;
    int64_t n_indexed = 0;
    int64_t n_buckets_used = 0;
    int64_t n_fallback = 0;  // queries answered by the global-histogram path
    DevBuf<unsigned long long> nz;
    DevBuf<unsigned long long> chk;  // aid_index_checksum result
    // query workspaces
    DevBuf<uint64_t> q_recs;
    DevBuf<int64_t> q_start, q_count;
    DevBuf<uint32_t> q_hist;
    DevBuf<int32_t> q_rows, q_nrows;
    DevBuf<uint32_t> q_hot;  // K5h hot-bucket bitmaps, [batch][2^bits / 32]
    DevBuf<uint32_t> q_dset;  // K5b retries: HBM distinct (slot, t_q) sets, [batch][2^dbits]
    DevBuf<uint64_t> q_ranges;  // K5: per query record its CSR range (k_query_votes -> k_match_lds)
    HostBuf<int64_t> hq_meta;   // run_queries: per query start, record count, exact votes (pinned: async D2H)
    HostBuf<int32_t> hq_n;      // run_queries: the LDS path's per-query row counts
    HostBuf<int32_t> hq_rows;   // run_queries: the LDS path's rows, [nq][max_results][5]
    HostBuf<int64_t> hq_start;  // the queries' record starts (clip_base) staged page-locked for their upload
    std::vector<aid_query_ticket *> ticket_pool;  // collected tickets, reused: their buffers and event stay allocated
    DevBuf<int64_t> q_votes;  // exact votes per query (LDS-histogram eligibility)
    DevBuf<int64_t> x_src, x_dst;
    // batched exact lane (aid_exact_lane): PCM staging, window descriptors, consensus output
    DevBuf<float> x_in, x_win;
    DevBuf<int64_t> x_wdesc;
    DevBuf<int32_t> x_order, x_clipwin, x_nout;
    DevBuf<double> x_out;  // aid_exact_row, 3 x 8 bytes each
    DevBuf<int64_t> g_meta;            // all-gather: (count, n_tracks) per rank
    std::map<std::pair<int32_t, int32_t>, float *> rs_taps;  // (up, down) -> device [up][J] taps
    // Chromaprint dedup catalog (insertion order) + scan scratch
    DevBuf<uint32_t> dd_words;
    DevBuf<int64_t> dd_off;
    DevBuf<double> dd_dur;
    int64_t dd_n = 0, dd_nw = 0;
    DevBuf<uint32_t> dq_words, dq_words2;
    DevBuf<int64_t> dq_off, dq_off2, dq_idx, dq_pidx;
    DevBuf<double> dq_lo, dq_hi, dq_sim, dq_psim;
    DevBuf<uint32_t> g_send, g_recv;   // all-gather: [3][max] SoA planes per rank
    DevBuf<uint32_t> x_tracks;
    size_t hist_zero_cap = 0;  // q_hist capacity known to be all-zero

    int64_t *h_stage = nullptr;  // pinned staging of aid_index_add_extracted
    size_t h_stage_cap = 0;
    ClipDesc *h_desc = nullptr;  // pinned
    size_t h_desc_cap = 0;
    // extraction call hazards, tracked with events instead of a stream sync per call:
    // h_desc is the source of an async H2D copy; pcm_stage is read by K1
    hipEvent_t desc_ev = nullptr, stage_ev = nullptr;
    bool desc_ev_live = false, stage_ev_live = false;
    hipStream_t stage_stream = nullptr;  // the stream whose K1 read pcm_stage last
    std::vector<int64_t> desc_key;  // offsets (+ pcm location) the device descriptors were built for
    ClipDesc *desc_dev_for_key = nullptr;
    std::vector<int64_t> clip_base;  // host copy of desc[c].hash_base
    std::vector<int64_t> clip_frames;
    int n_clips = 0;
    int64_t total_frames = 0, total_strips = 0, total_chunks = 0, total_records = 0;
    int64_t k2_slots = 1;  // resident K2 workgroups on the device (CUs x blocks per CU)
    int64_t k1_slots = 1;  // resident K1 waves (CUs x kStftWaves: one K1 workgroup per CU)
    int k5_path = 0;       // aid_engine_force K5_PATH: 0 auto, 1 LDS fast path first, 2 global path only (tests)
    int k5_parts = 0;      // aid_engine_force K5_PARTS: K5a key partitions per query (0 = by vote count)
    int lane_gather = 0;           // aid_engine_force LANE_GATHER: stage the exact lane's sub-windows (A/B)
    int64_t plane_rows = 0;        // aid_engine_force PLANE_ROWS: power rows per K1 -> K2 clip group (0 = kPlaneRows)
    int inject_exchange_fail = 0;  // aid_engine_force EXCHANGE_FAIL: the next exchange's prepare step fails (tests)
    // aid_match_stats: queries, exact votes, and the postings K5 read (a vote = one 8-B posting per pass)
    int64_t st_queries = 0, st_votes = 0, st_post_reads = 0, st_q_global = 0, st_q_lds = 0, st_records = 0;
    int64_t st_sig_reads = 0;  // 2-B posting signatures the LDS path read (two per vote: counting and insert passes)
    int64_t st_fb_reason[5] = {0, 0, 0, 0, 0};  // LDS-path fallbacks (speculative pass) by reason (index.hip)
    int64_t tomb_since_build = 0;  // removals after the last CSR build (queries must check tomb[])
    size_t k5_batch = 2048;        // global-path queries per launch
    hipStream_t last_stream = nullptr;
    bool have_result = false;

    bool profiling = false;
    uint32_t prof_mask = 0xFFFFFFFFu;  // bit k: kernel id k gets events (aid_profile_select)
    std::vector<ProfEvent> pending;
    std::vector<hipEvent_t> pool;
    double prof_ms[AID_K_COUNT] = {};
    int64_t prof_n[AID_K_COUNT] = {};
    std::mutex mu;
};

static hipEvent_t take_event(aid_engine *e) {
    if (!e->pool.empty()) {
        hipEvent_t ev = e->pool.back();
        e->pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    return ev;
}

// attached = the scope wraps exactly one timed_launch: its events are stamped by the dispatch itself
// (aidfp_device.h LaunchTiming); otherwise two hipEventRecord markers bracket the scope.
struct ProfScope {
    aid_engine *e;
    int k;
    hipStream_t s;
    bool attached;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(aid_engine *e_, int k_, hipStream_t s_, bool attached_ = false) : e(e_), k(k_), s(s_), attached(attached_) {
        if (!e->profiling || !((e->prof_mask >> k) & 1u) || !(a = take_event(e))) return;
        if (!attached) {
            (void)hipEventRecord(a, s);
            return;
        }
        if (!(b = take_event(e))) {
            e->pool.push_back(a);
            a = nullptr;
            return;
        }
        launch_timing().start = a;
        launch_timing().stop = b;
    }
    ~ProfScope() {
        if (!a) return;
        if (attached) {
            LaunchTiming &t = launch_timing();
            if (t.start) {  // nothing was launched: the events were never stamped
                t.start = t.stop = nullptr;
                e->pool.push_back(a);
                e->pool.push_back(b);
                return;
            }
        } else {
            if (!(b = take_event(e))) return;
            (void)hipEventRecord(b, s);
        }
        e->pending.push_back({k, a, b});
    }
};

static void build_tables(Tables &t) {
    auto tw = [](int j, int L) {
        return make_float2((float)cos(2.0 * M_PI * (double)j / (double)L),
                           (float)(-sin(2.0 * M_PI * (double)j / (double)L)));
    };
    for (int m = 0; m < 1024; ++m)
        t.win2[m] = make_float2((float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)(2 * m) / 2048.0)),
                                (float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)(2 * m + 1) / 2048.0)));
    for (int j = 0; j < 16; ++j) t.t16[j] = tw(j, 16);
    for (int j = 0; j < 64; ++j) t.t64[j] = tw(j, 64);
    for (int j = 0; j < 1024; ++j) t.t1k[j] = tw(j, 1024);
    for (int j = 0; j < 1024; ++j) t.t2k[j] = tw(j, 2048);
}

static hipStream_t pick_stream(aid_engine *e, void *stream) {
    return stream ? (hipStream_t)stream : e->own_stream;
}

// A host-PCM call copies the caller's samples with ONE hipMemcpyAsync on the call's stream; from page-locked
// memory that copy is a real DMA that can still be running when the call returns. On success the caller syncs
// before reusing its buffer (include/aidfp.h); on an error return the engine drains the stream itself, so a
// caller that reuses or frees its buffer after a failed call cannot race the copy. Returns rc.
static int drain_host_copy(aid_engine *e, int32_t loc, void *stream, int rc) {
    if (rc != AID_OK && loc == AID_PCM_HOST && e) (void)hipStreamSynchronize(pick_stream(e, stream));
    return rc;
}

extern "C" {

int32_t aid_abi_version(void) { return AID_ABI_VERSION; }

const char *aid_last_error(void) { return g_err.c_str(); }

int aid_config_default(int32_t sample_rate, aid_config *out) {
    if (!out || sample_rate <= 0) return fail(AID_ERR_INVALID, "aid_config_default: bad argument");
    std::memset(out, 0, sizeof(*out));
    out->sample_rate = sample_rate;
    out->hop = sample_rate >= 32000 ? 512 : 256;
    out->peak_threshold = 4.0f;
    out->device = -1;
    out->min_match = 10;
    out->max_results = 50;
    return AID_OK;
}

int aid_engine_create(const aid_config *cfg, aid_engine **out) {
    if (!cfg || !out) return fail(AID_ERR_INVALID, "aid_engine_create: null argument");
    *out = nullptr;
    aid_config c = *cfg;
    if (c.sample_rate <= 0) return fail(AID_ERR_INVALID, "sample_rate must be > 0");
    if (c.hop == 0) c.hop = c.sample_rate >= 32000 ? 512 : 256;
    if (c.hop != 128 && c.hop != 256 && c.hop != 512 && c.hop != 1024 && c.hop != 2048)
        return fail(AID_ERR_INVALID, "hop must be one of 128, 256, 512, 1024, 2048");
    if (c.peak_threshold == 0.0f) c.peak_threshold = 4.0f;
    // [2^-124, 2^100]: K1/K2 compare the plane's Q = 4P against 4 thr. In that range 4 thr is exact and
    // any Q of a candidate (Q > 4 thr) is normal, so Q-order and P-order decide every comparison alike
    if (!(c.peak_threshold >= 0x1p-124f) || c.peak_threshold > 0x1p100f)
        return fail(AID_ERR_INVALID, "peak_threshold must be in [2^-124, 2^100]");
    if (c.min_match <= 0) c.min_match = 10;
    if (c.max_results <= 0) c.max_results = 50;
    if (c.flags & ~AID_FLAG_KEEP_POWER) return fail(AID_ERR_INVALID, "unknown aid_config.flags bits");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (ndev <= 0) return fail(AID_ERR_DEVICE, "no HIP device visible");
    int dev = c.device;
    if (dev < 0) HIP_TRY(hipGetDevice(&dev));
    if (dev >= ndev) return fail(AID_ERR_INVALID, "device ordinal out of range");
    HIP_TRY(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(AID_ERR_DEVICE, std::string("libaidfp is built for gfx950, device is ") + prop.gcnArchName);
    c.device = dev;

    aid_engine *e = new aid_engine();
    e->cfg = c;
    e->device = dev;
    e->k2_slots = (int64_t)prop.multiProcessorCount * peak_pick_blocks_per_cu();
    e->k1_slots = (int64_t)prop.multiProcessorCount * kStftWaves;
    // blocking stream: ordered against the legacy default stream (torch's default), so device
    // buffers the caller filled there without a stream handle are complete before NULL-stream calls
    hipError_t he = hipStreamCreateWithFlags(&e->own_stream, hipStreamDefault);
    if (he != hipSuccess) {
        delete e;
        return fail(AID_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(he));
    }
    Tables *h = new Tables();
    build_tables(*h);
    // K1 derives the real split's mirror twiddle T2K[1024-k] as (-re, im) of T2K[k]
    for (int k = 1; k < 512; ++k)
        if (!(h->t2k[1024 - k].x == -h->t2k[k].x && h->t2k[1024 - k].y == h->t2k[k].y)) {
            delete h;
            (void)hipStreamDestroy(e->own_stream);
            delete e;
            return fail(AID_ERR_DEVICE, "twiddle table lacks the mirror symmetry K1 relies on");
        }
    // K1's DFT16 (aidfp_device.h) shares one product in the cmuls by T16[2], T16[4], T16[6]
    {
        const float2 w2 = h->t16[2], w4 = h->t16[4], w6 = h->t16[6];
        if (!(w2.y == -w2.x && w6.x == w6.y && w6.x == -w2.x && w4.y == -1.0f)) {
            delete h;
            (void)hipStreamDestroy(e->own_stream);
            delete e;
            return fail(AID_ERR_DEVICE, "DFT16 twiddle table lacks the symmetry K1 relies on");
        }
    }
    std::vector<int16_t> sin_tab(4096);
    for (int k = 0; k < 4096; ++k) sin_tab[k] = (int16_t)nearbyint(32767.0 * sin(2.0 * M_PI * (double)k / 4096.0));
    he = hipMalloc(&e->d_tab, sizeof(Tables));
    if (he == hipSuccess) he = hipMemcpy(e->d_tab, h, sizeof(Tables), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMalloc(&e->d_sin, 4096 * sizeof(int16_t));
    if (he == hipSuccess) he = hipMemcpy(e->d_sin, sin_tab.data(), 4096 * sizeof(int16_t), hipMemcpyHostToDevice);
    delete h;
    if (he != hipSuccess) {
        aid_engine_destroy(e);
        return fail(AID_ERR_DEVICE, std::string("table upload: ") + hipGetErrorString(he));
    }
    *out = e;
    return AID_OK;
}

void aid_engine_destroy(aid_engine *e) {
    if (!e) return;
    // a call still running on another thread (ctypes releases the GIL) holds e->mu: it finishes before anything
    // is freed; the lock is released before the engine itself is deleted below
    std::unique_lock<std::mutex> destroy_lk(e->mu);
    (void)hipSetDevice(e->device);
    if (e->own_stream) (void)hipStreamSynchronize(e->own_stream);
    (void)hipDeviceSynchronize();
    for (auto &p : e->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto ev : e->pool) (void)hipEventDestroy(ev);
    e->pcm_stage.release();
    e->power.release();
    e->k2_cold.release();
    if (e->h_cold) (void)hipHostFree(e->h_cold);
    e->mask.release();
    e->desc.release();
    e->chunk_counts.release();
    e->records.release();
    e->counts.release();
    e->synth_tracks.release();
    e->synth_starts.release();
    e->p_hash.release();
    e->p_track.release();
    e->p_t.release();
    e->tomb.release();
    e->idx_cnt.release();
    e->idx_off.release();
    e->scan_tmp.release();
    e->idx_post.release();
    e->idx_sig.release();
    e->srt_k0.release();
    e->srt_k1.release();
    e->srt_v.release();
    e->srt_tmp.release();
    e->srt_scratch.release();
    e->nz.release();
    e->q_recs.release();
    e->q_start.release();
    e->q_count.release();
    e->q_hist.release();
    e->q_hot.release();
    e->q_dset.release();
    e->q_ranges.release();
    e->hq_meta.release();
    e->hq_n.release();
    e->hq_rows.release();
    e->hq_start.release();
    free_ticket_pool(e);
    e->q_rows.release();
    e->q_nrows.release();
    e->x_src.release();
    e->x_dst.release();
    e->x_in.release();
    e->x_win.release();
    e->x_wdesc.release();
    e->x_order.release();
    e->x_clipwin.release();
    e->x_nout.release();
    e->x_out.release();
    e->g_meta.release();
    for (auto &kv : e->rs_taps) (void)hipFree(kv.second);
    e->dd_words.release();
    e->dd_off.release();
    e->dd_dur.release();
    e->dq_words.release();
    e->dq_words2.release();
    e->dq_off.release();
    e->dq_off2.release();
    e->dq_idx.release();
    e->dq_pidx.release();
    e->dq_lo.release();
    e->dq_hi.release();
    e->dq_sim.release();
    e->dq_psim.release();
    e->g_send.release();
    e->g_recv.release();
    e->x_tracks.release();
    e->chk.release();
    if (e->h_desc) (void)hipHostFree(e->h_desc);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->h_synth) (void)hipHostFree(e->h_synth);
    if (e->h_npost) (void)hipHostFree(e->h_npost);
    e->d_npost.release();
    if (e->synth_ev) (void)hipEventDestroy(e->synth_ev);
    if (e->add_ev) (void)hipEventDestroy(e->add_ev);
    if (e->desc_ev) (void)hipEventDestroy(e->desc_ev);
    if (e->stage_ev) (void)hipEventDestroy(e->stage_ev);
    if (e->d_tab) (void)hipFree(e->d_tab);
    if (e->d_sin) (void)hipFree(e->d_sin);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    destroy_lk.unlock();
    delete e;
}

int aid_engine_config(const aid_engine *e, aid_config *out) {
    if (!e || !out) return fail(AID_ERR_INVALID, "null argument");
    *out = e->cfg;
    return AID_OK;
}

int aid_engine_force(aid_engine *e, int32_t what, int32_t value) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    switch (what) {
        case AID_FORCE_K5_PATH:
            if (value < 0 || value > 2) return fail(AID_ERR_INVALID, "K5_PATH: 0 auto, 1 LDS first, 2 global");
            e->k5_path = value;
            return AID_OK;
        case AID_FORCE_K5_PARTS:
            if (value != 0 && value != 1 && value != 2 && value != 4) return fail(AID_ERR_INVALID, "K5_PARTS: 0, 1, 2 or 4");
            e->k5_parts = value;
            return AID_OK;
        case AID_FORCE_K5_BATCH:
            if (value < 0) return fail(AID_ERR_INVALID, "K5_BATCH must be >= 0");
            e->k5_batch = value ? (size_t)value : 2048;
            return AID_OK;
        case AID_FORCE_K2_STRIPS_X100:
            if (value < 0) return fail(AID_ERR_INVALID, "K2_STRIPS_X100 must be >= 0");
            e->k2_slots_x = value / 100.0;
            e->desc_dev_for_key = nullptr;  // strip bases change: rebuild the descriptors
            return AID_OK;
        case AID_FORCE_K4_BUILD:
            if (value < 0 || value > 4)
                return fail(AID_ERR_INVALID, "K4_BUILD: 0 default, 1 radix, 2 atomic, 3 rocPRIM, 4 radix with ballot ranks");
            if (value == 3 && !k4_ab_sort_built())
                return fail(AID_ERR_INVALID, "K4_BUILD 3: the rocPRIM A/B build is only in the diagnostic variant "
                                             "library (build_ext.build(variant=\"k4rocprim\"), -DAID_K4_ROCPRIM_AB)");
            e->k4_mode = value == 2 ? 0 : value == 3 ? 1 : 2;
            e->k4_rank = value == 4 ? 1 : 0;
            e->index_dirty = true;
            return AID_OK;
        case AID_FORCE_EXCHANGE_FAIL:
            if (value != 0 && value != 1) return fail(AID_ERR_INVALID, "EXCHANGE_FAIL: 0 or 1");
            e->inject_exchange_fail = value;
            return AID_OK;
        case AID_FORCE_LANE_GATHER:
            if (value != 0 && value != 1) return fail(AID_ERR_INVALID, "LANE_GATHER: 0 or 1");
            e->lane_gather = value;
            return AID_OK;
        case AID_FORCE_PLANE_ROWS:
            if (value < 0) return fail(AID_ERR_INVALID, "PLANE_ROWS must be >= 0");
            e->plane_rows = value;
            return AID_OK;
        default:
            return fail(AID_ERR_INVALID, "aid_engine_force: unknown path id");
    }
}

int64_t aid_num_frames(const aid_engine *e, int64_t n) { return e ? num_frames(n, e->cfg.hop) : 0; }

int64_t aid_hash_capacity(const aid_engine *e, int64_t n) { return e ? hash_capacity(num_frames(n, e->cfg.hop)) : 0; }

static int extract_locked(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                          void *stream, const int64_t *ends = nullptr);

// power rows per K1 -> K2 clip group of one extraction call (3 GB of plane; extract_locked)
constexpr int64_t kPlaneRows = (int64_t)3 << 18;

int aid_extract(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc, void *stream) {
    if (!e || !offsets || n_clips < 0) return fail(AID_ERR_INVALID, "aid_extract: bad argument");
    if (loc != AID_PCM_HOST && loc != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "aid_extract: bad pcm_location");
    if (n_clips > 0 && !pcm && offsets[n_clips] > offsets[0]) return fail(AID_ERR_INVALID, "aid_extract: null pcm");
    for (int c = 0; c < n_clips; ++c)
        if (offsets[c + 1] < offsets[c] || offsets[c] < 0)
            return fail(AID_ERR_INVALID, "aid_extract: offsets must be non-decreasing and >= 0");
    std::lock_guard<std::mutex> lk(e->mu);
    return drain_host_copy(e, loc, stream, extract_locked(e, pcm, offsets, n_clips, loc, stream));
}

// Clip c is pcm[offsets[c], offsets[c + 1]); with `ends` (device PCM only) it is pcm[offsets[c], ends[c]), so
// clips may overlap (the exact lane's sub-windows are read in place).
static int extract_locked(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                          void *stream, const int64_t *ends) {
    if (ends && loc != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "extract: clip ends need device PCM");
    HIP_TRY(hipSetDevice(e->device));
    auto clip_len = [&](int c) { return (ends ? ends[c] : offsets[c + 1]) - offsets[c]; };
    hipStream_t s = pick_stream(e, stream);
    const int hop = e->cfg.hop;

    // descriptors; host PCM is staged as one copy of the clips' span
    if ((size_t)n_clips + 1 > e->h_desc_cap) {
        if (e->h_desc) HIP_TRY(hipHostFree(e->h_desc));
        e->h_desc = nullptr;
        e->h_desc_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&e->h_desc, sizeof(ClipDesc) * ((size_t)n_clips + 1)));
        e->h_desc_cap = (size_t)n_clips + 1;
    }
    // a different stream than the previous call's: order against it the simple way
    if (e->last_stream && e->last_stream != s) HIP_TRY(hipStreamSynchronize(e->last_stream));
    // same clips, PCM location and strip length as the descriptors already on the device: no re-upload
    // key: [offset, length] per clip, the PCM location, then the K2 strip length of every clip group (below)
    bool desc_same = e->desc_dev_for_key == e->desc.p && e->desc.p && e->desc_key.size() > 2 * (size_t)n_clips + 1 &&
                     e->desc_key[2 * n_clips] == loc;
    for (int c = 0; desc_same && c < n_clips; ++c)
        desc_same = e->desc_key[2 * c] == offsets[c] && e->desc_key[2 * c + 1] == clip_len(c);
    // h_desc is rewritten below: the previous descriptor upload must have left it
    if (e->desc_ev_live) {
        HIP_TRY(hipEventSynchronize(e->desc_ev));
        e->desc_ev_live = false;
    }
    e->clip_base.assign(n_clips, 0);
    e->clip_frames.assign(n_clips, 0);
    int64_t frames = 0, strips = 0, chunks = 0, recs = 0, staged = 0, kstrips = 0;
    bool empty_clip = false;  // a clip without frames gets no count from K3: zero the counts first
    // K3 (landmarks.hip): a clip of several chunks needs the COUNT pass for its chunk bases; when every clip is
    // exactly one chunk, a workgroup's clip is its chunk index. Neither follows from the totals alone: a clip
    // too short for a frame has no chunk, so [short, two-chunk] also has as many chunks as clips
    bool multi_chunk = false, one_chunk_each = n_clips > 0;
    for (int c = 0; c < n_clips; ++c) e->clip_frames[c] = num_frames(clip_len(c), hop);
    // K2 strips per resident workgroup slot. Strip-cold K2 waves exit (peaks.hip) and their
    // registers admit more workgroups per CU (LDS allows 7 instead of the 4 of an all-hot CU): with the
    // fraction c of cold waves counted in earlier calls (K3 stores it in pinned memory; read without a sync,
    // so it lags a few calls), the strips are made shorter and more numerous, 0.75 / (1 - c) per slot,
    // quantised to 1, 1.25, 1.5 (a stable key for the cached descriptors)
    double kx = e->k2_slots_x;
    if (kx <= 0.0) {
        kx = 1.0;
        const uint64_t cw = e->h_cold ? *reinterpret_cast<volatile uint64_t *>(e->h_cold) : 0;
        if (cw >> 32) {
            const double c = std::min(1.0, (double)(uint32_t)cw / (double)(cw >> 32));
            kx = c >= 0.45 ? 1.5 : c >= 0.3 ? 1.25 : 1.0;
        }
    }
    // clip groups: consecutive clips whose frames fit kPlaneRows power rows each run K1 -> K2 on one power buffer.
    // K1 and K2 run 5-14 % slower per audio-second on a 10.8 GB plane than on a 2.7 GB one
    // (profiles/r05zo_catalog_batch.txt); a call within the bound (the headline's 256 x 10 s, one catalog batch, a
    // stream push) is one group, as before. K3 runs once over the whole call's mask. AID_FLAG_KEEP_POWER keeps
    // every row for aid_result_power: one group.
    std::vector<int> gstart{0};
    {
        const bool keep_all = (e->cfg.flags & AID_FLAG_KEEP_POWER) != 0;
        const int64_t cap = e->plane_rows > 0 ? e->plane_rows : kPlaneRows;
        int64_t acc = 0;
        for (int c = 0; c < n_clips; ++c) {
            if (!keep_all && acc > 0 && acc + e->clip_frames[c] > cap) {
                gstart.push_back(c);
                acc = 0;
            }
            acc += e->clip_frames[c];
        }
        gstart.push_back(n_clips);
    }
    const int n_groups = (int)gstart.size() - 1;
    std::vector<int> glen(n_groups);
    std::vector<int64_t> gfirst(n_groups), gframes(n_groups, 0), gstrips(n_groups, 0), gk(n_groups, 0);
    for (int g = 0; g < n_groups; ++g)  // K2 strips per resident slot, per group (strip_base restarts at 0 in each)
        glen[g] = peak_strip_len(e->clip_frames.data() + gstart[g], gstart[g + 1] - gstart[g],
                                 std::max<int64_t>(1, (int64_t)(e->k2_slots * kx)));
    // strip bases follow the groups and their strip lengths: (first clip, strip length) per group in the key
    desc_same = desc_same && e->desc_key.size() == 2 * (size_t)n_clips + 1 + 2 * (size_t)n_groups;
    for (int g = 0; desc_same && g < n_groups; ++g)
        desc_same = e->desc_key[2 * n_clips + 1 + 2 * g] == gstart[g] && e->desc_key[2 * n_clips + 2 + 2 * g] == glen[g];
    for (int c = 0, g = 0; c < n_clips; ++c) {
        const int64_t n = clip_len(c);
        const int64_t F = num_frames(n, hop);
        ClipDesc &d = e->h_desc[c];
        while (c == gstart[g + 1]) ++g;
        if (c == gstart[g]) gfirst[g] = frames;
        if (loc == AID_PCM_DEVICE) {
            d.pcm_off = offsets[c];  // odd: K1's float2 frame loads are then 4-byte aligned (dword alignment suffices)
        } else {
            d.pcm_off = offsets[c] - offsets[0];  // the clips' span is staged as one copy
            staged = offsets[c] + n - offsets[0];
        }
        d.frames = F;
        d.frame_base = frames;
        d.strip_base = gstrips[g];  // within the clip's group (K2 runs per group)
        d.chunk_base = chunks;
        d.hash_base = recs;
        d.hash_cap = hash_capacity(F);
        d.stft_base = kstrips;
        e->clip_base[c] = recs;
        e->clip_frames[c] = F;
        empty_clip |= F == 0;
        const int64_t nck = (F + kHashChunk - 1) / kHashChunk;
        multi_chunk |= nck > 1;
        one_chunk_each &= nck == 1;
        frames += F;
        gframes[g] += F;
        gstrips[g] += (F + glen[g] - 1) / glen[g];
        strips += (F + glen[g] - 1) / glen[g];
        chunks += (F + kHashChunk - 1) / kHashChunk;
        recs += d.hash_cap;
        gk[g] += (F + kStftStrip - 1) / kStftStrip;
        kstrips += (F + kStftStrip - 1) / kStftStrip;
    }
    HIP_TRY(e->desc.reserve((size_t)n_clips + 1));
    HIP_TRY(e->power.reserve((size_t)std::max<int64_t>(1, *std::max_element(gframes.begin(), gframes.end())) * kBins));
    HIP_TRY(e->mask.reserve((size_t)frames * kMaskWords));
    HIP_TRY(e->hotw.reserve((size_t)frames + 1));
    if (!e->k2_cold.p) {
        HIP_TRY(e->k2_cold.reserve(64));
        HIP_TRY(hipMemsetAsync(e->k2_cold.p, 0, 64 * sizeof(uint32_t), s));
    }
    if (!e->h_cold) {
        HIP_TRY(hipHostMalloc((void **)&e->h_cold, sizeof(uint64_t), hipHostMallocMapped));
        *e->h_cold = 0;
        HIP_TRY(hipHostGetDevicePointer((void **)&e->h_cold_dev, e->h_cold, 0));
    }
    HIP_TRY(e->chunk_counts.reserve((size_t)chunks + 1));
    HIP_TRY(e->records.reserve((size_t)recs + 1));
    HIP_TRY(e->counts.reserve((size_t)n_clips + 1));
    const float *dpcm = pcm;
    if (loc == AID_PCM_HOST && staged > 0) {
        // K1 of an earlier call may still read the staging buffer: on the same stream the new copy is ordered after
        // it (a pipelined submit must not wait for the previous batch's K1), on another stream the host waits
        if (e->stage_ev_live && e->stage_stream != s) HIP_TRY(hipEventSynchronize(e->stage_ev));
        e->stage_ev_live = false;
        // one copy of the clips' whole span (clips at odd offsets are read with dword-aligned float2 loads; a copy
        // per clip cost ~10-20 us of call overhead each: 64 coalesced service queries ~1 ms)
        HIP_TRY(e->pcm_stage.reserve((size_t)staged));
        HIP_TRY(hipMemcpyAsync(e->pcm_stage.p, pcm + offsets[0], staged * sizeof(float), hipMemcpyHostToDevice, s));
        dpcm = e->pcm_stage.p;
    }
    if (n_clips > 0 && !desc_same) {
        if (!e->desc_ev) HIP_TRY(hipEventCreateWithFlags(&e->desc_ev, hipEventDisableTiming));
        HIP_TRY(hipMemcpyAsync(e->desc.p, e->h_desc, sizeof(ClipDesc) * n_clips, hipMemcpyHostToDevice, s));
        HIP_TRY(hipEventRecord(e->desc_ev, s));
        e->desc_ev_live = true;
        e->desc_key.resize(2 * (size_t)n_clips);
        for (int c = 0; c < n_clips; ++c) {
            e->desc_key[2 * c] = offsets[c];
            e->desc_key[2 * c + 1] = clip_len(c);
        }
        e->desc_key.push_back(loc);
        for (int g = 0; g < n_groups; ++g) {
            e->desc_key.push_back(gstart[g]);
            e->desc_key.push_back(glen[g]);
        }
        e->desc_dev_for_key = e->desc.p;
    }
    if (empty_clip || frames == 0) HIP_TRY(hipMemsetAsync(e->counts.p, 0, sizeof(int64_t) * ((size_t)n_clips + 1), s));
    e->n_clips = n_clips;
    e->total_frames = frames;
    e->total_strips = strips;
    e->total_chunks = chunks;
    e->total_records = recs;
    if (frames > 0) {
        for (int g = 0; g < n_groups; ++g) {  // K1 -> K2 per clip group, on one power buffer
            const int ca = gstart[g], ng = gstart[g + 1] - ca;
            if (gframes[g] == 0) continue;
            {
                ProfScope ps(e, AID_K_STFT, s, true);
                launch_stft_power(dpcm, e->desc.p + ca, ng, gfirst[g], gframes[g], gk[g], e->k1_slots, hop, e->d_tab,
                                  e->power.p, false, e->hotw.p, e->cfg.peak_threshold,
                                  (e->cfg.flags & AID_FLAG_KEEP_POWER) != 0, s);
            }
            if (loc == AID_PCM_HOST && g == n_groups - 1) {
                if (!e->stage_ev) HIP_TRY(hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming));
                HIP_TRY(hipEventRecord(e->stage_ev, s));
                e->stage_ev_live = true;
                e->stage_stream = s;
            }
            {
                ProfScope ps(e, AID_K_PEAKS, s, true);
                launch_peak_pick(e->power.p, e->desc.p + ca, ng, gfirst[g], gstrips[g], glen[g], e->cfg.peak_threshold,
                                 e->hotw.p, e->mask.p, e->k2_cold.p, s);
            }
        }
        if (multi_chunk) {  // some clip spans several K3 chunks: their bases need the COUNT pass
            ProfScope ps(e, AID_K_LANDMARK_COUNT, s, true);
            launch_landmarks(e->mask.p, e->desc.p, n_clips, chunks, e->chunk_counts.p, e->records.p, e->counts.p,
                             false, nullptr, nullptr, 0u, one_chunk_each, s);
        }
        {
            ProfScope ps(e, AID_K_LANDMARK_WRITE, s, true);
            launch_landmarks(e->mask.p, e->desc.p, n_clips, chunks, e->chunk_counts.p, e->records.p, e->counts.p,
                             true, e->h_cold_dev ? e->k2_cold.p : nullptr, e->h_cold_dev, (uint32_t)(4 * strips),
                             one_chunk_each, s);
        }
    }
    HIP_TRY(hipGetLastError());
    e->last_stream = s;
    e->have_result = true;
    return AID_OK;
}

int aid_sync(aid_engine *e) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->last_stream ? e->last_stream : e->own_stream));
    return AID_OK;
}

int aid_result_counts(aid_engine *e, int64_t *counts) {
    if (!e || (!counts && e->n_clips > 0)) return fail(AID_ERR_INVALID, "null argument");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction yet");
    if (int rc = aid_sync(e)) return rc;
    if (e->n_clips > 0) HIP_TRY(hipMemcpy(counts, e->counts.p, sizeof(int64_t) * e->n_clips, hipMemcpyDeviceToHost));
    return AID_OK;
}

int aid_result_hashes(aid_engine *e, int32_t clip, aid_hash *out, int64_t cap, int64_t *n_out) {
    if (!e || !n_out) return fail(AID_ERR_INVALID, "null argument");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction yet");
    if (clip < 0 || clip >= e->n_clips) return fail(AID_ERR_INVALID, "clip index out of range");
    if (int rc = aid_sync(e)) return rc;
    int64_t n = 0;
    HIP_TRY(hipMemcpy(&n, e->counts.p + clip, sizeof(int64_t), hipMemcpyDeviceToHost));
    *n_out = n;
    if (n > cap) return fail(AID_ERR_INVALID, "output capacity too small");
    if (n > 0) {
        if (!out) return fail(AID_ERR_INVALID, "null output");
        HIP_TRY(hipMemcpy(out, e->records.p + e->clip_base[clip], n * sizeof(aid_hash), hipMemcpyDeviceToHost));
    }
    return AID_OK;
}

int aid_result_device(aid_engine *e, const aid_hash **records, const int64_t **counts_dev,
                      const int64_t **clip_base_host, int32_t *n_clips) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction yet");
    if (records) *records = reinterpret_cast<const aid_hash *>(e->records.p);
    if (counts_dev) *counts_dev = e->counts.p;
    if (clip_base_host) *clip_base_host = e->clip_base.data();
    if (n_clips) *n_clips = e->n_clips;
    return AID_OK;
}

int aid_result_power(aid_engine *e, int32_t clip, float *out, int64_t cap) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction yet");
    if (clip < 0 || clip >= e->n_clips) return fail(AID_ERR_INVALID, "clip index out of range");
    if (!(e->cfg.flags & AID_FLAG_KEEP_POWER))
        return fail(AID_ERR_STATE, "aid_result_power: engine created without AID_FLAG_KEEP_POWER (cold blocks not stored)");
    const int64_t F = e->clip_frames[clip];
    if (F * kBins > cap) return fail(AID_ERR_INVALID, "output capacity too small");
    if (int rc = aid_sync(e)) return rc;
    if (F > 0) {
        int64_t fb = 0;
        for (int c = 0; c < clip; ++c) fb += e->clip_frames[c];
        HIP_TRY(hipMemcpy(out, e->power.p + fb * kBins, F * kBins * sizeof(float), hipMemcpyDeviceToHost));
        // K1 stores Q = fma(Xr, Xr, Xi*Xi) = 4P; FPSPEC 4's P is Q * 0.25f, the same binary32 op
        for (int64_t i = 0; i < F * kBins; ++i) out[i] = out[i] * 0.25f;
    }
    return AID_OK;
}

int aid_result_peakmask(aid_engine *e, int32_t clip, uint64_t *out, int64_t cap) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction yet");
    if (clip < 0 || clip >= e->n_clips) return fail(AID_ERR_INVALID, "clip index out of range");
    const int64_t F = e->clip_frames[clip];
    if (F * kMaskWords > cap) return fail(AID_ERR_INVALID, "output capacity too small");
    if (int rc = aid_sync(e)) return rc;
    if (F > 0) {
        int64_t fb = 0;
        for (int c = 0; c < clip; ++c) fb += e->clip_frames[c];
        HIP_TRY(hipMemcpy(out, e->mask.p + fb * kMaskWords, F * kMaskWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    return AID_OK;
}

int aid_spectrogram(aid_engine *e, const float *pcm, int64_t n, float *out, int64_t cap) {
    if (!e || (n > 0 && !pcm) || n < 0) return fail(AID_ERR_INVALID, "aid_spectrogram: bad argument");
    const int64_t F = num_frames(n, e->cfg.hop);
    if (F * kBins > cap) return fail(AID_ERR_INVALID, "output capacity too small");
    if (F == 0) return AID_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    float *d_pcm = nullptr, *d_out = nullptr;
    ClipDesc *d_desc = nullptr;
    ClipDesc d{};
    d.frames = F;
    HIP_TRY(hipMalloc(&d_pcm, n * sizeof(float)));
    hipError_t he = hipMalloc(&d_out, F * kBins * sizeof(float));
    if (he == hipSuccess) he = hipMalloc(&d_desc, sizeof(ClipDesc));
    if (he == hipSuccess) he = hipMemcpy(d_pcm, pcm, n * sizeof(float), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(d_desc, &d, sizeof(ClipDesc), hipMemcpyHostToDevice);
    if (he == hipSuccess) {
        launch_stft_power(d_pcm, d_desc, 1, 0, F, (F + kStftStrip - 1) / kStftStrip, e->k1_slots, e->cfg.hop, e->d_tab,
                          d_out, true, nullptr, e->cfg.peak_threshold, true, s);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he == hipSuccess) he = hipMemcpy(out, d_out, F * kBins * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d_pcm);
    (void)hipFree(d_out);
    (void)hipFree(d_desc);
    if (he != hipSuccess) return fail(AID_ERR_DEVICE, std::string("aid_spectrogram: ") + hipGetErrorString(he));
    return AID_OK;
}

int aid_synth_rate(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips,
                   int64_t n, int32_t sample_rate, int32_t noise_a, uint32_t salt, int32_t fmax_hz, int32_t flags,
                   void *stream) {
    if (!e || !dst || !tracks || !starts || n_clips < 0 || n < 0 || noise_a < 0 || sample_rate <= 0)
        return fail(AID_ERR_INVALID, "aid_synth: bad argument");
    if (flags & ~(AID_SYNTH_STATIONARY | AID_SYNTH_ASYNC)) return fail(AID_ERR_INVALID, "aid_synth: unknown flags");
    if (sample_rate > 384000) return fail(AID_ERR_INVALID, "aid_synth: sample_rate above 384 kHz");
    if (fmax_hz <= 100 || 2 * (int64_t)fmax_hz > sample_rate)
        return fail(AID_ERR_INVALID, "aid_synth: fmax_hz must be in (100, sample_rate / 2]");
    if (n_clips == 0 || n == 0) return AID_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    const bool async = (flags & AID_SYNTH_ASYNC) != 0;
    // the engine's last work on another stream may still read dst; on the same stream it is ordered already
    if (e->last_stream && (!async || e->last_stream != s)) HIP_TRY(hipStreamSynchronize(e->last_stream));
    // the previous call's copies and kernel must have left the pinned staging and the device arrays before a
    // reserve may reallocate them or the copies below overwrite them
    if (e->synth_ev_live) {
        HIP_TRY(hipEventSynchronize(e->synth_ev));
        e->synth_ev_live = false;
    }
    HIP_TRY(e->synth_tracks.reserve(n_clips));
    HIP_TRY(e->synth_starts.reserve(n_clips));
    // tracks + starts go up from pinned staging (the caller's arrays may be gone when an async copy runs)
    const size_t tb = ((size_t)n_clips * sizeof(uint32_t) + 7) & ~(size_t)7, need = tb + (size_t)n_clips * sizeof(int64_t);
    if (need > e->h_synth_cap) {
        if (e->h_synth) HIP_TRY(hipHostFree(e->h_synth));
        e->h_synth = nullptr;
        e->h_synth_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&e->h_synth, need));
        e->h_synth_cap = need;
    }
    std::memcpy(e->h_synth, tracks, (size_t)n_clips * sizeof(uint32_t));
    std::memcpy(e->h_synth + tb, starts, (size_t)n_clips * sizeof(int64_t));
    HIP_TRY(hipMemcpyAsync(e->synth_tracks.p, e->h_synth, n_clips * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->synth_starts.p, e->h_synth + tb, n_clips * sizeof(int64_t), hipMemcpyHostToDevice, s));
    {
        ProfScope ps(e, AID_K_SYNTH, s);
        launch_synth(dst, e->synth_tracks.p, e->synth_starts.p, n_clips, n, sample_rate, noise_a, salt, fmax_hz,
                     !(flags & AID_SYNTH_STATIONARY), e->d_sin, s);
    }
    HIP_TRY(hipGetLastError());
    // the event covers the kernel's reads of synth_tracks / synth_starts as well as the copies into them, so the
    // next call (any stream) waits for both before it reuses the pinned staging or the device arrays; last_stream
    // makes every later call on another stream wait for this one too
    if (!e->synth_ev) HIP_TRY(hipEventCreateWithFlags(&e->synth_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(e->synth_ev, s));
    e->synth_ev_live = true;
    e->last_stream = s;
    if (!async) HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_synth_band(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips,
                   int64_t n, int32_t noise_a, uint32_t salt, int32_t fmax_hz, void *stream) {
    if (!e) return fail(AID_ERR_INVALID, "aid_synth: null engine");
    return aid_synth_rate(e, dst, tracks, starts, n_clips, n, e->cfg.sample_rate, noise_a, salt, fmax_hz, 0, stream);
}

int aid_synth(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips, int64_t n,
              int32_t noise_a, uint32_t salt, void *stream) {
    return aid_synth_band(e, dst, tracks, starts, n_clips, n, noise_a, salt, 8000, stream);
}

int aid_resample_plan(int32_t sr_in, int32_t sr_out, int32_t *up, int32_t *down, int32_t *hl, int32_t *J) {
    ResamplePlan p;
    if (!resample_plan(sr_in, sr_out, p)) return 0;
    if (up) *up = p.up;
    if (down) *down = p.down;
    if (hl) *hl = p.hl;
    if (J) *J = p.J;
    return 1;
}

int64_t aid_resample_len(int64_t n, int32_t sr_in, int32_t sr_out) {
    ResamplePlan p;
    if (n <= 0 || !resample_plan(sr_in, sr_out, p)) return 0;
    return (n * p.up + p.down - 1) / p.down;
}

static int resample_taps_dev(aid_engine *e, const ResamplePlan &p, float **out) {
    auto it = e->rs_taps.find({p.up, p.down});
    if (it != e->rs_taps.end()) {
        *out = it->second;
        return AID_OK;
    }
    const std::vector<float> h = resample_phase_taps(p);
    float *taps = nullptr;
    HIP_TRY(hipMalloc(&taps, h.size() * sizeof(float)));
    hipError_t he = hipMemcpy(taps, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
    if (he != hipSuccess) {
        (void)hipFree(taps);
        return fail(AID_ERR_DEVICE, std::string("aid_resample: ") + hipGetErrorString(he));
    }
    e->rs_taps[{p.up, p.down}] = taps;
    *out = taps;
    return AID_OK;
}

int aid_resample_range(aid_engine *e, const float *src, int64_t in_base, int64_t n, int32_t channels, int32_t sr_in,
                       int32_t sr_out, int64_t m_first, int64_t count, float *dst, void *stream) {
    return aid_resample_batch(e, src, 0, 1, in_base, n, channels, sr_in, sr_out, m_first, count, dst, 0, stream);
}

static int resample_batch(aid_engine *e, const float *src, int64_t src_stride, int32_t n_streams, int64_t in_base,
                          int64_t n, int32_t channels, int32_t sr_in, int32_t sr_out, int64_t m_first, int64_t count,
                          float *dst, int64_t dst_stride, void *stream, const float *hist, int64_t hist_n,
                          int64_t hist_stride) {
    if (!e || n < 0 || in_base < 0 || m_first < 0 || count < 0 || (channels != 1 && channels != 2) || n_streams < 0 ||
        n_streams > 65535 || src_stride < 0 || dst_stride < 0 || hist_n < 0 || hist_n > in_base || hist_stride < 0)
        return fail(AID_ERR_INVALID, "aid_resample: bad argument");
    if (n_streams > 1 && (src_stride < n * channels || dst_stride < count || (channels == 2 && (src_stride & 1))))
        return fail(AID_ERR_INVALID, "aid_resample_batch: strides must cover one stream (stereo: even)");
    if (hist_n > 0 && (!hist || (n_streams > 1 && hist_stride < hist_n * channels) ||
                       (channels == 2 && ((hist_stride & 1) || (reinterpret_cast<uintptr_t>(hist) & 7)))))
        return fail(AID_ERR_INVALID, "aid_resample_batch_split: bad history (null, stride, or stereo alignment)");
    if (n_streams == 0) return AID_OK;
    ResamplePlan p;
    if (!resample_plan(sr_in, sr_out, p)) return fail(AID_ERR_INVALID, "aid_resample: sample rates must be > 0");
    if (count == 0) return AID_OK;
    if (!dst || (n > 0 && !src)) return fail(AID_ERR_INVALID, "aid_resample: null buffer");
    if (channels == 2 && (reinterpret_cast<uintptr_t>(src) & 7))
        return fail(AID_ERR_INVALID, "aid_resample: stereo src must be 8-byte aligned");
    if (resample_lds_floats(p.up, p.down, p.J) * 4 > 65536)
        return fail(AID_ERR_INVALID, "aid_resample: down/up ratio too large (LDS window > 64 KB)");
    if ((int64_t)p.up * p.J > (1 << 24)) return fail(AID_ERR_INVALID, "aid_resample: tap table too large");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    float *taps = nullptr;
    if (int rc = resample_taps_dev(e, p, &taps)) return rc;
    {
        ProfScope ps(e, AID_K_RESAMPLE, s);
        launch_resample(src, in_base, n, channels, p.up, p.down, p.hl, p.J, taps, dst, m_first, count, s, n_streams,
                        src_stride, dst_stride, hist, hist_n, hist_stride);
    }
    HIP_TRY(hipGetLastError());
    return AID_OK;
}

int aid_resample_batch(aid_engine *e, const float *src, int64_t src_stride, int32_t n_streams, int64_t in_base, int64_t n,
                       int32_t channels, int32_t sr_in, int32_t sr_out, int64_t m_first, int64_t count, float *dst,
                       int64_t dst_stride, void *stream) {
    return resample_batch(e, src, src_stride, n_streams, in_base, n, channels, sr_in, sr_out, m_first, count, dst,
                          dst_stride, stream, nullptr, 0, 0);
}

int aid_resample_batch_split(aid_engine *e, const float *hist, int64_t hist_stride, int64_t hist_n, const float *src,
                             int64_t src_stride, int32_t n_streams, int64_t in_base, int64_t n, int32_t channels,
                             int32_t sr_in, int32_t sr_out, int64_t m_first, int64_t count, float *dst,
                             int64_t dst_stride, void *stream) {
    return resample_batch(e, src, src_stride, n_streams, in_base, n, channels, sr_in, sr_out, m_first, count, dst,
                          dst_stride, stream, hist, hist_n, hist_stride);
}

int aid_resample(aid_engine *e, const float *src, int64_t n, int32_t channels, int32_t sr_in, int32_t sr_out,
                 float *dst, int64_t cap, int64_t *n_out, void *stream) {
    if (!e || n < 0 || (channels != 1 && channels != 2)) return fail(AID_ERR_INVALID, "aid_resample: bad argument");
    const int64_t m = aid_resample_len(n, sr_in, sr_out);
    if (n > 0 && m == 0) return fail(AID_ERR_INVALID, "aid_resample: sample rates must be > 0");
    if (n_out) *n_out = m;
    if (m > cap) return fail(AID_ERR_INVALID, "aid_resample: output capacity too small");
    if (m == 0) return AID_OK;
    if (sr_in == sr_out && channels == 1) {  // same rate, mono: a copy
        if (!src || !dst) return fail(AID_ERR_INVALID, "aid_resample: null buffer");
        std::lock_guard<std::mutex> lk(e->mu);
        HIP_TRY(hipSetDevice(e->device));
        HIP_TRY(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, pick_stream(e, stream)));
        return AID_OK;
    }
    return aid_resample_range(e, src, 0, n, channels, sr_in, sr_out, 0, m, dst, stream);
}

}  // extern "C"

// grow a device buffer to hold `want` elements, keeping the first `keep` (stream-ordered copy)
template <typename T>
static int grow_keep(DevBuf<T> &b, size_t keep, size_t want, hipStream_t s) {
    if (want <= b.n) return AID_OK;
    size_t cap = std::max(want, b.n * 2);
    T *p = nullptr;
    HIP_TRY(hipMalloc(&p, cap * sizeof(T)));
    keep = b.p ? std::min(keep, b.n) : 0;  // nothing stored yet on the first growth
    if (keep) HIP_TRY(hipMemcpyAsync(p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (b.p) (void)hipFree(b.p);
    b.p = p;
    b.n = cap;
    return AID_OK;
}

extern "C" {

int aid_dedup_reset(aid_engine *e) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    e->dd_n = 0;
    e->dd_nw = 0;
    return AID_OK;
}

int aid_dedup_count(aid_engine *e, int64_t *n_entries, int64_t *n_words) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (n_entries) *n_entries = e->dd_n;
    if (n_words) *n_words = e->dd_nw;
    return AID_OK;
}

static int check_offsets(const int64_t *off, int32_t n, const char *what) {
    if (off[0] != 0) return fail(AID_ERR_INVALID, std::string(what) + ": offsets[0] must be 0");
    for (int32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return fail(AID_ERR_INVALID, std::string(what) + ": offsets must be non-decreasing");
    return AID_OK;
}

int aid_dedup_add(aid_engine *e, const uint32_t *words, const int64_t *offsets, const double *durations, int32_t n) {
    if (!e || n < 0 || (n > 0 && (!offsets || !durations))) return fail(AID_ERR_INVALID, "aid_dedup_add: bad argument");
    if (n == 0) return AID_OK;
    if (int rc = check_offsets(offsets, n, "aid_dedup_add")) return rc;
    const int64_t nw = offsets[n];
    if (nw > 0 && !words) return fail(AID_ERR_INVALID, "aid_dedup_add: null words");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    if (int rc = grow_keep(e->dd_words, (size_t)e->dd_nw, (size_t)(e->dd_nw + nw + 1), s)) return rc;
    if (int rc = grow_keep(e->dd_off, (size_t)e->dd_n + 1, (size_t)(e->dd_n + n + 1), s)) return rc;
    if (int rc = grow_keep(e->dd_dur, (size_t)e->dd_n, (size_t)(e->dd_n + n), s)) return rc;
    std::vector<int64_t> off(n + 1);
    for (int32_t i = 0; i <= n; ++i) off[i] = e->dd_nw + offsets[i];
    if (nw > 0) HIP_TRY(hipMemcpyAsync(e->dd_words.p + e->dd_nw, words, nw * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dd_off.p + e->dd_n, off.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dd_dur.p + e->dd_n, durations, n * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->dd_n += n;
    e->dd_nw += nw;
    return AID_OK;
}

int aid_dedup_scan(aid_engine *e, const uint32_t *words, const int64_t *offsets, const double *durations, int32_t nq,
                   int64_t *best_idx, double *best_sim) {
    if (!e || nq < 0 || (nq > 0 && (!offsets || !durations || !best_idx || !best_sim)))
        return fail(AID_ERR_INVALID, "aid_dedup_scan: bad argument");
    if (nq == 0) return AID_OK;
    if (int rc = check_offsets(offsets, nq, "aid_dedup_scan")) return rc;
    const int64_t nw = offsets[nq];
    if (nw > 0 && !words) return fail(AID_ERR_INVALID, "aid_dedup_scan: null words");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    const int nc = std::max(1, dedup_chunks(e->dd_n));
    std::vector<double> lo(nq), hi(nq);
    for (int32_t q = 0; q < nq; ++q) {  // the reference's SQL bounds (dedup.py:193-194)
        lo[q] = durations[q] * 0.9;
        hi[q] = durations[q] * 1.1;
    }
    HIP_TRY(e->dq_words.reserve((size_t)nw + 1));
    HIP_TRY(e->dq_off.reserve((size_t)nq + 1));
    HIP_TRY(e->dq_lo.reserve((size_t)nq));
    HIP_TRY(e->dq_hi.reserve((size_t)nq));
    HIP_TRY(e->dq_sim.reserve((size_t)nq));
    HIP_TRY(e->dq_idx.reserve((size_t)nq));
    HIP_TRY(e->dq_psim.reserve((size_t)nq * nc));
    HIP_TRY(e->dq_pidx.reserve((size_t)nq * nc));
    if (nw > 0) HIP_TRY(hipMemcpyAsync(e->dq_words.p, words, nw * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dq_off.p, offsets, (nq + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dq_lo.p, lo.data(), nq * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dq_hi.p, hi.data(), nq * sizeof(double), hipMemcpyHostToDevice, s));
    {
        ProfScope ps(e, AID_K_DEDUP, s);
        launch_dedup_scan(e->dd_words.p, e->dd_off.p, e->dd_dur.p, e->dd_n, e->dq_words.p, e->dq_off.p, e->dq_lo.p,
                          e->dq_hi.p, nq, e->dq_psim.p, e->dq_pidx.p, e->dq_sim.p, e->dq_idx.p, s);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(best_idx, e->dq_idx.p, nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(best_sim, e->dq_sim.p, nq * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_dedup_pairs(aid_engine *e, const uint32_t *a, const int64_t *a_off, const uint32_t *b, const int64_t *b_off,
                    int32_t n, double *sim) {
    if (!e || n < 0 || (n > 0 && (!a_off || !b_off || !sim))) return fail(AID_ERR_INVALID, "aid_dedup_pairs: bad argument");
    if (n == 0) return AID_OK;
    if (int rc = check_offsets(a_off, n, "aid_dedup_pairs")) return rc;
    if (int rc = check_offsets(b_off, n, "aid_dedup_pairs")) return rc;
    const int64_t na = a_off[n], nb = b_off[n];
    if ((na > 0 && !a) || (nb > 0 && !b)) return fail(AID_ERR_INVALID, "aid_dedup_pairs: null words");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    HIP_TRY(e->dq_words.reserve((size_t)na + 1));
    HIP_TRY(e->dq_words2.reserve((size_t)nb + 1));
    HIP_TRY(e->dq_off.reserve((size_t)n + 1));
    HIP_TRY(e->dq_off2.reserve((size_t)n + 1));
    HIP_TRY(e->dq_sim.reserve((size_t)n));
    if (na > 0) HIP_TRY(hipMemcpyAsync(e->dq_words.p, a, na * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    if (nb > 0) HIP_TRY(hipMemcpyAsync(e->dq_words2.p, b, nb * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dq_off.p, a_off, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->dq_off2.p, b_off, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    launch_dedup_pairs(e->dq_words.p, e->dq_off.p, e->dq_words2.p, e->dq_off2.p, n, e->dq_sim.p, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(sim, e->dq_sim.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_profile_enable(aid_engine *e, int32_t on) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    e->profiling = on != 0;
    return AID_OK;
}

int aid_profile_select(aid_engine *e, uint32_t kernel_mask) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    e->prof_mask = kernel_mask;
    return AID_OK;
}

int aid_profile_read(aid_engine *e, double *ms, int64_t *launches, int32_t reset) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    for (auto &p : e->pending) {
        HIP_TRY(hipEventSynchronize(p.b));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, p.a, p.b));
        e->prof_ms[p.kernel] += t;
        e->prof_n[p.kernel] += 1;
        e->pool.push_back(p.a);
        e->pool.push_back(p.b);
    }
    e->pending.clear();
    for (int k = 0; k < AID_K_COUNT; ++k) {
        if (ms) ms[k] = e->prof_ms[k];
        if (launches) launches[k] = e->prof_n[k];
    }
    if (reset)
        for (int k = 0; k < AID_K_COUNT; ++k) {
            e->prof_ms[k] = 0;
            e->prof_n[k] = 0;
        }
    return AID_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- index + query

static int grow_copy_u32(DevBuf<uint32_t> &b, size_t keep, size_t want, hipStream_t s) {
    if (want <= b.n) return AID_OK;
    size_t cap = std::max(want, b.n * 2);
    uint32_t *p = nullptr;
    HIP_TRY(hipMalloc(&p, cap * sizeof(uint32_t)));
    if (keep) HIP_TRY(hipMemcpyAsync(p, b.p, keep * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (b.p) (void)hipFree(b.p);
    b.p = p;
    b.n = cap;
    return AID_OK;
}

static int reserve_postings(aid_engine *e, int64_t extra, hipStream_t s) {
    const size_t want = (size_t)(e->n_post + extra);
    if (int rc = grow_copy_u32(e->p_hash, e->n_post, want, s)) return rc;
    if (int rc = grow_copy_u32(e->p_track, e->n_post, want, s)) return rc;
    if (int rc = grow_copy_u32(e->p_t, e->n_post, want, s)) return rc;
    return AID_OK;
}

// wait for the engine's own streams (not the whole device: torch streams, other engines and ranks on the
// same GPU keep running) before a buffer that in-flight engine work may read is freed
static void sync_engine_streams(aid_engine *e, hipStream_t s) {
    if (e->last_stream && e->last_stream != s) (void)hipStreamSynchronize(e->last_stream);
    if (e->own_stream && e->own_stream != s) (void)hipStreamSynchronize(e->own_stream);
    (void)hipStreamSynchronize(s);
}

// capacity of the track tables for max_track_plus1 ids, without changing the index: the new tombstone
// buffer is allocated (and filled) before the old one goes, so a failed growth leaves the engine as it was
static int reserve_tracks(aid_engine *e, uint32_t max_track_plus1, hipStream_t s) {
    const size_t want = std::max<size_t>(max_track_plus1, 1024);
    if (want <= e->tomb.n) return AID_OK;
    DevBuf<uint8_t> nb;
    HIP_TRY(nb.reserve(std::max(want, 2 * e->tomb.n)));
    if (e->tomb.p) sync_engine_streams(e, s);  // in-flight queries may still read the old tombstones
    if (e->n_tracks) {
        // synchronous: the engine's tombstones must be whole in the new buffer before it replaces the old one
        hipError_t he = hipMemcpyAsync(nb.p, e->h_tomb.data(), e->n_tracks, hipMemcpyHostToDevice, s);
        if (he == hipSuccess) he = hipStreamSynchronize(s);
        if (he != hipSuccess) {
            nb.release();
            return fail(AID_ERR_DEVICE, std::string("reserve_tracks: ") + hipGetErrorString(he));
        }
    }
    std::swap(e->tomb, nb);
    nb.release();
    return AID_OK;
}

// grow the track tables to max_track_plus1 ids (reserve first: nothing changes if that fails)
static int ensure_tracks(aid_engine *e, uint32_t max_track_plus1, hipStream_t s) {
    if (max_track_plus1 <= e->n_tracks) return AID_OK;
    if (int rc = reserve_tracks(e, max_track_plus1, s)) return rc;
    e->h_tomb.resize(max_track_plus1, 0);
    e->n_tracks = max_track_plus1;
    HIP_TRY(hipMemcpyAsync(e->tomb.p, e->h_tomb.data(), e->n_tracks, hipMemcpyHostToDevice, s));
    return AID_OK;
}

// the posting count of the last aid_index_add_extracted, if still in flight, made exact (the append's own
// kernels are ordered before the event; a reader of n_post or of the planes calls this first)
static int settle_postings(aid_engine *e) {
    if (!e->add_live) return AID_OK;
    HIP_TRY(hipEventSynchronize(e->add_ev));
    e->add_live = false;
    if (e->post_pend) e->n_post = *e->h_npost;
    e->post_pend = false;
    return AID_OK;
}

extern "C" {

int aid_index_reset(aid_engine *e) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    e->n_post = 0;
    e->n_tracks = 0;
    e->h_tomb.clear();
    e->index_built = false;
    e->index_dirty = true;
    e->n_indexed = 0;
    return AID_OK;
}

int aid_index_add_extracted(aid_engine *e, const uint32_t *track_ids) {
    if (!e || (!track_ids && e->n_clips > 0)) return fail(AID_ERR_INVALID, "aid_index_add_extracted: bad argument");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction to index");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->last_stream ? e->last_stream : e->own_stream;
    const int n = e->n_clips;
    if (n == 0) return AID_OK;
    // the previous call's count (normally long arrived: this batch's extraction was queued behind it) and its
    // pinned staging, whose H2D copies precede that call's event
    if (int rc = settle_postings(e)) return rc;
    // pinned staging [counts n][src n][dst n][tracks n/2+1] (int64 slots)
    const size_t need = 3 * (size_t)n + (size_t)n / 2 + 1;
    if (need > e->h_stage_cap) {
        if (e->h_stage) HIP_TRY(hipHostFree(e->h_stage));
        e->h_stage = nullptr;
        e->h_stage_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&e->h_stage, need * sizeof(int64_t)));
        e->h_stage_cap = need;
    }
    int64_t *counts = e->h_stage, *src = counts + n, *dst = src + n;
    uint32_t *trk = reinterpret_cast<uint32_t *>(dst + n);
    uint32_t mx = 0;
    for (int c = 0; c < n; ++c) {
        src[c] = e->clip_base[c];
        trk[c] = track_ids[c];
        mx = std::max(mx, track_ids[c] + 1);
    }
    if (int rc = ensure_tracks(e, mx, s)) return rc;
    HIP_TRY(e->x_src.reserve(n));
    HIP_TRY(e->x_dst.reserve(n));
    HIP_TRY(e->x_tracks.reserve(n));
    // the batch's postings are at most its hash capacity: when the planes hold that much more, the append is
    // scanned on the device and nothing waits for it; otherwise the counts come back first and the planes grow
    // to the exact need plus one batch's hash capacity (1.5x the records buffer the extraction already holds),
    // so the following appends of such batches are asynchronous again (growth doubles: this path runs
    // O(log n) times), unless that headroom would take more than a quarter of the free device memory
    const int64_t bound = e->total_records;
    const int64_t cap = (int64_t)std::min({e->p_hash.n, e->p_track.n, e->p_t.n});
    if (!e->add_ev) HIP_TRY(hipEventCreateWithFlags(&e->add_ev, hipEventDisableTiming));
    if (e->n_post + bound <= cap) {
        if (!e->h_npost) HIP_TRY(hipHostMalloc((void **)&e->h_npost, sizeof(int64_t)));
        HIP_TRY(e->d_npost.reserve(1));
        HIP_TRY(hipMemcpyAsync(e->x_src.p, src, n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(e->x_tracks.p, trk, n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        launch_append_offsets(e->counts.p, n, e->n_post, e->x_dst.p, e->d_npost.p, s);
        launch_records_to_postings(e->records.p, e->x_src.p, e->counts.p, e->x_dst.p, e->x_tracks.p, n, e->p_hash.p,
                                   e->p_track.p, e->p_t.p, s);
        HIP_TRY(hipMemcpyAsync(e->h_npost, e->d_npost.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(e->add_ev, s));
        HIP_TRY(hipGetLastError());
        e->add_live = e->post_pend = true;
    } else {
        HIP_TRY(hipMemcpyAsync(counts, e->counts.p, n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        int64_t tot = 0;
        for (int c = 0; c < n; ++c) {
            dst[c] = e->n_post + tot;
            tot += counts[c];
        }
        size_t free_b = 0, total_b = 0;
        HIP_TRY(hipMemGetInfo(&free_b, &total_b));
        const bool room = (size_t)bound * 3 * sizeof(uint32_t) <= free_b / 4;
        if (int rc = reserve_postings(e, tot + (room ? bound : 0), s)) return rc;
        HIP_TRY(hipMemcpyAsync(e->x_src.p, src, n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(e->x_dst.p, dst, n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(e->x_tracks.p, trk, n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        launch_records_to_postings(e->records.p, e->x_src.p, e->counts.p, e->x_dst.p, e->x_tracks.p, n, e->p_hash.p,
                                   e->p_track.p, e->p_t.p, s);
        HIP_TRY(hipEventRecord(e->add_ev, s));  // the staging's copies (the next call waits for them)
        HIP_TRY(hipGetLastError());  // no sync: every reader of the posting planes syncs last_stream first
        e->add_live = true;
        e->n_post += tot;
    }
    e->index_dirty = true;
    return AID_OK;
}

int aid_index_add_postings(aid_engine *e, const uint32_t *hash, const uint32_t *track, const uint32_t *t, int64_t n,
                           int32_t location) {
    if (!e || n < 0 || (n > 0 && (!hash || !track || !t))) return fail(AID_ERR_INVALID, "aid_index_add_postings: bad argument");
    if (location != AID_PCM_HOST && location != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "bad location");
    if (n == 0) return AID_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (int rc = settle_postings(e)) return rc;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    uint32_t mx = 0;
    if (location == AID_PCM_HOST) {
        for (int64_t i = 0; i < n; ++i) mx = std::max(mx, track[i] + 1);
    } else {
        // device track ids: one max-reduction via a host copy of the track column
        std::vector<uint32_t> tr(n);
        HIP_TRY(hipMemcpy(tr.data(), track, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n; ++i) mx = std::max(mx, tr[i] + 1);
    }
    if (int rc = reserve_postings(e, n, s)) return rc;
    if (int rc = ensure_tracks(e, mx, s)) return rc;
    const hipMemcpyKind k = location == AID_PCM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(e->p_hash.p + e->n_post, hash, n * sizeof(uint32_t), k, s));
    HIP_TRY(hipMemcpyAsync(e->p_track.p + e->n_post, track, n * sizeof(uint32_t), k, s));
    HIP_TRY(hipMemcpyAsync(e->p_t.p + e->n_post, t, n * sizeof(uint32_t), k, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->n_post += n;
    e->index_dirty = true;
    return AID_OK;
}

int aid_index_add_track(aid_engine *e, uint32_t track) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (track == 0xFFFFFFFFu) return fail(AID_ERR_INVALID, "aid_index_add_track: bad track id");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    if (int rc = ensure_tracks(e, track + 1, s)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_index_remove(aid_engine *e, uint32_t track) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (track >= e->n_tracks || e->h_tomb[track]) return fail(AID_ERR_INVALID, "track not indexed");
    HIP_TRY(hipSetDevice(e->device));
    e->h_tomb[track] = 1;
    ++e->tomb_since_build;  // the CSR still holds its postings until the next finalize
    HIP_TRY(hipMemcpy(e->tomb.p + track, &e->h_tomb[track], 1, hipMemcpyHostToDevice));
    return AID_OK;
}

int aid_index_compact(aid_engine *e, int64_t *n_removed) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    if (n_removed) *n_removed = 0;
    bool any = false;
    for (uint8_t t : e->h_tomb) any = any || t;
    if (!any || e->n_post == 0) return AID_OK;
    if (e->n_post > 0xFFFFFFFFll) return fail(AID_ERR_INVALID, "index holds more than 2^32 postings");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    const int64_t nb = (e->n_post + 1023) / 1024;
    DevBuf<uint32_t> cnt, off, tmp, nh, ntr, nt;
    struct Release {  // every scratch buffer goes on every return path
        DevBuf<uint32_t> *b[6];
        ~Release() {
            for (auto *x : b) x->release();
        }
    } release_all{{&cnt, &off, &tmp, &nh, &ntr, &nt}};
    HIP_TRY(cnt.reserve((size_t)nb));
    HIP_TRY(off.reserve((size_t)nb));
    HIP_TRY(tmp.reserve(4 * ((size_t)nb / 1024 + 2) + 4096));
    HIP_TRY(nh.reserve((size_t)e->n_post));
    HIP_TRY(ntr.reserve((size_t)e->n_post));
    HIP_TRY(nt.reserve((size_t)e->n_post));
    launch_compact(e->p_hash.p, e->p_track.p, e->p_t.p, e->n_post, e->tomb.p, e->n_tracks, cnt.p, off.p, tmp.p, nh.p,
                   ntr.p, nt.p, s);
    HIP_TRY(hipGetLastError());
    uint32_t last_off = 0, last_cnt = 0;
    HIP_TRY(hipMemcpyAsync(&last_off, off.p + (nb - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&last_cnt, cnt.p + (nb - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int64_t live = (int64_t)last_off + last_cnt;
    if (n_removed) *n_removed = e->n_post - live;
    std::swap(e->p_hash, nh);
    std::swap(e->p_track, ntr);
    std::swap(e->p_t, nt);  // the old planes are released with the scratch buffers
    e->n_post = live;  // tombstones stay: removed ids are never reused, and the CSR skips nothing new
    e->index_dirty = true;
    return AID_OK;
}

static int finalize_locked(aid_engine *e) {
    HIP_TRY(hipSetDevice(e->device));
    if (int rc = settle_postings(e)) return rc;
    hipStream_t s = e->own_stream;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    if (e->n_post > 0xFFFFFFFFll) return fail(AID_ERR_INVALID, "index holds more than 2^32 postings");
    const size_t K = (size_t)index_keys() + 1;
    HIP_TRY(e->idx_cnt.reserve(K));
    HIP_TRY(e->idx_off.reserve(K));
    HIP_TRY(e->scan_tmp.reserve(4 * (K / 1024 + 2) + 4096));
    HIP_TRY(e->idx_post.reserve((size_t)std::max<int64_t>(e->n_post, 1)));
    // + 8: K5's LDS path reads the signatures in aligned chunks of 4 or 8; a record's last chunk may reach past the end
    HIP_TRY(e->idx_sig.reserve((size_t)std::max<int64_t>(e->n_post, 1) + 8));
    if (e->n_tracks == 0) HIP_TRY(e->tomb.reserve(1024));
    HIP_TRY(hipMemsetAsync(e->idx_cnt.p, 0, K * sizeof(uint32_t), s));
    HIP_TRY(e->nz.reserve(1));
    HIP_TRY(hipMemsetAsync(e->nz.p, 0, sizeof(unsigned long long), s));
    if (e->k4_mode >= 1 && e->n_post > 0) {
        // sort build (index_sort.hip): stable radix sort of (key27, track | t << 32) -> run ends -> max-scan
        const size_t np = (size_t)e->n_post;
        const bool rocprim_ab = e->k4_mode == 1;
        size_t tb = 0;
        if (rocprim_ab) {
            tb = index_sort_temp_bytes(e->n_post);
            if (tb == 0) return fail(AID_ERR_DEVICE, "radix sort: temporary storage query failed");
            HIP_TRY(e->srt_tmp.reserve(tb));
        }
        HIP_TRY(e->srt_scratch.reserve(radix_scratch_u32(e->n_post)));
        HIP_TRY(e->srt_k0.reserve(np));
        HIP_TRY(e->srt_k1.reserve(np));
        HIP_TRY(e->srt_v.reserve(np));
        uint64_t *sorted = nullptr;
        {
            ProfScope ps(e, AID_K_INDEX_BUILD, s);
            bool any_removed = false;
            for (uint8_t t : e->h_tomb) any_removed = any_removed || t;
            HIP_TRY(launch_index_sort_build(e->p_hash.p, e->p_track.p, e->p_t.p, e->n_post,
                                            any_removed ? e->tomb.p : nullptr, e->n_tracks,
                                            e->srt_k0.p, e->srt_k1.p, e->srt_v.p, e->idx_post.p, e->srt_tmp.p, tb,
                                            rocprim_ab, e->srt_scratch.p, e->idx_cnt.p, e->idx_off.p, e->nz.p, &sorted,
                                            e->idx_sig.p, e->k4_rank, s));
            if (sorted == e->srt_v.p) std::swap(e->srt_v, e->idx_post);  // the CSR's post array is where the sort ended
        }
    } else {
        launch_index_count(e->p_hash.p, e->p_track.p, e->n_post, e->tomb.p, e->n_tracks, e->idx_cnt.p, s);
        launch_count_nonzero(e->idx_cnt.p, (int64_t)K, e->nz.p, s);
        launch_scan(e->idx_cnt.p, e->idx_off.p, (int64_t)K, e->scan_tmp.p, s);
        HIP_TRY(hipMemcpyAsync(e->idx_cnt.p, e->idx_off.p, K * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        launch_index_scatter(e->p_hash.p, e->p_track.p, e->p_t.p, e->n_post, e->tomb.p, e->n_tracks, e->idx_cnt.p,
                             e->idx_post.p, s);
        launch_make_sig(e->idx_post.p, e->n_post, e->idx_sig.p, s);  // (only the first n_indexed are read)
    }
    HIP_TRY(hipGetLastError());
    uint32_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, e->idx_off.p + (K - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    unsigned long long used = 0;
    HIP_TRY(hipMemcpyAsync(&used, e->nz.p, sizeof(used), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->n_buckets_used = (int64_t)used;
    e->n_indexed = total;
    e->index_built = true;
    e->index_dirty = false;
    e->tomb_since_build = 0;  // the build skipped every removed track's postings
    // the sort's double buffers are 16 B per posting (15 GB at the 100k-track catalog): kept for the next build
    // of a small index (a store + query cycle rebuilds it), released above 1 GiB
    if ((e->srt_k0.n + e->srt_k1.n) * 4 + e->srt_v.n * 8 + e->srt_tmp.n + e->srt_scratch.n * 4 > ((size_t)1 << 30)) {
        e->srt_k0.release();
        e->srt_k1.release();
        e->srt_v.release();
        e->srt_tmp.release();
        e->srt_scratch.release();
    }
    return AID_OK;
}

int aid_index_finalize(aid_engine *e) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    return finalize_locked(e);
}

int aid_match_stats(aid_engine *e, int64_t *out, int32_t n, int32_t reset) {
    if (!e || (n > 0 && !out)) return fail(AID_ERR_INVALID, "aid_match_stats: bad argument");
    std::lock_guard<std::mutex> lk(e->mu);
    const int64_t v[13] = {e->st_queries,     e->st_votes,   e->st_post_reads, e->st_q_lds,
                           e->st_q_global,    e->st_records, e->st_sig_reads,  (int64_t)match_lds_blocks_per_cu(),
                           e->st_fb_reason[0], e->st_fb_reason[1], e->st_fb_reason[2], e->st_fb_reason[3],
                           e->st_fb_reason[4]};
    for (int i = 0; i < n && i < 13; ++i) out[i] = v[i];
    if (reset) {
        e->st_queries = e->st_votes = e->st_post_reads = e->st_q_lds = e->st_q_global = e->st_records = e->st_sig_reads = 0;
        for (auto &r : e->st_fb_reason) r = 0;
    }
    return AID_OK;
}

int aid_index_stats(aid_engine *e, int64_t *n_postings, int64_t *n_live, uint32_t *n_tracks) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    if (n_postings) *n_postings = e->n_post;
    if (n_live) *n_live = e->index_built && !e->index_dirty ? e->n_indexed : -1;
    if (n_tracks) *n_tracks = e->n_tracks;
    return AID_OK;
}

}  // extern "C"

struct aid_comm {
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0, device = -1;
};

#define NCCL_TRY(expr)                                                                              \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) return fail(AID_ERR_DEVICE, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)

extern "C" {

int aid_comm_id(uint8_t id[AID_COMM_ID_BYTES]) {
    if (!id) return fail(AID_ERR_INVALID, "null id");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    static_assert(sizeof(u.internal) == AID_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, u.internal, AID_COMM_ID_BYTES);
    return AID_OK;
}

int aid_comm_create(aid_engine *e, const uint8_t id[AID_COMM_ID_BYTES], int32_t world, int32_t rank, aid_comm **out) {
    if (!e || !id || !out || world <= 0 || rank < 0 || rank >= world) return fail(AID_ERR_INVALID, "aid_comm_create: bad argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(e->device));
    {
        std::lock_guard<std::mutex> lk(e->mu);
        HIP_TRY(e->g_meta.reserve(2 * (size_t)world + 2));  // the exchange's (count, n_tracks) and ok rounds
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, AID_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    NCCL_TRY(ncclCommInitRank(&c, world, u, rank));
    aid_comm *ac = new aid_comm();
    ac->comm = c;
    ac->world = world;
    ac->rank = rank;
    ac->device = e->device;
    *out = ac;
    return AID_OK;
}

void aid_comm_destroy(aid_comm *c) {
    if (!c) return;
    if (c->comm) {
        (void)hipSetDevice(c->device);
        (void)ncclCommDestroy(c->comm);
    }
    delete c;
}

int aid_comm_size(const aid_comm *c, int32_t *world, int32_t *rank) {
    if (!c || !c->comm) return fail(AID_ERR_INVALID, "aid_comm_size: null comm");
    int n = 0, r = 0;
    NCCL_TRY(ncclCommCount(c->comm, &n));
    NCCL_TRY(ncclCommUserRank(c->comm, &r));
    if (world) *world = n;
    if (rank) *rank = r;
    return AID_OK;
}

// the exchange in three steps (aid_index_allgather runs them around two RCCL all-gathers; a host-driven
// exchange, e.g. torch.distributed over gloo, runs them around its own collectives)
static int shard_info_locked(aid_engine *e, int64_t first, int64_t *count, uint32_t *n_tracks) {
    if (int rc = settle_postings(e)) return rc;
    if (first < 0 || first > e->n_post) return fail(AID_ERR_INVALID, "index exchange: first out of range");
    *count = e->n_post - first;
    *n_tracks = e->n_tracks;
    return AID_OK;
}

static int pack_locked(aid_engine *e, int64_t first, uint32_t *planes, int64_t stride, hipStream_t s) {
    if (e->inject_exchange_fail) {  // test hook: this rank's prepare step fails as a device OOM would
        e->inject_exchange_fail = 0;
        return fail(AID_ERR_NOMEM, "index exchange: injected failure of this rank's pack (aid_engine_force)");
    }
    if (int rc = settle_postings(e)) return rc;
    const int64_t n = e->n_post - first;
    if (n > stride) return fail(AID_ERR_INVALID, "aid_index_pack: stride below the shard's count");
    const uint32_t *src[3] = {e->p_hash.p, e->p_track.p, e->p_t.p};
    for (int q = 0; q < 3 && n > 0; ++q)
        HIP_TRY(hipMemcpyAsync(planes + q * stride, src[q] + first, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (stride > n)  // padding: defined bytes on the wire
        for (int q = 0; q < 3; ++q)
            HIP_TRY(hipMemsetAsync(planes + q * stride + n, 0, (stride - n) * sizeof(uint32_t), s));
    return AID_OK;
}

// everything a splice of `tot` postings at `first` (and n_tracks ids) can fail on, done before the exchange:
// the posting planes and the tombstone buffer grow keeping every stored posting (n_post, not first) and
// every tombstone; the index itself (n_post, n_tracks, the CSR) does not change
static int splice_reserve_locked(aid_engine *e, int64_t first, int64_t tot, uint32_t n_tracks, hipStream_t s) {
    if (int rc = settle_postings(e)) return rc;
    if (first < 0 || first > e->n_post) return fail(AID_ERR_INVALID, "index exchange: first out of range");
    if (tot < 0) return fail(AID_ERR_INVALID, "index exchange: negative posting count");
    if (first + tot > 0xFFFFFFFFll) return fail(AID_ERR_INVALID, "index exchange: more than 2^32 postings");
    const size_t want = (size_t)std::max<int64_t>(first + tot, e->n_post);
    if (int rc = grow_copy_u32(e->p_hash, e->n_post, want, s)) return rc;
    if (int rc = grow_copy_u32(e->p_track, e->n_post, want, s)) return rc;
    if (int rc = grow_copy_u32(e->p_t, e->n_post, want, s)) return rc;
    return n_tracks > e->n_tracks ? reserve_tracks(e, n_tracks, s) : AID_OK;
}

// failure-atomic: everything that can fail (growth of the posting planes and track tables) happens before
// the index changes; the union then replaces [first, n_post) in one stream-ordered pass
static int splice_locked(aid_engine *e, int64_t first, const uint32_t *recv, int32_t world, int64_t stride,
                         const int64_t *counts, uint32_t n_tracks, hipStream_t s) {
    if (int rc = settle_postings(e)) return rc;
    if (first < 0 || first > e->n_post) return fail(AID_ERR_INVALID, "aid_index_splice: first out of range");
    int64_t tot = 0;
    for (int r = 0; r < world; ++r) {
        if (counts[r] < 0 || counts[r] > stride) return fail(AID_ERR_INVALID, "aid_index_splice: bad count");
        tot += counts[r];
    }
    if (int rc = splice_reserve_locked(e, first, tot, n_tracks, s)) return rc;
    if (int rc = ensure_tracks(e, n_tracks, s)) return rc;  // capacity reserved: only the commit is left
    uint32_t *dst[3] = {e->p_hash.p, e->p_track.p, e->p_t.p};
    int64_t at = first;
    for (int r = 0; r < world; ++r) {
        const int64_t n = counts[r];
        for (int q = 0; q < 3 && n > 0; ++q)
            HIP_TRY(hipMemcpyAsync(dst[q] + at, recv + ((size_t)r * 3 + q) * stride, n * sizeof(uint32_t),
                                   hipMemcpyDeviceToDevice, s));
        at += n;
    }
    HIP_TRY(hipStreamSynchronize(s));
    e->n_post = at;
    e->index_dirty = true;
    return AID_OK;
}

int aid_index_shard_info(aid_engine *e, int64_t first, int64_t *count, uint32_t *n_tracks) {
    if (!e || !count || !n_tracks) return fail(AID_ERR_INVALID, "aid_index_shard_info: null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return shard_info_locked(e, first, count, n_tracks);
}

int aid_index_reserve(aid_engine *e, int64_t first, int64_t total, uint32_t n_tracks, void *stream) {
    if (!e) return fail(AID_ERR_INVALID, "aid_index_reserve: null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    if (e->last_stream && e->last_stream != s) HIP_TRY(hipStreamSynchronize(e->last_stream));
    return splice_reserve_locked(e, first, total, n_tracks, s);
}

int aid_index_pack(aid_engine *e, int64_t first, uint32_t *planes, int64_t stride, void *stream) {
    if (!e || (!planes && stride > 0) || stride < 0) return fail(AID_ERR_INVALID, "aid_index_pack: bad argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    if (first < 0 || first > e->n_post) return fail(AID_ERR_INVALID, "aid_index_pack: first out of range");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    if (e->last_stream && e->last_stream != s) HIP_TRY(hipStreamSynchronize(e->last_stream));
    if (int rc = pack_locked(e, first, planes, stride, s)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_index_splice(aid_engine *e, int64_t first, const uint32_t *recv, int32_t world, int64_t stride,
                     const int64_t *counts, uint32_t n_tracks, void *stream) {
    if (!e || world <= 0 || stride < 0 || !counts || (!recv && stride > 0))
        return fail(AID_ERR_INVALID, "aid_index_splice: bad argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    if (e->last_stream && e->last_stream != s) HIP_TRY(hipStreamSynchronize(e->last_stream));
    return splice_locked(e, first, recv, world, stride, counts, n_tracks, s);
}

// one all-gather of an int64 pair per rank over the engine's meta buffer (reserved by aid_comm_create);
// every rank calls it the same number of times, whatever its own state
static int allgather_pair(aid_engine *e, aid_comm *c, int64_t a, int64_t b, std::vector<int64_t> &out, hipStream_t s) {
    const int W = c->world;
    const int64_t mine[2] = {a, b};
    HIP_TRY(hipMemcpyAsync(e->g_meta.p, mine, sizeof(mine), hipMemcpyHostToDevice, s));
    NCCL_TRY(ncclAllGather(e->g_meta.p, e->g_meta.p + 2, 2, ncclInt64, c->comm, s));
    out.assign(2 * (size_t)W, 0);
    HIP_TRY(hipMemcpyAsync(out.data(), e->g_meta.p + 2, out.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_index_allgather(aid_engine *e, aid_comm *c, int64_t first, int64_t *n_total) {
    if (!e || !c || !c->comm) return fail(AID_ERR_INVALID, "aid_index_allgather: null argument");
    if (c->device != e->device) return fail(AID_ERR_INVALID, "aid_index_allgather: comm and engine on different devices");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->own_stream;
    if (int rc = settle_postings(e)) return rc;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    const int W = c->world;
    // aid_comm_create reserved this engine's meta buffer; a comm made with another engine gets it here (16 B per
    // rank: returning early instead would leave the other ranks blocked in the first all-gather)
    HIP_TRY(e->g_meta.reserve(2 * (size_t)W + 2));
    // Every rank runs the same collectives whatever happens locally: (1) (count, n_tracks), (2) one ok flag
    // per rank after every step that can fail locally, (3) the payload only when every rank is ready. A
    // rank-local failure (bad arguments, OOM of the exchange buffers or the grown index, the pack) is
    // therefore seen by all ranks before the payload all-gather, and every rank returns an error with its
    // index unchanged instead of leaving its peers blocked in RCCL.
    int64_t n_local = -1;
    uint32_t nt = 0;
    const int bad = shard_info_locked(e, first, &n_local, &nt);
    std::vector<int64_t> meta;
    if (int rc = allgather_pair(e, c, bad ? -1 : n_local, (int64_t)nt, meta, s)) return rc;
    int64_t mx = 0, tot = 0;
    uint32_t tracks = 0;
    std::vector<int64_t> counts(W);
    for (int r = 0; r < W; ++r) {
        if (meta[2 * r] < 0) return bad ? bad : fail(AID_ERR_INVALID, "aid_index_allgather: another rank's shard is invalid");
        counts[r] = meta[2 * r];
        mx = std::max(mx, counts[r]);
        tot += counts[r];
        tracks = std::max(tracks, (uint32_t)meta[2 * r + 1]);
    }
    // 2. local preparation: the exchange buffers ([3][mx] own planes, [W][3][mx] received; scratch of this
    //    call only: ~(W + 1) x 12 B per largest-shard posting), the grown index, the pack of the own shard
    int rc = AID_OK;
    if (mx > 0) {
        hipError_t he = e->g_send.reserve(3 * (size_t)mx);
        if (he == hipSuccess) he = e->g_recv.reserve(3 * (size_t)mx * W);
        if (he != hipSuccess)
            rc = fail(he == hipErrorOutOfMemory ? AID_ERR_NOMEM : AID_ERR_DEVICE,
                      std::string("index exchange buffers: ") + hipGetErrorString(he));
        if (!rc) rc = splice_reserve_locked(e, first, tot, tracks, s);
        if (!rc) rc = pack_locked(e, first, e->g_send.p, mx, s);
        if (!rc) {
            he = hipStreamSynchronize(s);
            if (he != hipSuccess) rc = fail(AID_ERR_DEVICE, std::string("index exchange pack: ") + hipGetErrorString(he));
        }
    } else {
        rc = splice_reserve_locked(e, first, 0, tracks, s);
    }
    const std::string local_err = rc ? g_err : std::string();
    std::vector<int64_t> ok;
    if (int rc2 = allgather_pair(e, c, rc ? 0 : 1, (int64_t)rc, ok, s)) {
        e->g_send.release();
        e->g_recv.release();
        return rc2;
    }
    int failed = -1;
    for (int r = 0; r < W && failed < 0; ++r)
        if (!ok[2 * r]) failed = r;
    if (failed >= 0) {
        e->g_send.release();
        e->g_recv.release();
        if (rc) return fail(rc, local_err);
        return fail(AID_ERR_STATE, "index exchange aborted: rank " + std::to_string(failed) +
                                       " failed to prepare (error " + std::to_string(ok[2 * failed + 1]) +
                                       "); this rank's index is unchanged");
    }
    if (mx > 0) {
        // 3. one all-gather of the padded planes, then the union in rank order replaces this rank's shard
        NCCL_TRY(ncclAllGather(e->g_send.p, e->g_recv.p, 3 * (size_t)mx, ncclUint32, c->comm, s));
        rc = splice_locked(e, first, e->g_recv.p, W, mx, counts.data(), tracks, s);
        e->g_send.release();
        e->g_recv.release();
        if (rc) return rc;
    } else if (int rc3 = ensure_tracks(e, tracks, s)) {
        return rc3;
    }
    if (n_total) *n_total = e->n_post;
    return AID_OK;
}

int aid_index_export(aid_engine *e, uint32_t *hash, uint32_t *track, uint32_t *t, int64_t first, int64_t count,
                     int32_t location) {
    if (!e || first < 0 || count < 0) return fail(AID_ERR_INVALID, "aid_index_export: bad range");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    if (first + count > e->n_post) return fail(AID_ERR_INVALID, "aid_index_export: bad range");
    if (count == 0) return AID_OK;
    HIP_TRY(hipSetDevice(e->device));
    // the posting append of aid_index_add_extracted runs asynchronously on the caller's stream
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    const hipMemcpyKind k = location == AID_PCM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpy(hash, e->p_hash.p + first, count * sizeof(uint32_t), k));
    HIP_TRY(hipMemcpy(track, e->p_track.p + first, count * sizeof(uint32_t), k));
    HIP_TRY(hipMemcpy(t, e->p_t.p + first, count * sizeof(uint32_t), k));
    return AID_OK;
}

int aid_index_checksum(aid_engine *e, int64_t first, int64_t count, uint64_t *out) {
    if (!e || !out || first < 0 || count < 0) return fail(AID_ERR_INVALID, "aid_index_checksum: bad range");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = settle_postings(e)) return rc;
    if (first + count > e->n_post) return fail(AID_ERR_INVALID, "aid_index_checksum: bad range");
    HIP_TRY(hipSetDevice(e->device));
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    HIP_TRY(e->chk.reserve(1));
    hipStream_t s = e->own_stream;
    HIP_TRY(hipMemsetAsync(e->chk.p, 0, sizeof(unsigned long long), s));
    launch_index_checksum(e->p_hash.p, e->p_track.p, e->p_t.p, first, count, e->chk.p, s);
    HIP_TRY(hipGetLastError());
    unsigned long long v = 0;
    HIP_TRY(hipMemcpyAsync(&v, e->chk.p, sizeof(v), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out = (uint64_t)v;
    return AID_OK;
}

int aid_index_csr_export(aid_engine *e, uint32_t *offsets, int64_t n_offsets, uint64_t *posts, int64_t cap,
                         int64_t *n_out) {
    if (!e || !n_out || n_offsets < 0 || cap < 0 || (!offsets && n_offsets > 0) || (!posts && cap > 0))
        return fail(AID_ERR_INVALID, "aid_index_csr_export: bad argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (!e->index_built || e->index_dirty) return fail(AID_ERR_STATE, "aid_index_csr_export: the index is not finalized");
    HIP_TRY(hipSetDevice(e->device));
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    const int64_t K = (int64_t)index_keys() + 1;
    *n_out = e->n_indexed;
    if (offsets && n_offsets > 0) {
        if (n_offsets < K) return fail(AID_ERR_INVALID, "aid_index_csr_export: offsets need 2^26 + 1 entries");
        HIP_TRY(hipMemcpy(offsets, e->idx_off.p, K * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    if (posts && cap > 0) {
        const int64_t n = std::min<int64_t>(cap, e->n_indexed);
        if (n > 0) HIP_TRY(hipMemcpy(posts, e->idx_post.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    return AID_OK;
}

static const char kIdxMagic[8] = {'A', 'I', 'D', 'F', 'P', 'I', 'X', '1'};

int aid_index_save(aid_engine *e, const char *path) {
    if (!e || !path) return fail(AID_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    if (int rc = settle_postings(e)) return rc;
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    FILE *f = std::fopen(path, "wb");
    if (!f) return fail(AID_ERR_INVALID, std::string("cannot open ") + path);
    int64_t hdr[6] = {AID_ABI_VERSION, e->cfg.sample_rate, e->cfg.hop, e->n_post, (int64_t)e->n_tracks, 0};
    bool ok = std::fwrite(kIdxMagic, 1, 8, f) == 8 && std::fwrite(hdr, sizeof(hdr), 1, f) == 1;
    std::vector<uint32_t> buf((size_t)std::min<int64_t>(e->n_post, 1 << 24));
    DevBuf<uint32_t> *cols[3] = {&e->p_hash, &e->p_track, &e->p_t};
    for (int c = 0; c < 3 && ok; ++c)
        for (int64_t o = 0; o < e->n_post && ok; o += (int64_t)buf.size()) {
            const int64_t m = std::min<int64_t>((int64_t)buf.size(), e->n_post - o);
            if (hipMemcpy(buf.data(), cols[c]->p + o, m * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) ok = false;
            else ok = std::fwrite(buf.data(), sizeof(uint32_t), m, f) == (size_t)m;
        }
    if (ok && e->n_tracks) ok = std::fwrite(e->h_tomb.data(), 1, e->n_tracks, f) == e->n_tracks;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) return fail(AID_ERR_DEVICE, std::string("failed writing ") + path);
    return AID_OK;
}

int aid_index_load(aid_engine *e, const char *path) {
    if (!e || !path) return fail(AID_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    if (int rc = settle_postings(e)) return rc;
    // Everything is validated and read into scratch buffers first; the engine's index changes only
    // once the whole file has been read (a failed load leaves the previous index untouched).
    struct File {
        FILE *f;
        ~File() {
            if (f) std::fclose(f);
        }
    } file{std::fopen(path, "rb")};
    FILE *f = file.f;
    if (!f) return fail(AID_ERR_INVALID, std::string("cannot open ") + path);
    char magic[8];
    int64_t hdr[6];
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kIdxMagic, 8) != 0 || std::fread(hdr, sizeof(hdr), 1, f) != 1)
        return fail(AID_ERR_INVALID, "not an aidfp index file");
    if (hdr[0] != AID_ABI_VERSION) return fail(AID_ERR_INVALID, "index file written by another ABI version");
    if (hdr[1] != e->cfg.sample_rate || hdr[2] != e->cfg.hop)
        return fail(AID_ERR_INVALID, "index sample_rate/hop differ from the engine's");
    const int64_t n = hdr[3];
    if (n < 0 || n > 0xFFFFFFFFll || hdr[4] < 0 || hdr[4] > 0xFFFFFFFFll || hdr[5] != 0)
        return fail(AID_ERR_INVALID, "corrupt index header");
    const uint32_t nt = (uint32_t)hdr[4];
    if (std::fseek(f, 0, SEEK_END) != 0) return fail(AID_ERR_INVALID, "cannot size index file");
    const long long fsize = (long long)ftello(f);
    const long long want = 8 + (long long)sizeof(hdr) + 12ll * n + (long long)nt;
    if (fsize != want) return fail(AID_ERR_INVALID, fsize < want ? "truncated index file" : "index file has trailing bytes");
    if (std::fseek(f, 8 + (long)sizeof(hdr), SEEK_SET) != 0) return fail(AID_ERR_INVALID, "cannot read index file");
    HIP_TRY(hipSetDevice(e->device));
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    DevBuf<uint32_t> cols[3];
    struct Release {
        DevBuf<uint32_t> *c;
        ~Release() {
            for (int i = 0; i < 3; ++i) c[i].release();
        }
    } release_cols{cols};
    std::vector<uint32_t> buf((size_t)std::min<int64_t>(std::max<int64_t>(n, 1), 1 << 24));
    for (int c = 0; c < 3; ++c) {
        HIP_TRY(cols[c].reserve((size_t)std::max<int64_t>(n, 1)));
        for (int64_t o = 0; o < n; o += (int64_t)buf.size()) {
            const int64_t m = std::min<int64_t>((int64_t)buf.size(), n - o);
            if (std::fread(buf.data(), sizeof(uint32_t), m, f) != (size_t)m) return fail(AID_ERR_INVALID, "truncated index file");
            HIP_TRY(hipMemcpy(cols[c].p + o, buf.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
    }
    std::vector<uint8_t> tomb(nt);
    if (nt && std::fread(tomb.data(), 1, nt, f) != nt) return fail(AID_ERR_INVALID, "truncated index file");
    DevBuf<uint8_t> dtomb;
    struct ReleaseTomb {
        DevBuf<uint8_t> *b;
        ~ReleaseTomb() { b->release(); }
    } release_tomb{&dtomb};
    HIP_TRY(dtomb.reserve(std::max<size_t>(nt, 1024)));
    if (nt) HIP_TRY(hipMemcpy(dtomb.p, tomb.data(), nt, hipMemcpyHostToDevice));
    // commit: swap the new planes in (the old ones are released with the scratch)
    std::swap(e->tomb, dtomb);
    std::swap(e->p_hash, cols[0]);
    std::swap(e->p_track, cols[1]);
    std::swap(e->p_t, cols[2]);
    e->h_tomb = std::move(tomb);
    e->n_tracks = nt;
    e->n_post = n;
    e->tomb_since_build = 0;
    e->index_dirty = true;
    e->index_built = false;
    return AID_OK;
}

constexpr double kForwardedPerBucket = 2.0;  // forwarded votes (1-bit filter estimate) per global histogram bucket
// run K5 over nq queries whose records are at device ranges (q_start/q_count device arrays).
// Exact per-query vote counts (k_query_votes) choose the path and size the vote histogram;
// queries whose exact LDS table overflowed are re-run with 4x the buckets. rec_cap: elements of `recs` (the per-record
// CSR range cache the vote count writes for the LDS path has one entry per record index).
// rows == nullptr: device mode, every query's rows end in e->q_rows ([nq][max_results][5] int32);
// nrows (host) is always filled

static int run_queries(aid_engine *e, const uint64_t *recs, const int64_t *qstart_dev, const int64_t *qcount_dev,
                       int nq, int64_t rec_cap, aid_match_row *rows, int32_t *nrows, hipStream_t s) {
    const int mr = e->cfg.max_results;
    HIP_TRY(e->q_rows.reserve((size_t)std::max(nq, 1) * mr * 5));
    HIP_TRY(e->q_nrows.reserve((size_t)std::max(nq, 1)));
    std::vector<int> todo(nq);
    for (int q = 0; q < nq; ++q) todo[q] = q;
    std::vector<int64_t> h_start(nq), h_count(nq), h_votes(nq, 0);
    // the per-query metadata and (below) the LDS path's rows come back through page-locked buffers: the copies are
    // queued behind the kernels and the call waits ONCE (a pageable destination made each copy a host wait, so K5
    // was launched only after a round trip behind the extraction)
    HIP_TRY(e->hq_meta.reserve((size_t)3 * nq));
    int64_t *p_start = e->hq_meta.p, *p_count = p_start + nq, *p_votes = p_count + nq;
    HIP_TRY(hipMemcpyAsync(p_start, qstart_dev, nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(p_count, qcount_dev, nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    {  // exact vote counts: path choice and the global histogram's size
        HIP_TRY(e->q_votes.reserve((size_t)nq));
        const bool ranges = e->k5_path == 0 || e->k5_path == 1;  // the LDS path reads them
        if (ranges) HIP_TRY(e->q_ranges.reserve((size_t)std::max<int64_t>(rec_cap, 1)));
        launch_query_votes(recs, qstart_dev, qcount_dev, nq, e->idx_off.p, e->q_votes.p, ranges ? e->q_ranges.p : nullptr,
                           s);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(p_votes, e->q_votes.p, nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    }
    // the LDS path is launched right away, in the same round trip as the vote counts instead of after them (one
    // host sync less per call). It routes each query by its own count (K5 reads q_votes on the device): a query
    // above kLdsMaxVotes is handed back (nrows -1) without an LDS run, and one that overflows its counters reports
    // -1 too; both fall through to the global path below. Round 2 did this for batches of <= 16 queries, gated on
    // the previous batch's heaviest query, because the LDS kernel then ran heavy queries too; with per-query
    // routing (round 5) a batch of any size takes it, the coalesced service batches and the stream pushes included
    const bool speculate = e->k5_path == 0;
    std::vector<int32_t> spec_n;
    if (speculate) {
        {
            ProfScope ps(e, AID_K_MATCH, s, true);
            launch_match_lds(recs, qstart_dev, qcount_dev, nq, e->idx_off.p, e->idx_post.p, e->tomb.p, e->n_tracks,
                             e->cfg.min_match, mr, e->q_rows.p, e->q_nrows.p, e->tomb_since_build > 0, e->q_votes.p,
                             e->idx_sig.p, e->q_ranges.p, s);
        }
        HIP_TRY(hipGetLastError());
        spec_n.resize(nq);
        if (rows) {
            HIP_TRY(e->hq_rows.reserve((size_t)nq * mr * 5));
            HIP_TRY(hipMemcpyAsync(e->hq_rows.p, e->q_rows.p, (size_t)nq * mr * sizeof(aid_match_row),
                                   hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(e->hq_n.reserve((size_t)nq));
        HIP_TRY(hipMemcpyAsync(e->hq_n.p, e->q_nrows.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(h_start.data(), p_start, nq * sizeof(int64_t));
    std::memcpy(h_count.data(), p_count, nq * sizeof(int64_t));
    std::memcpy(h_votes.data(), p_votes, nq * sizeof(int64_t));
    if (speculate) {
        std::memcpy(spec_n.data(), e->hq_n.p, nq * sizeof(int32_t));
        if (rows) std::memcpy(rows, e->hq_rows.p, (size_t)nq * mr * sizeof(aid_match_row));
        std::vector<int> again;
        for (int q = 0; q < nq; ++q) {
            if (spec_n[q] < 0) {
                again.push_back(q);
                ++e->st_fb_reason[std::min(-spec_n[q], 5) - 1];
            } else {
                nrows[q] = spec_n[q];
            }
        }
        todo.swap(again);
        e->n_fallback += (int64_t)todo.size();
    }
    int64_t vmax = 1;
    for (int q = 0; q < nq; ++q) vmax = std::max(vmax, h_votes[q]);
    const double votes = (double)vmax;
    e->st_queries += nq;
    for (int q = 0; q < nq; ++q) {
        e->st_votes += h_votes[q];
        e->st_records += h_count[q];
    }
    if (speculate)  // the LDS path ran every light query once: two enumerations (counting, then the exact inserts)
        for (int q = 0; q < nq; ++q) e->st_sig_reads += h_votes[q] <= kLdsMaxVotes ? 2 * h_votes[q] : 0;
    // global histogram, sized for the votes that pass K5a's 2^20-bit seen filter (all but the
    // distinct bits: v - m(1 - e^{-v/m})) at ~2 per bucket: a chance bucket reaching
    // min_match - 1 then has probability ~1e-5. Sizing it for ALL votes (2 buckets each: 2 MB rows on
    // config 4) spread K5a's random atomics over ~4 GB of rows, all HBM round trips: 16 bits
    // (256 KB rows, 64 MB for the 256 resident queries: Infinity-Cache resident) took 0.295 s
    // against 0.383 s for 19 bits on config 4 (37.3k against 28.8k clips/s; 20 bits: 23.4k).
    // K5a key partitions (a workgroup and a 2^20-bit seen filter each): two once the filter
    // saturates (> 2^18 votes; config 4's ~540k: 46.6k -> 60.2k clips/s), else one
    const int parts = e->k5_parts > 0 ? e->k5_parts : votes > (double)(1 << 18) ? 2 : 1;
    const double m_seen = (double)(1 << 20), vp = votes / parts;
    const double fwd = parts * (vp - m_seen * (1.0 - std::exp(-vp / m_seen)));
    int bits = 15;
    while (bits < 24 && (double)(1ull << bits) < fwd / kForwardedPerBucket) ++bits;
    // LDS fast path while its 2^16 counters stay sparse enough. It is exact for heavier queries too (overflows
    // fall back; tests/test_gpu_match_load.py) but one query per CU cannot keep enough posting reads in flight:
    // round-1 config 4 (v0 catalog, ~540k votes per window) took 48.6 s on it against 1.43 s on the global path.
    // On the v2 catalog (~84.5k votes per window, probes/k5_path_probe.py) it is the faster path (201k against
    // 185k clips/s, rows equal), so a batch goes to it when its mean query has <= 2^17 votes (2 per counter) and
    // none has more than 2^20 (a heavier one falls back to the global path after its LDS run)
    // Each query is routed by its own vote count: k_match_lds answers the queries with <= kLdsMaxVotes
    // (2^18 votes over the 2^16 4-bit counters of its filter = 4 per counter, aidfp_layout.h) and hands heavier ones
    // straight back (nrows -1, no LDS run), so the batch takes
    // the LDS launch whenever some query is light enough for it; the heavy ones run on the global path below
    int n_light = 0;
    for (int q = 0; q < nq; ++q) n_light += h_votes[q] <= kLdsMaxVotes;
    const bool fast = !speculate && (e->k5_path == 1 || (e->k5_path == 0 && n_light > 0));
    // fast path: the whole vote filter in LDS (K5 `k_match_lds`); overflowed queries fall
    // through to the global-histogram path below
    if (fast) {
        {
            ProfScope ps(e, AID_K_MATCH, s, true);
            launch_match_lds(recs, qstart_dev, qcount_dev, nq, e->idx_off.p, e->idx_post.p, e->tomb.p, e->n_tracks,
                             e->cfg.min_match, mr, e->q_rows.p, e->q_nrows.p, e->tomb_since_build > 0, e->q_votes.p,
                             e->idx_sig.p, e->q_ranges.p, s);
        }
        HIP_TRY(hipGetLastError());
        std::vector<int32_t> got_n(nq);
        if (rows)
            HIP_TRY(hipMemcpyAsync(rows, e->q_rows.p, (size_t)nq * mr * sizeof(aid_match_row), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(got_n.data(), e->q_nrows.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<int> again;
        for (int q = 0; q < nq; ++q) {
            if (got_n[q] < 0) again.push_back(q);
            else nrows[q] = got_n[q];
        }
        todo.swap(again);
        e->n_fallback += (int64_t)todo.size();
        for (int q = 0; q < nq; ++q)  // counting pass + insert pass (2 B each), light queries only
            e->st_sig_reads += h_votes[q] <= kLdsMaxVotes ? 2 * h_votes[q] : 0;
        e->st_q_lds += n_light;
    }
    if (speculate) e->st_q_lds += n_light;
    for (int attempt = 1; !todo.empty(); ++attempt, bits += 2) {
        for (int q : todo) e->st_post_reads += h_votes[q] * (parts + 1);  // K5a once per key partition, K5b once
        e->st_q_global += (int64_t)todo.size();
        if (bits > 26) return fail(AID_ERR_STATE, "query vote table overflow (too many candidate votes)");
        const size_t H = (size_t)1 << bits;
        const int batch = (int)std::max<size_t>(1, std::min<size_t>(e->k5_batch, ((size_t)4 << 30) / (H * 4)));
        HIP_TRY(e->q_hist.reserve((size_t)std::min<int>((int)todo.size(), batch) * H));
        HIP_TRY(e->q_hot.reserve((size_t)std::min<int>((int)todo.size(), batch) * (H / 32)));
        if (e->hist_zero_cap != e->q_hist.n) {  // fresh allocation; K5h re-zeroes its rows afterwards
            HIP_TRY(hipMemsetAsync(e->q_hist.p, 0, e->q_hist.n * sizeof(uint32_t), s));
            e->hist_zero_cap = e->q_hist.n;
        }
        const int64_t *qs = qstart_dev, *qc = qcount_dev;
        int32_t *out_rows = e->q_rows.p, *out_n = e->q_nrows.p;
        std::vector<int> order = todo;
        if (attempt > 0) {  // gather the overflowed queries' ranges into the scratch arrays' tail
            HIP_TRY(e->x_src.reserve(2 * order.size()));
            std::vector<int64_t> st(order.size()), ct(order.size());
            for (size_t i = 0; i < order.size(); ++i) { st[i] = h_start[order[i]]; ct[i] = h_count[order[i]]; }
            HIP_TRY(hipMemcpyAsync(e->x_src.p, st.data(), st.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->x_src.p + order.size(), ct.data(), ct.size() * sizeof(int64_t),
                                   hipMemcpyHostToDevice, s));
            qs = e->x_src.p;
            qc = e->x_src.p + order.size();
            HIP_TRY(e->x_dst.reserve(((size_t)order.size() * mr * 5 + 1) / 2 + order.size()));
            out_rows = reinterpret_cast<int32_t *>(e->x_dst.p);
            out_n = out_rows + (size_t)order.size() * mr * 5;
        }
        const int n = (int)order.size();
        // from the second global attempt on, the distinct (slot, t_q) sets live in HBM (2^dbits entries per query,
        // 4x more per attempt): a query that overflowed k_vote_final's LDS set is a long one with a strong match
        // (FPSPEC v1 7), which more histogram buckets do not help
        const int dbits = attempt >= 2 ? std::min(12 + 2 * attempt, 26) : 0;
        int dbatch = batch;
        if (dbits) {
            dbatch = (int)std::max<size_t>(1, std::min<size_t>((size_t)batch, ((size_t)1 << 30) / ((size_t)4 << dbits)));
            HIP_TRY(e->q_dset.reserve((size_t)std::min(dbatch, n) << dbits));
        }
        for (int q0 = 0; q0 < n; q0 += dbatch) {
            const int nb = std::min(dbatch, n - q0);
            if (dbits) HIP_TRY(hipMemsetAsync(e->q_dset.p, 0xFF, ((size_t)nb << dbits) * sizeof(uint32_t), s));
            // K5a, K5h, K5b, each with its own dispatch-attached events when profiled
            for (int stage = 1; stage <= 3; ++stage) {
                ProfScope ps(e, stage == 1 ? AID_K_VOTE_HIST : stage == 2 ? AID_K_HOT_SCAN : AID_K_VOTE_FINAL, s, true);
                launch_query(recs, qs + q0, qc + q0, nb, e->idx_off.p, e->idx_post.p, e->tomb.p, e->n_tracks,
                             e->cfg.min_match, mr, e->q_hist.p, bits, e->q_hot.p, out_rows + (size_t)q0 * mr * 5,
                             out_n + q0, e->tomb_since_build > 0, parts, stage, dbits ? e->q_dset.p : nullptr, dbits,
                             s);
            }
            HIP_TRY(hipGetLastError());
        }
        std::vector<int32_t> got_n(n);
        std::vector<aid_match_row> got;
        if (rows) {
            got.resize((size_t)n * mr);
            HIP_TRY(hipMemcpyAsync(got.data(), out_rows, (size_t)n * mr * sizeof(aid_match_row), hipMemcpyDeviceToHost, s));
        } else {  // device mode: the batch's rows go to their queries' slots of q_rows
            HIP_TRY(e->x_order.reserve(order.size()));
            HIP_TRY(hipMemcpyAsync(e->x_order.p, order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
            launch_rows_scatter(out_rows, e->x_order.p, n, mr, e->q_rows.p, s);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipMemcpyAsync(got_n.data(), out_n, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<int> again;
        for (int i = 0; i < n; ++i) {
            const int q = order[i];
            if (got_n[i] < 0) {
                again.push_back(q);
                continue;
            }
            nrows[q] = got_n[i];
            if (rows) std::memcpy(rows + (size_t)q * mr, got.data() + (size_t)i * mr, (size_t)mr * sizeof(aid_match_row));
        }
        todo.swap(again);
    }
    return AID_OK;
}

// K5 keys its distinct-frame sets by (table slot << 20 | t_q) (index.hip distinct_first): a query's anchor frames must
// stay below 2^20 - 1 (3.4 h of audio at 44.1 kHz, 4.6 h at 16 kHz)
constexpr int64_t kMaxQueryFrame = ((int64_t)1 << 20) - 2;
static int check_query_frames(const aid_engine *e) {
    for (int c = 0; c < e->n_clips; ++c)
        if (e->clip_frames[c] > kMaxQueryFrame + 1)
            return fail(AID_ERR_INVALID, "query clip longer than 2^20 - 1 frames (FPSPEC v1 7)");
    return AID_OK;
}

static int ensure_index(aid_engine *e) {
    if (e->index_dirty || !e->index_built) return finalize_locked(e);
    return AID_OK;
}

int aid_query(aid_engine *e, const aid_hash *recs, const int64_t *qoff, int32_t nq, aid_match_row *rows,
              int32_t *nrows) {
    if (!e || nq < 0 || !qoff || (nq > 0 && (!rows || !nrows))) return fail(AID_ERR_INVALID, "aid_query: bad argument");
    if (nq == 0) return AID_OK;
    for (int q = 0; q < nq; ++q)
        if (qoff[q + 1] < qoff[q]) return fail(AID_ERR_INVALID, "aid_query: offsets must be non-decreasing");
    for (int64_t i = qoff[0]; i < qoff[nq]; ++i)
        if ((int64_t)recs[i].t1 > kMaxQueryFrame)
            return fail(AID_ERR_INVALID, "aid_query: record anchor frame >= 2^20 - 1 (FPSPEC v1 7)");
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = ensure_index(e)) return rc;
    hipStream_t s = e->own_stream;
    const int64_t n = qoff[nq] - qoff[0];
    HIP_TRY(e->q_recs.reserve((size_t)std::max<int64_t>(n, 1)));
    HIP_TRY(e->q_start.reserve(nq));
    HIP_TRY(e->q_count.reserve(nq));
    std::vector<int64_t> st(nq), ct(nq);
    for (int q = 0; q < nq; ++q) {
        st[q] = qoff[q] - qoff[0];
        ct[q] = qoff[q + 1] - qoff[q];
    }
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->q_recs.p, recs + qoff[0], n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->q_start.p, st.data(), nq * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->q_count.p, ct.data(), nq * sizeof(int64_t), hipMemcpyHostToDevice, s));
    int64_t mx = 0;
    for (int q = 0; q < nq; ++q) mx = std::max(mx, ct[q]);
    (void)mx;
    return run_queries(e, e->q_recs.p, e->q_start.p, e->q_count.p, nq, std::max<int64_t>(n, 1), rows, nrows, s);
}

// q_start <- clip_base through page-locked staging: from the engine's std::vector (pageable) the copy could hold
// the host until the stream had drained the extraction queued before it. Every caller waits for its stream before
// returning, so the staging is free again at the next call.
static hipError_t upload_clip_base(aid_engine *e, int n, hipStream_t s) {
    hipError_t he = e->hq_start.reserve((size_t)n);
    if (he != hipSuccess) return he;
    std::memcpy(e->hq_start.p, e->clip_base.data(), (size_t)n * sizeof(int64_t));
    return hipMemcpyAsync(e->q_start.p, e->hq_start.p, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, s);
}

static int query_extracted_locked(aid_engine *e, aid_match_row *rows, int32_t *nrows) {
    if (int rc = check_query_frames(e)) return rc;
    if (int rc = ensure_index(e)) return rc;
    hipStream_t s = e->last_stream ? e->last_stream : e->own_stream;
    const int nq = e->n_clips;
    if (nq == 0) return AID_OK;
    if (!rows || !nrows) return fail(AID_ERR_INVALID, "null output");
    HIP_TRY(e->q_start.reserve(nq));
    HIP_TRY(upload_clip_base(e, nq, s));
    return run_queries(e, e->records.p, e->q_start.p, e->counts.p, nq, (int64_t)e->records.n, rows, nrows, s);
}

int aid_query_extracted(aid_engine *e, aid_match_row *rows, int32_t *nrows) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    if (!e->have_result) return fail(AID_ERR_STATE, "no extraction to query with");
    std::lock_guard<std::mutex> lk(e->mu);
    return query_extracted_locked(e, rows, nrows);
}

int aid_query_pcm(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                  aid_match_row *rows, int32_t *nrows, void *stream) {
    if (!e || !offsets || n_clips < 0) return fail(AID_ERR_INVALID, "aid_query_pcm: bad argument");
    if (loc != AID_PCM_HOST && loc != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "aid_query_pcm: bad pcm_location");
    if (n_clips > 0 && !pcm && offsets[n_clips] > offsets[0]) return fail(AID_ERR_INVALID, "aid_query_pcm: null pcm");
    for (int c = 0; c < n_clips; ++c)
        if (offsets[c + 1] < offsets[c] || offsets[c] < 0)
            return fail(AID_ERR_INVALID, "aid_query_pcm: offsets must be non-decreasing and >= 0");
    if (n_clips > 0 && (!rows || !nrows)) return fail(AID_ERR_INVALID, "aid_query_pcm: null output");
    if (n_clips == 0) return AID_OK;
    // one critical section: no other thread's extraction can land between this batch's K1-K3 and K5
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = ensure_index(e)) return rc;
    if (int rc = extract_locked(e, pcm, offsets, n_clips, loc, stream)) return drain_host_copy(e, loc, stream, rc);
    return drain_host_copy(e, loc, stream, query_extracted_locked(e, rows, nrows));
}

// ---- asynchronous windowed query: submit enqueues the extraction, K5's LDS path and the result
// copies and returns; collect waits for the ticket's event. The ticket owns page-locked result buffers and a device copy
// of its records (the next submit reuses the engine's extraction buffers in stream order), so a query the LDS path
// hands back can still be answered on the global path at collect time.
struct aid_query_ticket {
    int nq = 0;
    int64_t nrec = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    HostBuf<int32_t> rows, nrows;
    HostBuf<int64_t> meta;  // [0, nq) record starts, [nq, 2nq) record counts, [2nq, 3nq) exact votes
    DevBuf<uint64_t> recs;
    DevBuf<int64_t> qsc;    // device record starts and counts of the ticket's queries ([0, nq), [nq, 2nq))
    ~aid_query_ticket() {
        if (ev) (void)hipEventDestroy(ev);
        rows.release();
        nrows.release();
        meta.release();
        recs.release();
        qsc.release();
    }
};

static void free_ticket_pool(aid_engine *e) {
    for (aid_query_ticket *t : e->ticket_pool) delete t;
    e->ticket_pool.clear();
}

static aid_query_ticket *take_ticket(aid_engine *e) {
    // a pooled ticket keeps its page-locked and device buffers and its event: allocating them per call (hipHostMalloc,
    // hipMalloc, and the hipFree that synchronises the device on release) had cost more than the overlap gained
    if (e->ticket_pool.empty()) return new aid_query_ticket();
    aid_query_ticket *t = e->ticket_pool.back();
    e->ticket_pool.pop_back();
    return t;
}

// the body both submit entries share (engine lock held): the extraction of n clips, K5's LDS pass over the ticket's
// own copy of the records, the result copies into its page-locked buffers and its event
static int submit_locked(aid_engine *e, const float *pcm, const int64_t *offsets, const int64_t *ends, int32_t n,
                         int32_t loc, void *stream, aid_query_ticket *t) {
    t->nq = n;
    t->nrec = 0;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc = ensure_index(e)) return rc;
    if (n == 0) return AID_OK;
    if (int rc = extract_locked(e, pcm, offsets, n, loc, stream, ends)) return rc;
    if (int rc = check_query_frames(e)) return rc;
    hipStream_t s = e->last_stream ? e->last_stream : e->own_stream;
    t->s = s;
    const int nq = n, mr = e->cfg.max_results;
    t->nrec = e->clip_base[nq - 1] + hash_capacity(e->clip_frames[nq - 1]);
    HIP_TRY(t->meta.reserve((size_t)3 * nq));
    HIP_TRY(t->rows.reserve((size_t)nq * mr * 5));
    HIP_TRY(t->nrows.reserve((size_t)nq));
    HIP_TRY(t->recs.reserve((size_t)std::max<int64_t>(t->nrec, 1)));
    HIP_TRY(t->qsc.reserve((size_t)2 * nq));
    std::memcpy(t->meta.p, e->clip_base.data(), (size_t)nq * sizeof(int64_t));
    // the ticket's own copies: record starts (from its page-locked meta), counts and records (device to device)
    HIP_TRY(hipMemcpyAsync(t->qsc.p, t->meta.p, (size_t)nq * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(t->qsc.p + nq, e->counts.p, (size_t)nq * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemcpyAsync(t->recs.p, e->records.p, (size_t)t->nrec * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemcpyAsync(t->meta.p + nq, e->counts.p, (size_t)nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(e->q_votes.reserve((size_t)nq));
    HIP_TRY(e->q_ranges.reserve((size_t)std::max<int64_t>(t->nrec, 1)));
    HIP_TRY(e->q_rows.reserve((size_t)nq * mr * 5));
    HIP_TRY(e->q_nrows.reserve((size_t)nq));
    launch_query_votes(t->recs.p, t->qsc.p, t->qsc.p + nq, nq, e->idx_off.p, e->q_votes.p, e->q_ranges.p, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(t->meta.p + 2 * nq, e->q_votes.p, (size_t)nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    {
        ProfScope ps(e, AID_K_MATCH, s, true);
        launch_match_lds(t->recs.p, t->qsc.p, t->qsc.p + nq, nq, e->idx_off.p, e->idx_post.p, e->tomb.p, e->n_tracks,
                         e->cfg.min_match, mr, e->q_rows.p, e->q_nrows.p, e->tomb_since_build > 0, e->q_votes.p,
                         e->idx_sig.p, e->q_ranges.p, s);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(t->rows.p, e->q_rows.p, (size_t)nq * mr * sizeof(aid_match_row), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(t->nrows.p, e->q_nrows.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (!t->ev) HIP_TRY(hipEventCreateWithFlags(&t->ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(t->ev, s));
    return AID_OK;
}

extern "C" int aid_query_windows_submit(aid_engine *e, const float *pcm, const int64_t *starts, const int64_t *ends,
                                        int32_t n_windows, void *stream, aid_query_ticket **out) {
    if (!e || n_windows < 0 || !out || (n_windows > 0 && (!starts || !ends || !pcm)))
        return fail(AID_ERR_INVALID, "aid_query_windows_submit: bad argument");
    *out = nullptr;
    for (int c = 0; c < n_windows; ++c)
        if (starts[c] < 0 || ends[c] < starts[c]) return fail(AID_ERR_INVALID, "aid_query_windows_submit: bad window");
    std::lock_guard<std::mutex> lk(e->mu);
    std::unique_ptr<aid_query_ticket> t(take_ticket(e));
    if (int rc = submit_locked(e, pcm, starts, ends, n_windows, AID_PCM_DEVICE, stream, t.get())) return rc;
    *out = t.release();
    return AID_OK;
}

// aid_query_pcm in two halves (the query coalescer's pipelined batches): host PCM must stay unchanged until the ticket
// is collected (its one H2D copy is queued, not waited for)
extern "C" int aid_query_pcm_submit(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips,
                                    int32_t loc, void *stream, aid_query_ticket **out) {
    if (!e || !offsets || n_clips < 0 || !out) return fail(AID_ERR_INVALID, "aid_query_pcm_submit: bad argument");
    *out = nullptr;
    if (loc != AID_PCM_HOST && loc != AID_PCM_DEVICE)
        return fail(AID_ERR_INVALID, "aid_query_pcm_submit: bad pcm_location");
    if (n_clips > 0 && !pcm && offsets[n_clips] > offsets[0])
        return fail(AID_ERR_INVALID, "aid_query_pcm_submit: null pcm");
    for (int c = 0; c < n_clips; ++c)
        if (offsets[c + 1] < offsets[c] || offsets[c] < 0)
            return fail(AID_ERR_INVALID, "aid_query_pcm_submit: offsets must be non-decreasing and >= 0");
    std::lock_guard<std::mutex> lk(e->mu);
    std::unique_ptr<aid_query_ticket> t(take_ticket(e));
    if (int rc = submit_locked(e, pcm, offsets, nullptr, n_clips, loc, stream, t.get()))
        return drain_host_copy(e, loc, stream, rc);
    *out = t.release();
    return AID_OK;
}

extern "C" int aid_query_windows_collect(aid_engine *e, aid_query_ticket *t, aid_match_row *rows, int32_t *nrows) {
    if (!e || !t) {
        delete t;
        return fail(AID_ERR_INVALID, "aid_query_windows_collect: bad argument");
    }
    if (t->nq > 0 && (!rows || !nrows)) {
        if (t->ev) (void)hipEventSynchronize(t->ev);
        std::lock_guard<std::mutex> lk(e->mu);
        e->ticket_pool.push_back(t);
        return fail(AID_ERR_INVALID, "aid_query_windows_collect: bad argument");
    }
    if (t->nq > 0) {
        const hipError_t we = hipEventSynchronize(t->ev);
        if (we != hipSuccess) {
            delete t;
            return fail(AID_ERR_DEVICE, std::string("aid_query_windows_collect: ") + hipGetErrorString(we));
        }
    }
    std::lock_guard<std::mutex> lk(e->mu);
    struct Back {  // back to the pool on every return below (the ticket's work has completed)
        aid_engine *e;
        aid_query_ticket *t;
        ~Back() { e->ticket_pool.push_back(t); }
    } back{e, t};
    if (t->nq == 0) return AID_OK;
    const int nq = t->nq, mr = e->cfg.max_results;
    std::memcpy(rows, t->rows.p, (size_t)nq * mr * sizeof(aid_match_row));
    const int64_t *starts = t->meta.p, *counts = starts + nq, *votes = counts + nq;
    std::vector<int> again;
    int n_light = 0;
    for (int q = 0; q < nq; ++q) {
        const int32_t n = t->nrows.p[q];
        if (n < 0) {
            again.push_back(q);
            ++e->st_fb_reason[std::min(-n, 5) - 1];
        } else {
            nrows[q] = n;
        }
        e->st_votes += votes[q];
        e->st_records += counts[q];
        e->st_sig_reads += votes[q] <= kLdsMaxVotes ? 2 * votes[q] : 0;
        n_light += votes[q] <= kLdsMaxVotes;
    }
    e->st_queries += nq;
    e->st_q_lds += n_light;
    e->n_fallback += (int64_t)again.size();
    if (again.empty()) return AID_OK;
    // the queries the LDS path handed back: the global path over the ticket's own copy of their records
    HIP_TRY(hipSetDevice(e->device));
    const int na = (int)again.size();
    std::vector<int64_t> sc(2 * (size_t)na);
    for (int i = 0; i < na; ++i) {
        sc[i] = starts[again[i]];
        sc[na + i] = counts[again[i]];
    }
    HIP_TRY(t->qsc.reserve((size_t)2 * nq));
    HIP_TRY(hipMemcpyAsync(t->qsc.p, sc.data(), sc.size() * sizeof(int64_t), hipMemcpyHostToDevice, t->s));
    std::vector<aid_match_row> sub((size_t)na * mr);
    std::vector<int32_t> subn(na, 0);
    const int keep_path = e->k5_path;
    const int64_t q0 = e->st_queries, v0 = e->st_votes, r0 = e->st_records;
    e->k5_path = 2;
    const int rc = run_queries(e, t->recs.p, t->qsc.p, t->qsc.p + na, na, t->nrec, sub.data(), subn.data(), t->s);
    e->k5_path = keep_path;
    e->st_queries = q0;  // counted above already
    e->st_votes = v0;
    e->st_records = r0;
    if (rc) return rc;
    for (int i = 0; i < na; ++i) {
        nrows[again[i]] = subn[i];
        std::memcpy(rows + (size_t)again[i] * mr, sub.data() + (size_t)i * mr, (size_t)mr * sizeof(aid_match_row));
    }
    return AID_OK;
}

int aid_query_windows(aid_engine *e, const float *pcm, const int64_t *starts, const int64_t *ends, int32_t n_windows,
                      aid_match_row *rows, int32_t *nrows, void *stream) {
    if (!e || n_windows < 0 || (n_windows > 0 && (!starts || !ends || !rows || !nrows)))
        return fail(AID_ERR_INVALID, "aid_query_windows: bad argument");
    for (int c = 0; c < n_windows; ++c)
        if (starts[c] < 0 || ends[c] < starts[c]) return fail(AID_ERR_INVALID, "aid_query_windows: bad window");
    if (n_windows > 0 && !pcm) return fail(AID_ERR_INVALID, "aid_query_windows: null pcm");
    if (n_windows == 0) return AID_OK;
    // one critical section, as aid_query_pcm: K1 reads every window in place (they may overlap), then K5
    std::lock_guard<std::mutex> lk(e->mu);
    if (int rc = ensure_index(e)) return rc;
    if (int rc = extract_locked(e, pcm, starts, n_windows, AID_PCM_DEVICE, stream, ends)) return rc;
    return query_extracted_locked(e, rows, nrows);
}

}  // extern "C"

extern "C" int aid_downmix(aid_engine *e, const float *stereo, int64_t n_frames, float *mono, void *stream) {
    if (!e || n_frames < 0 || (n_frames > 0 && (!stereo || !mono))) return fail(AID_ERR_INVALID, "aid_downmix: bad argument");
    if (((uintptr_t)stereo & 15) || ((uintptr_t)mono & 7)) return fail(AID_ERR_INVALID, "aid_downmix: misaligned buffers");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    launch_downmix(stereo, n_frames, mono, s);
    HIP_TRY(hipGetLastError());
    return AID_OK;
}

// ---------------------------------------------------------------- batched exact lane

extern "C" int aid_exact_windows(int64_t n, int32_t sample_rate, int64_t *lo, int64_t *len, int32_t *mode) {
    if (n < 0 || sample_rate <= 0 || !lo || !len || !mode) return fail(AID_ERR_INVALID, "aid_exact_windows: bad argument");
    // app/search/exact.py: duration = samples / SAMPLE_RATE (:389-390); <= 5.0 s -> SUB_WINDOWS
    // (:48-52, :103), stop = min(b, duration), piece = _extract_pcm_window(a, stop) if a < stop
    // (:150-160), whose byte bounds are int(t * SAMPLE_RATE) * 4 clamped to the data (:374-399)
    static const double kSub[3][2] = {{0.0, 3.5}, {0.75, 4.25}, {1.5, 5.0}};
    const double sr = (double)sample_rate, dur = (double)n / sr;
    if (!(dur <= 5.0)) {
        *mode = 0;
        lo[0] = 0;
        len[0] = n;
        return 1;
    }
    *mode = 1;
    for (int w = 0; w < 3; ++w) {
        const double a = kSub[w][0], stop = std::min(kSub[w][1], dur);
        int64_t l = 0, h = 0;
        if (a < stop) {
            l = std::min(std::max<int64_t>((int64_t)(a * sr), 0), n);
            h = std::max(l, std::min<int64_t>((int64_t)(stop * sr), n));
        }
        lo[w] = l;
        len[w] = h - l;  // 0: the reference sends no query for this window
    }
    return 3;
}

static int exact_lane_locked(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                             int32_t max_out, aid_exact_row *out, int32_t *n_out, void *stream);

extern "C" int aid_exact_lane(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                              int32_t max_out, aid_exact_row *out, int32_t *n_out, void *stream) {
    if (!e || !offsets || n_clips < 0 || max_out <= 0 || (n_clips > 0 && (!out || !n_out)))
        return fail(AID_ERR_INVALID, "aid_exact_lane: bad argument");
    if (loc != AID_PCM_HOST && loc != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "aid_exact_lane: bad pcm_location");
    for (int c = 0; c < n_clips; ++c)
        if (offsets[c + 1] < offsets[c] || offsets[c] < 0)
            return fail(AID_ERR_INVALID, "aid_exact_lane: offsets must be non-decreasing and >= 0");
    if (n_clips > 0 && !pcm && offsets[n_clips] > offsets[0]) return fail(AID_ERR_INVALID, "aid_exact_lane: null pcm");
    if (e->cfg.max_results > 256) return fail(AID_ERR_INVALID, "aid_exact_lane: engine max_results must be <= 256");
    if (n_clips == 0) return AID_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    return drain_host_copy(e, loc, stream, exact_lane_locked(e, pcm, offsets, n_clips, loc, max_out, out, n_out, stream));
}

static int exact_lane_locked(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc,
                             int32_t max_out, aid_exact_row *out, int32_t *n_out, void *stream) {
    HIP_TRY(hipSetDevice(e->device));
    if (int rc = ensure_index(e)) return rc;
    hipStream_t s = pick_stream(e, stream);
    if (e->last_stream && e->last_stream != s) HIP_TRY(hipStreamSynchronize(e->last_stream));
    // fan-out plan (host): clip_win = (first window, windows, mode). A window of odd length n is
    // extracted as n - 1 samples: with an even hop, frames(n) = frames(n - 1) for odd n and no
    // frame reaches the last sample, so the records are the same. K1 reads the windows in place
    // (wstart / wend into the clips' PCM; at 44.1 kHz the 0.75 s window starts at an odd sample);
    // the LANE_GATHER A/B copies them to even offsets of a staging buffer first (xoff)
    std::vector<int64_t> wdesc, xoff(1, 0), wstart, wend;
    std::vector<int32_t> clipwin(3 * (size_t)n_clips);
    int64_t staged = 0, max_len = 0;
    for (int c = 0; c < n_clips; ++c) {
        int64_t lo[3], len[3];
        int32_t mode = 0;
        const int nw = aid_exact_windows(offsets[c + 1] - offsets[c], e->cfg.sample_rate, lo, len, &mode);
        clipwin[3 * c] = (int32_t)(xoff.size() - 1);
        int used = 0;
        for (int w = 0; w < nw; ++w) {
            if (len[w] <= 0) continue;  // the reference sends no query for an empty piece
            const int64_t m = len[w] & ~(int64_t)1;
            wdesc.push_back(offsets[c] - offsets[0] + lo[w]);
            wdesc.push_back(m);
            wdesc.push_back(staged);
            wstart.push_back(offsets[c] - offsets[0] + lo[w]);
            wend.push_back(offsets[c] - offsets[0] + lo[w] + m);
            staged += m;
            xoff.push_back(staged);
            max_len = std::max(max_len, m);
            ++used;
        }
        clipwin[3 * c + 1] = used;
        clipwin[3 * c + 2] = mode;
    }
    const int n_win = (int)(xoff.size() - 1);
    const float *src = pcm + offsets[0];
    if (loc == AID_PCM_HOST) {
        const int64_t n_all = offsets[n_clips] - offsets[0];
        HIP_TRY(e->x_in.reserve((size_t)std::max<int64_t>(n_all, 1)));
        if (n_all > 0) HIP_TRY(hipMemcpyAsync(e->x_in.p, src, n_all * sizeof(float), hipMemcpyHostToDevice, s));
        src = e->x_in.p;
    }
    HIP_TRY(e->x_clipwin.reserve(clipwin.size()));
    HIP_TRY(hipMemcpyAsync(e->x_clipwin.p, clipwin.data(), clipwin.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(e->x_nout.reserve((size_t)n_clips));
    HIP_TRY(e->x_out.reserve((size_t)n_clips * max_out * 3));
    std::vector<int32_t> nrows(std::max(n_win, 1), 0);
    const int mr = e->cfg.max_results;
    if (n_win > 0) {
        if (e->lane_gather) {
            HIP_TRY(e->x_wdesc.reserve(wdesc.size()));
            HIP_TRY(hipMemcpyAsync(e->x_wdesc.p, wdesc.data(), wdesc.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIP_TRY(e->x_win.reserve((size_t)std::max<int64_t>(staged, 2)));
            launch_window_gather(src, e->x_wdesc.p, n_win, max_len, e->x_win.p, s);
            HIP_TRY(hipGetLastError());
            if (int rc = extract_locked(e, e->x_win.p, xoff.data(), n_win, AID_PCM_DEVICE, s)) return rc;
        } else {
            if (int rc = extract_locked(e, src, wstart.data(), n_win, AID_PCM_DEVICE, s, wend.data())) return rc;
        }
        if (int rc = check_query_frames(e)) return rc;
        HIP_TRY(e->q_start.reserve(n_win));
        HIP_TRY(upload_clip_base(e, n_win, s));
        if (int rc = run_queries(e, e->records.p, e->q_start.p, e->counts.p, n_win, (int64_t)e->records.n, nullptr,
                                 nrows.data(), s))
            return rc;
        HIP_TRY(e->q_nrows.reserve((size_t)n_win));
        HIP_TRY(hipMemcpyAsync(e->q_nrows.p, nrows.data(), n_win * sizeof(int32_t), hipMemcpyHostToDevice, s));
    } else {
        HIP_TRY(e->q_nrows.reserve(1));
        HIP_TRY(e->q_rows.reserve((size_t)mr * 5));
        HIP_TRY(hipMemsetAsync(e->q_nrows.p, 0, sizeof(int32_t), s));
    }
    const double sec = (double)e->cfg.hop / (double)e->cfg.sample_rate;
    launch_exact_consensus(e->q_rows.p, e->q_nrows.p, mr, e->x_clipwin.p, n_clips, sec, max_out, e->x_out.p, e->x_nout.p,
                           s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(n_out, e->x_nout.p, (size_t)n_clips * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out, e->x_out.p, (size_t)n_clips * max_out * sizeof(aid_exact_row), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->last_stream = s;
    return AID_OK;
}

