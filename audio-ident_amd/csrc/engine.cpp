// engine.cpp -- host side of libaidfp.so: the C ABI of include/aidfp.h.
//
// Owns one GPU's tables and workspaces, builds the per-call clip descriptors
// (one small H2D copy), launches K1..K3 on the caller's stream and exposes the
// results. Replaces the `olaf_c` process boundary of the reference
// (audio-ident-service/app/audio/fingerprint.py:87-270).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/aidfp.h"
#include "aidfp_device.h"
#include "aidfp_layout.h"

namespace aid {
void launch_stft_power(const float *pcm, const ClipDesc *clips, int n_clips, int64_t total_strips, int hop,
                       const Tables *tab, float *out, bool logmag, hipStream_t s);
void launch_peak_pick(const float *power, const ClipDesc *clips, int n_clips, int64_t total_strips, float thr,
                      uint64_t *mask, hipStream_t s);
void launch_landmarks(const uint64_t *mask, const ClipDesc *clips, int n_clips, int64_t total_chunks,
                      int64_t *chunk_counts, uint64_t *records, int64_t *clip_counts, bool write, hipStream_t s);
void launch_synth(float *out, const uint32_t *tracks, const int64_t *starts, int n_clips, int64_t n, int sr,
                  int noise_a, uint32_t salt, const int16_t *sin_tab, hipStream_t s);
}  // namespace aid

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
        if (p) (void)hipFree(p);
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

struct ProfEvent {
    int kernel;
    hipEvent_t a, b;
};

}  // namespace

struct aid_engine {
    aid_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    Tables *d_tab = nullptr;
    int16_t *d_sin = nullptr;

    DevBuf<float> pcm_stage;
    DevBuf<float> power;
    DevBuf<uint64_t> mask;
    DevBuf<ClipDesc> desc;
    DevBuf<int64_t> chunk_counts;
    DevBuf<uint64_t> records;
    DevBuf<int64_t> counts;
    DevBuf<uint32_t> synth_tracks;
    DevBuf<int64_t> synth_starts;

    ClipDesc *h_desc = nullptr;  // pinned
    size_t h_desc_cap = 0;
    std::vector<int64_t> clip_base;  // host copy of desc[c].hash_base
    std::vector<int64_t> clip_frames;
    int n_clips = 0;
    int64_t total_frames = 0, total_strips = 0, total_chunks = 0, total_records = 0;
    hipStream_t last_stream = nullptr;
    bool have_result = false;

    bool profiling = false;
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

struct ProfScope {
    aid_engine *e;
    int k;
    hipStream_t s;
    hipEvent_t a = nullptr;
    ProfScope(aid_engine *e_, int k_, hipStream_t s_) : e(e_), k(k_), s(s_) {
        if (e->profiling && (a = take_event(e))) (void)hipEventRecord(a, s);
    }
    ~ProfScope() {
        if (!a) return;
        hipEvent_t b = take_event(e);
        if (!b) return;
        (void)hipEventRecord(b, s);
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
    out->min_match = 5;
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
    if (!(c.peak_threshold > 0.0f)) return fail(AID_ERR_INVALID, "peak_threshold must be > 0");
    if (c.min_match <= 0) c.min_match = 5;
    if (c.max_results <= 0) c.max_results = 50;
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
    hipError_t he = hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        delete e;
        return fail(AID_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(he));
    }
    Tables *h = new Tables();
    build_tables(*h);
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
    e->mask.release();
    e->desc.release();
    e->chunk_counts.release();
    e->records.release();
    e->counts.release();
    e->synth_tracks.release();
    e->synth_starts.release();
    if (e->h_desc) (void)hipHostFree(e->h_desc);
    if (e->d_tab) (void)hipFree(e->d_tab);
    if (e->d_sin) (void)hipFree(e->d_sin);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
}

int aid_engine_config(const aid_engine *e, aid_config *out) {
    if (!e || !out) return fail(AID_ERR_INVALID, "null argument");
    *out = e->cfg;
    return AID_OK;
}

int64_t aid_num_frames(const aid_engine *e, int64_t n) { return e ? num_frames(n, e->cfg.hop) : 0; }

int64_t aid_hash_capacity(const aid_engine *e, int64_t n) { return e ? hash_capacity(num_frames(n, e->cfg.hop)) : 0; }

int aid_extract(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t loc, void *stream) {
    if (!e || !offsets || n_clips < 0) return fail(AID_ERR_INVALID, "aid_extract: bad argument");
    if (loc != AID_PCM_HOST && loc != AID_PCM_DEVICE) return fail(AID_ERR_INVALID, "aid_extract: bad pcm_location");
    if (n_clips > 0 && !pcm && offsets[n_clips] > offsets[0]) return fail(AID_ERR_INVALID, "aid_extract: null pcm");
    for (int c = 0; c < n_clips; ++c)
        if (offsets[c + 1] < offsets[c] || offsets[c] < 0)
            return fail(AID_ERR_INVALID, "aid_extract: offsets must be non-decreasing and >= 0");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    const int hop = e->cfg.hop;

    // descriptors; host PCM is re-packed at even offsets
    if ((size_t)n_clips + 1 > e->h_desc_cap) {
        if (e->h_desc) HIP_TRY(hipHostFree(e->h_desc));
        e->h_desc = nullptr;
        e->h_desc_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&e->h_desc, sizeof(ClipDesc) * ((size_t)n_clips + 1)));
        e->h_desc_cap = (size_t)n_clips + 1;
    }
    // host PCM staging goes through the previous call's buffers: make sure they are idle
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    e->clip_base.assign(n_clips, 0);
    e->clip_frames.assign(n_clips, 0);
    int64_t frames = 0, strips = 0, chunks = 0, recs = 0, staged = 0, kstrips = 0;
    for (int c = 0; c < n_clips; ++c) {
        const int64_t n = offsets[c + 1] - offsets[c];
        const int64_t F = num_frames(n, hop);
        ClipDesc &d = e->h_desc[c];
        if (loc == AID_PCM_DEVICE) {
            if (offsets[c] & 1) return fail(AID_ERR_INVALID, "aid_extract: device clip offsets must be even");
            d.pcm_off = offsets[c];
        } else {
            d.pcm_off = staged;
            staged += (n + 1) & ~(int64_t)1;
        }
        d.frames = F;
        d.frame_base = frames;
        d.strip_base = strips;
        d.chunk_base = chunks;
        d.hash_base = recs;
        d.hash_cap = hash_capacity(F);
        d.stft_base = kstrips;
        e->clip_base[c] = recs;
        e->clip_frames[c] = F;
        frames += F;
        strips += (F + kPeakStrip - 1) / kPeakStrip;
        chunks += (F + kHashChunk - 1) / kHashChunk;
        recs += d.hash_cap;
        kstrips += (F + kStftStrip - 1) / kStftStrip;
    }
    HIP_TRY(e->desc.reserve((size_t)n_clips + 1));
    HIP_TRY(e->power.reserve((size_t)frames * kBins));
    HIP_TRY(e->mask.reserve((size_t)frames * kMaskWords));
    HIP_TRY(e->chunk_counts.reserve((size_t)chunks + 1));
    HIP_TRY(e->records.reserve((size_t)recs + 1));
    HIP_TRY(e->counts.reserve((size_t)n_clips + 1));
    const float *dpcm = pcm;
    if (loc == AID_PCM_HOST && staged > 0) {
        HIP_TRY(e->pcm_stage.reserve((size_t)staged));
        for (int c = 0; c < n_clips; ++c) {
            const int64_t n = offsets[c + 1] - offsets[c];
            if (n > 0)
                HIP_TRY(hipMemcpyAsync(e->pcm_stage.p + e->h_desc[c].pcm_off, pcm + offsets[c], n * sizeof(float),
                                       hipMemcpyHostToDevice, s));
        }
        dpcm = e->pcm_stage.p;
    }
    if (n_clips > 0)
        HIP_TRY(hipMemcpyAsync(e->desc.p, e->h_desc, sizeof(ClipDesc) * n_clips, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(e->counts.p, 0, sizeof(int64_t) * ((size_t)n_clips + 1), s));
    e->n_clips = n_clips;
    e->total_frames = frames;
    e->total_strips = strips;
    e->total_chunks = chunks;
    e->total_records = recs;
    if (frames > 0) {
        {
            ProfScope ps(e, AID_K_STFT, s);
            launch_stft_power(dpcm, e->desc.p, n_clips, kstrips, hop, e->d_tab, e->power.p, false, s);
        }
        {
            ProfScope ps(e, AID_K_PEAKS, s);
            launch_peak_pick(e->power.p, e->desc.p, n_clips, strips, e->cfg.peak_threshold, e->mask.p, s);
        }
        {
            ProfScope ps(e, AID_K_LANDMARK_COUNT, s);
            launch_landmarks(e->mask.p, e->desc.p, n_clips, chunks, e->chunk_counts.p, e->records.p, e->counts.p,
                             false, s);
        }
        {
            ProfScope ps(e, AID_K_LANDMARK_WRITE, s);
            launch_landmarks(e->mask.p, e->desc.p, n_clips, chunks, e->chunk_counts.p, e->records.p, e->counts.p,
                             true, s);
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
    const int64_t F = e->clip_frames[clip];
    if (F * kBins > cap) return fail(AID_ERR_INVALID, "output capacity too small");
    if (int rc = aid_sync(e)) return rc;
    if (F > 0) {
        int64_t fb = 0;
        for (int c = 0; c < clip; ++c) fb += e->clip_frames[c];
        HIP_TRY(hipMemcpy(out, e->power.p + fb * kBins, F * kBins * sizeof(float), hipMemcpyDeviceToHost));
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
        launch_stft_power(d_pcm, d_desc, 1, (F + kStftStrip - 1) / kStftStrip, e->cfg.hop, e->d_tab, d_out, true, s);
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

int aid_synth(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips, int64_t n,
              int32_t noise_a, uint32_t salt, void *stream) {
    if (!e || !dst || !tracks || !starts || n_clips < 0 || n < 0 || noise_a < 0)
        return fail(AID_ERR_INVALID, "aid_synth: bad argument");
    if (n_clips == 0 || n == 0) return AID_OK;
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = pick_stream(e, stream);
    if (e->last_stream) HIP_TRY(hipStreamSynchronize(e->last_stream));
    HIP_TRY(e->synth_tracks.reserve(n_clips));
    HIP_TRY(e->synth_starts.reserve(n_clips));
    HIP_TRY(hipMemcpyAsync(e->synth_tracks.p, tracks, n_clips * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->synth_starts.p, starts, n_clips * sizeof(int64_t), hipMemcpyHostToDevice, s));
    {
        ProfScope ps(e, AID_K_SYNTH, s);
        launch_synth(dst, e->synth_tracks.p, e->synth_starts.p, n_clips, n, e->cfg.sample_rate, noise_a, salt,
                     e->d_sin, s);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    return AID_OK;
}

int aid_profile_enable(aid_engine *e, int32_t on) {
    if (!e) return fail(AID_ERR_INVALID, "null engine");
    e->profiling = on != 0;
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
