// exact.hip -- batched exact lane: sub-window fan-out + consensus +
// thresholds + ranking for a batch of clips, on the device.
//
// Reference: audio-ident-service/app/search/exact.py
//   * clips of at most 5 s are queried as three overlapping sub-windows (SUB_WINDOWS :48-52,
//     the loop :132-173, _extract_pcm_window :374-399); longer clips whole (:176-191);
//   * _consensus_score (:220-293): per track (first-appearance order over window 0, 1, 2 rows)
//     the summed match_count; tracks seen in one window only keep max(total // 2, 1); the
//     offset is the median of the raw reference_start values (statistics.median);
//   * _matches_to_candidates (:296-332) for whole clips: summed count, median start;
//   * MIN_ALIGNED_HASHES = 8 (:33, :109), confidence = min(h / 20, 1) (:340-353), stable sort
//     by confidence descending, top-N (:118-121).
// Metadata enrichment (:447-496) stays with the caller (Python, Postgres in the reference).
//
// The lane extracts its sub-windows in place (K1's clip table takes overlapping windows); K8a
// `window_gather`, which copies each sub-window to an even offset of a staging buffer first, is
// the A/B behind aid_engine_force(LANE_GATHER). K8b `exact_consensus` runs one wave per clip over
// the K5 rows of its windows (<= 3 x max_results rows, staged in LDS).
#include "aidfp_device.h"

namespace aid {

struct ExactRow {  // == aid_exact_row (include/aidfp.h)
    uint32_t track;
    int32_t aligned_hashes;
    double offset_seconds;
    double confidence;
};

__global__ __launch_bounds__(256) void k_window_gather(const float *__restrict__ src, const int64_t *__restrict__ win,
                                                       int n_win, float *__restrict__ dst) {
    // win[3*w] = source offset, win[3*w+1] = length (even), win[3*w+2] = destination offset (even): float2
    // stores; float2 loads when the source is 8-B aligned too (every other window at 44.1 kHz starts odd)
    for (int w = blockIdx.y; w < n_win; w += gridDim.y) {
        const int64_t so = win[3 * w], n2 = win[3 * w + 1] >> 1, d = win[3 * w + 2];
        float2 *__restrict__ d2 = reinterpret_cast<float2 *>(dst + d);
        const float *s = src + so;
        const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
        if ((reinterpret_cast<uintptr_t>(s) & 7) == 0) {
            const float2 *__restrict__ s2 = reinterpret_cast<const float2 *>(s);
            for (int64_t i = i0; i < n2; i += step) d2[i] = s2[i];
        } else {
            for (int64_t i = i0; i < n2; i += step) d2[i] = make_float2(s[2 * i], s[2 * i + 1]);
        }
    }
}

constexpr int kExactMaxRows = 3 * 256;  // rows of one clip's windows staged in LDS (max_results <= 256)

__global__ __launch_bounds__(64) void k_exact_consensus(const int32_t *__restrict__ rows, const int32_t *__restrict__ nrows,
                                                        int mr, const int32_t *__restrict__ clip_win, double sec,
                                                        int max_out, ExactRow *__restrict__ out,
                                                        int32_t *__restrict__ n_out) {
    // clip_win[3*c] = first window (query) of clip c, [3*c+1] = windows (0..3), [3*c+2] = 1 for the
    // sub-window consensus (clip <= 5 s), 0 for the whole-clip aggregation
    __shared__ uint32_t s_track[kExactMaxRows];
    __shared__ int32_t s_count[kExactMaxRows];
    __shared__ int8_t s_win[kExactMaxRows];
    __shared__ double s_start[kExactMaxRows];
    __shared__ int32_t s_aligned[kExactMaxRows];  // per leader (first row of its track), -1 otherwise
    __shared__ double s_off[kExactMaxRows];
    __shared__ int s_n;
    const int c = blockIdx.x, lane = threadIdx.x;
    const int w0 = clip_win[3 * c], nw = clip_win[3 * c + 1], sub = clip_win[3 * c + 2];
    if (lane == 0) {
        int n = 0;
        for (int w = 0; w < nw; ++w) n += max(0, nrows[w0 + w]);
        s_n = n;
    }
    __syncthreads();
    const int n = s_n;
    // stage rows in first-appearance order: window 0's rows in K5 order, then window 1, 2
    for (int w = 0, base = 0; w < nw; ++w) {
        const int q = w0 + w, nq = max(0, nrows[q]);
        for (int i = lane; i < nq; i += 64) {
            const int32_t *r = rows + ((size_t)q * mr + i) * 5;  // count, track, d, tq_min, tq_max
            s_count[base + i] = r[0];
            s_track[base + i] = (uint32_t)r[1];
            s_win[base + i] = (int8_t)w;
            // reference_start = (tq0 + d) * sec, as the adapter builds OlafMatch (binary64)
            s_start[base + i] = (double)(r[3] + r[2]) * sec;
        }
        base += nq;
    }
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        const uint32_t t = s_track[i];
        bool leader = true;
        for (int j = 0; j < i && leader; ++j) leader = s_track[j] != t;
        int32_t aligned = -1;
        double off = 0.0;
        if (leader) {
            // K5 emits one row per track per query, so a track has <= 3 rows (one per window)
            double a = 0.0, b = 0.0, c3 = 0.0;
            int m = 0, total = 0, wins = 0, wmask = 0;
            for (int j = i; j < n; ++j) {
                if (s_track[j] != t) continue;
                total += s_count[j];
                const double x = s_start[j];
                if (m == 0) a = x;
                else if (m == 1) b = x;
                else c3 = x;
                ++m;
                if (!(wmask >> s_win[j] & 1)) { wmask |= 1 << s_win[j]; ++wins; }
            }
            // statistics.median: sorted; odd -> middle, even -> (lo + hi) / 2
            const double lo = fmin(a, b), hi = fmax(a, b);
            off = m == 1 ? a : m == 2 ? (lo + hi) / 2.0 : fmax(lo, fmin(hi, c3));
            aligned = (!sub || wins >= 2) ? total : max(total / 2, 1);
            if (aligned < 8) aligned = -1;  // MIN_ALIGNED_HASHES
        }
        s_aligned[i] = aligned;
        s_off[i] = off;
    }
    __syncthreads();
    int kept = 0;
    for (int i = lane; i < n; i += 64) {
        const int32_t a = s_aligned[i];
        if (a < 0) continue;
        ++kept;
        const double conf = min((double)a / 20.0, 1.0);
        // stable sort by confidence, descending: rank = higher confidences + equal ones listed earlier
        int rank = 0;
        for (int j = 0; j < n; ++j) {
            const int32_t b = s_aligned[j];
            if (b < 0 || j == i) continue;
            const double cj = min((double)b / 20.0, 1.0);
            rank += (cj > conf) || (cj == conf && j < i);
        }
        if (rank < max_out) {
            ExactRow o;
            o.track = s_track[i];
            o.aligned_hashes = a;
            o.offset_seconds = s_off[i];
            o.confidence = conf;
            out[(size_t)c * max_out + rank] = o;
        }
    }
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
    if (lane == 0) n_out[c] = min(kept, max_out);
}

// Rows of a K5 batch written to scratch (x_dst) land at their query's slot of the device row
// table, so the consensus reads every query's rows from one place.
__global__ __launch_bounds__(256) void k_rows_scatter(const int32_t *__restrict__ src, const int32_t *__restrict__ order,
                                                      int n, int mr, int32_t *__restrict__ dst) {
    for (int i = blockIdx.y; i < n; i += gridDim.y) {
        const int q = order[i];
        for (int k = threadIdx.x; k < mr * 5; k += blockDim.x) dst[(size_t)q * mr * 5 + k] = src[(size_t)i * mr * 5 + k];
    }
}

void launch_window_gather(const float *src, const int64_t *win, int n_win, int64_t max_len, float *dst, hipStream_t s) {
    if (n_win <= 0 || max_len <= 0) return;
    int64_t bx = (max_len + 1023) / 1024;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(k_window_gather, dim3((unsigned)bx, (unsigned)(n_win < 65535 ? n_win : 65535)), dim3(256), 0, s,
                       src, win, n_win, dst);
}

void launch_exact_consensus(const int32_t *rows, const int32_t *nrows, int mr, const int32_t *clip_win, int n_clips,
                            double sec, int max_out, void *out, int32_t *n_out, hipStream_t s) {
    if (n_clips <= 0) return;
    hipLaunchKernelGGL(k_exact_consensus, dim3((unsigned)n_clips), dim3(64), 0, s, rows, nrows, mr, clip_win, sec,
                       max_out, reinterpret_cast<ExactRow *>(out), n_out);
}

void launch_rows_scatter(const int32_t *src, const int32_t *order, int n, int mr, int32_t *dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rows_scatter, dim3(1, (unsigned)(n < 65535 ? n : 65535)), dim3(256), 0, s, src, order, n, mr,
                       dst);
}

}  // namespace aid
