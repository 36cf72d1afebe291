/* fp_dedup.c -- CPU oracle for K7 `dedup_scan`. TEST INFRASTRUCTURE ONLY (tests/ and the
 * cpu_baseline leg of bench_dedup.py). Restates audio-ident-service/app/audio/dedup.py:
 * `_fingerprint_similarity` (:127-166) -- (matching / (min_len*32)) * (min_len / max_len) in
 * binary64 -- and the scan of `check_content_duplicate` (:169-222): candidates with
 * duration*0.9 <= d <= duration*1.1 in catalog order, best by strict > from 0.0. Pinned to the
 * reference by tests/golden/ref_dedup.json (vectors captured from the reference itself). */
#include <stdint.h>

double fp_dedup_similarity(const uint32_t *a, int64_t la, const uint32_t *b, int64_t lb) {
    const int64_t mn = la < lb ? la : lb, mx = la < lb ? lb : la;
    if (mn == 0) return 0.0;
    uint64_t diff = 0;
    for (int64_t i = 0; i < mn; ++i) diff += (uint64_t)__builtin_popcount(a[i] ^ b[i]);
    const uint64_t matching = (uint64_t)mn * 32 - diff;
    return ((double)matching / (double)(mn * 32)) * ((double)mn / (double)mx);
}

void fp_dedup_scan(const uint32_t *cw, const int64_t *coff, const double *cdur, int64_t n, const uint32_t *qw,
                   const int64_t *qoff, const double *qdur, int64_t nq, int64_t *best_idx, double *best_sim) {
    for (int64_t q = 0; q < nq; ++q) {
        const double lo = qdur[q] * 0.9, hi = qdur[q] * 1.1;
        double best = 0.0;
        int64_t bi = -1;
        for (int64_t e = 0; e < n; ++e) {
            if (!(lo <= cdur[e] && cdur[e] <= hi)) continue;
            const double s = fp_dedup_similarity(qw + qoff[q], qoff[q + 1] - qoff[q], cw + coff[e], coff[e + 1] - coff[e]);
            if (s > best) {
                best = s;
                bi = e;
            }
        }
        best_idx[q] = bi;
        best_sim[q] = best;
    }
}
