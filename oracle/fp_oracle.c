/*
 * fp_oracle.c -- CPU restatement of spec/FPSPEC.md (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline -- never as the product
 * path. The product path is audio-ident_amd/csrc (HIP, gfx950).
 *
 * What it restates: the fingerprint arithmetic that the reference delegates to
 * the external `olaf_c` binary (audio-ident-service/app/audio/fingerprint.py:
 * 117-125 store, 185-193 query). Olaf is not vendored in /root/reference and is
 * not installed in this image, so the hash arithmetic is
 * **parity unpinned by the reference**: this file follows the build-owned
 * spec/FPSPEC.md and is pinned instead by (a) a float64 numpy spectrogram
 * (tolerance), (b) a brute-force peak definition and (c) known-answer tests in
 * tests/test_oracle.py.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; every float op below is
 * one correctly rounded binary32 op, fmaf is the single-rounding FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define FP_N 2048
#define FP_M 1024
#define FP_BINS 1024
#define FP_PEAK_DT 7
#define FP_PEAK_DF 15
#define FP_ZONE_DT 63
#define FP_ZONE_DF 127
#define FP_FAN 10

typedef struct { float re, im; } cpx;

static float g_win[FP_N];
static cpx g_t16[16], g_t64[64], g_t1k[1024], g_t2k[1024];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static cpx tw(int j, int L) {
    cpx w;
    w.re = (float)cos(2.0 * M_PI * (double)j / (double)L);
    w.im = (float)(-sin(2.0 * M_PI * (double)j / (double)L));
    return w;
}

static void init_tables(void) {
    for (int j = 0; j < FP_N; ++j)
        g_win[j] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)j / 2048.0));
    for (int j = 0; j < 16; ++j) g_t16[j] = tw(j, 16);
    for (int j = 0; j < 64; ++j) g_t64[j] = tw(j, 64);
    for (int j = 0; j < 1024; ++j) g_t1k[j] = tw(j, 1024);
    for (int j = 0; j < 1024; ++j) g_t2k[j] = tw(j, 2048);
}

static inline cpx cadd(cpx a, cpx b) { cpx r = {a.re + b.re, a.im + b.im}; return r; }
static inline cpx csub(cpx a, cpx b) { cpx r = {a.re - b.re, a.im - b.im}; return r; }
static inline cpx cmul(cpx x, cpx w) {
    cpx r;
    r.re = fmaf(x.re, w.re, -(x.im * w.im));
    r.im = fmaf(x.re, w.im, x.im * w.re);
    return r;
}

/* FPSPEC 3: DFT4 */
static inline void dft4(cpx x0, cpx x1, cpx x2, cpx x3, cpx *y) {
    cpx t0 = cadd(x0, x2), t1 = csub(x0, x2), t2 = cadd(x1, x3), t3 = csub(x1, x3);
    y[0] = cadd(t0, t2);
    y[2] = csub(t0, t2);
    y[1].re = t1.re + t3.im; y[1].im = t1.im - t3.re;
    y[3].re = t1.re - t3.im; y[3].im = t1.im + t3.re;
}

/* FPSPEC 3: DFT16 (radix 4x4) */
static void dft16(const cpx *v, cpx *out) {
    cpx s[4][4];
    for (int b = 0; b < 4; ++b) {
        dft4(v[b], v[b + 4], v[b + 8], v[b + 12], s[b]);
        for (int c = 0; c < 4; ++c)
            if (b * c) s[b][c] = cmul(s[b][c], g_t16[b * c]);
    }
    for (int c = 0; c < 4; ++c) {
        cpx y[4];
        dft4(s[0][c], s[1][c], s[2][c], s[3][c], y);
        for (int d = 0; d < 4; ++d) out[c + 4 * d] = y[d];
    }
}

/* FPSPEC 4: power spectrum of one frame (bins 0..1023) */
static void frame_power(const float *x, float *P) {
    cpx z[FP_M], A[16][64], Z[FP_M];
    for (int m = 0; m < FP_M; ++m) {
        z[m].re = x[2 * m] * g_win[2 * m];
        z[m].im = x[2 * m + 1] * g_win[2 * m + 1];
    }
    for (int n2 = 0; n2 < 64; ++n2) {
        cpx v[16], o[16];
        for (int n1 = 0; n1 < 16; ++n1) v[n1] = z[64 * n1 + n2];
        dft16(v, o);
        for (int k1 = 0; k1 < 16; ++k1)
            A[k1][n2] = (n2 * k1) ? cmul(o[k1], g_t1k[n2 * k1]) : o[k1];
    }
    for (int k1 = 0; k1 < 16; ++k1) {
        cpx B[4][16];
        for (int m2 = 0; m2 < 4; ++m2) {
            cpx v[16];
            for (int m1 = 0; m1 < 16; ++m1) v[m1] = A[k1][4 * m1 + m2];
            dft16(v, B[m2]);
            for (int j1 = 0; j1 < 16; ++j1)
                if (m2 * j1) B[m2][j1] = cmul(B[m2][j1], g_t64[m2 * j1]);
        }
        for (int j1 = 0; j1 < 16; ++j1) {
            cpx y[4];
            dft4(B[0][j1], B[1][j1], B[2][j1], B[3][j1], y);
            for (int j2 = 0; j2 < 4; ++j2) Z[k1 + 16 * j1 + 256 * j2] = y[j2];
        }
    }
    for (int k = 0; k < FP_BINS; ++k) {
        cpx p = Z[k], q = Z[(FP_M - k) & (FP_M - 1)];
        cpx o; o.re = p.im + q.im; o.im = q.re - p.re;
        float er = p.re + q.re, ei = p.im - q.im;
        cpx t = cmul(o, g_t2k[k]);
        float xr = er + t.re, xi = ei + t.im;
        P[k] = fmaf(xr, xr, xi * xi) * 0.25f;
    }
}

int64_t fp_num_frames(int64_t n, int hop) {
    if (hop <= 0 || n < FP_N) return 0;
    return 1 + (n - FP_N) / hop;
}

/* power spectrogram [F][1024] */
int64_t fp_stft_power(const float *x, int64_t n, int hop, float *P) {
    pthread_once(&g_once, init_tables);
    int64_t F = fp_num_frames(n, hop);
    for (int64_t t = 0; t < F; ++t) frame_power(x + t * hop, P + t * FP_BINS);
    return F;
}

/* FPSPEC 5, separable form: before-max must be < p, after-max must be <= p */
int64_t fp_peaks(const float *P, int64_t F, float thr, int32_t *pt, int32_t *pk, int64_t cap) {
    if (F <= 0) return 0;
    float *Lm = (float *)malloc(sizeof(float) * F * FP_BINS);
    float *Rm = (float *)malloc(sizeof(float) * F * FP_BINS);
    float *Fm = (float *)malloc(sizeof(float) * F * FP_BINS);
    for (int64_t t = 0; t < F; ++t) {
        const float *row = P + t * FP_BINS;
        for (int k = 0; k < FP_BINS; ++k) {
            float l = 0.0f, r = 0.0f;
            for (int d = 1; d <= FP_PEAK_DF; ++d) {
                if (k - d >= 0 && row[k - d] > l) l = row[k - d];
                if (k + d < FP_BINS && row[k + d] > r) r = row[k + d];
            }
            Lm[t * FP_BINS + k] = l;
            Rm[t * FP_BINS + k] = r;
            float f = row[k] > l ? row[k] : l;
            Fm[t * FP_BINS + k] = f > r ? f : r;
        }
    }
    int64_t n = 0;
    for (int64_t t = 0; t < F; ++t) {
        for (int k = 1; k < FP_BINS; ++k) {
            float p = P[t * FP_BINS + k];
            if (!(p > thr)) continue;
            float before = Lm[t * FP_BINS + k], after = Rm[t * FP_BINS + k];
            for (int d = 1; d <= FP_PEAK_DT; ++d) {
                if (t - d >= 0 && Fm[(t - d) * FP_BINS + k] > before) before = Fm[(t - d) * FP_BINS + k];
                if (t + d < F && Fm[(t + d) * FP_BINS + k] > after) after = Fm[(t + d) * FP_BINS + k];
            }
            if (p > before && p >= after) {
                if (n < cap) { pt[n] = (int32_t)t; pk[n] = k; }
                ++n;
            }
        }
    }
    free(Lm); free(Rm); free(Fm);
    return n;
}

/* FPSPEC 5, literal definition (O(F*B*465)): used only to pin fp_peaks on small cases */
int64_t fp_peaks_bruteforce(const float *P, int64_t F, float thr, int32_t *pt, int32_t *pk, int64_t cap) {
    int64_t n = 0;
    for (int64_t t = 0; t < F; ++t)
        for (int k = 1; k < FP_BINS; ++k) {
            float p = P[t * FP_BINS + k];
            if (!(p > thr)) continue;
            int ok = 1;
            for (int64_t u = t - FP_PEAK_DT; u <= t + FP_PEAK_DT && ok; ++u) {
                if (u < 0 || u >= F) continue;
                for (int j = k - FP_PEAK_DF; j <= k + FP_PEAK_DF; ++j) {
                    if (j < 0 || j >= FP_BINS || (u == t && j == k)) continue;
                    float q = P[u * FP_BINS + j];
                    int after = (u > t) || (u == t && j > k);
                    if (q > p || (q == p && !after)) { ok = 0; break; }
                }
            }
            if (ok) {
                if (n < cap) { pt[n] = (int32_t)t; pk[n] = k; }
                ++n;
            }
        }
    return n;
}

/* FPSPEC 6 */
int64_t fp_hashes(const int32_t *pt, const int32_t *pk, int64_t np, uint32_t *hash, uint32_t *t1, int64_t cap) {
    int64_t n = 0;
    for (int64_t i = 0; i < np; ++i) {
        int got = 0;
        for (int64_t j = i + 1; j < np && got < FP_FAN; ++j) {
            int32_t dt = pt[j] - pt[i];
            if (dt <= 0) continue;
            if (dt > FP_ZONE_DT) break;
            int32_t df = pk[j] - pk[i];
            if (df < -FP_ZONE_DF || df > FP_ZONE_DF) continue;
            if (n < cap) {
                hash[n] = ((uint32_t)(pk[i] & 0x3FF) << 22) | ((uint32_t)(pk[j] & 0x3FF) << 12) |
                          ((uint32_t)dt & 0xFFF);
                t1[n] = (uint32_t)pt[i];
            }
            ++n; ++got;
        }
    }
    return n;
}

int64_t fp_peak_capacity(int64_t F) { return 64 * ((F + 7) / 8); }

/* whole pipeline for one clip; returns number of hashes (or -1 on alloc failure) */
int64_t fp_fingerprint(const float *x, int64_t n, int hop, float thr, uint32_t *hash, uint32_t *t1, int64_t cap) {
    int64_t F = fp_num_frames(n, hop);
    if (F <= 0) return 0;
    float *P = (float *)malloc(sizeof(float) * F * FP_BINS);
    int64_t pc = fp_peak_capacity(F);
    int32_t *pt = (int32_t *)malloc(sizeof(int32_t) * pc), *pk = (int32_t *)malloc(sizeof(int32_t) * pc);
    if (!P || !pt || !pk) { free(P); free(pt); free(pk); return -1; }
    fp_stft_power(x, n, hop, P);
    int64_t np = fp_peaks(P, F, thr, pt, pk, pc);
    if (np > pc) np = pc; /* cannot happen (packing bound) */
    int64_t nh = fp_hashes(pt, pk, np, hash, t1, cap);
    free(P); free(pt); free(pk);
    return nh;
}

/* ---- multi-threaded batch (CPU baseline): clips of equal length n ---- */
typedef struct {
    const float *x; int64_t n; int hop; float thr; int clips;
    uint32_t *hash, *t1; int64_t cap; int64_t *counts;
    int next; pthread_mutex_t mu;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int c = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (c >= j->clips) break;
        j->counts[c] = fp_fingerprint(j->x + (int64_t)c * j->n, j->n, j->hop, j->thr,
                                      j->hash + (int64_t)c * j->cap, j->t1 + (int64_t)c * j->cap, j->cap);
    }
    return NULL;
}

int fp_fingerprint_batch(const float *x, int64_t n, int clips, int hop, float thr, uint32_t *hash,
                         uint32_t *t1, int64_t cap, int64_t *counts, int threads) {
    pthread_once(&g_once, init_tables);
    if (threads < 1) threads = 1;
    batch_job j = {x, n, hop, thr, clips, hash, t1, cap, counts, 0, PTHREAD_MUTEX_INITIALIZER};
    pthread_t th[256];
    if (threads > 256) threads = 256;
    for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, batch_worker, &j);
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    return 0;
}
