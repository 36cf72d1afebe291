/* fp_resample.c -- CPU oracle for the PCM front-end (spec/FPSPEC.md 8): stereo downmix +
 * rational polyphase resampling. TEST INFRASTRUCTURE ONLY: called by tests/ (and nowhere
 * in the product path) to check the GPU kernel (audio-ident_amd/csrc/resample.hip).
 *
 * Replaces ffmpeg's `-ac 1 -ar <rate>` in the reference
 * (audio-ident-service/app/audio/decode.py:41-60). ffmpeg's swr filter is not reproducible
 * here, so the filter restates scipy.signal.resample_poly (scipy 1.15.3, signal/_signaltools.py:
 * firwin(2*hl+1, 1/max(up,down), window=('kaiser', 5.0)) * up, output c = m*down + hl), pinned
 * against scipy itself by tests/test_resample_oracle.py (float64 scipy vs this binary32 code).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a;
}

/* I0(z) = sum_j ((z/2)^j / j!)^2, in j order, until a term drops below 1e-17 of the sum */
static double bessel_i0(double z) {
    const double q = 0.25 * z * z;
    double term = 1.0, sum = 1.0;
    for (int j = 1; j < 500; ++j) {
        term = term * q / ((double)j * (double)j);
        sum += term;
        if (term < 1e-17 * sum) break;
    }
    return sum;
}

/* ratio of sr_in -> sr_out: up/down, taps per phase J; returns 0 on bad rates */
int fp_resample_ratio(int32_t sr_in, int32_t sr_out, int32_t *up, int32_t *down, int32_t *hl, int32_t *J) {
    if (sr_in <= 0 || sr_out <= 0) return 0;
    const int64_t g = gcd64(sr_in, sr_out);
    *up = (int32_t)(sr_out / g);
    *down = (int32_t)(sr_in / g);
    const int32_t R = *up > *down ? *up : *down;
    *hl = 10 * R;
    const int32_t N = 2 * *hl + 1;
    *J = (N + *up - 1) / *up;
    return 1;
}

/* taps[k], k < 2*hl+1 (binary64 design, rounded once) */
void fp_resample_taps(int32_t up, int32_t down, float *taps) {
    const int32_t R = up > down ? up : down;
    const int32_t hl = 10 * R, N = 2 * hl + 1;
    const double fc = 1.0 / (double)R, i0b = bessel_i0(5.0);
    double *h = (double *)malloc(sizeof(double) * N);
    double s = 0.0;
    for (int32_t k = 0; k < N; ++k) {
        const double m = (double)(k - hl);
        const double u = fc * m;
        const double sn = (u == 0.0) ? 1.0 : sin(M_PI * u) / (M_PI * u);
        const double r = m / (double)hl;
        const double w = bessel_i0(5.0 * sqrt(1.0 - r * r)) / i0b;
        h[k] = fc * sn * w;
    }
    for (int32_t k = 0; k < N; ++k) s += h[k];
    for (int32_t k = 0; k < N; ++k) taps[k] = (float)(h[k] / s * (double)up);
    free(h);
}

int64_t fp_resample_len(int64_t n, int32_t sr_in, int32_t sr_out) {
    int32_t up, down, hl, J;
    if (n <= 0 || !fp_resample_ratio(sr_in, sr_out, &up, &down, &hl, &J)) return 0;
    return (n * up + down - 1) / down;
}

/* x: n frames of `channels` (1 or 2, interleaved) float32; y: fp_resample_len(n) samples */
int64_t fp_resample(const float *x, int64_t n, int32_t channels, int32_t sr_in, int32_t sr_out, float *y) {
    int32_t up, down, hl, J;
    if (n <= 0 || (channels != 1 && channels != 2) || !fp_resample_ratio(sr_in, sr_out, &up, &down, &hl, &J))
        return 0;
    float *mono = (float *)malloc(sizeof(float) * n);
    for (int64_t i = 0; i < n; ++i) mono[i] = channels == 2 ? (x[2 * i] + x[2 * i + 1]) * 0.5f : x[i];
    const int64_t n_out = (n * up + down - 1) / down;
    if (up == down) {
        memcpy(y, mono, sizeof(float) * n);
        free(mono);
        return n;
    }
    const int32_t N = 2 * hl + 1;
    float *taps = (float *)malloc(sizeof(float) * N);
    fp_resample_taps(up, down, taps);
    for (int64_t m = 0; m < n_out; ++m) {
        const int64_t c = m * down + hl;
        const int64_t p = c % up, i0 = c / up;
        float acc = 0.0f;
        for (int32_t j = 0; j < J; ++j) {
            const int64_t k = p + (int64_t)j * up, i = i0 - j;
            const float t = k < N ? taps[k] : 0.0f;
            const float v = (i >= 0 && i < n) ? mono[i] : 0.0f;
            acc = fmaf(t, v, acc);
        }
        y[m] = acc;
    }
    free(taps);
    free(mono);
    return n_out;
}
