// resample_design.h -- host-side filter design of the PCM front-end (spec/FPSPEC.md 8):
// scipy.signal.resample_poly's Kaiser(5) windowed-sinc low-pass (firwin(2*hl+1, 1/max(up,down))
// * up), designed in binary64 in a pinned order and rounded once to binary32, then laid out
// per phase for the GPU: row p holds taps[p + j*up] for j < J (zero past the filter).
#pragma once
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

namespace aid {

struct ResamplePlan {
    int32_t up = 1, down = 1, hl = 0, J = 0;
};

inline bool resample_plan(int32_t sr_in, int32_t sr_out, ResamplePlan &p) {
    if (sr_in <= 0 || sr_out <= 0) return false;
    const int64_t g = std::gcd((int64_t)sr_in, (int64_t)sr_out);
    p.up = (int32_t)(sr_out / g);
    p.down = (int32_t)(sr_in / g);
    const int32_t R = std::max(p.up, p.down);
    p.hl = 10 * R;
    p.J = (2 * p.hl + 1 + p.up - 1) / p.up;
    return true;
}

inline double resample_i0(double z) {  // sum_j ((z/2)^j / j!)^2 in j order
    const double q = 0.25 * z * z;
    double term = 1.0, sum = 1.0;
    for (int j = 1; j < 500; ++j) {
        term = term * q / ((double)j * (double)j);
        sum += term;
        if (term < 1e-17 * sum) break;
    }
    return sum;
}

// phase-major table [up][J]
inline std::vector<float> resample_phase_taps(const ResamplePlan &p) {
    const int32_t R = std::max(p.up, p.down), N = 2 * p.hl + 1;
    const double fc = 1.0 / (double)R, i0b = resample_i0(5.0);
    std::vector<double> h(N);
    for (int32_t k = 0; k < N; ++k) {
        const double m = (double)(k - p.hl);
        const double u = fc * m;
        const double sn = (u == 0.0) ? 1.0 : std::sin(M_PI * u) / (M_PI * u);
        const double r = m / (double)p.hl;
        const double w = resample_i0(5.0 * std::sqrt(1.0 - r * r)) / i0b;
        h[k] = fc * sn * w;
    }
    double s = 0.0;
    for (int32_t k = 0; k < N; ++k) s += h[k];
    std::vector<float> t((size_t)p.up * p.J, 0.0f);
    for (int32_t ph = 0; ph < p.up; ++ph)
        for (int32_t j = 0; j < p.J; ++j) {
            const int64_t k = ph + (int64_t)j * p.up;
            if (k < N) t[(size_t)ph * p.J + j] = (float)(h[k] / s * (double)p.up);
        }
    return t;
}

}  // namespace aid
