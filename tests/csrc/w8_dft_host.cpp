// Host check of the in-register DFTs (fft_common.h dft<16>/dft<32>) and their W_8 forms
// (fft_w8.h dft16w/dft32w, S0 inputs): prints the max relative error of each against a
// double-precision DFT of the same float inputs.  Built and run by tests/test_w8_host.py.
#include <cmath>
#include <complex>
#include <cstdio>
#include <random>

#include "fft_w8.h"

using cd = std::complex<double>;

template <int R>
static double err(const float2 *in, const float2 *out) {
    double worst = 0, norm = 0;
    for (int k = 0; k < R; k++) {
        cd s = 0;
        for (int n = 0; n < R; n++) s += cd(in[n].x, in[n].y) * std::polar(1.0, -2 * M_PI * n * k / R);
        norm = std::max(norm, std::abs(s));
        worst = std::max(worst, std::abs(s - cd(out[k].x, out[k].y)));
    }
    return worst / norm;
}

int main() {
    std::mt19937 g(5);
    std::normal_distribution<float> d(0.f, 1.f);
    double e16 = 0, e16w = 0, e16s = 0, e32 = 0, e32w = 0;
    const float r2 = 0.707106781186547524f;
    for (int trial = 0; trial < 200; trial++) {
        float2 x[32], u[32];
        for (auto &v : x) v = make_float2(d(g), d(g));
        for (int i = 0; i < 16; i++) u[i] = x[i];
        rfa::dft<16>(u);
        e16 = std::max(e16, err<16>(x, u));
        for (int i = 0; i < 16; i++) u[i] = x[i];
        rfa::dft16w<0>(u);
        e16w = std::max(e16w, err<16>(x, u));
        // S0: u[4], u[12] arrive as p with x = sqrt(1/2) p (exact inputs: x built from p)
        float2 xs[16];
        for (int i = 0; i < 16; i++) xs[i] = x[i];
        for (int i : {4, 12}) {
            u[i] = x[i];
            xs[i] = make_float2(r2 * x[i].x, r2 * x[i].y);  // the value the S0 form transforms (as float products)
        }
        for (int i = 0; i < 16; i++) if (i != 4 && i != 12) u[i] = x[i];
        rfa::dft16w<0, true>(u);
        e16s = std::max(e16s, err<16>(xs, u));
        for (int i = 0; i < 32; i++) u[i] = x[i];
        rfa::dft<32>(u);
        e32 = std::max(e32, err<32>(x, u));
        for (int i = 0; i < 32; i++) u[i] = x[i];
        rfa::dft32w(u);
        e32w = std::max(e32w, err<32>(x, u));
    }
    std::printf("%.3e %.3e %.3e %.3e %.3e\n", e16, e16w, e16s, e32, e32w);
    return 0;
}
