// N = 2^18 .. 2^20 (BASELINE config 5, 1 M-point FFT): decimation in time over
// S = N / M sub-frames, M = 32768.
//
// Kernel A (fft_wide.hip, dit_ss = S): sub-frame (f, r) = samples x_f[S m + r],
// m < M, is converted, windowed (w[S m + r], the [S][M] permuted window) and
// transformed by the 32 K-point workgroup: Y_r[k] = sum_m x[S m + r] w W_M^{m k},
// written unscaled to scratch [f][r][k].
//
// Kernel B (here): X[k + M s] = sum_r (W_N^{r k} Y_r[k]) W_S^{r s}.  One thread
// per k: S coalesced loads (consecutive k across lanes), exact twiddles
// W_N^{r k} = C[r][k >> 7] * D[r][k & 127] (both from double), an in-register
// DFT-S, then the reference's epilogue (nativedsp.cpp:72-79: 10*log10 of
// |X|/N, fft-shift) -- every store is coalesced across lanes (k consecutive).
// Scratch traffic is 16 B per sample (write + read); the engine sizes batches so
// the scratch stays in the 256 MB Infinity Cache.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "fft_common.h"
#include "fft_kernels.h"

namespace rfa {

template <int S, bool CO>
__global__ void __launch_bounds__(256) dit_combine_kernel(DitLaunch a) {
    const int M = 1 << a.logm, n = 1 << a.logn;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int f = blockIdx.y;
    if (k >= M) return;
    const float2 *y = a.y + (size_t)f * S * M + k;
    float2 v[S];
#pragma unroll
    for (int r = 0; r < S; r++) v[r] = y[(size_t)r * M];
    const int khi = k >> 7, klo = k & 127, mc = M >> 7;
#pragma unroll
    for (int r = 1; r < S; r++) v[r] = cmul(v[r], cmul(a.tw_c[r * mc + khi], a.tw_d[r * 128 + klo]));
    dft<S>(v);  // v[s] = X[k + M s]
    if constexpr (CO) {
        float2 *o = a.complex_out + (size_t)f * n + k;
#pragma unroll
        for (int s = 0; s < S; s++) o[(size_t)s * M] = v[s];
    } else {
        const int frame = a.frame0 + f;
        float *row = a.rows ? a.rows + (size_t)f * n : nullptr;
        float *ring = nullptr;
        if (a.ring && frame >= a.ring_first) {
            int rr = (a.ring_base - frame) % a.ring_rows;
            if (rr < 0) rr += a.ring_rows;
            ring = a.ring + (size_t)rr * n;
        }
        const float db_off = db_offset(a.logn);
#pragma unroll
        for (int s = 0; s < S; s++) {
            const float db = db_unscaled(v[s], db_off);      // nativedsp.cpp:73-78
            const int o = (k + M * s + (n >> 1)) & (n - 1);  // fft-shift, nativedsp.cpp:77
            if (row) row[o] = db;
            if (ring) ring[o] = db;
        }
    }
}

template <int S>
static hipError_t launch_s(const DitLaunch &a) {
    const dim3 grid((1 << a.logm) / 256, a.n_frames);
    if (a.complex_out) hipLaunchKernelGGL((dit_combine_kernel<S, true>), grid, dim3(256), 0, a.stream, a);
    else hipLaunchKernelGGL((dit_combine_kernel<S, false>), grid, dim3(256), 0, a.stream, a);
    return hipGetLastError();
}

hipError_t launch_dit_combine(const DitLaunch &a) {
    if (a.n_frames <= 0) return hipSuccess;
    switch (a.logn - a.logm) {
    case 3: return launch_s<8>(a);
    case 4: return launch_s<16>(a);
    case 5: return launch_s<32>(a);
    default: return hipErrorInvalidValue;
    }
}

void dit_twiddles(int logn, std::vector<float2> &c, std::vector<float2> &d) {
    const int m = 1 << kDitLogM, s = 1 << (logn - kDitLogM), mc = m >> 7;
    const double n = (double)(1 << logn);
    auto w = [&](double e) {  // exp(-2 pi i e / N), correctly rounded from double
        const double ang = -2.0 * M_PI * e / n;
        return make_float2((float)std::cos(ang), (float)std::sin(ang));
    };
    c.assign((size_t)s * mc, make_float2(1.f, 0.f));
    d.assign((size_t)s * 128, make_float2(1.f, 0.f));
    for (int r = 0; r < s; r++) {
        for (int h = 0; h < mc; h++) c[(size_t)r * mc + h] = w(std::fmod((double)r * 128.0 * h, n));
        for (int l = 0; l < 128; l++) d[(size_t)r * 128 + l] = w((double)r * l);
    }
}

}  // namespace rfa
