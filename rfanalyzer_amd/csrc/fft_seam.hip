// fft_seam.hip -- the reference's legacy FFT seam at every length its pffft
// accepts (include/rfa.h, rfa_seam_*).
//
// The reference's JNI symbols (nativedsp.cpp:19-81, NativeDsp.kt:43-62) build a
// pffft setup for whatever array length they are given: any N that is a
// multiple of 16 whose N / 4 factors into 2, 3, 4 and 5, up to 2^26
// (pffft.c:1231-1280, decompose :1073-1095).  The streaming handle (rfa_create)
// only takes powers of two in 64 .. 2^20, the sizes of its fused spectrum
// kernels.  This file serves the rest -- N = 16, 32, 2^21 .. 2^26 and every
// mixed length such as 48, 80, 1000 * 16 or 3 * 2^20 -- on the GPU, with no
// CPU fallback.
//
// Algorithm: a self-sorting (Stockham) mixed-radix transform, one kernel per
// radix pass, ping-ponging between two HBM buffers.  Pass p with radix R and
// span S (the product of the earlier radices) reads the R points
// j + r N/R (coalesced for every pass), multiplies point r by W_{S R}^{r k}
// (k = j mod S, from one table W_N^t correctly rounded from double), runs an
// in-register DFT-R and writes its outputs to (j - k) R + k + r S: after the
// last pass the spectrum is in natural order.  The first pass fuses the input
// side of the seam (NativeDsp.kt's Blackman window times planar re / im, or
// the interleaved floats as they are), the last one the output side (the
// complex spectrum, or nativedsp.cpp:72-79's fft-shifted 10 log10(|X| / N)).
// Radix 8 first, then 4 / 2 for the rest of the twos, then 3 and 5, so N = 2^k
// takes ceil(k / 3) passes.  Each pass moves 16 B per point; this path is the
// reference's single-frame legacy call, not the streaming hot path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rfa.h"
#include "fft_common.h"

struct rfa_seam {
    int n = 0;
    int device = 0;
    std::vector<int> radix;           // pass radices, first pass first
    hipStream_t stream = nullptr;
    float2 *d_tw = nullptr;           // W_N^t, t in [0, N)
    float *d_win = nullptr;           // Blackman (NativeDsp.kt:14-21), made on the first planar call
    float2 *d_a = nullptr, *d_b = nullptr;
    void *h_pinned = nullptr;
    size_t h_cap = 0;
    std::string err;
};

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 8192;  // grid-stride beyond 2 M threads

// ---------------------------------------------------------------- DFT-3 / DFT-5
// Y_q = sum_t x_t W_R^{t q}, natural order, W_R = exp(-2 pi i / R).
RFA_HD void dft3(float2 *u) {
    constexpr float kS = 0.866025403784438647f;  // sin(2 pi / 3)
    const float2 s = rfa::cadd(u[1], u[2]), d = rfa::csub(u[1], u[2]);
    const float2 m = make_float2(u[0].x - 0.5f * s.x, u[0].y - 0.5f * s.y);
    const float2 r = make_float2(kS * d.y, -kS * d.x);  // -i sin(2 pi / 3) d
    u[0] = rfa::cadd(u[0], s);
    u[1] = rfa::cadd(m, r);
    u[2] = rfa::csub(m, r);
}

RFA_HD void dft5(float2 *u) {
    constexpr float c1 = 0.309016994374947424f, c2 = -0.809016994374947424f;  // cos(2 pi / 5), cos(4 pi / 5)
    constexpr float s1 = 0.951056516295153572f, s2 = 0.587785252292473129f;   // sin(2 pi / 5), sin(4 pi / 5)
    const float2 t1 = rfa::cadd(u[1], u[4]), t3 = rfa::csub(u[1], u[4]);
    const float2 t2 = rfa::cadd(u[2], u[3]), t4 = rfa::csub(u[2], u[3]);
    const float2 a1 = make_float2(u[0].x + c1 * t1.x + c2 * t2.x, u[0].y + c1 * t1.y + c2 * t2.y);
    const float2 a2 = make_float2(u[0].x + c2 * t1.x + c1 * t2.x, u[0].y + c2 * t1.y + c1 * t2.y);
    const float2 b1 = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);
    const float2 b2 = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
    u[0] = rfa::cadd(u[0], rfa::cadd(t1, t2));
    u[1] = rfa::cadd(a1, rfa::mul_mi(b1));  // a1 - i b1
    u[4] = rfa::cadd(a1, rfa::mul_pi(b1));  // a1 + i b1
    u[2] = rfa::cadd(a2, rfa::mul_mi(b2));
    u[3] = rfa::cadd(a2, rfa::mul_pi(b2));
}

template <int R>
RFA_HD void dft_any(float2 *u) {
    if constexpr (R == 3) dft3(u);
    else if constexpr (R == 5) dft5(u);
    else rfa::dft<R>(u);
}

enum { kInBuf = 0, kInPlanarWin = 1 };      // first-pass input: float2 buffer / planar re, im x window
enum { kOutBuf = 0, kOutDbShift = 1 };      // last-pass output: float2 buffer / fft-shifted dB row

// One Stockham pass.  src holds N complex points (or, for kInPlanarWin, N re
// floats then N im floats); tw = W_N^t.  span = S (1 on the first pass).
template <int R, int IN, int OUT>
__global__ void __launch_bounds__(kThreads) seam_pass_kernel(const float2 *__restrict__ src,
                                                             const float *__restrict__ win,
                                                             const float2 *__restrict__ tw, float2 *__restrict__ dst,
                                                             float *__restrict__ db, int n, int span, float db_off) {
    const int nr = n / R;
    const int tstep = n / (span * R);  // W_{S R}^{r k} = W_N^{r k tstep}
    const int half = n >> 1;
    for (int j = blockIdx.x * kThreads + threadIdx.x; j < nr; j += gridDim.x * kThreads) {
        float2 u[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int i = j + r * nr;
            if constexpr (IN == kInPlanarWin) {
                const float *p = reinterpret_cast<const float *>(src);
                const float w = win[i];
                u[r] = make_float2(p[i] * w, p[n + i] * w);  // NativeDsp.kt:55-58, one rounding each
            } else {
                u[r] = src[i];
            }
        }
        const int k = j % span;
        if (span > 1) {
#pragma unroll
            for (int r = 1; r < R; r++) u[r] = rfa::cmul(u[r], tw[r * k * tstep]);
        }
        dft_any<R>(u);
        const int base = (j - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int o = base + r * span;
            if constexpr (OUT == kOutDbShift) {
                const int t = o < half ? o + half : o - half;  // nativedsp.cpp:77
                db[t] = rfa::db_unscaled(u[r], db_off);
            } else {
                dst[o] = u[r];
            }
        }
    }
}

__global__ void seam_twiddle_kernel(float2 *tw, int n) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= n) return;
    double s, c;
    sincospi(-2.0 * (double)t / (double)n, &s, &c);
    tw[t] = make_float2((float)c, (float)s);
}

template <int R>
hipError_t launch_pass_r(int in_mode, int out_mode, const float2 *src, const float *win, const float2 *tw,
                         float2 *dst, float *db, int n, int span, float db_off, hipStream_t st) {
    const int nr = n / R;
    const int blocks = (int)std::min<long long>(kMaxBlocks, ((long long)nr + kThreads - 1) / kThreads);
    const dim3 g(blocks), b(kThreads);
    if (in_mode == kInPlanarWin) {
        if (out_mode == kOutDbShift)
            hipLaunchKernelGGL((seam_pass_kernel<R, kInPlanarWin, kOutDbShift>), g, b, 0, st, src, win, tw, dst, db, n, span, db_off);
        else
            hipLaunchKernelGGL((seam_pass_kernel<R, kInPlanarWin, kOutBuf>), g, b, 0, st, src, win, tw, dst, db, n, span, db_off);
    } else {
        if (out_mode == kOutDbShift)
            hipLaunchKernelGGL((seam_pass_kernel<R, kInBuf, kOutDbShift>), g, b, 0, st, src, win, tw, dst, db, n, span, db_off);
        else
            hipLaunchKernelGGL((seam_pass_kernel<R, kInBuf, kOutBuf>), g, b, 0, st, src, win, tw, dst, db, n, span, db_off);
    }
    return hipGetLastError();
}

hipError_t launch_pass(int radix, int in_mode, int out_mode, const float2 *src, const float *win, const float2 *tw,
                       float2 *dst, float *db, int n, int span, float db_off, hipStream_t st) {
    switch (radix) {
    case 2: return launch_pass_r<2>(in_mode, out_mode, src, win, tw, dst, db, n, span, db_off, st);
    case 3: return launch_pass_r<3>(in_mode, out_mode, src, win, tw, dst, db, n, span, db_off, st);
    case 4: return launch_pass_r<4>(in_mode, out_mode, src, win, tw, dst, db, n, span, db_off, st);
    case 5: return launch_pass_r<5>(in_mode, out_mode, src, win, tw, dst, db, n, span, db_off, st);
    case 8: return launch_pass_r<8>(in_mode, out_mode, src, win, tw, dst, db, n, span, db_off, st);
    default: return hipErrorInvalidValue;
    }
}

// pffft.c:1231-1280: N > 0, N % 16 == 0 (PFFFT_COMPLEX, SIMD_SZ 4), N <= 2^26,
// N / 4 a product of 2, 3, 4, 5.  Returns the pass radices or an empty list.
std::vector<int> plan_radices(long long n) {
    if (n <= 0 || n % 16 || n > (1LL << 26)) return {};
    long long m = n;
    int twos = 0, threes = 0, fives = 0;
    while (m % 2 == 0) { m /= 2; twos++; }
    while (m % 3 == 0) { m /= 3; threes++; }
    while (m % 5 == 0) { m /= 5; fives++; }
    if (m != 1) return {};
    std::vector<int> r;
    for (; twos >= 3; twos -= 3) r.push_back(8);
    if (twos == 2) r.push_back(4);
    if (twos == 1) r.push_back(2);
    for (int i = 0; i < threes; i++) r.push_back(3);
    for (int i = 0; i < fives; i++) r.push_back(5);
    return r;
}

int seam_fail(rfa_seam *s, int code, const std::string &msg) {
    if (s) s->err = msg;
    return code;
}

#define SEAMCHK(s, expr)                                                                          \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) return seam_fail((s), RFA_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

int ensure_pinned(rfa_seam *s, size_t bytes) {
    if (s->h_cap >= bytes) return RFA_OK;
    if (s->h_pinned) hipHostFree(s->h_pinned);
    s->h_pinned = nullptr;
    s->h_cap = 0;
    if (hipHostMalloc(&s->h_pinned, bytes, hipHostMallocDefault) != hipSuccess)
        return seam_fail(s, RFA_ERR_NOMEM, "hipHostMalloc staging");
    s->h_cap = bytes;
    return RFA_OK;
}

// Upload the host input (in0 then in1, 2 N floats together) into d_a, run
// every pass, copy the result (N float2 or N dB floats) back into `out`.
int run(rfa_seam *s, const float *in0, const float *in1, int in_mode, int out_mode, void *out) {
    if (hipSetDevice(s->device) != hipSuccess) return seam_fail(s, RFA_ERR_NODEVICE, "hipSetDevice");
    const int n = s->n;
    const size_t in_bytes = 2 * (size_t)n * sizeof(float);
    int rc = ensure_pinned(s, in_bytes);
    if (rc) return rc;
    float *pin = static_cast<float *>(s->h_pinned);
    if (in1) {
        std::memcpy(pin, in0, (size_t)n * sizeof(float));
        std::memcpy(pin + n, in1, (size_t)n * sizeof(float));
    } else {
        std::memcpy(pin, in0, in_bytes);
    }
    SEAMCHK(s, hipMemcpyAsync(s->d_a, s->h_pinned, in_bytes, hipMemcpyHostToDevice, s->stream));
    // -(5 log10 2) * log2(N^2): the 1 / N of nativedsp.cpp:73,75 applied in the log domain
    const float db_off = (float)(-rfa::kDbPerLog2 * 2.0 * std::log2((double)n));
    float2 *src = s->d_a, *dst = s->d_b;
    int span = 1;
    const int passes = (int)s->radix.size();
    for (int p = 0; p < passes; p++) {
        const bool last = p == passes - 1;
        const int im = p == 0 ? in_mode : kInBuf;
        const int om = last ? out_mode : kOutBuf;
        SEAMCHK(s, launch_pass(s->radix[p], im, om, src, s->d_win, s->d_tw, dst, reinterpret_cast<float *>(dst), n,
                               span, db_off, s->stream));
        span *= s->radix[p];
        std::swap(src, dst);
    }
    const size_t out_bytes = out_mode == kOutDbShift ? (size_t)n * sizeof(float) : (size_t)n * sizeof(float2);
    SEAMCHK(s, hipMemcpyAsync(s->h_pinned, src, out_bytes, hipMemcpyDeviceToHost, s->stream));
    SEAMCHK(s, hipStreamSynchronize(s->stream));
    std::memcpy(out, s->h_pinned, out_bytes);
    return RFA_OK;
}

}  // namespace

extern "C" {

RFA_API int rfa_seam_supported(int32_t n) { return plan_radices(n).empty() ? 0 : 1; }

RFA_API int rfa_seam_create(int32_t n, int32_t device_id, rfa_seam **out) {
    if (!out) return RFA_ERR_INVALID;
    *out = nullptr;
    std::vector<int> radix = plan_radices(n);
    if (radix.empty()) return RFA_ERR_UNSUPPORTED;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RFA_ERR_NODEVICE;
    if (device_id < 0 || device_id >= ndev) return RFA_ERR_NODEVICE;
    if (hipSetDevice(device_id) != hipSuccess) return RFA_ERR_NODEVICE;
    rfa_seam *s = new (std::nothrow) rfa_seam();
    if (!s) return RFA_ERR_NOMEM;
    s->n = n;
    s->device = device_id;
    s->radix = radix;
    auto bail = [&](int code) { rfa_seam_destroy(s); return code; };
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return bail(RFA_ERR_HIP);
    const size_t cbytes = (size_t)n * sizeof(float2);
    if (hipMalloc(&s->d_tw, cbytes) != hipSuccess || hipMalloc(&s->d_a, cbytes) != hipSuccess ||
        hipMalloc(&s->d_b, cbytes) != hipSuccess)
        return bail(RFA_ERR_NOMEM);
    hipLaunchKernelGGL(seam_twiddle_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, s->stream, s->d_tw, n);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s->stream) != hipSuccess) return bail(RFA_ERR_HIP);
    *out = s;
    return RFA_OK;
}

RFA_API int rfa_seam_destroy(rfa_seam *s) {
    if (!s) return RFA_ERR_INVALID;
    hipSetDevice(s->device);
    if (s->stream) hipStreamSynchronize(s->stream);
    hipFree(s->d_tw);
    hipFree(s->d_win);
    hipFree(s->d_a);
    hipFree(s->d_b);
    if (s->h_pinned) hipHostFree(s->h_pinned);
    if (s->stream) hipStreamDestroy(s->stream);
    delete s;
    return RFA_OK;
}

RFA_API const char *rfa_seam_last_error(const rfa_seam *s) { return s ? s->err.c_str() : "null seam"; }

RFA_API int rfa_seam_get_plan(const rfa_seam *s, int32_t *radices, int32_t cap, int32_t *count) {
    if (!s || !count || (cap > 0 && !radices) || cap < 0) return RFA_ERR_INVALID;
    *count = (int32_t)s->radix.size();
    for (int32_t i = 0; i < cap && i < *count; i++) radices[i] = s->radix[i];
    return RFA_OK;
}

// NativeDsp.kt:43-62 (window, then nativedsp.cpp:44-81)
RFA_API int rfa_seam_windowed_fft_mag_planar(rfa_seam *s, const float *re, const float *im, float *mag_out, size_t n) {
    if (!s || !re || !im || !mag_out) return RFA_ERR_INVALID;
    if (n != (size_t)s->n) return seam_fail(s, RFA_ERR_SIZE, "array length != fft size");  // NativeDsp.kt:45-46
    if (!s->d_win) {
        std::vector<float> w((size_t)n);
        for (size_t i = 0; i < n; i++) {  // NativeDsp.kt:19-20: double, cast once
            const double x = 2.0 * M_PI * (double)i / (double)(n - 1);
            w[i] = (float)(0.42 - 0.5 * std::cos(x) + 0.08 * std::cos(2.0 * x));
        }
        if (hipSetDevice(s->device) != hipSuccess) return seam_fail(s, RFA_ERR_NODEVICE, "hipSetDevice");
        if (hipMalloc(&s->d_win, n * sizeof(float)) != hipSuccess) return seam_fail(s, RFA_ERR_NOMEM, "window");
        SEAMCHK(s, hipMemcpy(s->d_win, w.data(), n * sizeof(float), hipMemcpyHostToDevice));
    }
    return run(s, re, im, kInPlanarWin, kOutDbShift, mag_out);  // planar staging: re[N] then im[N]
}

// nativedsp.cpp:44-81
RFA_API int rfa_seam_fft_logmag_interleaved(rfa_seam *s, const float *in, float *mag_out, size_t n) {
    if (!s || !in || !mag_out) return RFA_ERR_INVALID;
    if (n != (size_t)s->n) return seam_fail(s, RFA_ERR_SIZE, "array length != fft size");
    return run(s, in, nullptr, kInBuf, kOutDbShift, mag_out);
}

// nativedsp.cpp:19-42
RFA_API int rfa_seam_fft_ordered(rfa_seam *s, const float *in, float *out, size_t n) {
    if (!s || !in || !out) return RFA_ERR_INVALID;
    if (n != (size_t)s->n) return seam_fail(s, RFA_ERR_SIZE, "array length != fft size");
    return run(s, in, nullptr, kInBuf, kOutBuf, out);
}

}  // extern "C"
