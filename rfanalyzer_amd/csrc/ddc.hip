// ddc.hip -- demod-branch front end on gfx950.
//
// One fused kernel per call: every workgroup owns P consecutive decimated
// outputs, stages the raw IQ bytes they depend on through LDS -- converted and
// NCO-mixed on the way in (IQConverter.mixPacketIntoSamplePacket,
// source/Signed8BitIQConverter.java:101-130, Signed16BitIQConverter.kt:126-181)
// -- and each lane then runs the FIR dot product of one output
// (FirFilter.filter, dsp/FirFilter.kt:63-107) over LDS.  Raw bytes are read from
// HBM once plus a halo of T-1 samples per workgroup; only the decimated outputs
// are written.  The T-1 newest mixed samples of every call are kept on the
// device as the next call's history (the reference's circular delay line).
//
// Bit-exactness: products and sums are separate float roundings in the
// reference's order (no FMA contraction, taps summed k = 0..T-1, newest sample
// first), the mixer's lut(b) * cos_t product is the value the reference stores
// in its table, and the host design code below follows the JVM's float/double
// promotions step by step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rfa.h"

#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 256;           // largest workgroup
constexpr int kLdsBytes = 160 * 1024;    // LDS per CU on gfx950
constexpr int kMaxWavesPerCu = 32;
// Mixer tables are sized by their length.  calcOptimalCosineLength
// (IQConverter.java:64-76) after the fold of generateMixerLookupTable never
// exceeds MAX_COSINE_LENGTH (an unfolded cycle is sr/|f| < 501 samples, the
// search stops below 500), but nothing here relies on it: a table only has to
// fit the LDS beside one staged output window (plan_tiles checks).
constexpr int kDynLds = kLdsBytes;      // taps + mixer table + staged samples, all dynamic
constexpr int kMaxCosineLength = 500;   // IQConverter.java:39

struct DdcLaunch {
    const void *raw;
    long long S;                   // input samples this call
    const float *hist;             // [re T-1 | im T-1], oldest first, precedes raw[0]
    float *new_hist;
    const float *taps;
    int T;
    const float *cosv, *sinv;
    int L, ci;                     // mixer table length, cosine index of raw[0]
    int D;
    long long n0, in0, n_out;      // global index of this call's first output / first input
    long long off;                 // output n's newest input is (n*Dd + off) / I, phase (n*Dd + off) % I
    int I, Dd;                     // interpolation, decimation (decimator: 1, D)
    int P, KC;                     // outputs per workgroup, taps per LDS chunk
    int threads, lds_bytes;        // workgroup size (P rounded up to 64), dynamic LDS
    int pad;                       // LDS row pitch D + pad is odd
    int vec4;                      // raw buffer aligned for 4-sample loads
    int kc_pad;                    // floats reserved for the chunk's taps (multiple of 4)
    int cs_v2;                     // LDS slots (8 B) of the mixer table, L rounded up to even
    float *out_re, *out_im;
};

template <int FMT> struct RawOf { using type = unsigned; };
template <> struct RawOf<RFA_IN_F32_INTERLEAVED> { using type = float2; };
// Four consecutive samples as one load.
template <int FMT> struct Raw4Of { using type = uint2; };        // 8-bit I,Q x 4
template <> struct Raw4Of<RFA_IN_S16LE> { using type = uint4; };  // int16 I,Q x 4

template <int FMT>
__device__ __forceinline__ unsigned raw4_elem(typename Raw4Of<FMT>::type v, int e) {
    if constexpr (FMT == RFA_IN_S16LE) return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
    else return ((e < 2 ? v.x : v.y) >> (16 * (e & 1))) & 0xffffu;
}

// One complex input sample as stored (I,Q bytes / int16 pair / float pair).
template <int FMT>
__device__ __forceinline__ typename RawOf<FMT>::type load_raw(const DdcLaunch &a, long long g) {
    if constexpr (FMT == RFA_IN_F32_INTERLEAVED) return static_cast<const float2 *>(a.raw)[g];
    else if constexpr (FMT == RFA_IN_S16LE) return static_cast<const unsigned *>(a.raw)[g];
    else return static_cast<const unsigned short *>(a.raw)[g];
}

// LUT conversion + NCO mix of one raw sample with the table entry (c, s).
template <int FMT>
__device__ __forceinline__ void mix_raw(typename RawOf<FMT>::type v, float c, float s, float &re, float &im) {
    if constexpr (FMT == RFA_IN_F32_INTERLEAVED) {
        re = v.x;
        im = v.y;
    } else {
        float i, q;
        if constexpr (FMT == RFA_IN_S16LE) {
            i = (float)(short)(v & 0xffffu) / 32768.0f;
            q = (float)(short)(v >> 16) / 32768.0f;
        } else if constexpr (FMT == RFA_IN_S8) {
            i = (float)(signed char)(v & 0xffu) / 128.0f;
            q = (float)(signed char)(v >> 8) / 128.0f;
        } else {
            i = ((float)(v & 0xffu) - 127.4f) / 128.0f;
            q = ((float)(v >> 8) - 127.4f) / 128.0f;
        }
        re = i * c - q * s;
        im = q * c + i * s;
    }
}

template <int FMT>
__device__ __forceinline__ void ddc_sample(const DdcLaunch &a, long long g, int t, float &re, float &im) {
    if (g < 0) {
        re = a.hist[a.T - 1 + g];
        im = a.hist[2 * (a.T - 1) + g];
        return;
    }
    const float c = FMT == RFA_IN_F32_INTERLEAVED ? 0.0f : a.cosv[t];
    const float s = FMT == RFA_IN_F32_INTERLEAVED ? 0.0f : a.sinv[t];
    mix_raw<FMT>(load_raw<FMT>(a, g), c, s, re, im);
}

// Table index (cosineIndex) of extended-sequence sample g, for any g.
__device__ __forceinline__ int cos_index(const DdcLaunch &a, long long g) {
    if (a.L <= 0) return 0;
    const long long r = ((long long)a.ci + g) % a.L;
    return (int)(r < 0 ? r + a.L : r);
}

typedef float v2f __attribute__((ext_vector_type(2)));

// One staged (re, im) pair as its own ds_read_b64.  A volatile LDS access keeps
// the compiler from fusing neighbours into ds_read2_b64, which moves half the
// bytes per LDS cycle on gfx950 (MI355X_MICROARCH.md, LDS table); the loads
// still issue back to back with counted waits (measured 3-9 % faster,
// profiles/r01o/ddc_unfused_lds_reads_ab.txt).
__device__ __forceinline__ v2f lds_ld(const v2f *p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const volatile __attribute__((address_space(3))) v2f *)(p);
#else
    return *p;
#endif
}

// One lane per decimated output; blockDim = P rounded up to a wave.  The
// samples all P outputs need for taps [k0, k1) are one contiguous run of
// (P-1)*D + (k1-k0) samples, staged (converted + mixed) into LDS as (re, im)
// pairs in rows of D samples with a row pitch Dp = D + pad, pad making Dp odd:
// at a given tap the lanes read samples exactly D apart, so an odd pitch puts
// the 32 lanes of a half-wave on 32 different bank pairs (an even D would give
// up to a 32-way conflict).  Each lane accumulates its taps in the reference's
// order with packed fp32 multiply and add (v_pk_mul_f32 / v_pk_add_f32: two
// separately rounded operations, exactly the JVM's tap * delay then +=); the
// tap loop runs in segments that stay inside one row, so the LDS pointer just
// walks down.
template <int FMT>
__global__ __launch_bounds__(kThreads) void ddc_fir_kernel(DdcLaunch a) {
    extern __shared__ __attribute__((aligned(16))) v2f dyn[];
    // [taps of the chunk | mixer table (cos, sin), L entries | staged samples]
    float *wl = reinterpret_cast<float *>(dyn);
    float2 *cs = reinterpret_cast<float2 *>(dyn + a.kc_pad / 2);
    v2f *xs = dyn + a.kc_pad / 2 + a.cs_v2;
    const int tid = threadIdx.x;
    const int nth = blockDim.x;
    for (int i = tid; i < a.L; i += nth) cs[i] = float2{a.cosv[i], a.sinv[i]};
    __syncthreads();
    const int D = a.D, Dp = a.D + a.pad;                   // LDS layout: rows of D samples
    const long long m0 = (long long)blockIdx.x * a.P;
    const int nloc = (int)min((long long)a.P, a.n_out - m0);
    const bool valid = tid < nloc;
    // newest input of output n (global indices), RationalResampler / FirFilter counters closed-form
    const long long nf = a.n0 + m0, nl = nf + (nloc - 1), nt = nf + (valid ? tid : 0);
    const long long cf = (nf * a.Dd + a.off) / a.I, cl = (nl * a.Dd + a.off) / a.I;
    const long long pos_t = nt * a.Dd + a.off;
    const int lane_off = (int)(pos_t / a.I - cf);          // decimator: tid * D
    const int phase = (int)(pos_t % a.I);
    const long long jb = cf - a.in0;                        // call-relative input index of output m0
    const int step = a.L > 0 ? nth % a.L : 0;
    const int srow = nth / D, scol = nth % D;
    v2f acc = {0.0f, 0.0f};
    for (int k0 = 0; k0 < a.T; k0 += a.KC) {
        const int k1 = min(a.T, k0 + a.KC);
        const long long lo = jb - (k1 - 1);                 // oldest sample any lane needs
        const int span = (int)(cl - cf) + (k1 - k0);         // fits the LDS the host sized
        if (a.I == 1)
            for (int i = tid; i < k1 - k0; i += nth) wl[i] = a.taps[k0 + i];
        // leading samples older than this call come from the history (first workgroups only)
        const int nh = (int)min((long long)span, max(0LL, -lo));
        for (int i = tid; i < nh; i += nth) {
            float re, im;
            ddc_sample<FMT>(a, lo + i, 0, re, im);
            xs[(i / D) * Dp + i % D] = v2f{re, im};
        }
        // raw part: U loads in flight per lane before any is converted
        constexpr int U = 8;
        bool staged = false;
        if constexpr (FMT != RFA_IN_F32_INTERLEAVED) {
            if (a.vec4) {
                // 4 consecutive samples per load (8 B for 8-bit IQ, 16 B for int16): four
                // times the bytes in flight of the per-sample loop, which left HBM latency
                // exposed.  Groups are aligned in the raw buffer; samples outside
                // [lo + nh, lo + span) are skipped.
                using R4 = typename Raw4Of<FMT>::type;
                const long long gA = lo + nh, gB = lo + span;     // gA >= 0 whenever gA < gB
                const long long q0 = gA >> 2;
                // whole groups inside the buffer only; the last < 4 samples of the call
                // (a group that would run past raw[S-1]) go through scalar loads below
                const long long qend = min((gB + 3) >> 2, a.S >> 2);
                const int nq = gA < gB ? (int)max(0LL, qend - q0) : 0;
                const int step4 = (4 * nth) % max(a.L, 1);
                const int srow4 = (4 * nth) / D, scol4 = (4 * nth) % D;
                const int i0 = (int)((q0 + tid) * 4 - lo);          // may be negative for the first group
                int tq = cos_index(a, lo + i0);
                int rq = (i0 >= 0 ? i0 / D : -((-i0 + D - 1) / D)), cq = i0 - rq * D;
                for (int qb = tid; qb < nq; qb += U * nth) {
                    R4 v[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int q = qb + u * nth;
                        if (q < nq) v[u] = static_cast<const R4 *>(a.raw)[q0 + q];
                    }
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int q = qb + u * nth;
                        if (q < nq) {
                            const int ib = (int)((q0 + q) * 4 - lo);
                            // the group's four table entries are read before any is used, so
                            // one LDS round trip covers the group instead of four
                            float2 cst[4];
                            int t = tq;
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                cst[e] = cs[t];
                                if (++t >= a.L) t = 0;
                            }
                            int r = rq, c = cq;
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const int i = ib + e;
                                if (i >= nh && i < span) {
                                    float re, im;
                                    mix_raw<FMT>(raw4_elem<FMT>(v[u], e), cst[e].x, cst[e].y, re, im);
                                    xs[r * Dp + c] = v2f{re, im};
                                }
                                if (++c >= D) c = 0, r++;
                            }
                        }
                        tq += step4;
                        if (tq >= a.L) tq -= a.L;
                        rq += srow4;
                        cq += scol4;
                        if (cq >= D) cq -= D, rq++;
                    }
                }
                const long long gt = max(gA, (a.S >> 2) << 2);     // scalar tail [gt, gB)
                for (long long g = gt + tid; g < gB; g += nth) {
                    const int i = (int)(g - lo);
                    float re, im;
                    ddc_sample<FMT>(a, g, cos_index(a, g), re, im);
                    xs[(i / D) * Dp + i % D] = v2f{re, im};
                }
                staged = true;
            }
        }
        if (!staged) {
            const int i0 = nh + tid;
            int t = cos_index(a, lo + i0);
            int row = i0 / D, col = i0 % D;
            for (int base = i0; base < span; base += U * nth) {
                typename RawOf<FMT>::type v[U];
    #pragma unroll
                for (int u = 0; u < U; u++) {
                    const int i = base + u * nth;
                    if (i < span) v[u] = load_raw<FMT>(a, lo + i);
                }
    #pragma unroll
                for (int u = 0; u < U; u++) {
                    const int i = base + u * nth;
                    if (i < span) {
                        float re, im;
                        const float2 cst = FMT == RFA_IN_F32_INTERLEAVED ? float2{0.0f, 0.0f} : cs[t];
                        mix_raw<FMT>(v[u], cst.x, cst.y, re, im);
                        xs[row * Dp + col] = v2f{re, im};
                    }
                    t += step;
                    if (t >= a.L) t -= a.L;
                    row += srow;
                    col += scol;
                    if (col >= D) col -= D, row++;
                }
            }
        }
        __syncthreads();
        if (valid && a.pad) {
            // decimator, even D: tap k reads staged sample tid*D + rel, rel = k1-1-k, in row segments
            int k = k0;
            while (k < k1) {
                const int rel = k1 - 1 - k;
                const int r = rel / D, c = rel - r * D;
                const int seg = min(c + 1, k1 - k);
                const v2f *x = xs + (tid + r) * Dp + c;
                const float *w = wl + (k - k0);
#pragma unroll 8
                for (int u = 0; u < seg; u++) acc = acc + w[u] * lds_ld(x - u);
                k += seg;
            }
        } else if (valid) {
            // linear layout: one contiguous walk; taps shared (I == 1, LDS) or this lane's phase row
            const v2f *x = xs + lane_off + (k1 - 1 - k0);
            if (a.I == 1) {
#pragma unroll 8
                for (int u = 0; u < k1 - k0; u++) acc = acc + wl[u] * lds_ld(x - u);
            } else {
                const float *w = a.taps + (long long)phase * a.T + k0;
#pragma unroll 8
                for (int u = 0; u < k1 - k0; u++) acc = acc + w[u] * lds_ld(x - u);
            }
        }
        __syncthreads();
    }
    if (valid) {
        a.out_re[m0 + tid] = acc.x;
        a.out_im[m0 + tid] = acc.y;
    }
}

// new_hist[t] = sample S - (T-1) + t of the extended sequence [hist | raw].
template <int FMT>
__global__ __launch_bounds__(kThreads) void ddc_hist_kernel(DdcLaunch a) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= a.T - 1) return;
    const long long g = a.S - (a.T - 1) + t;
    float re, im;
    ddc_sample<FMT>(a, g, cos_index(a, g), re, im);
    a.new_hist[t] = re;
    a.new_hist[a.T - 1 + t] = im;
}

template <int FMT>
hipError_t launch_ddc(const DdcLaunch &a, hipStream_t st) {
    if (a.n_out > 0) {
        const long long blocks = (a.n_out + a.P - 1) / a.P;
        static bool attr_set = false;
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(ddc_fir_kernel<FMT>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kDynLds);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
        hipLaunchKernelGGL(ddc_fir_kernel<FMT>, dim3((unsigned)blocks), dim3(a.threads), a.lds_bytes, st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (a.T > 1) {
        hipLaunchKernelGGL(ddc_hist_kernel<FMT>, dim3((a.T - 1 + kThreads - 1) / kThreads), dim3(kThreads), 0, st, a);
        return hipGetLastError();
    }
    return hipSuccess;
}

// ---------------------------------------------------------------- host design

// Java/Kotlin (int) of a double: truncation, saturation, NaN -> 0.
int32_t jtoint(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

// BlackmanWindow.value (WindowFunctions.kt:44-49).
float blackman(int n, int N) {
    const float c1 = (float)std::cos(2.0 * M_PI * n / (N - 1));
    const float c2 = (float)std::cos(4.0 * M_PI * n / (N - 1));
    return 0.42f - 0.5f * c1 + 0.08f * c2;
}

// KaiserWindow (WindowFunctions.kt:63-99): izero series as GNU Radio's.
double kaiser_izero(double x) {
    double sum = 1.0, term = 1.0;
    const double half = x / 2.0;
    for (int k = 1;; k++) {
        const double tmp = half / k;
        term *= tmp * tmp;
        sum += term;
        if (term < 1e-12) break;
    }
    return sum;
}

float kaiser(int n, int N, double beta) {
    const double ibeta = 1.0 / kaiser_izero(beta);
    if (n == 0 || n == N - 1) return (float)ibeta;
    const double inm1 = 1.0 / (double)(N - 1);
    const double temp = 2.0 * n * inm1 - 1.0;
    return (float)(kaiser_izero(beta * std::sqrt(1.0 - temp * temp)) * ibeta);
}

enum { kWinBlackman = 0, kWinKaiser7 = 1 };

// FirFilter.createLowPassTaps (FirFilter.kt:134-195).  false where it returns null.
bool design_low_pass(float gain, float fs, float fc, float tw, float att, int max_taps, std::vector<float> &taps,
                     int window = kWinBlackman) {
    if (fs <= 0.0f || fc <= 0.0f || fc > fs / 2 || tw <= 0.0f) return false;
    int ntaps = jtoint((double)(att * fs) / (22.0 * (double)tw));
    if (max_taps > 0) ntaps = std::min(ntaps, max_taps);
    if ((ntaps & 1) == 0) ntaps++;
    if (ntaps <= 0 || ntaps > (1 << 24)) return false;
    taps.assign(ntaps, 0.0f);
    const float pi = (float)M_PI;
    const int M = (ntaps - 1) / 2;
    const float fwT0 = 2 * pi * fc / fs;
    for (int n = -M; n <= M; n++) {
        const float w = window == kWinKaiser7 ? kaiser(n + M, ntaps, 7.0) : blackman(n + M, ntaps);
        if (n == 0) taps[n + M] = fwT0 / pi * w;
        else taps[n + M] = (float)std::sin((double)((float)n * fwT0)) / ((float)n * pi) * w;
    }
    float fmx = taps[M];
    for (int n = 1; n <= M; n++) fmx += 2 * taps[n + M];
    const float g = gain / fmx;
    for (float &t : taps) t *= g;
    return true;
}

int gcd_i(int a, int b) {  // RationalResampler.gcd
    int x = std::abs(a), y = std::abs(b);
    while (y != 0) {
        const int t = y;
        y = x % y;
        x = t;
    }
    return x;
}

// RationalResampler.limitDenominator (RationalResampler.kt:165-203).
void limit_denominator(int num, int den, int max_den, int &out_i, int &out_d) {
    const double target = (double)num / (double)den;
    const int g0 = gcd_i(num, den);
    if (den / g0 <= max_den) {
        out_i = num / g0;
        out_d = den / g0;
        return;
    }
    int ln = 0, ld = 1, un = 1, ud = 0;
    while (true) {
        const int mn = ln + un, md = ld + ud;
        if (md > max_den) break;
        if ((double)mn / md < target) ln = mn, ld = md;
        else un = mn, ud = md;
    }
    const double le = std::fabs(target - (double)ln / ld), ue = std::fabs(target - (double)un / ud);
    if (le < ue) out_i = ln, out_d = ld;
    else out_i = un, out_d = ud;
}

// RationalResampler.designResamplerTaps (RationalResampler.kt:210-235): Kaiser(7) low-pass at
// gain = fs = interpolation; empty where createLowPassTaps returns null.
void design_resampler_taps(int I, int D, float fbw, int max_taps, std::vector<float> &taps) {
    const double halfband = 0.5;
    const float rate = (float)I / (float)D;
    float tw, mid;
    if (rate >= 1.0f) {
        tw = (float)(halfband - fbw);
        mid = (float)(halfband - tw / 2.0);
    } else {
        tw = (float)(rate * (halfband - fbw));
        mid = (float)(rate * halfband - tw / 2.0);
    }
    if (!design_low_pass((float)I, (float)I, mid, tw, 72.22087f, max_taps * I, taps, kWinKaiser7)) taps.clear();
}

// (int)(frequency - channelFrequency) and the fold of generateMixerLookupTable
// (Signed8BitIQConverter.java:55-57, Signed16BitIQConverter.kt:62-64).
int32_t fold_mix(int64_t frequency, int64_t channel, int32_t sr) {
    int32_t mix = (int32_t)(uint32_t)((uint64_t)frequency - (uint64_t)channel);
    const int32_t a = mix == INT32_MIN ? INT32_MIN : (mix < 0 ? -mix : mix);
    const int32_t q = a != 0 ? sr / a : 0;
    if (mix == 0 || q > kMaxCosineLength) mix = (int32_t)((uint32_t)mix + (uint32_t)sr);
    return mix;
}

// IQConverter.calcOptimalCosineLength (IQConverter.java:64-76).
int optimal_cosine_length(int32_t sr, int32_t cf) {
    const double cycle = (double)sr / std::fabs((double)cf);
    int best = jtoint(cycle);
    double err = std::fabs(best - cycle);
    for (int i = 1; i * cycle < kMaxCosineLength; i++) {
        const double ic = i * cycle;
        if (std::fabs(ic - jtoint(ic)) < err) {
            best = jtoint(ic);
            err = std::fabs(best - ic);
        }
    }
    return best;
}

void mixer_table(int fmt, int32_t sr, int32_t cf, std::vector<float> &c, std::vector<float> &s) {
    const int n = std::max(0, optimal_cosine_length(sr, cf));
    c.assign(n, 0.0f);
    s.assign(n, 0.0f);
    if (fmt == RFA_IN_S16LE) {  // Signed16BitIQConverter.kt:73-81
        const double w = (2.0 * M_PI * cf) / (double)sr;
        for (int t = 0; t < n; t++) {
            c[t] = (float)std::cos(w * t);
            s[t] = (float)std::sin(w * t);
        }
    } else {                    // Signed8BitIQConverter.java:68-70
        for (int t = 0; t < n; t++) {
            const double x = 2 * M_PI * cf * t / (double)(float)sr;
            c[t] = (float)std::cos(x);
            s[t] = (float)std::sin(x);
        }
    }
}

}  // namespace

struct rfa_ddc {
    int device = 0;
    int fmt = 0;
    int32_t sample_rate = 0, out_rate = 0;
    hipStream_t stream = nullptr;       // where work is enqueued (own_stream or the caller's)
    hipStream_t own_stream = nullptr;   // created by the handle; set once rfa_ddc_set_stream is used
    std::string err;
    // mixer (IQConverter state)
    bool mixer_valid = false;
    int32_t cos_freq = 0;
    int ci = 0;
    std::vector<float> cos_t, sin_t;
    float *d_cos = nullptr;   // [cos L | sin L], capacity d_cos_cap entries each
    size_t d_cos_cap = 0;
    std::vector<float> fir_taps;  // mode 2: caller's FirFilter taps
    int fir_decimation = 1;
    // filter: Decimator/FirFilter (mode 0) or Resampler/RationalResampler (mode 1)
    int mode = 0;
    int D = 0;                // decimation (mode 1: of the reduced ratio I/D)
    int I = 1;                // interpolation
    std::vector<float> taps;  // mode 0: the taps; mode 1: polyphase bank [I][T], phase-major
    std::vector<float> proto; // mode 1: prototype taps padded to a multiple of I
    int T = 0;                // taps per output
    float *d_taps = nullptr;
    size_t taps_cap = 0;
    long long n_done = 0, in_done = 0;   // outputs produced / inputs consumed since the filter was built
    float *d_hist[2] = {nullptr, nullptr};
    int cur = 0;
    // staging for the _host entry point
    void *d_in = nullptr;
    size_t d_in_cap = 0;
    float *d_out = nullptr;
    size_t d_out_cap = 0;
};

namespace {

int dfail(rfa_ddc *d, int code, const std::string &msg) {
    if (d) d->err = msg;
    return code;
}

#define DHIP(d, expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) return dfail((d), RFA_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

size_t ddc_sample_bytes(int fmt) {
    switch (fmt) {
    case RFA_IN_S8:
    case RFA_IN_U8: return 2;
    case RFA_IN_S16LE: return 4;
    case RFA_IN_F32_INTERLEAVED: return 8;
    default: return 0;
    }
}

// (Re)build the filter for the current rates with a zeroed delay line:
// mode 0 Decimator.java:177-181 (decimationCounter 1: first output at input
// D-1), mode 1 Resampler.kt:102-110 + RationalResampler.kt:27-60 (ctr 0).
int rebuild_filter(rfa_ddc *d) {
    std::vector<float> taps, proto;
    int I = 1, D, T;
    if (d->mode == 2) {  // FirFilter(taps, decimation) as given (FirFilter.kt:34-46)
        taps = d->fir_taps;
        D = d->fir_decimation;
        T = (int)taps.size();
    } else if (d->mode == 0) {
        D = d->sample_rate / d->out_rate;
        if (!design_low_pass(1.0f, (float)d->sample_rate, d->out_rate * 0.75f, d->out_rate * 0.25f, 60.0f, 0, taps))
            return dfail(d, RFA_ERR_INVALID, "low-pass design rejected the rates (createLowPassTaps returns null)");
        if (D < 1) return dfail(d, RFA_ERR_INVALID, "output rate above input rate");
        T = (int)taps.size();
    } else {
        limit_denominator(d->out_rate, d->sample_rate, 10000, I, D);
        const int g = gcd_i(I, D);
        I /= g;
        D /= g;
        if (I < 1 || D < 1) return dfail(d, RFA_ERR_INVALID, "rate ratio");
        if (I > D) return dfail(d, RFA_ERR_UNSUPPORTED, "upsampling (the reference resampler only guarantees downsampling)");
        design_resampler_taps(I, D, 0.4f, 500, proto);
        if (proto.empty()) return dfail(d, RFA_ERR_INVALID, "resampler design rejected the rates");
        while (proto.size() % I) proto.push_back(0.0f);
        T = (int)(proto.size() / I);
        taps.resize(proto.size());
        for (int ph = 0; ph < I; ph++)
            for (int i = 0; i < T; i++) taps[(size_t)ph * T + i] = proto[(size_t)i * I + ph];
    }
    const size_t bank = taps.size(), H = (size_t)T;
    if (bank > d->taps_cap || 2 * H > d->taps_cap * 2) {
        if (d->d_taps) (void)hipFree(d->d_taps);
        for (float *&h : d->d_hist)
            if (h) (void)hipFree(h), h = nullptr;
        d->d_taps = nullptr;
        d->taps_cap = 0;
        const size_t cap = std::max(bank, H);
        if (hipMalloc(&d->d_taps, cap * sizeof(float)) != hipSuccess) return dfail(d, RFA_ERR_NOMEM, "hipMalloc taps");
        for (float *&h : d->d_hist)
            if (hipMalloc(&h, 2 * cap * sizeof(float)) != hipSuccess) return dfail(d, RFA_ERR_NOMEM, "hipMalloc history");
        d->taps_cap = cap;
    }
    DHIP(d, hipMemcpyAsync(d->d_taps, taps.data(), bank * sizeof(float), hipMemcpyHostToDevice, d->stream));
    DHIP(d, hipMemsetAsync(d->d_hist[0], 0, 2 * H * sizeof(float), d->stream));
    DHIP(d, hipStreamSynchronize(d->stream));
    d->taps = std::move(taps);
    d->proto = std::move(proto);
    d->I = I;
    d->D = D;
    d->T = T;
    d->n_done = d->in_done = 0;
    d->cur = 0;
    return RFA_OK;
}

// Offset of the newest-input formula c_n = (n*Dd + off) / I: the decimator's
// counter starts at 1, so its outputs fire at inputs D-1, 2D-1, ...; with D = 1
// the initial 1 is checked once before it wraps to 0, so the first output is at
// input 1 (FirFilter.kt:46,78,101-103; ApplicationTest.kt testFirFilter2 has 63
// outputs for 64 inputs).
// Mode 0 (Decimator) and mode 2 (FirFilter with explicit taps) share FirFilter's counter.
long long out_offset(const rfa_ddc *d) { return d->mode != 1 ? (d->D >= 2 ? d->D - 1 : 1) : 0; }

// Outputs available once `in_total` inputs have been consumed: every n with
// c_n < in_total (FirFilter.kt:75-98, RationalResampler.kt:80-123).
long long outputs_for(const rfa_ddc *d, long long in_total) {
    const long long lim = in_total * d->I - out_offset(d);
    return lim > 0 ? (lim + d->D - 1) / d->D : 0;
}

// Outputs per workgroup: the P whose LDS run (P-1)*D + T samples lets the most
// output lanes be resident per CU (LDS and wave limits); P = 1 with the taps
// split into LDS-sized chunks when even one output's window does not fit.
void plan_tiles(DdcLaunch &a) {
    a.D = std::max(1, a.Dd / a.I);              // LDS row length (outputs are Dd/I inputs apart)
    a.pad = (a.I == 1 && !(a.D & 1)) ? 1 : 0;
    const long long Dp = a.D + a.pad;
    // dynamic LDS of a workgroup: kc taps (padded to 4) + rows of staged samples
    a.cs_v2 = (a.L + 1) / 2 * 2;
    const long long cs_b = a.cs_v2 * 8LL;
    auto lds_of = [&](int P, long long kc) {
        const long long span = ((long long)(P - 1) * a.Dd + a.I - 1) / a.I + 1 + kc;
        return (span + a.D - 1) / a.D * Dp * (long long)sizeof(float2) + (kc + 3) / 4 * 16 + cs_b;
    };
    int best_p = 1, best_lanes = -1;
    for (int P = 1; P <= kThreads; P++) {
        const long long lds = lds_of(P, a.T);
        if (lds > kDynLds) break;
        const int threads = (P + 63) / 64 * 64;
        const int by_lds = (int)(kLdsBytes / lds);
        const int blocks = std::min(by_lds, kMaxWavesPerCu / (threads / 64));
        const int lanes = P * blocks;
        if (lanes >= best_lanes) best_lanes = lanes, best_p = P;
    }
    a.P = best_p;
    a.threads = (best_p + 63) / 64 * 64;
    long long kc = a.T;                     // all taps in one pass when they fit, else chunks
    while (kc > 1 && lds_of(a.P, kc) > kDynLds) kc = std::max(1LL, kc - a.D);
    a.KC = (int)kc;
    a.kc_pad = (a.KC + 3) / 4 * 4;
    a.lds_bytes = (int)lds_of(a.P, a.KC);
}

template <int FMT>
hipError_t dispatch(const DdcLaunch &a, hipStream_t st) {
    return launch_ddc<FMT>(a, st);
}

}  // namespace

extern "C" {

int rfa_lowpass_taps(float gain, float sample_rate, float cutoff, float transition, float attenuation,
                     int32_t max_taps, float *taps, size_t capacity, int32_t *num_taps) {
    if (!num_taps) return RFA_ERR_INVALID;
    std::vector<float> t;
    *num_taps = 0;
    if (!design_low_pass(gain, sample_rate, cutoff, transition, attenuation, max_taps, t)) return RFA_ERR_INVALID;
    *num_taps = (int32_t)t.size();
    if (taps) {
        if (capacity < t.size()) return RFA_ERR_SIZE;
        std::memcpy(taps, t.data(), t.size() * sizeof(float));
    }
    return RFA_OK;
}

static int ddc_create(int mode, int device, int input_format, int32_t sample_rate, int32_t output_sample_rate,
                      rfa_ddc **out, const float *fir_taps = nullptr, int fir_ntaps = 0, int fir_decimation = 1) {
    if (!out) return RFA_ERR_INVALID;
    *out = nullptr;
    if (ddc_sample_bytes(input_format) == 0 || sample_rate <= 0 || output_sample_rate <= 0) return RFA_ERR_INVALID;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return RFA_ERR_NODEVICE;
    if (device < 0 || device >= count) return RFA_ERR_INVALID;
    rfa_ddc *d = new (std::nothrow) rfa_ddc();
    if (!d) return RFA_ERR_NOMEM;
    d->device = device;
    d->mode = mode;
    d->fmt = input_format;
    d->sample_rate = sample_rate;
    d->out_rate = output_sample_rate;
    if (mode == 2) {
        d->fir_taps.assign(fir_taps, fir_taps + fir_ntaps);
        d->fir_decimation = fir_decimation;
    }
    int rc = RFA_OK;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess)
        rc = RFA_ERR_HIP;
    else
        rc = rebuild_filter(d);
    if (rc != RFA_OK) {
        rfa_ddc_destroy(d);
        return rc;
    }
    *out = d;
    return RFA_OK;
}

int rfa_ddc_create(int device, int input_format, int32_t sample_rate, int32_t output_sample_rate, rfa_ddc **out) {
    return ddc_create(0, device, input_format, sample_rate, output_sample_rate, out);
}

int rfa_ddc_create_resampler(int device, int input_format, int32_t sample_rate, int32_t output_sample_rate,
                             rfa_ddc **out) {
    return ddc_create(1, device, input_format, sample_rate, output_sample_rate, out);
}

int rfa_ddc_create_fir(int device, int input_format, int32_t sample_rate, const float *taps, int32_t num_taps,
                       int32_t decimation, rfa_ddc **out) {
    if (!out) return RFA_ERR_INVALID;
    *out = nullptr;
    if (!taps || num_taps < 1 || decimation < 1 || sample_rate <= 0) return RFA_ERR_INVALID;
    return ddc_create(2, device, input_format, sample_rate, std::max(1, sample_rate / decimation), out, taps, num_taps,
                      decimation);
}

int rfa_ddc_set_stream(rfa_ddc *d, void *stream) {
    if (!d) return RFA_ERR_INVALID;
    // the filter history and mixer uploads are ordered on the handle's stream: drain it first
    DHIP(d, hipSetDevice(d->device));
    DHIP(d, hipStreamSynchronize(d->stream));
    if (d->own_stream == nullptr) d->own_stream = d->stream;
    d->stream = stream ? (hipStream_t)stream : d->own_stream;
    return RFA_OK;
}

int rfa_ddc_get_ratio(const rfa_ddc *d, int32_t *interpolation, int32_t *decimation, int32_t *taps_per_output) {
    if (!d) return RFA_ERR_INVALID;
    if (interpolation) *interpolation = d->I;
    if (decimation) *decimation = d->D;
    if (taps_per_output) *taps_per_output = d->T;
    return RFA_OK;
}

int rfa_ddc_get_format(const rfa_ddc *d, int32_t *input_format) {
    if (!d || !input_format) return RFA_ERR_INVALID;
    *input_format = d->fmt;
    return RFA_OK;
}

int rfa_resampler_design(int32_t output_rate, int32_t input_rate, int32_t max_denominator, float fractional_bw,
                         int32_t max_taps, int32_t *interpolation, int32_t *decimation, float *taps, size_t capacity,
                         int32_t *num_taps) {
    if (output_rate <= 0 || input_rate <= 0 || max_denominator <= 0 || !interpolation || !decimation || !num_taps)
        return RFA_ERR_INVALID;
    int I, D;
    limit_denominator(output_rate, input_rate, max_denominator, I, D);
    const int g = gcd_i(I, D);
    if (I <= 0 || D <= 0 || g == 0) return RFA_ERR_INVALID;
    I /= g;
    D /= g;
    if (fractional_bw <= 0 || fractional_bw >= 0.5f) fractional_bw = 0.4f;   // RationalResampler.kt:35-37
    std::vector<float> t;
    design_resampler_taps(I, D, fractional_bw, max_taps, t);
    *interpolation = I;
    *decimation = D;
    *num_taps = (int32_t)t.size();
    if (t.empty()) return RFA_ERR_INVALID;
    if (taps) {
        if (capacity < t.size()) return RFA_ERR_SIZE;
        std::memcpy(taps, t.data(), t.size() * sizeof(float));
    }
    return RFA_OK;
}

int rfa_ddc_destroy(rfa_ddc *d) {
    if (!d) return RFA_ERR_INVALID;
    hipSetDevice(d->device);
    if (d->stream) hipStreamSynchronize(d->stream);
    for (void *p : {(void *)d->d_cos, (void *)d->d_taps, (void *)d->d_hist[0], (void *)d->d_hist[1], d->d_in,
                    (void *)d->d_out})
        if (p) hipFree(p);
    hipStream_t own = d->own_stream ? d->own_stream : d->stream;
    if (own) hipStreamDestroy(own);
    delete d;
    return RFA_OK;
}

const char *rfa_ddc_last_error(const rfa_ddc *d) { return d ? d->err.c_str() : "null handle"; }

int rfa_ddc_set_sample_rate(rfa_ddc *d, int32_t sample_rate) {
    if (!d || sample_rate <= 0) return RFA_ERR_INVALID;
    if (sample_rate == d->sample_rate) return RFA_OK;
    DHIP(d, hipSetDevice(d->device));
    const int32_t old = d->sample_rate;
    d->sample_rate = sample_rate;
    d->mixer_valid = false;                      // IQConverter.setSampleRate: cosineFrequency = -1
    // Decimator: rebuilt only when the integer decimation changes (Decimator.java:177-178);
    // Resampler: whenever the input rate changes (Resampler.kt:102)
    if (d->mode == 1 || (d->mode == 0 && sample_rate / d->out_rate != d->D)) {
        const int rc = rebuild_filter(d);
        if (rc != RFA_OK) {
            d->sample_rate = old;
            return rc;
        }
    }
    return RFA_OK;
}

int rfa_ddc_set_frequencies(rfa_ddc *d, int64_t frequency, int64_t channel_frequency) {
    if (!d) return RFA_ERR_INVALID;
    if (d->fmt == RFA_IN_F32_INTERLEAVED) return RFA_OK;  // samples arrive mixed
    const int32_t mf = fold_mix(frequency, channel_frequency, d->sample_rate);
    if (d->mixer_valid && mf == d->cos_freq) return RFA_OK;
    std::vector<float> c, s;
    mixer_table(d->fmt, d->sample_rate, mf, c, s);
    if (c.size() * 8 > (size_t)kDynLds / 2) return dfail(d, RFA_ERR_UNSUPPORTED, "mixer table larger than half the LDS");
    DHIP(d, hipSetDevice(d->device));
    if (!c.empty()) {
        if (c.size() > d->d_cos_cap) {
            DHIP(d, hipStreamSynchronize(d->stream));
            if (d->d_cos) (void)hipFree(d->d_cos);
            d->d_cos = nullptr;
            d->d_cos_cap = 0;
            if (hipMalloc(&d->d_cos, 2 * c.size() * sizeof(float)) != hipSuccess)
                return dfail(d, RFA_ERR_NOMEM, "hipMalloc mixer table");
            d->d_cos_cap = c.size();
        }
        DHIP(d, hipMemcpyAsync(d->d_cos, c.data(), c.size() * sizeof(float), hipMemcpyHostToDevice, d->stream));
        DHIP(d, hipMemcpyAsync(d->d_cos + d->d_cos_cap, s.data(), s.size() * sizeof(float), hipMemcpyHostToDevice,
                               d->stream));
        DHIP(d, hipStreamSynchronize(d->stream));
    }
    d->cos_t = std::move(c);
    d->sin_t = std::move(s);
    d->cos_freq = mf;
    d->ci = 0;
    d->mixer_valid = true;
    return RFA_OK;
}

int rfa_ddc_process(rfa_ddc *d, const void *in, size_t n_samples, float *out_re, float *out_im, size_t out_capacity,
                    size_t *n_out) {
    if (!d || !n_out) return RFA_ERR_INVALID;
    *n_out = 0;
    if (n_samples == 0) return RFA_OK;
    const size_t sb = ddc_sample_bytes(d->fmt);
    if (!in || (uintptr_t)in % std::min<size_t>(sb, 8) != 0) return dfail(d, RFA_ERR_INVALID, "input pointer null or misaligned");
    if (n_samples > (size_t)1 << 40) return dfail(d, RFA_ERR_INVALID, "n_samples too large");
    const bool mixed = d->fmt != RFA_IN_F32_INTERLEAVED;
    if (mixed && !d->mixer_valid) return dfail(d, RFA_ERR_STATE, "rfa_ddc_set_frequencies not called");
    if (mixed && d->cos_t.empty()) return RFA_OK;   // empty table: the reference mixes nothing
    const long long S = (long long)n_samples;
    const long long n = outputs_for(d, d->in_done + S) - d->n_done;
    if ((size_t)n > out_capacity) return dfail(d, RFA_ERR_SIZE, "output capacity too small");
    if (n > 0 && (!out_re || !out_im)) return RFA_ERR_INVALID;
    DHIP(d, hipSetDevice(d->device));
    DdcLaunch a{};
    a.raw = in;
    a.S = S;
    a.hist = d->d_hist[d->cur];
    a.new_hist = d->d_hist[d->cur ^ 1];
    a.taps = d->d_taps;
    a.T = d->T;
    a.cosv = d->d_cos;
    a.sinv = d->d_cos + d->d_cos_cap;
    a.L = mixed ? (int)d->cos_t.size() : 0;
    a.ci = d->ci;
    a.n0 = d->n_done;
    a.in0 = d->in_done;
    a.off = out_offset(d);
    a.I = d->I;
    a.Dd = d->D;
    a.n_out = n;
    plan_tiles(a);
    a.vec4 = mixed && ((uintptr_t)in % (4 * sb) == 0);
    if ((n + a.P - 1) / a.P > (long long)INT32_MAX) return dfail(d, RFA_ERR_INVALID, "call too large for one grid");
    a.out_re = out_re;
    a.out_im = out_im;
    hipError_t e = hipSuccess;
    switch (d->fmt) {
    case RFA_IN_S8: e = dispatch<RFA_IN_S8>(a, d->stream); break;
    case RFA_IN_U8: e = dispatch<RFA_IN_U8>(a, d->stream); break;
    case RFA_IN_S16LE: e = dispatch<RFA_IN_S16LE>(a, d->stream); break;
    default: e = dispatch<RFA_IN_F32_INTERLEAVED>(a, d->stream); break;
    }
    if (e != hipSuccess) return dfail(d, RFA_ERR_HIP, std::string("ddc launch: ") + hipGetErrorString(e));
    if (a.T > 1) d->cur ^= 1;
    d->n_done += n;
    d->in_done += S;
    if (mixed) d->ci = (int)(((long long)d->ci + S) % (long long)d->cos_t.size());
    *n_out = (size_t)n;
    return RFA_OK;
}

int rfa_ddc_process_host(rfa_ddc *d, const void *in, size_t n_samples, float *out_re, float *out_im,
                         size_t out_capacity, size_t *n_out) {
    if (!d || !n_out || (n_samples && !in)) return RFA_ERR_INVALID;
    *n_out = 0;
    if (n_samples == 0) return RFA_OK;
    DHIP(d, hipSetDevice(d->device));
    const size_t bytes = n_samples * ddc_sample_bytes(d->fmt);
    const size_t most = (size_t)(outputs_for(d, d->in_done + (long long)n_samples) - d->n_done) + 1;
    if (bytes > d->d_in_cap) {
        if (d->d_in) hipFree(d->d_in);
        d->d_in = nullptr;
        d->d_in_cap = 0;
        if (hipMalloc(&d->d_in, bytes) != hipSuccess) return dfail(d, RFA_ERR_NOMEM, "hipMalloc input staging");
        d->d_in_cap = bytes;
    }
    if (2 * most > d->d_out_cap) {
        if (d->d_out) hipFree(d->d_out);
        d->d_out = nullptr;
        d->d_out_cap = 0;
        if (hipMalloc(&d->d_out, 2 * most * sizeof(float)) != hipSuccess) return dfail(d, RFA_ERR_NOMEM, "hipMalloc output staging");
        d->d_out_cap = 2 * most;
    }
    DHIP(d, hipMemcpyAsync(d->d_in, in, bytes, hipMemcpyHostToDevice, d->stream));
    size_t n = 0;
    const int rc = rfa_ddc_process(d, d->d_in, n_samples, d->d_out, d->d_out + most, out_capacity, &n);
    if (rc != RFA_OK) return rc;
    if (n) {
        DHIP(d, hipMemcpyAsync(out_re, d->d_out, n * sizeof(float), hipMemcpyDeviceToHost, d->stream));
        DHIP(d, hipMemcpyAsync(out_im, d->d_out + most, n * sizeof(float), hipMemcpyDeviceToHost, d->stream));
    }
    DHIP(d, hipStreamSynchronize(d->stream));
    *n_out = n;
    return RFA_OK;
}

int rfa_ddc_synchronize(rfa_ddc *d) {
    if (!d) return RFA_ERR_INVALID;
    DHIP(d, hipSetDevice(d->device));
    DHIP(d, hipStreamSynchronize(d->stream));
    return RFA_OK;
}

int rfa_ddc_get_stream(const rfa_ddc *d, void **stream) {
    if (!d || !stream) return RFA_ERR_INVALID;
    *stream = (void *)d->stream;
    return RFA_OK;
}

int rfa_ddc_get_taps(const rfa_ddc *d, float *taps, size_t capacity, int32_t *num_taps, int32_t *decimation) {
    if (!d) return RFA_ERR_INVALID;
    // decimator / explicit FirFilter taps as given; resampler: the prototype filter as designed
    const std::vector<float> &t = d->mode == 1 ? d->proto : d->taps;
    if (num_taps) *num_taps = (int32_t)t.size();
    if (decimation) *decimation = d->D;
    if (taps) {
        if (capacity < t.size()) return RFA_ERR_SIZE;
        std::memcpy(taps, t.data(), t.size() * sizeof(float));
    }
    return RFA_OK;
}

int rfa_ddc_get_mixer(const rfa_ddc *d, float *cos_t, float *sin_t, size_t capacity, int32_t *length,
                      int32_t *mix_frequency, int32_t *cosine_index) {
    if (!d) return RFA_ERR_INVALID;
    if (d->fmt != RFA_IN_F32_INTERLEAVED && !d->mixer_valid) return RFA_ERR_STATE;
    if (length) *length = (int32_t)d->cos_t.size();
    if (mix_frequency) *mix_frequency = d->cos_freq;
    if (cosine_index) *cosine_index = d->ci;
    if (cos_t || sin_t) {
        if (capacity < d->cos_t.size()) return RFA_ERR_SIZE;
        if (cos_t) std::memcpy(cos_t, d->cos_t.data(), d->cos_t.size() * sizeof(float));
        if (sin_t) std::memcpy(sin_t, d->sin_t.data(), d->sin_t.size() * sizeof(float));
    }
    return RFA_OK;
}

}  // extern "C"
