// gfx950 (MI355X / CDNA4) kernels of the spectrum hot path.
//
// One workgroup "slot" owns one M-point sub-FFT (M <= 16384) entirely on chip:
//   global raw IQ  --(convert: Signed8BitIQConverter.java:48-50 / Unsigned8Bit..:48-50 /
//                     Signed16BitIQConverter.kt:52-55; window: NativeDsp.kt:55-58)-->
//   registers --(radix-16 Stockham passes, LDS exchange between passes)-->
//   registers --(10*log10(sqrt((Re/N)^2+(Im/N)^2)), fft-shift: nativedsp.cpp:72-79)--> rows / ring
// Each thread holds 16 complex points in VGPRs; one Stockham pass = twiddle +
// in-register DFT-16 (4x4) + one LDS round trip.  The forward transform has
// sign -1 and is unscaled, natural output order (pffft.h:117, pffft.c:1660).
//
// N > 16384 (N = RS*M, RS in {2,4,8}): RS workgroups share one frame.  Workgroup
// r computes the decimation-in-frequency residue class X[r + RS*k]: it reads
// the WHOLE frame, forms y_r[m] = W_N^{m r} * sum_j x[m + jM] W_RS^{j r}, and runs
// the M-point FFT of y_r.  The RS workgroups of a frame get block ids that are
// congruent mod 8 so that, under the observed round-robin XCD placement, they
// share one L2 and the re-reads of the frame hit there (speed only).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstdlib>

#include "fft_common.h"
#include "fft_kernels.h"
#include "wave.h"

namespace rfa {
// ----------------------------------------------------------------- geometry
template <int LOGM>
struct Geo {
    static constexpr int M = 1 << LOGM;
    static constexpr int TPF = M / 16;                      // threads per sub-FFT, 16 points each
    static constexpr int SLOTS = TPF >= 256 ? 1 : 256 / TPF;  // sub-FFTs per workgroup
    static constexpr int THREADS = TPF * SLOTS;
    static constexpr int PADM = M + M / 8;                  // LDS words (float2) per slot
    static constexpr int NP16 = LOGM / 4;                   // radix-16 passes
    static constexpr int LASTR = 1 << (LOGM % 4);           // trailing small radix (1 = none)
    static constexpr int NPASS = NP16 + (LASTR > 1 ? 1 : 0);
};

// Padded LDS address: two float2 of padding per 16 keeps the first pass's
// 16-consecutive-point writes (stride 144 B between lanes) conflict-free.
__device__ __forceinline__ int pad(int e) { return e + ((e >> 4) << 1); }

template <int Q, int LOGM>
struct PassInfo {
    using G = Geo<LOGM>;
    static constexpr int R = (Q < G::NP16) ? 16 : G::LASTR;
    static constexpr int PREV_LOG = 4 * (Q < G::NP16 ? Q : G::NP16);
    static constexpr int P = 1 << PREV_LOG;  // product of earlier radices
    static constexpr int NB = 16 / R;        // butterflies per thread
};

// Read the inputs of pass Q from LDS into v.
template <int Q, int LOGM>
__device__ __forceinline__ void lds_read(float2 (&v)[16], const float2 *buf, int tid) {
    using PI = PassInfo<Q, LOGM>;
    using G = Geo<LOGM>;
#pragma unroll
    for (int b = 0; b < PI::NB; b++) {
        const int i = tid + b * G::TPF;
#pragma unroll
        for (int t = 0; t < PI::R; t++) v[b * PI::R + t] = buf[pad(i + t * (G::M / PI::R))];
    }
}

// Apply the data twiddles of pass Q and its in-register DFTs.
template <int Q, int LOGM>
__device__ __forceinline__ void butterflies(float2 (&v)[16], int tid, const float2 *twc, const float2 *twf,
                                            int shift, int tw_scale) {
    using PI = PassInfo<Q, LOGM>;
    using G = Geo<LOGM>;
#pragma unroll
    for (int b = 0; b < PI::NB; b++) {
        const int i = tid + b * G::TPF;
        if constexpr (PI::P > 1) {
            const int k = i & (PI::P - 1);
            // W_{P R}^{t k} = W_N^{t k N/(P R)};  tw_scale = N / M
            const int base = k * (G::M / (PI::P * PI::R)) * tw_scale;
#pragma unroll
            for (int t = 1; t < PI::R; t++) v[b * PI::R + t] = cmul(v[b * PI::R + t], tw(twc, twf, t * base, shift));
        }
        dft<PI::R>(&v[b * PI::R]);
    }
}

// Write the outputs of pass Q into LDS (Stockham autosort destination).
template <int Q, int LOGM>
__device__ __forceinline__ void lds_write(const float2 (&v)[16], float2 *buf, int tid) {
    using PI = PassInfo<Q, LOGM>;
    using G = Geo<LOGM>;
#pragma unroll
    for (int b = 0; b < PI::NB; b++) {
        const int i = tid + b * G::TPF;
        const int k = i & (PI::P - 1);
        const int j = (i - k) * PI::R + k;
#pragma unroll
        for (int t = 0; t < PI::R; t++) buf[pad(j + t * PI::P)] = v[b * PI::R + t];
    }
}

#ifndef RFA_ROWS_WAVESYNC
#define RFA_ROWS_WAVESYNC 1
#endif
// The exchange of a sub-FFT of <= 64 threads stays inside one wave (its slot's LDS region is its
// own): a wave's DS instructions execute in order, so its writes are visible to its later reads
// and its reads precede its later writes -- a compiler fence and the lgkmcnt wait replace the
// workgroup barrier, and the workgroup's waves run their passes independently.
template <int LOGM>
__device__ __forceinline__ void exchange_sync() {
    if constexpr (RFA_ROWS_WAVESYNC && Geo<LOGM>::TPF <= 64) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else lds_barrier();
}

template <int Q, int LOGM, int DIAG>
__device__ __forceinline__ void run_passes(float2 (&v)[16], float2 *buf, int tid, const float2 *twc,
                                           const float2 *twf, int shift, int tw_scale) {
    using G = Geo<LOGM>;
    if constexpr (DIAG & 4) {  // ablation: no FFT work, one LDS round trip only
        if constexpr (Q == 0) {
            lds_write<0, LOGM>(v, buf, tid);
            lds_barrier();
            lds_read<G::NPASS - 1, LOGM>(v, buf, tid);
            lds_barrier();
        }
        return;
    } else {
        butterflies<Q, LOGM>(v, tid, twc, twf, shift, tw_scale);
        if constexpr (Q + 1 < G::NPASS) {
            lds_write<Q, LOGM>(v, buf, tid);
            exchange_sync<LOGM>();
            lds_read<Q + 1, LOGM>(v, buf, tid);
            exchange_sync<LOGM>();
            run_passes<Q + 1, LOGM, DIAG>(v, buf, tid, twc, twf, shift, tw_scale);
        }
    }
}

// ----------------------------------------------------------------- main kernel
// Persistent: each workgroup walks work items u = blockIdx.x + k*gridDim.x.
// RS == 1: item = SLOTS frames (one per slot); the next item's raw samples are
//          prefetched into VGPRs while the current one is transformed.
// RS  > 1: item = (frame, residue r); the RS items of a frame are taken by
//          blocks that are congruent mod 8 in the same round (gridDim.x is a
//          multiple of 8*RS), i.e. one XCD under round-robin placement.
// Persistence (grid = CUs x occupancy, register prefetch of the next item) is
// used where the prefetch fits the VGPR budget: RS == 1 and <= 256 threads.
template <int LOGM, int RS>
struct Persist {
    static constexpr bool value = false;  // see DESIGN.md: register prefetch exceeds the VGPR budget
};

template <int LOGM, int RS, int FMT, bool COMPLEX_OUT, int DIAG>
__global__ void __launch_bounds__(Geo<LOGM>::THREADS, 4) fft_rows_kernel(FftLaunch a) {
    using G = Geo<LOGM>;
    constexpr bool PERSIST = Persist<LOGM, RS>::value;
    using RT = typename Raw<FMT>::T;
    constexpr int M = G::M;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int n = M * RS;
    const int shift = a.tw_shift;
    const int nc = n >> shift, nf = 1 << shift;
    float2 *twc = lds;
    float2 *twf = lds + nc;
    float2 *data = lds + ((nc + nf + 1) & ~1);

    for (int e = threadIdx.x; e < nc; e += G::THREADS) twc[e] = a.tw_coarse[e];
    for (int e = threadIdx.x; e < nf; e += G::THREADS) twf[e] = a.tw_fine[e];

    const int slot = threadIdx.x / G::TPF;
    const int tid = threadIdx.x - slot * G::TPF;
    float2 *buf = data + slot * G::PADM;
    const int items = (RS == 1) ? (a.n_frames + G::SLOTS - 1) / G::SLOTS : ((a.n_frames + 7) / 8) * 8 * RS;

    auto decode = [&](int u, int &frame, int &r) {
        if constexpr (RS == 1) {
            frame = u * G::SLOTS + slot;
            r = 0;
        } else {
            const int g = u / (8 * RS), rem = u - g * (8 * RS);
            r = rem >> 3;
            frame = g * 8 + (rem & 7);
        }
    };

    // frame-invariant per-thread window values
    float wv[PERSIST ? 16 : 1];
    if constexpr (PERSIST) {
#pragma unroll
        for (int t = 0; t < 16; t++) wv[t] = a.window[tid + t * G::TPF];
    }

    RT raw[RS == 1 ? 16 : 1];
    auto issue = [&](int u) {
        int fr, rr;
        decode(u, fr, rr);
        const bool act = fr < a.n_frames;
        const uint8_t *fb = a.in + (size_t)(act ? fr : 0) * (size_t)a.frame_stride;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const int m = tid + t * G::TPF;
            if constexpr (DIAG & 1) raw[t] = synth_raw<FMT>(m + fr);
            else raw[t] = load_raw<FMT>(fb, m, n);
        }
    };
    if constexpr (RS == 1) {
        if ((int)blockIdx.x < items) issue(blockIdx.x);
    }
    __syncthreads();

    auto body = [&](int u) {
        int frame, r;
        decode(u, frame, r);
        const bool active = frame < a.n_frames;
        float2 v[16];
        if constexpr (RS == 1) {
#pragma unroll
            for (int t = 0; t < 16; t++) {
                const float2 x = convert_raw<FMT>(raw[t]);
                const float w = PERSIST ? wv[t] : a.window[tid + t * G::TPF];
                v[t] = make_float2(x.x * w, x.y * w);  // NativeDsp.kt:55-58 (fp32 multiply)
            }
            if constexpr (PERSIST) {
                if (u + (int)gridDim.x < items) issue(u + gridDim.x);  // prefetch the next item
            }
        } else {
            const uint8_t *fb = a.in + (size_t)(active ? frame : 0) * (size_t)a.frame_stride;
            float2 wr[RS];  // W_RS^{j r}: wave-uniform
#pragma unroll
            for (int j = 0; j < RS; j++) wr[j] = kW8[((j * r) * (8 / RS)) & 7];
#pragma unroll
            for (int t = 0; t < 16; t++) {
                const int m = tid + t * G::TPF;
                float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                for (int j = 0; j < RS; j++) {
                    const int s = m + j * M;
                    const float w = a.window[s];
                    RT rv;
                    if constexpr (DIAG & 1) rv = synth_raw<FMT>(s + frame);
                    else rv = load_raw<FMT>(fb, s, n);
                    const float2 x = convert_raw<FMT>(rv);
                    const float2 xw = make_float2(x.x * w, x.y * w);
                    acc = (j == 0) ? xw : cadd(acc, cmul(xw, wr[j]));
                }
                v[t] = (r == 0) ? acc : cmul(acc, tw(twc, twf, m * r, shift));
                if (t & 1) __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight (VGPRs)
            }
        }

        run_passes<0, LOGM, DIAG>(v, buf, tid, twc, twf, shift, RS);

        using PL = PassInfo<G::NPASS - 1, LOGM>;
        if constexpr (DIAG & 2) {
#pragma unroll
            for (int q = 0; q < 16; q++) asm volatile("" ::"v"(v[q].x), "v"(v[q].y));
            return;
        }
        if (!active) return;
        if constexpr (COMPLEX_OUT) {
            float2 *out = a.complex_out + (size_t)frame * n;
#pragma unroll
            for (int b = 0; b < PL::NB; b++) {
#pragma unroll
                for (int t = 0; t < PL::R; t++) {
                    const int ks = tid + b * G::TPF + t * PL::P;
                    out[r + RS * ks] = v[b * PL::R + t];
                }
            }
        } else {
            const float db_off = db_offset(a.logn);
            float *row = a.rows ? a.rows + (size_t)frame * n : nullptr;
            float *ring = nullptr;
            if (a.ring && frame >= a.ring_first) {
                int rr = (a.ring_base - frame) % a.ring_rows;
                if (rr < 0) rr += a.ring_rows;
                ring = a.ring + (size_t)rr * n;
            }
            auto store = [&](float *dst, float *dst2) {
#pragma unroll
                for (int b = 0; b < PL::NB; b++) {
#pragma unroll
                    for (int t = 0; t < PL::R; t++) {
                        const int ks = tid + b * G::TPF + t * PL::P;
                        const int kk = r + RS * ks;
                        const float2 x = v[b * PL::R + t];
                        const float db = db_unscaled(x, db_off);  // nativedsp.cpp:73-78
                        const int o = (kk + (n >> 1)) & (n - 1);  // fft-shift, nativedsp.cpp:77
                        dst[o] = db;
                        if (dst2) dst2[o] = db;
                    }
                }
            };
            if (row && ring) store(row, ring);
            else if (row) store(row, nullptr);
            else if (ring) store(ring, nullptr);
        }
    };
    if constexpr (PERSIST) {
        for (int u = blockIdx.x; u < items; u += gridDim.x) body(u);
    } else {
        if ((int)blockIdx.x < items) body(blockIdx.x);
    }
}

// ----------------------------------------------------------------- dispatch
static int g_cus = 0;

template <int LOGM, int RS, int FMT, bool CO, int DIAG>
static hipError_t launch_one(const FftLaunch &a) {
    using G = Geo<LOGM>;
    auto kern = &fft_rows_kernel<LOGM, RS, FMT, CO, DIAG>;
    const int n = G::M * RS;
    const int nc = n >> a.tw_shift, nf = 1 << a.tw_shift;
    const size_t lds = (size_t)(((nc + nf + 1) & ~1) + G::SLOTS * G::PADM) * sizeof(float2);
    static int per_cu = 0;
    if (per_cu == 0) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        if (g_cus == 0) {
            int dev = 0;
            hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) g_cus = 256;
        }
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, G::THREADS, lds) != hipSuccess || occ < 1) occ = 1;
        per_cu = occ;
    }
    const int items = (RS == 1) ? (a.n_frames + G::SLOTS - 1) / G::SLOTS : ((a.n_frames + 7) / 8) * 8 * RS;
    if (items <= 0) return hipSuccess;
    int grid = items;
    if (Persist<LOGM, RS>::value) grid = std::min(items, (a.cus > 0 ? a.cus : g_cus) * per_cu);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::THREADS), lds, a.stream, a);
    return hipGetLastError();
}

template <int LOGM, int RS, bool CO>
static hipError_t by_fmt(const FftLaunch &a) {
    if constexpr (!CO) {
#ifdef RFA_AB_BUILD
        if (a.diag) {  // ablation builds (profiling only): 16K/64K, s8 and f32
            if constexpr (LOGM == 14 && (RS == 1 || RS == 4)) {
#define RFA_DIAG(D)                                                   \
    case D:                                                           \
        return a.fmt == 0 ? launch_one<LOGM, RS, 0, false, D>(a)     \
                          : launch_one<LOGM, RS, 3, false, D>(a);
                if (a.fmt != 0 && a.fmt != 3) return hipErrorInvalidValue;
                switch (a.diag) { RFA_DIAG(1) RFA_DIAG(2) RFA_DIAG(3) RFA_DIAG(4) RFA_DIAG(6) RFA_DIAG(7)
                default: return hipErrorInvalidValue; }
#undef RFA_DIAG
            }
            return hipErrorInvalidValue;
        }
#endif
    }
    switch (a.fmt) {
    case 0: return launch_one<LOGM, RS, 0, CO, 0>(a);
    case 1: return launch_one<LOGM, RS, 1, CO, 0>(a);
    case 2: return launch_one<LOGM, RS, 2, CO, 0>(a);
    case 3: return launch_one<LOGM, RS, 3, CO, 0>(a);
    case 4: return launch_one<LOGM, RS, 4, CO, 0>(a);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fft(const FftLaunch &a) {
    if (a.variant != 1 && wide_supported(a.logn)) return launch_fft_wide(a);
    if (a.complex_out) {
        if (a.fmt != 3) return hipErrorInvalidValue;
        switch (a.logn) {  // complex output: f32 interleaved only
#define RFA_CO(L, RS) \
    case (L + (RS == 1 ? 0 : (RS == 2 ? 1 : (RS == 4 ? 2 : 3)))): return launch_one<L, RS, 3, true, 0>(a);
            RFA_CO(6, 1) RFA_CO(7, 1) RFA_CO(8, 1) RFA_CO(9, 1) RFA_CO(10, 1) RFA_CO(11, 1) RFA_CO(12, 1)
            RFA_CO(13, 1) RFA_CO(14, 1) RFA_CO(14, 2) RFA_CO(14, 4) RFA_CO(14, 8)
#undef RFA_CO
        default: return hipErrorInvalidValue;
        }
    }
    switch (a.logn) {
    case 6: return by_fmt<6, 1, false>(a);
    case 7: return by_fmt<7, 1, false>(a);
    case 8: return by_fmt<8, 1, false>(a);
    case 9: return by_fmt<9, 1, false>(a);
    case 10: return by_fmt<10, 1, false>(a);
    case 11: return by_fmt<11, 1, false>(a);
    case 12: return by_fmt<12, 1, false>(a);
    case 13: return by_fmt<13, 1, false>(a);
    case 14: return by_fmt<14, 1, false>(a);
    case 15: return by_fmt<14, 2, false>(a);
    case 16: return by_fmt<14, 4, false>(a);
    case 17: return by_fmt<14, 8, false>(a);
    default: return hipErrorInvalidValue;
    }
}

// ----------------------------------------------------------------- state / ring kernels
// Peak-hold (FftProcessor.kt:241-242) and EMA (extension; GlobalPerformanceData.kt:44-50
// idiom, -inf/uninitialised state re-seeded by the next frame), frame by frame.
__device__ __forceinline__ const float *state_row(const StateLaunch &a, int f) {
    if (a.ring_rows > 0) {
        int rr = (a.ring_base - f) % a.ring_rows;
        return a.rows + (size_t)(rr < 0 ? rr + a.ring_rows : rr) * a.n;
    }
    return a.rows + (size_t)((long long)f * a.row_stride);
}
// ring_pos order of the rows the state kernels read (the ring's; caller rows are natural)
__device__ __forceinline__ int state_logrs(const StateLaunch &a) { return a.ring_rows > 0 ? a.ring_logrs : 0; }
__device__ __forceinline__ int ilog2_dev(int n) { return 31 - __clz(n); }

// The state kernels walk the rows in STORAGE order (ring_pos order when they read
// the ring, natural order for caller / staging rows): every row load is a
// contiguous 16-B load, and the element at storage position p updates the peak /
// EMA of natural bin ring_bin(p) (peaks and EMA are kept in natural order).

// Sequential peak-hold / EMA over the batch (one thread per bin, frames in order).
// Peak: FftProcessor.kt:229-232.  EMA (extension): em += alpha (x - em); an
// uninitialised (-inf) average takes the frame's value.
__global__ void state_kernel(StateLaunch a) {
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;  // storage position
    if (pos >= a.n) return;
    const int lr = state_logrs(a), bin = ring_bin(pos, lr, ring_logm(lr, ilog2_dev(a.n)));
    float pk = a.peaks ? a.peaks[bin] : 0.f;
    float em = a.ema ? a.ema[bin] : 0.f;
    const float al = a.ema_alpha;
#pragma unroll 8
    for (int f = 0; f < a.n_frames; f++) {
        const float x = state_row(a, f)[pos];
        pk = fmaxf(pk, x);
        em = (em > -INFINITY) ? em + al * (x - em) : x;
    }
    if (a.peaks) a.peaks[bin] = pk;
    if (a.ema) a.ema[bin] = em;
}

// The same sequential recursion for a ring in column order with RS = 2^lr >= 8
// residue blocks (N >= 256 K): storage position s*M + q holds natural bin q*RS + s,
// so a thread walking storage order would touch peaks / EMA RS floats apart (one
// cache line per lane).  A workgroup takes the tile q in [q0, q0 + 64) of the
// eight blocks s in [s0, s0 + 8): its row loads stay 256-B coalesced (lane = q),
// and its natural bins are 64 runs of 8 consecutive bins (q*RS + s0 ...), moved
// through LDS (pitch 9, bank conflict free) in and out.  Thread (w = wave,
// l = lane) owns blocks s0 + w and s0 + w + 4.
template <int LR>
__global__ void __launch_bounds__(256) state_tile_kernel(StateLaunch a) {
    constexpr int RS = 1 << LR, SB = 8, SPT = SB / 4, TILE = 64 * SB;
    __shared__ float pk_l[64 * (SB + 1)], em_l[64 * (SB + 1)];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m = a.n >> LR, q0 = blockIdx.x * 64, s0 = blockIdx.y * SB;
    for (int i = threadIdx.x; i < TILE; i += 256) {
        const size_t g = (size_t)(q0 + i / SB) * RS + s0 + i % SB;  // natural bin
        const int li = (i / SB) * (SB + 1) + i % SB;
        pk_l[li] = a.peaks ? a.peaks[g] : 0.f;
        em_l[li] = a.ema ? a.ema[g] : 0.f;
    }
    __syncthreads();
    float pk[SPT], em[SPT];
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        pk[j] = pk_l[l * (SB + 1) + w + 4 * j];
        em[j] = em_l[l * (SB + 1) + w + 4 * j];
    }
    const float al = a.ema_alpha;
    constexpr int FR = 8;  // frames whose loads are in flight together
    for (int f0 = 0; f0 < a.n_frames; f0 += FR) {
        float x[FR][SPT];
#pragma unroll
        for (int k = 0; k < FR; k++) {
            if (f0 + k < a.n_frames) {
                const float *row = state_row(a, f0 + k);
#pragma unroll
                for (int j = 0; j < SPT; j++) x[k][j] = row[(size_t)(s0 + w + 4 * j) * m + q0 + l];
            }
        }
#pragma unroll
        for (int k = 0; k < FR; k++) {
            if (f0 + k >= a.n_frames) break;
#pragma unroll
            for (int j = 0; j < SPT; j++) {
                pk[j] = fmaxf(pk[j], x[k][j]);
                em[j] = (em[j] > -INFINITY) ? em[j] + al * (x[k][j] - em[j]) : x[k][j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < SPT; j++) {
        pk_l[l * (SB + 1) + w + 4 * j] = pk[j];
        em_l[l * (SB + 1) + w + 4 * j] = em[j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TILE; i += 256) {
        const size_t g = (size_t)(q0 + i / SB) * RS + s0 + i % SB;
        const int li = (i / SB) * (SB + 1) + i % SB;
        if (a.peaks) a.peaks[g] = pk_l[li];
        if (a.ema) a.ema[g] = em_l[li];
    }
}

// Chunked form of the same recursions for large batches: blockIdx.y = chunk of
// chunk_len frames.  Per (chunk, bin) it stores
//   x: max over the chunk,
//   y: (1-alpha)^L, or -1 if some frame of the chunk is -inf (the EMA restarts there),
//   z: b with  em_out = y * em_in + b  for a finite em_in and no restart,
//   w: the chunk's EMA started from -inf (= em_out whenever em_in is -inf or the
//      chunk restarts: after a -inf frame both runs are identical).
__global__ void state_partial_kernel(StateLaunch a, int chunk_len) {
    // 4 adjacent bins per thread: one 16-B row load per frame (N is a multiple of 64)
    const int bin = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    const int c = blockIdx.y;
    if (bin >= a.n) return;
    const int f0 = c * chunk_len, f1 = min(a.n_frames, f0 + chunk_len);
    const float al = a.ema_alpha, keep = 1.0f - al;
    float pk[4], emi[4], b[4];
    bool restart[4];
#pragma unroll
    for (int k = 0; k < 4; k++) pk[k] = emi[k] = -INFINITY, b[k] = 0.0f, restart[k] = false;
    float am = 1.0f;
#pragma unroll 4
    for (int f = f0; f < f1; f++) {
        const float4 x4 = *reinterpret_cast<const float4 *>(state_row(a, f) + bin);  // storage positions
        const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
        for (int k = 0; k < 4; k++) state_step(pk[k], emi[k], b[k], restart[k], xs[k], al);
        am *= keep;
    }
    float4 *out = a.part + (size_t)c * a.n + bin;
#pragma unroll
    for (int k = 0; k < 4; k++) out[k] = make_float4(pk[k], restart[k] ? -1.0f : am, b[k], emi[k]);
}

__global__ void state_combine_kernel(StateLaunch a, int chunks) {
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;  // storage position of the partials
    if (pos >= a.n) return;
    const int lr = state_logrs(a), bin = ring_bin(pos, lr, ring_logm(lr, ilog2_dev(a.n)));
    float pk = a.peaks ? a.peaks[bin] : 0.f;
    float em = a.ema ? a.ema[bin] : 0.f;
    for (int c = 0; c < chunks; c++) {
        const float4 p = a.part[(size_t)c * a.n + pos];
        pk = fmaxf(pk, p.x);
        em = (em == -INFINITY || p.y < 0.0f) ? p.w : fmaf(p.y, em, p.z);
    }
    if (a.peaks) a.peaks[bin] = pk;
    if (a.ema) a.ema[bin] = em;
}

// One launch for the chunked scan: a block owns 1024/CH bins (4 per thread) and
// all CH chunks of frames; the chunk summaries meet in LDS and the block folds
// them in frame order into peaks / EMA (same algebra as state_combine_kernel),
// so no summary buffer round trip and no second launch.
#ifndef RFA_STATE_BUF
#define RFA_STATE_BUF 1
#endif
#ifndef RFA_STATE_UNROLL
#define RFA_STATE_UNROLL 4
#endif
#ifndef RFA_STATE_LOAD_AUX
#define RFA_STATE_LOAD_AUX 0  // cache policy of the ring-row loads (A/B: 2 = nt)
#endif
template <int CH>
__global__ void __launch_bounds__(256) state_fused_kernel(StateLaunch a, int chunk_len) {
    constexpr int TPC = 256 / CH, BPB = 4 * TPC;  // threads per chunk, bins per block
    __shared__ float4 part[CH][BPB];
    const int c = threadIdx.x / TPC, l = threadIdx.x % TPC;
    const int bin = blockIdx.x * BPB + 4 * l;
    {
        const int f0 = c * chunk_len, f1 = min(a.n_frames, f0 + chunk_len);
        const float al = a.ema_alpha, keep = 1.0f - al;
        float pk[4], emi[4], b[4];
        bool restart[4];
#pragma unroll
        for (int k = 0; k < 4; k++) pk[k] = emi[k] = -INFINITY, b[k] = 0.0f, restart[k] = false;
        float am = 1.0f;
        auto step = [&](float4 x4) {
            const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
            for (int k = 0; k < 4; k++) state_step(pk[k], emi[k], b[k], restart[k], xs[k], al);
            am *= keep;
        };
        if (RFA_STATE_BUF && a.ring_rows > 0 && (long long)a.ring_rows * a.n * 4 < (1ll << 31)) {
            // ring rows: the chunk's first row once, then one row down per frame with the wrap
            // (FftProcessor.kt:226-227 writeIndex--), as 32-bit buffer offsets -- not a modulo
            // and a 64-bit address per frame (four chunks share a wave, so they are per lane)
            const unsigned rowb = (unsigned)a.n * 4u;
            const rsrc_t rs = make_rsrc(a.rows, (unsigned)a.ring_rows * rowb);
            int rr = (a.ring_base - f0) % a.ring_rows;
            if (rr < 0) rr += a.ring_rows;
#pragma unroll RFA_STATE_UNROLL
            for (int f = f0; f < f1; f++) {
                step(__builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((unsigned)rr * rowb + (unsigned)bin * 4u), 0, RFA_STATE_LOAD_AUX)));
                rr = rr == 0 ? a.ring_rows - 1 : rr - 1;
            }
        } else {
#pragma unroll 4  // frames in flight per thread (profiles/r02c/state_unroll_ab.txt)
            for (int f = f0; f < f1; f++) step(*reinterpret_cast<const float4 *>(state_row(a, f) + bin));  // storage positions
        }
#pragma unroll
        for (int k = 0; k < 4; k++) part[c][4 * l + k] = make_float4(pk[k], restart[k] ? -1.0f : am, b[k], emi[k]);
    }
    __syncthreads();
    const int lr = state_logrs(a), lm = ring_logm(lr, ilog2_dev(a.n));
    for (int i = threadIdx.x; i < BPB; i += 256) {
        const int gb = ring_bin(blockIdx.x * BPB + i, lr, lm);  // natural bin of storage position
        float p = a.peaks ? a.peaks[gb] : 0.f;
        float em = a.ema ? a.ema[gb] : 0.f;
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            const float4 q = part[cc][i];
            p = fmaxf(p, q.x);
            em = (em == -INFINITY || q.y < 0.0f) ? q.w : fmaf(q.y, em, q.z);
        }
        if (a.peaks) a.peaks[gb] = p;
        if (a.ema) a.ema[gb] = em;
    }
}

#ifdef RFA_AB_BUILD
static const bool kStateTileOff = std::getenv("RFA_STATE_TILE") && std::atoi(std::getenv("RFA_STATE_TILE")) == 0;
#else
static constexpr bool kStateTileOff = false;
#endif

bool state_fused_plan(int n, int n_frames, int max_chunks, int fused, int *chunks, int *chunk_len) {
    const int c = std::min(max_chunks, (n_frames + 7) / 8);
    if (c < 8 || !fused) return false;
    const int ch = c >= 32 ? 32 : c >= 16 ? 16 : 8;
    if (n % (1024 / ch)) return false;
    *chunks = ch;
    *chunk_len = (n_frames + ch - 1) / ch;
    return true;
}

hipError_t launch_state(const StateLaunch &a) {
    if (a.n_frames <= 0) return hipSuccess;
    const int tpb = 256;
    if (a.ring_rows > 0 && !(a.ring_logrs & kRingTile) && a.ring_logrs >= 3 && a.ring_logrs <= 5 && !kStateTileOff) {
        // column-order ring (N >= 256 K): tiled sequential update (RFA_STATE_TILE=0: A/B off)
        const int m = a.n >> a.ring_logrs;
        if (m % 64 == 0) {
            auto k = a.ring_logrs == 5 ? state_tile_kernel<5> : a.ring_logrs == 4 ? state_tile_kernel<4>
                                                                                  : state_tile_kernel<3>;
            hipLaunchKernelGGL(k, dim3(m / 64, (1 << a.ring_logrs) / 8), dim3(256), 0, a.stream, a);
            return hipGetLastError();
        }
    }
    const int bx = (a.n + tpb - 1) / tpb;
    int chunks = a.part ? std::min(a.max_chunks, (a.n_frames + 7) / 8) : 1;
    int ch = 0, len = 0;
    if (a.part && state_fused_plan(a.n, a.n_frames, a.max_chunks, a.fused, &ch, &len)) {
        // single-launch form: CH = 8, 16 or 32 chunks
        auto k = ch == 32 ? state_fused_kernel<32> : ch == 16 ? state_fused_kernel<16> : state_fused_kernel<8>;
        hipLaunchKernelGGL(k, dim3(a.n / (1024 / ch)), dim3(256), 0, a.stream, a, len);
        return hipGetLastError();
    }
    if (chunks > 1) {
        const int len = (a.n_frames + chunks - 1) / chunks;
        chunks = (a.n_frames + len - 1) / len;
        hipLaunchKernelGGL(state_partial_kernel, dim3((a.n / 4 + tpb - 1) / tpb, chunks), dim3(tpb), 0, a.stream, a,
                           len);
        hipLaunchKernelGGL(state_combine_kernel, dim3(bx), dim3(tpb), 0, a.stream, a, chunks);
    } else {
        hipLaunchKernelGGL(state_kernel, dim3(bx), dim3(tpb), 0, a.stream, a);
    }
    return hipGetLastError();
}

// FftProcessor.kt:143-157: mean of the channel's dB bins per frame (the squelch input).
// One workgroup per frame: thread t adds bins first + t, first + t + 256, ... in that
// order (each wave instruction reads 64 consecutive natural bins of the row), then the
// 256 partial sums are folded in a fixed order (wavefront shuffles, wave.h, then the
// four waves).  Deterministic, and within a few fp32 ulps of the reference's sequential fp32 loop (:150-152) -- which is itself only one
// rounding order of the sum; the rows it averages already differ from pffft's by up to
// the FFT tolerance.  Round 2 kept that loop's order exactly, one lane per frame: a
// dependent add per bin behind a load that gathers 64 rows per wave instruction,
// +64 us per 500-frame 64 K step for a 1000-bin channel and +2.1 ms for 32000 bins
// (profiles/r03/channel_mean_ab.txt).
__global__ void __launch_bounds__(256) channel_mean_kernel(StateLaunch a, int first, int last, int span, float *out,
                                                          float *partial) {
    __shared__ float part[4];
    const int f = blockIdx.x, t = threadIdx.x;
    const float *row = state_row(a, f);
    const int lr = state_logrs(a), lm = ring_logm(lr, ilog2_dev(a.n));
    // wide channels: blockIdx.y takes bins [lo, hi) of the channel (span bins each)
    const int lo = first + blockIdx.y * span, hi = min(last, lo + span);
    float s = 0.0f;
    int i = lo + t;
    for (; i + 3 * 256 < hi; i += 4 * 256) {  // four loads in flight per thread
        const float x0 = row[ring_pos(i, lr, lm)], x1 = row[ring_pos(i + 256, lr, lm)];
        const float x2 = row[ring_pos(i + 512, lr, lm)], x3 = row[ring_pos(i + 768, lr, lm)];
        s = (((s + x0) + x1) + x2) + x3;
    }
    for (; i < hi; i += 256) s += row[ring_pos(i, lr, lm)];
    // wave sums by cross-lane moves (wave.h), then the four waves' in order
    s = wave_reduce(s, [](float x, float y) { return x + y; });
    if ((t & 63) == 0) part[t >> 6] = s;
    __syncthreads();
    if (t == 0) {
        const float sum = ((part[0] + part[1]) + part[2]) + part[3];
        if (gridDim.y == 1) out[f] = sum / (float)(last - first);
        else partial[(size_t)f * gridDim.y + blockIdx.y] = sum;
    }
}

// wide channels: the per-span sums of a frame folded in span order
__global__ void channel_mean_fold_kernel(int n_frames, int spans, int width, const float *partial, float *out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    float s = 0.0f;
    for (int k = 0; k < spans; k++) s += partial[(size_t)f * spans + k];
    out[f] = s / (float)width;
}

int channel_mean_spans(int width) { return std::min(64, std::max(1, (width + 16383) / 16384)); }

hipError_t launch_channel_mean(const StateLaunch &a, int first, int last, float *out, float *partial) {
    if (a.n_frames <= 0 || last <= first) return hipSuccess;
    const int width = last - first, spans = channel_mean_spans(width), span = (width + spans - 1) / spans;
    if (spans > 1 && !partial) return hipErrorInvalidValue;
    hipLaunchKernelGGL(channel_mean_kernel, dim3(a.n_frames, spans), dim3(256), 0, a.stream, a, first, last, span, out,
                       partial);
    if (spans > 1)
        hipLaunchKernelGGL(channel_mean_fold_kernel, dim3((a.n_frames + 255) / 256), dim3(256), 0, a.stream, a.n_frames,
                           spans, width, partial, out);
    return hipGetLastError();
}

__global__ void fill_kernel(float *p, long long count, float value) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < count;
         i += (long long)gridDim.x * blockDim.x)
        p[i] = value;
}

hipError_t launch_fill(float *p, long long count, float value, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, count, value);
    return hipGetLastError();
}

// dst[row][i] = src[row][i - shift] (fill outside) -- FftProcessor.kt:202-209; bins
// i addressed through the ring's storage order (ring_pos)
__global__ void ring_shift_kernel(const float *src, float *dst, int n, int logrs, int shift, float fill) {
    const int row = blockIdx.y;
    const int lm = ring_logm(logrs, ilog2_dev(n));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int s = i - shift;
        dst[(size_t)row * n + ring_pos(i, logrs, lm)] =
            (s >= 0 && s < n) ? src[(size_t)row * n + ring_pos(s, logrs, lm)] : fill;
    }
}

hipError_t launch_ring_shift(const float *src, float *dst, int rows, int n, int logrs, int shift, float fill,
                             hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    int bx = (n + 255) / 256;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(ring_shift_kernel, dim3(bx, rows), dim3(256), 0, s, src, dst, n, logrs, shift, fill);
    return hipGetLastError();
}

__global__ void ring_natural_kernel(const float *src, float *dst, int n, int logrs) {
    const int row = blockIdx.y;
    const int lm = ring_logm(logrs, ilog2_dev(n));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        dst[(size_t)row * n + i] = src[(size_t)row * n + ring_pos(i, logrs, lm)];
}

hipError_t launch_ring_natural(const float *src, float *dst, int rows, int n, int logrs, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    int bx = (n + 255) / 256;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(ring_natural_kernel, dim3(bx, rows), dim3(256), 0, s, src, dst, n, logrs);
    return hipGetLastError();
}

// FftProcessor.kt:185-195: the resized ring keeps the history rotated so the
// next write (writeIndex = 0) lands on the oldest row.
__global__ void ring_rotate_kernel(const float *src, int src_rows, float *dst, int n, int write_index, float fill) {
    const int row = blockIdx.y;
    const float4 *s4 = row < src_rows
                           ? reinterpret_cast<const float4 *>(src + (size_t)((write_index + row) % src_rows) * n)
                           : nullptr;
    float4 *d4 = reinterpret_cast<float4 *>(dst + (size_t)row * n);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += gridDim.x * blockDim.x)
        d4[i] = s4 ? s4[i] : make_float4(fill, fill, fill, fill);
}

hipError_t launch_ring_rotate(const float *src, int src_rows, float *dst, int dst_rows, int n, int write_index,
                              float fill, hipStream_t s) {
    if (dst_rows <= 0) return hipSuccess;
    int bx = (n / 4 + 255) / 256;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(ring_rotate_kernel, dim3(bx, dst_rows), dim3(256), 0, s, src, src ? src_rows : 0, dst, n,
                       write_index, fill);
    return hipGetLastError();
}

// AnalyzerSurface.kt:710-714 at bin resolution: fp32 sum newest-first, / (L+1).
__global__ void boxcar_kernel(const float *ring, int rows, int n, int logrs, int read_index, int length, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = ring_pos(i, logrs, ring_logm(logrs, ilog2_dev(n)));
    float acc = 0.f;
    for (int r = 0; r <= length; r++) acc += ring[(size_t)((read_index + r) % rows) * n + p];
    out[i] = acc / (float)(length + 1);
}

hipError_t launch_boxcar(const float *ring, int rows, int n, int logrs, int read_index, int length, float *out,
                         hipStream_t s) {
    hipLaunchKernelGGL(boxcar_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ring, rows, n, logrs, read_index,
                       length, out);
    return hipGetLastError();
}

// Streaming copy at the HBM ceiling (bench denominator): one float4 per lane, one
// pass over the buffer (the fastest of the shapes in
// profiles/r02a/copy_kernel_variants.txt: 6.2 TB/s read + write on MI355X).
__global__ void __launch_bounds__(256) stream_copy_kernel(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                          long long n4) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) dst[i] = src[i];
}

hipError_t launch_stream_copy(void *dst, const void *src, size_t bytes, hipStream_t s) {
    const long long n4 = (long long)(bytes / 16);
    if (n4 <= 0) return hipSuccess;
    for (long long off = 0; off < n4; off += (long long)0x7fffffff / 256 * 256) {  // grid.x limit
        const long long cnt = std::min<long long>(n4 - off, (long long)0x7fffffff / 256 * 256);
        hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s,
                           static_cast<float4 *>(dst) + off, static_cast<const float4 *>(src) + off, cnt);
    }
    return hipGetLastError();
}

}  // namespace rfa
