// gfx950 "wide" sub-FFT kernel: one M-point sub-FFT (M = 8192, 16384 or 32768)
// per work item, 32 points per thread in VGPRs, M/32 threads per workgroup (256
// for 8 K, 512 for 16 K, 1024 for 32 K).
//
// Shape (measured): 32 points per thread keeps the
// kernel at 128 VGPRs (4 waves per SIMD), an M-point FFT needs three in-register
// radix-32/16 passes and two LDS exchanges, and each exchange runs in two
// half-rounds through an M/2 buffer (66 KiB for 16 K: two workgroups per CU;
// 132 KiB for 32 K: one).  N = 64 K / 128 K run as RS = 2 / 4 residue work
// items of the 32 K workgroup (decimation-in-frequency pre-stage below).
//
// Per work item (frame, residue r) the pipeline is the same as the narrow
// kernel (fft_kernels.hip): raw IQ -> LUT-exact convert -> window (fp32
// multiply, NativeDsp.kt:55-58) [-> decimation-in-frequency pre-stage for
// N = RS*M] -> FFT (sign -1, unscaled, natural order: pffft.h:117) ->
// 10*log10(sqrt((Re/N)^2+(Im/N)^2)) + fft-shift (nativedsp.cpp:72-79) -> rows/ring.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "fft_common.h"
#include "fft_kernels.h"

namespace rfa {

template <int LOGM, int PT>
struct WGeo {
    static constexpr int M = 1 << LOGM;
    static constexpr int TPF = M / PT;           // threads per sub-FFT (PT points per thread)
    static constexpr int THREADS = TPF < 256 ? 256 : TPF;
    static constexpr int SLOTS = THREADS / TPF;  // sub-FFTs per workgroup
    static constexpr int HALF = M / 2;           // exchange buffer (float2) per slot ...
    static constexpr int HALFP = HALF + HALF / 32;  // ... with one float2 of padding per 32
    static constexpr int R1 = LOGM >= 14 ? 32 : 16;  // radix of pass 1 (pass 0: 32)
    static constexpr int R2 = M / (32 * R1);          // radix of pass 2: 16 (8 K, 16 K) or 32 (32 K)
    // LDS twiddle tables (float2, t = 1..R-1 only).  Odd row strides (R-1)
    // spread the rows read by one lane group over distinct banks.
    static constexpr int P1_ROW = R1 - 1;        // pass 1: [k = tid & 31][t]
    static constexpr int TW_P1 = 32 * P1_ROW;
    static constexpr int LO = TPF > 256 ? 32 : 16;  // pass 2: tid = hi*LO + lo
    static constexpr int P2_ROW = R2 - 1;
    static constexpr int TW_P2A = (TPF / LO) * P2_ROW;  // A[hi][t] = W_M^{t hi LO}
    static constexpr int TW_P2B = LO * P2_ROW;          // B[lo][t] = W_M^{t lo}
    static constexpr int TW_LDS = TW_P1 + TW_P2A + TW_P2B;
    static constexpr int LDS_BYTES = (TW_LDS + SLOTS * HALFP) * 8;
    // staged kernels: + 16 B for the work-queue slot (next item index)
    static constexpr int LDS_Q_BYTES = 16;
};

template <int Q, int LOGM, int PT>
struct WPass {
    using G = WGeo<LOGM, PT>;
    static constexpr int R = Q == 0 ? 32 : (Q == 1 ? G::R1 : G::R2);
    static constexpr int P = Q == 0 ? 1 : (Q == 1 ? 32 : 32 * G::R1);  // product of earlier radices
    static constexpr int NB = PT / R;                                 // butterflies per thread
    static constexpr int STRIDE = G::M / R;                           // input stride of a butterfly
};

// Padded exchange-buffer index (one float2 per 32): every access pattern of
// the three passes is bank-conflict free, and because all lane
// bases have zero low-5 bits w.r.t. the compile-time parts, pad(base + c) =
// pad(base) + pad(c): LDS addresses are lane base + immediate.
__device__ __forceinline__ constexpr int padw(int e) { return e + (e >> 5); }

// Exchange pass Q's outputs (v) for pass Q+1's inputs through the M/2 LDS
// buffer in two half-rounds.  Round h moves the outputs that land in
// [h*M/2, (h+1)*M/2) -- butterflies [h*NB/2, (h+1)*NB/2), or, with one
// butterfly per thread, the threads with (tid >= TPF/2) == h (wave-uniform) --
// and the inputs with t' in [h*R'/2, (h+1)*R'/2), which come from the same
// half.  Reads go to fresh SSA temporaries (compile-time renaming), so round-1
// outputs are never overwritten by round-0 inputs.
// LDS pointer the compiler cannot see through: per-thread LDS bases built
// inside a work item are then not hoisted out of the item loop (and spilled).
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lds_opaque(T *p) {
    auto q = (__attribute__((address_space(3))) T *)p;
    asm volatile("" : "+v"(q));
    return q;
}
#else
template <typename T>
__device__ __forceinline__ T *lds_opaque(T *p) { return p; }  // host pass: never executed
#endif

template <int Q, int LOGM, int PT, int KR = 2>
__device__ __forceinline__ void exchange(float2 (&v)[PT], float2 *buf, int tid) {
    // KR rounds (2: the M/2 buffer; 4: an M/4 buffer, RFA_SPLIT_STAGE) -- round h
    // moves the outputs landing in [h*M/KR, (h+1)*M/KR) and the inputs t' in
    // [h*R'/KR, (h+1)*R'/KR), which come from the same part
    using G = WGeo<LOGM, PT>;
    using W = WPass<Q, LOGM, PT>;
    using N = WPass<Q + 1, LOGM, PT>;
    static_assert(N::R >= KR && (W::NB == 1 || W::NB % KR == 0), "round split needs radix >= KR");
    constexpr int PART = G::M / KR, PARTP = PART + PART / 32;
    float2 in[KR][PT / KR];
    const int wk = tid & (W::P - 1);
    const int wbase = padw((tid - wk) * W::R + wk);  // butterfly b adds R*TPF*b
    const int rbase = padw(tid);                     // butterfly b adds TPF*b
    const int my_part = tid / (G::TPF / KR);         // NB == 1 writers only
#pragma unroll
    for (int h = 0; h < KR; h++) {
        if constexpr (W::NB == 1) {
            if (my_part == h) {
#pragma unroll
                for (int t = 0; t < W::R; t++) buf[wbase + padw(t * W::P) - h * PARTP] = v[t];
            }
        } else {
#pragma unroll
            for (int b = h * W::NB / KR; b < (h + 1) * W::NB / KR; b++) {
#pragma unroll
                for (int t = 0; t < W::R; t++)
                    buf[wbase + padw(W::R * G::TPF * b + t * W::P - h * PART)] = v[b * W::R + t];
            }
        }
        lds_barrier();
#pragma unroll
        for (int b = 0; b < N::NB; b++) {
#pragma unroll
            for (int t = h * N::R / KR; t < (h + 1) * N::R / KR; t++)
                in[h][b * (N::R / KR) + (t - h * N::R / KR)] =
                    buf[rbase + padw(G::TPF * b + t * N::STRIDE - h * PART)];
        }
        lds_barrier();
    }
#pragma unroll
    for (int b = 0; b < N::NB; b++) {
#pragma unroll
        for (int t = 0; t < N::R; t++) {
            const int h = t / (N::R / KR);
            v[b * N::R + t] = in[h][b * (N::R / KR) + (t - h * N::R / KR)];
        }
    }
}

// Pass 1: k = tid & 31 is the same for every butterfly of the thread; its
// twiddles W_{32 R}^{t k} sit contiguously at twp1[k][t-1] (exact, from double).
template <int LOGM, int PT>
__device__ __forceinline__ void pass1(float2 (&v)[PT], int tid, const float2 *twp1) {
    using W = WPass<1, LOGM, PT>;
    const float2 *row = twp1 + (tid & 31) * WGeo<LOGM, PT>::P1_ROW - 1;
#pragma unroll
    for (int b = 0; b < W::NB; b++) {
        v[b * W::R + 1] = cmul(v[b * W::R + 1], row[1]);
#pragma unroll
        for (int t = 2; t < W::R; t += 2) cmul2(v[b * W::R + t], row[t], v[b * W::R + t + 1], row[t + 1]);
    }
#pragma unroll
    for (int b = 0; b < W::NB; b++) dft<W::R>(&v[b * W::R]);
}

// Pass 2 (last, radix R2): k = i = tid + TPF*b.  W_M^{t i} = W_M^{t tid} * W_PT^{t b}
// (M / TPF = PT); W_M^{t tid} = A[tid/LO][t] * B[tid%LO][t] from two exact
// tables, the b-dependent factor is a compile-time constant.
template <int PT, int R2, int T, int B>
__device__ __forceinline__ void p2_const(float2 (&v)[PT]) {
    v[B * R2 + T] = w64<T * B * (64 / PT)>(v[B * R2 + T]);
}
template <int PT, int R2, int T, int... Bs>
__device__ __forceinline__ void p2_const_t(float2 (&v)[PT], std::integer_sequence<int, Bs...>) {
    (p2_const<PT, R2, T, Bs + 1>(v), ...);
}
template <int PT, int R2, int... Ts>
__device__ __forceinline__ void p2_const_all(float2 (&v)[PT], std::integer_sequence<int, Ts...>) {
    (p2_const_t<PT, R2, Ts>(v, std::make_integer_sequence<int, PT / R2 - 1>{}), ...);
}

template <int LOGM, int PT>
__device__ __forceinline__ void pass2(float2 (&v)[PT], int tid, const float2 *twp2) {
    using G = WGeo<LOGM, PT>;
    using W = WPass<2, LOGM, PT>;
    constexpr int R2 = G::R2;
    const float2 *ra = twp2 + (tid / G::LO) * G::P2_ROW - 1;
    const float2 *rb = twp2 + G::TW_P2A + (tid % G::LO) * G::P2_ROW - 1;
    {
        const float2 w1 = cmul(ra[1], rb[1]);
#pragma unroll
        for (int b = 0; b < W::NB; b++) v[b * R2 + 1] = cmul(v[b * R2 + 1], w1);
    }
#pragma unroll
    for (int t = 2; t < R2; t += 2) {  // twiddle pairs built and applied in place (no table in VGPRs)
        float2 w0 = ra[t], w1 = ra[t + 1];
        cmul2(w0, rb[t], w1, rb[t + 1]);
#pragma unroll
        for (int b = 0; b < W::NB; b++) cmul2(v[b * R2 + t], w0, v[b * R2 + t + 1], w1);
    }
    if constexpr (W::NB > 1) p2_const_all<PT, R2>(v, std::make_integer_sequence<int, R2>{});
#pragma unroll
    for (int b = 0; b < W::NB; b++) dft<R2>(&v[b * R2]);
}

// x * W_16^q added to acc, with the rotation / sqrt(1/2) forms folded in.
template <int Q>
__device__ __forceinline__ float2 add_w16(float2 acc, float2 x) {
    constexpr int q = Q & 15;
    if constexpr ((q & 3) == 0) return padd<0, q / 4>(acc, x);
    else if constexpr ((q & 3) == 2) return from_v(__builtin_elementwise_fma(to_v(padd<(q - 2) / 4, (q + 2) / 4>(x, x)), (f2v){kR2, kR2}, to_v(acc)));
    else return cadd(acc, w16<q>(x));
}

// Decimation-in-frequency pre-stage for N = RS * M, residue R (compile-time):
//   y_R[m] = W_N^{m R} * sum_j x[m + jM] w[m + jM] W_RS^{j R},   m = tid + TPF b + (M/32) t
// W_N^{m R} = pre_a[R][tid + TPF b] * pre_b[R][t] (exact tables).  The RS raw
// samples of a point come from RS separate quarter-frames; the RS window values
// are adjacent in the interleaved window (one 8/16-byte load).  Loads run one
// chunk ahead of the arithmetic (software pipeline), so a wave keeps two
// chunks of L2 requests in flight instead of waiting a full round trip per chunk.
// 64 K, 8-bit input: stage the next frame in two halves, the first right after the
// pre-stage (exchanges then run in four rounds through a quarter buffer).  1 = on
// (default, -1..-4 % kernel time, profiles/r02g/split_stage_ab.txt), 0 = whole frame
// after exchange 1, 2 = first half after exchange 0 (+10 %, not kept), 3 = second half
// loaded directly by the pre-stage (+5..8 %, not kept, split_direct_ab.txt).
#ifndef RFA_SPLIT_STAGE
#define RFA_SPLIT_STAGE 1
#endif
// 8/16 K ... 32 K one-residue kernels, 8-bit input: with the exchanges in four rounds
// through region A the whole next frame fits region B and is staged right after the
// pre-stage (RFA_SPLIT_WHOLE=1).
#ifndef RFA_SPLIT_WHOLE
#define RFA_SPLIT_WHOLE 0
#endif
#ifndef PRE_DIST
#define PRE_DIST 1
#endif

// WP > 0 (RS = 2): the window pairs (w[m], w[m+M]) of the thread's first WP points
// arrive preloaded in wpre[idx] (issued by the previous item's tail, see
// fft_wide_kernel); the rest are loaded here, behind the preloaded chunks' work.
#ifndef RFA_WPRE
#define RFA_WPRE 0  // measured slower at 8/16/32 (profiles/r02a/window_preload_and_stagger_ab.txt): spills
#endif
// PADRAW (fft_w64_kernel): the staged frame sits in LDS as 8 KiB pieces at a
// 8448-B pitch (one piece per wave region), i.e. raw element e at e + (e >> 12) * 128.
template <int LOGM, int PT, int RS, int FMT, int R, bool STG = false, bool NOWIN = false, int WP = 0,
          bool PADRAW = false, int JS = 0, bool HI_DIRECT = false>
__device__ __forceinline__ void prestage(float2 (&v)[PT], const float *window_il, const float2 *wide_tw, rsrc_t in_rs,
                                         int tid, int planar_im, const typename Raw<FMT>::T *lraw = nullptr,
                                         const float2 *wpre = nullptr) {
    static_assert(WP == 0 || RS == 2, "preloaded window pairs: RS = 2 only");
    using G = WGeo<LOGM, PT>;
    constexpr int M = G::M;
    constexpr int SB = FMT == 4 ? 4 : ((FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8));  // bytes per sample (per plane)
    // points per chunk: two chunks of raw samples + window values in flight must
    // fit beside the PT points in the register budget (64 VGPRs at PT = 32)
    constexpr int C = (PT == 64 ? 16 : 8) / RS > 0 ? (PT == 64 ? 16 : 8) / RS : 1;
    constexpr int NCH = PT / C;
    auto lraw_t = [&] {  // this thread's samples in the staged frame (opaque base, see lds_opaque)
        if constexpr (STG) return lds_opaque(lraw + tid);
        else return lraw;
    }();
    const rsrc_t w_rs = make_rsrc(window_il, M * RS * 4);
    const rsrc_t pa_rs = make_rsrc(wide_tw + G::TW_LDS, RS * (M / 32) * 8);
    const float2 *pre_b = wide_tw + G::TW_LDS + RS * (M / 32) + R * 32;
    float2 pa[PT / 32];
    if constexpr (R != 0) {
#pragma unroll
        for (int b = 0; b < PT / 32; b++) pa[b] = buf_load_f32x2(pa_rs, (tid + G::TPF * b) * 8, R * (M / 32) * 8);
    }
    // loads run DIST chunks ahead of the arithmetic (RFA_PRE_DIST experiments: 1 or 2)
    constexpr int DIST = PRE_DIST;
    typename Raw<FMT>::T raw[DIST + 1][C][RS];
    float win[DIST + 1][C][RS];
    // c is a template parameter throughout: every register array index below is a
    // compile-time constant (a runtime index would move the arrays to scratch)
    auto issue = [&]<int c>() {
        constexpr int s = c % (DIST + 1);
#pragma unroll
        for (int q = 0; q < C; q++) {
            const int idx = c * C + q, b = idx >> 5, t = idx & 31;
            const int mo = G::TPF * b + (M / 32) * t;  // uniform part of m
#pragma unroll
            for (int j = 0; j < RS; j++) {
                if constexpr (STG) {  // frame staged in LDS
                    if (HI_DIRECT && j >= 1) {  // RFA_SPLIT_STAGE=3: the second half straight from memory
                        raw[s][q][j] = buf_load_raw<FMT>(in_rs, tid * SB, (mo + j * M) * SB, planar_im);
                    } else {
                        // JS != 0 (RFA_SPLIT_STAGE): the frame's halves sit JS raw elements apart
                        const int e = mo + j * (JS != 0 ? JS : M);
                        raw[s][q][j] = lraw_t[PADRAW ? e + (e >> 12) * 128 : e];
                    }
                }
                else raw[s][q][j] = buf_load_raw<FMT>(in_rs, tid * SB, (mo + j * M) * SB, planar_im);
            }
            if constexpr (NOWIN) {  // ablation (RFA_DIAG=16): constant window, no window loads
#pragma unroll
                for (int j = 0; j < RS; j++) win[s][q][j] = 1.0f / 128.0f;
            } else if (WP > 0 && c * C + q < WP) {
                win[s][q][0] = wpre[idx < WP ? idx : 0].x;
                win[s][q][1] = wpre[idx < WP ? idx : 0].y;
            } else if constexpr (RS == 2) {
                const f2v w = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(w_rs, tid * 8, mo * 8, 0));
                win[s][q][0] = w.x;
                win[s][q][1] = w.y;
            } else {
#pragma unroll
                for (int j4 = 0; j4 < RS; j4 += 4) {
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    const f4v w = __builtin_bit_cast(
                        f4v, __builtin_amdgcn_raw_buffer_load_b128(w_rs, tid * RS * 4, (mo * RS + j4) * 4, 0));
                    win[s][q][j4] = w.x;
                    win[s][q][j4 + 1] = w.y;
                    win[s][q][j4 + 2] = w.z;
                    win[s][q][j4 + 3] = w.w;
                }
            }
        }
    };
    auto compute = [&]<int c>() {
        constexpr int s = c % (DIST + 1);
        float2 accs[C];
#pragma unroll
        for (int q = 0; q < C; q++) {
            float2 &acc = accs[q];
            [&]<int... Js>(std::integer_sequence<int, Js...>) {
                (
                    [&] {
                        const float2 x = convert_raw<FMT>(raw[s][q][Js]);
                        const float2 xw = from_v(to_v(x) * win[s][q][Js]);  // NativeDsp.kt:55-58 (fp32 multiply)
                        if constexpr (Js == 0) acc = xw;
                        else acc = add_w16<(Js * R * (16 / RS)) & 15>(acc, xw);  // W_RS^{j R} = W_16^{j R 16/RS}
                    }(),
                    ...);
            }(std::make_integer_sequence<int, RS>{});
        }
        if constexpr (RS == 2 && R != 0) {
            // W_N^{m R} = pre_a[tid + TPF b] * W_64^{t R} (N = 2M: pre_b is a compile-time
            // rotation, no table reads / scalar address registers)
            [&]<int... Qs>(std::integer_sequence<int, Qs...>) {
                (
                    [&] {
                        constexpr int i0 = c * C + Qs;
                        v[i0] = w64<((i0 & 31) * R) & 63>(cmul(accs[Qs], pa[i0 >> 5]));
                    }(),
                    ...);
            }(std::make_integer_sequence<int, C>{});
            return;
        }
        // twiddle W_N^{m R} = pre_a * pre_b, then acc * twiddle: independent pairs interleaved
#pragma unroll
        for (int q = 0; q < C; q += 2) {
            const int i0 = c * C + q;
            if constexpr (R == 0) {
                v[i0] = accs[q];
                if (q + 1 < C) v[i0 + 1] = accs[q + 1];
            } else if (q + 1 < C) {
                float2 w0 = pa[i0 >> 5], w1 = pa[(i0 + 1) >> 5];
                cmul2(w0, pre_b[i0 & 31], w1, pre_b[(i0 + 1) & 31]);
                cmul2(accs[q], w0, accs[q + 1], w1);
                v[i0] = accs[q];
                v[i0 + 1] = accs[q + 1];
            } else {
                v[i0] = cmul(accs[q], cmul(pa[i0 >> 5], pre_b[i0 & 31]));
            }
        }
    };
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        ((Cs < DIST && Cs < NCH ? issue.template operator()<Cs>() : void()), ...);
    }(std::make_integer_sequence<int, DIST>{});
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        (
            [&] {
                if constexpr (Cs + DIST < NCH) issue.template operator()<Cs + DIST>();
                __builtin_amdgcn_sched_barrier(0);
                compute.template operator()<Cs>();
                __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
    }(std::make_integer_sequence<int, NCH>{});
}

// LDS-DMA staging of one frame's raw bytes (STG kernels): the frame's n*BPS
// bytes go HBM -> LDS exchange buffer in natural order, 1 KiB per wave
// instruction (buffer_load_dwordx4 ... lds: no VGPRs, 16 B per lane), issued
// for the NEXT work item right after the current item's last LDS exchange, so
// the loads fly during pass 2, the dB epilogue and the next item's start.
// cache policy of the staging DMA (A/B builds: -DSTG_POLICY='"nt "')
#ifndef STG_POLICY
#define STG_POLICY ""
#endif
template <int BYTES, int THREADS>
__device__ __forceinline__ void stage_frame(const void *src, float2 *buf) {
    static_assert(BYTES % (1024 * (THREADS / 64)) == 0, "whole 1 KiB pieces per wave");
    constexpr int NW = THREADS / 64, PER = BYTES / 1024 / NW;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const rsrc_t rs = make_rsrc(src, BYTES);
    // LDS byte address of the buffer (generic -> local address-space cast)
    const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) uint8_t *)(uint8_t *)buf;
    // Inline asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: hipcc treats a pending
    // LDS-DMA as aliasing every later ds_read and waits vmcnt(0) before pass 2's
    // twiddle reads, which would serialise the prefetch.  Its completion is waited
    // for explicitly (vmcnt(0) + barrier at the start of the next item).
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const int c = j * NW + w;  // wave-uniform 1 KiB piece
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %4 offen " STG_POLICY "lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(base + c * 1024), "v"(lane * 16), "s"(rs), "s"(c * 1024)
            : "memory");
    }
}

// DIAG (profiling-only ablations, RFA_DIAG): 1 synthetic input (no input loads),
// 2 no row stores, 4 no butterflies/twiddles, 8 no LDS exchanges, 16 no window loads.
// STG: raw input staged through LDS by LDS-DMA one work item ahead (8/16-bit
// formats, one sub-FFT per workgroup, frame fits the exchange buffer; the
// host launches a persistent grid and checks 16-byte alignment).
template <int LOGM, int PT, int RS, int FMT, bool COMPLEX_OUT, int DIAG = 0, bool STG = false>
__global__ void __launch_bounds__((WGeo<LOGM, PT>::THREADS), (PT == 64 ? 2 : 4)) fft_wide_kernel(FftLaunch a) {
    using G = WGeo<LOGM, PT>;
    constexpr int M = G::M;
    constexpr int BPS = (FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8);
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int n = M * RS;
    float2 *twp1 = lds;
    float2 *twp2 = lds + G::TW_P1;
    float2 *data = lds + G::TW_LDS;

    for (int e = threadIdx.x; e < G::TW_LDS; e += G::THREADS) lds[e] = a.wide_tw[e];

    // TPF >= 64: a wave never straddles slots, so slot (and hence every buffer
    // descriptor below) is wave-uniform -- say so, or hipcc wraps each buffer
    // access in a readfirstlane waterfall loop.
    const int slot = __builtin_amdgcn_readfirstlane(threadIdx.x / G::TPF);
    const int tid = threadIdx.x - slot * G::TPF;
    float2 *buf = data + slot * G::HALFP;

    // large-N kernel B (FMT == kFmtDif): S column residues per frame, one work item each
    constexpr bool dif = FMT == kFmtDif;
    static_assert(!dif || (RS == 1 && G::SLOTS == 1), "large-N kernel B: one 32 K residue per workgroup");
    const int work = dif ? a.n_frames * a.dif_ss : a.n_frames;
    const int items = RS == 1 ? (work + G::SLOTS - 1) / G::SLOTS : ((a.n_frames + 7) / 8) * 8 * RS;
    __syncthreads();  // twiddle tables in LDS

#ifdef RFA_DIAG_STG12  // A/B builds only: the staged kernel without butterflies / exchanges (DIAG 12)
    constexpr int STG_DIAG_OK = ~60;
#else
    constexpr int STG_DIAG_OK = ~48;
#endif
    // RFA_SPLIT_STAGE (A/B builds; RS = 2, 8-bit input): the exchanges run in four
    // rounds through the buffer's first M/4 region A, so the next frame's first half
    // is staged into region B right after this item's pre-stage (it flies during both
    // exchanges and passes) and only its second half waits for exchange 1 (into A).
    constexpr bool SPLIT = RFA_SPLIT_STAGE && STG && RS == 2 && LOGM == 15 && BPS == 2 && !COMPLEX_OUT;
    // RFA_SPLIT_STAGE=2: exchange 0 keeps two rounds over the whole buffer and the
    // first half is staged after it (fewer barriers, less time in flight)
    constexpr bool SPLIT_LATE = SPLIT && RFA_SPLIT_STAGE == 2;
    // RFA_SPLIT_STAGE=3: only the first half is staged (early); the pre-stage loads the
    // second half straight from memory (no late DMA to wait for)
    constexpr bool SPLIT_DIRECT = SPLIT && RFA_SPLIT_STAGE == 3;
    constexpr int QP = M / 4 + M / 128;              // region A (padded quarter, float2)
    constexpr bool WHOLE_B = RFA_SPLIT_WHOLE && STG && RS == 1 && LOGM >= 14 && BPS == 2 && !COMPLEX_OUT &&
                             M * BPS <= (G::HALFP - QP) * 8;
    constexpr int KR = (SPLIT || WHOLE_B) ? 4 : 2;   // exchange rounds (exchange 1; exchange 0 too unless SPLIT_LATE)
    constexpr int KR0 = SPLIT_LATE ? 2 : KR;
    constexpr int HALF_BYTES = M * RS * BPS / 2;
    constexpr int JS = SPLIT ? -(QP * 8) / BPS : 0;  // raw-element offset of the second half (A) from B
    static_assert(!SPLIT || (G::HALFP - QP) * 8 >= HALF_BYTES, "region B holds half a frame");
    static_assert(!STG || (G::SLOTS == 1 && FMT <= 2 && !COMPLEX_OUT && (DIAG & STG_DIAG_OK) == 0 &&
                           M * RS * BPS <= G::HALFP * 8), "STG: one sub-FFT per WG, 8/16-bit input fitting the buffer");
    // frame of work item u (same mapping as body())
    auto frame_of = [&](int u) {
        if constexpr (RS == 1) return u;
        else return (u / (8 * RS)) * 8 + (u & 7);
    };
    // Work distribution.  Static: items blockIdx.x, +grid, ...  Dynamic (staged
    // one-residue kernels with a.queue): every workgroup takes its next item from one
    // device-wide counter a.queue[0], so workgroups that run slow take fewer items
    // (8 K/16 K: -11 % kernel time).  The index of the next item travels to all waves
    // through an LDS slot.  The last workgroup to finish (a.queue[1] counts
    // finishers) zeroes both counters for the next launch.  Two-residue kernels keep
    // the static stride: it puts the residues of a frame on one XCD (shared L2), which
    // a single queue does not (+7 % at 64 K, measured).
    const bool dq = STG && RS == 1 && a.queue != nullptr;
    int *qslot = reinterpret_cast<int *>(data + G::SLOTS * G::HALFP);
    auto dequeue = [&]() -> int {
        const unsigned u = atomicAdd(a.queue, 1u);
        return u < (unsigned)items ? (int)u : items;
    };
    if (a.stagger_ns > 0 && (int)blockIdx.x >= (int)(gridDim.x >> 1)) {
        // the second half of the grid starts late so workgroups do not all stream HBM
        // and compute in the same phases (speed only; RFA_STAGGER_NS)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        while ((__builtin_amdgcn_s_memrealtime() - t0) * 10ull < (unsigned long long)a.stagger_ns)
            __builtin_amdgcn_s_sleep(32);
    }
    int u0 = blockIdx.x;  // first item of this workgroup
    if (dq) {
        if (threadIdx.x == 0) qslot[0] = dequeue();
        __syncthreads();
        u0 = qslot[0];
        __syncthreads();  // every wave has read the slot before it is rewritten
    }
    auto next_item = [&](int u) { return u + (int)gridDim.x; };
    // SPLIT: half 0 of a frame goes to region B, half 1 to region A
    auto stage_half = [&](int f, int half) {
        if constexpr (SPLIT)
            stage_frame<HALF_BYTES, G::THREADS>(a.in + (size_t)f * (size_t)a.frame_stride + (half ? HALF_BYTES : 0),
                                                half ? buf : buf + QP);
    };
    auto stage_b = [&](int f) {  // WHOLE_B: the whole frame into region B
        if constexpr (WHOLE_B) stage_frame<M * RS * BPS, G::THREADS>(a.in + (size_t)f * (size_t)a.frame_stride, buf + QP);
    };
    if constexpr (STG) {
        const int f0 = frame_of(u0);
        if (u0 < items && f0 < a.n_frames) {
            if constexpr (WHOLE_B) {
                stage_b(f0);
            } else if constexpr (SPLIT) {
                stage_half(f0, 0);
                if constexpr (!SPLIT_DIRECT) stage_half(f0, 1);
            } else {
                stage_frame<M * RS * BPS, G::THREADS>(a.in + (size_t)f0 * (size_t)a.frame_stride, buf);
            }
        }
    }

    // One work item (SLOTS frames, or one residue of a frame).  Between items no
    // extra barrier is needed: the last LDS reads of an item (exchange 1) are
    // followed by a barrier before anyone leaves the FFT.
    // DIAG & 32 (profiling only): s_memrealtime stamps of each item's phases by
    // thread 0 into a.stamps[block][item < 16][8] (engine: RFA_STAMPS_FILE)
    int it_count = 0;  // items this workgroup has started (stamps)
    auto stamp = [&](int u, int k) {
        if constexpr ((DIAG & 32) != 0) {
            const int it = it_count;
            if (threadIdx.x == 0 && it < 16)
                a.stamps[((size_t)blockIdx.x * 16 + it) * 8 + k] = __builtin_amdgcn_s_memrealtime();
        }
    };
    // stores the previous item's epilogue left in flight (STG: the wait for the
    // staged frame skips them -- vmcnt counts in issue order and they are younger
    // than the frame's LDS-DMA, so only the DMA and older operations are waited for)
    int pending_st = 0;
    // RS = 2, staged 8/16-bit input: the thread's window pairs are the same for every
    // item; they are (re)loaded at the tail of each item, after the epilogue has
    // freed the point registers, so the loads fly during the staged-frame wait
    constexpr int WP = (STG && RS == 2 && !COMPLEX_OUT && (DIAG & 16) == 0) ? RFA_WPRE : 0;
    float2 wpre[WP > 0 ? WP : 1];
    auto load_wpre = [&]() {
        if constexpr (WP > 0) {
            const rsrc_t w_rs = make_rsrc(a.window_il, M * RS * 4);
#pragma unroll
            for (int idx = 0; idx < WP; idx++)
                wpre[idx] = buf_load_f32x2(w_rs, tid * 8, (G::TPF * (idx >> 5) + (M / 32) * (idx & 31)) * 8);
        }
    };
    load_wpre();
    auto body = [&](int u, int &unext) {
        stamp(u, 0);
        // opaque zero: stops hipcc hoisting the (loop-invariant) twiddle-table
        // reads out of the item loop, which would need ~90 more VGPRs
        int z;
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const float2 *tp1 = twp1 + z, *tp2 = twp2 + z;
        int frame, r;
        int dif_r = 0;  // large-N kernel B: column residue s of the frame (bins S q + s)
        if constexpr (RS == 1) {
            frame = u * G::SLOTS + slot;
            r = 0;
            if constexpr (dif) {
                frame = u / a.dif_ss;
                dif_r = u - frame * a.dif_ss;
            }
        } else {
            // blocks b, b+8, b+16, ... share an XCD: put a frame's RS residues there (speed only)
            const int g = u / (8 * RS), rem = u - g * (8 * RS);
            r = rem >> 3;
            frame = g * 8 + (rem & 7);
        }
        const bool active = frame < a.n_frames;
        constexpr int SB0 = FMT == 4 ? 4 : BPS;
        // inactive slots read zeros (num_records = 0) and store nothing; kernel B's
        // residue s of a frame is the contiguous z_s block of the scratch
        const rsrc_t in_rs =
            make_rsrc(a.in + (size_t)(active ? frame : 0) * (size_t)a.frame_stride + (size_t)dif_r * (M * 8),
                      active ? (unsigned)(n * BPS) : 0u);
        const int planar_im = n * 4;

        // ---- pass-0 inputs: x[m], m = tid + TPF*b + (M/32)*t   (b < PT/32, t < 32)
        float2 v[PT];
        using RawT = typename Raw<FMT>::T;
        const RawT *lraw = reinterpret_cast<const RawT *>((SPLIT || WHOLE_B) ? buf + QP : buf);
        if constexpr (STG) {
            // this item's frame, staged by LDS-DMA during the previous item: wait for
            // this wave's pieces, then for every wave's (the barrier)
            // operations younger than the frame's LDS-DMA: the epilogue stores and the window preloads
            const int younger = pending_st + WP;
            if (younger >= 63) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else if (younger >= 32) asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            stamp(u, 1);
        }
        if constexpr (RS == 1) {
            // all PT raw samples of the thread in flight at once (buffer loads need
            // no address registers), then the window (L2-resident) and convert.
            const rsrc_t w_rs = make_rsrc(a.window, dif ? 0 : n * 4);
            constexpr int SB = SB0;  // bytes between consecutive samples
            typename Raw<FMT>::T raw[PT];
    #pragma unroll
            for (int idx = 0; idx < PT; idx++) {
                const int so = G::TPF * (idx >> 5) + (M / 32) * (idx & 31);
                if constexpr (DIAG & 1) raw[idx] = synth_raw<FMT>(so + tid);
                else if constexpr (STG) raw[idx] = lraw[so + tid];
                else raw[idx] = buf_load_raw<FMT>(in_rs, tid * SB, so * SB, planar_im);
            }
    #pragma unroll
            for (int idx = 0; idx < PT; idx++) {
                const int so = G::TPF * (idx >> 5) + (M / 32) * (idx & 31);
                // kernel B's input is already windowed (kernel A)
                const float w = ((DIAG & 16) || dif) ? 1.0f : buf_load_f32(w_rs, tid * 4, so * 4);
                const float2 x = convert_raw<FMT>(raw[idx]);
                v[idx] = make_float2(x.x * w, x.y * w);  // NativeDsp.kt:55-58 (fp32 multiply)
            }
        } else {
            // residue r is wave-uniform: instantiate the pre-stage per r so the
            // W_RS^{j r} factors are compile-time rotations
            const int planar = planar_im;
            [&]<int... Rs>(std::integer_sequence<int, Rs...>) {
                ((r == Rs ? prestage<LOGM, PT, RS, FMT, Rs, STG, (DIAG & 16) != 0, WP, false, JS, SPLIT_DIRECT>(v, a.window_il, a.wide_tw, in_rs,
                                                                                        tid, planar, lraw, wpre)
                          : void()), ...);
            }(std::make_integer_sequence<int, RS>{});
        }

        // ---- FFT: pass 0 (radix 32, no twiddles), exchange, pass 1, exchange, pass 2
    #pragma unroll
        for (int b = 0; b < PT / 32; b++)
            if constexpr (!(DIAG & 4)) dft<32>(&v[b * 32]);
        stamp(u, 2);
        if constexpr (STG) {
            // dynamic queue: thread 0 takes the next item now; the barrier publishes it
            if (dq && threadIdx.x == 0) qslot[0] = dequeue();
            lds_barrier();  // every wave has read the staged frame before exchange 0 reuses the buffer
            if (dq) unext = qslot[0];
            if constexpr (SPLIT && !SPLIT_LATE) {  // region B is free until the next item: its half of the next frame now
                const int fn = frame_of(unext);
                if (unext < items && fn < a.n_frames) stage_half(fn, 0);
            }
            if constexpr (WHOLE_B) {  // region B is free until the next item: the whole next frame now
                const int fn = frame_of(unext);
                if (unext < items && fn < a.n_frames) stage_b(fn);
            }
        }
        if constexpr (!(DIAG & 8)) exchange<0, LOGM, PT, KR0>(v, buf, tid);
        if constexpr (SPLIT_LATE) {  // exchange 0 ended with a barrier after its last reads
            const int fn = frame_of(unext);
            if (unext < items && fn < a.n_frames) stage_half(fn, 0);
        }
        stamp(u, 3);
        if constexpr (!(DIAG & 4)) pass1<LOGM, PT>(v, tid, tp1);
        if constexpr (!(DIAG & 8)) exchange<1, LOGM, PT, KR>(v, buf, tid);
        stamp(u, 4);
        if constexpr (STG) {
            // exchange 1 ended with a barrier after its last reads: the buffer is free
            // until the next item, so stage the next item's frame now
            const int fn = frame_of(unext);
            if (unext < items && fn < a.n_frames) {
                if constexpr (SPLIT) {
                    if constexpr (!SPLIT_DIRECT) stage_half(fn, 1);
                }
                else if constexpr (!WHOLE_B) stage_frame<M * RS * BPS, G::THREADS>(a.in + (size_t)fn * (size_t)a.frame_stride, buf);
            }
        }
        if constexpr (!(DIAG & 4)) pass2<LOGM, PT>(v, tid, tp2);
        stamp(u, 5);
        if constexpr ((DIAG & 12) != 0) {
    #pragma unroll
            for (int q = 0; q < PT; q++) asm volatile("" : "+v"(v[q].x), "+v"(v[q].y));
        }

        if (!active) {
            load_wpre();
            return;
        }
        // ---- epilogue: sub-bin i + t*M/16 (i = tid + TPF*b) is full bin kk = r + RS*(i + t*M/16)
        // (kernel B of the large-N pair: kk = s + S*(...) with the runtime S = dif_ss and
        // s = dif_r; the stride and frame length below are then uniform runtime values)
        const int ors = dif ? a.dif_ss : RS, orr = dif ? dif_r : r;
        const int on = dif ? M * a.dif_ss : n;
        if constexpr (COMPLEX_OUT) {
            const rsrc_t o_rs = make_rsrc(a.complex_out + (size_t)frame * on, on * 8);
    #pragma unroll
            for (int b = 0; b < PT / G::R2; b++)
    #pragma unroll
                for (int t = 0; t < G::R2; t++)
                    buf_store_f32x2(v[b * G::R2 + t], o_rs, (ors * tid + orr) * 8,
                                    ors * (G::TPF * b + t * (M / G::R2)) * 8);
        } else {
            constexpr float db_off_c = -kDbPerLog2 * (float)(2 * (LOGM + (RS == 1 ? 0 : RS == 2 ? 1 : RS == 4 ? 2 : 3)));
            const float db_off = dif ? db_offset(LOGM + (31 - __builtin_clz(a.dif_ss))) : db_off_c;
            const bool to_ring = a.ring && frame >= a.ring_first;
            int rr = 0;
            if (to_ring) {
                rr = (a.ring_base - frame) % a.ring_rows;
                if (rr < 0) rr += a.ring_rows;
            }
            // ring in residue-major order (ring_pos, fft_kernels.h) when the engine asks for
            // it: residue r's M bins are one contiguous block, so this workgroup's stores
            // cover whole lines; caller rows are always natural (fft-shifted) order
            const bool rm = (RS > 1 || dif) && a.ring_logrs > 0;
            // kernel B (dif): rows residue-major too, block s (the engine reorders them)
            const rsrc_t row_rs = make_rsrc(a.rows ? a.rows + (size_t)frame * on + (dif ? (size_t)orr * M : 0) : nullptr,
                                            a.rows ? (dif ? M : on) * 4 : 0);
            const rsrc_t ring_rs = make_rsrc(to_ring ? a.ring + (size_t)rr * on + (rm ? (size_t)orr * M : 0) : nullptr,
                                             to_ring ? (rm ? M : on) * 4 : 0);
            const int vo = (ors * tid + orr) * 4;
            // one uniform branch per item, not per store
            auto epilogue = [&](auto nat_c, auto ring_c, auto rm_c) {
    #pragma unroll
                for (int b = 0; b < PT / G::R2; b++) {
    #pragma unroll
                    for (int t = 0; t < G::R2; t++) {
                        const float2 x = v[b * G::R2 + t];
                        const float db = db_unscaled(x, db_off);  // nativedsp.cpp:73-78
                        // fft-shift (nativedsp.cpp:77): out[(kk + N/2) mod N]; the lane part never wraps
                        const int so = ((ors * (G::TPF * b + t * (M / G::R2)) + on / 2) & (on - 1)) * 4;
                        // residue-major: sub-bin i = tid + TPF b + t M/R2 at (i + M/2) mod M of the block
                        const int so_rm = ((G::TPF * b + t * (M / G::R2) + M / 2) & (M - 1)) * 4;
                        if constexpr (DIAG & 2) {
                            asm volatile("" ::"v"(db));
                        } else {
                            if constexpr (decltype(nat_c)::value) {
                                if constexpr (dif) buf_store_f32(db, row_rs, tid * 4, so_rm);
                                else buf_store_f32(db, row_rs, vo, so);
                            }
                            if constexpr (decltype(ring_c)::value) {
                                if constexpr (decltype(rm_c)::value) buf_store_f32(db, ring_rs, tid * 4, so_rm);
                                else buf_store_f32(db, ring_rs, vo, so);
                            }
                        }
                    }
                }
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            pending_st = (a.rows ? PT : 0) + (to_ring ? PT : 0);
            if (a.rows && to_ring) {
                if constexpr (RS > 1 || dif) {
                    if (rm) epilogue(T_{}, T_{}, T_{});
                    else epilogue(T_{}, T_{}, F_{});
                } else {
                    epilogue(T_{}, T_{}, F_{});
                }
            } else if (a.rows) {
                epilogue(T_{}, F_{}, F_{});
            } else if (to_ring) {
                if constexpr (RS > 1 || dif) {
                    if (rm) epilogue(F_{}, T_{}, T_{});
                    else epilogue(F_{}, T_{}, F_{});
                } else {
                    epilogue(F_{}, T_{}, F_{});
                }
            }
            stamp(u, 6);
        }
        load_wpre();  // next item's window pairs (the point registers are free now)
    };
    for (int u = u0; u < items; it_count++) {
        int un = dq ? items : next_item(u);  // with the queue, body() dequeues the next item into un
        body(u, un);
        u = un;
    }
    if (dq) {
        if (threadIdx.x == 0) {
            __threadfence();  // this workgroup's dequeues are done before it counts itself finished
            if (atomicAdd(a.queue + 1, 1u) == gridDim.x - 1) {  // last one out: reset for the next launch
                atomicExch(a.queue, 0u);
                atomicExch(a.queue + 1, 0u);
            }
        }
    }
}

template <int LOGM, int PT, int RS, int FMT, bool CO, int DIAG = 0, bool STG = false>
static hipError_t launch_wide_one(const FftLaunch &a) {
    using G = WGeo<LOGM, PT>;
    auto kern = &fft_wide_kernel<LOGM, PT, RS, FMT, CO, DIAG, STG>;
    const size_t lds = (size_t)G::LDS_BYTES + (STG ? G::LDS_Q_BYTES : 0);
    if (!a.wide_tw) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int work = FMT == kFmtDif ? a.n_frames * a.dif_ss : a.n_frames;
    const int items = RS == 1 ? (work + G::SLOTS - 1) / G::SLOTS : ((a.n_frames + 7) / 8) * 8 * RS;
    if (items <= 0) return hipSuccess;
    int blocks = items;
    if (a.persist > 0 || STG) {  // persistent: a.persist (STG: all resident) workgroups per CU
        static int cus = 0, occ = 0;
        if (!cus) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(kern), G::THREADS,
                                                             lds) != hipSuccess || occ < 1)
                occ = 1;
        }
        blocks = std::min(items, cus * (a.persist > 0 ? a.persist : occ));
    }
    FftLaunch b = a;
    if (!STG) b.queue = nullptr;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(G::THREADS), lds, a.stream, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// N = 64 K "wave" kernel.  The 32 K-point sub-FFT of residue r
// (same decimation-in-frequency pre-stage as fft_wide_kernel) runs as a four-step
// 32 x 1024 transform whose 1024-point halves belong to half-waves, so only ONE
// exchange needs the whole workgroup:
//   m = m1 + 1024 m2, k = k2 + 32 k1
//   step 1, thread m1 = tid:  z[k2] = DFT32_m2(y[m1 + 1024 m2]) * W_M^(m1 k2)
//   exchange 0 (workgroup, two half-rounds): half-wave k2 = tid >> 5 gathers z_m1[k2]
//   step 2, half-wave k2, lane a = tid & 31, m1 = a + 32 b, k1 = c + 32 d:
//     pass A: DFT32 over b, * W_1024^(a c); transpose inside the wave through its own
//     8 KiB of LDS (no s_barrier); pass B: DFT32 over a -> Y[k2 + 32 c + 1024 d] in lane c
// After its transpose a wave's LDS region is free and the wave stages its 8 KiB
// piece of the next frame there (LDS-DMA), then writes its outputs: residue r's
// bins k2 + 32 (c + 32 d) are ring block r + 2 k2 (ring_pos order, logrs 6), so
// every store instruction covers whole 128-B lines.  Caller rows (natural order)
// take scattered stores; that path is not the hot one.
// STATUS: opt-in (RFA_W64=1), measured SLOWER than fft_wide_kernel's residue path
// (134 vs 95 us per 500 frames, profiles/r02a/w64_wave_kernel_ab.txt): hipcc spills
// 29-40 dwords per thread here (ScratchSize 116 / 160 B), and every scratch reload
// behind the epilogue's stores waits for them (vmcnt counts in issue order).  Kept,
// tested (tests/test_gpu_state.py), for the next attempt at the register budget.
#ifndef RFA_W64_ABL
#define RFA_W64_ABL 0  // compile-time ablations (register-pressure study only): 1 no step-1 twiddle,
                       // 2 no exchange 0, 4 no transpose, 8 no pass-A twiddle, 16 ring-only epilogue
#endif
template <int FMT, bool STG>
__global__ void __launch_bounds__(1024, 4) fft_w64_kernel(FftLaunch a) {
    constexpr int LOGM = 15, PT = 32, RS = 2;
    using G = WGeo<LOGM, PT>;
    constexpr int M = G::M;    // 32768
    constexpr int n = M * RS;  // 65536
    constexpr int BPS = (FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8);
    static_assert(G::TPF == 1024 && G::R1 == 32 && G::R2 == 32, "32 x 32 x 32 plan");
    static_assert(!STG || n * BPS == 16 * 8192, "staged: one 8 KiB piece of the frame per wave");
    // per-wave LDS region: 1056 points (8 KiB + 256 B): the wave's staged piece, then
    // its transposes (two 16 x 33 blocks); 16 regions fill the exchange buffer
    constexpr int WREG = 1056;
    static_assert(16 * WREG <= G::HALFP && 16 * 1024 <= G::HALFP, "exchange buffer");
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2 *twp1 = lds;
    float2 *twp2 = lds + G::TW_P1;
    float2 *buf = lds + G::TW_LDS;  // 16 K points: staged frame / exchange 0 / per-wave transposes
    for (int e = threadIdx.x; e < G::TW_LDS; e += 1024) lds[e] = a.wide_tw[e];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int items = ((a.n_frames + 7) / 8) * 8 * RS;
    __syncthreads();  // twiddle tables in LDS
    if (a.prio && (wave & a.prio)) __builtin_amdgcn_s_setprio(1);
    // blocks b, b+8, ... share an XCD: a frame's two residues run there (speed only)
    auto frame_of = [&](int u) { return (u / (8 * RS)) * 8 + (u & 7); };
    // this wave's 8 KiB piece of a frame's raw bytes into its own region of buf
    // (1 KiB LDS-DMA per instruction; inline asm for the reason given at stage_frame)
    auto stage_piece = [&](int f) {
        if constexpr (STG) {
            const rsrc_t rs = make_rsrc(a.in + (size_t)f * (size_t)a.frame_stride, n * BPS);
            const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) uint8_t *)(uint8_t *)buf;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int c = wave * 8 + j;  // 1 KiB piece c of the frame -> this wave's region
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                    "buffer_load_dwordx4 %2, %3, %4 offen " STG_POLICY "lds\n\ts_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "s"(base + wave * (WREG * 8) + j * 1024), "v"((tid & 63) * 16), "s"(rs), "s"(c * 1024)
                    : "memory");
            }
        }
    };
    const int u0 = blockIdx.x;
    if (u0 < items && frame_of(u0) < a.n_frames) stage_piece(frame_of(u0));
    int pending = 0;  // this wave's vector-memory operations issued after its last DMA piece
    for (int u = u0; u < items; u += gridDim.x) {
        int z;  // opaque zero: keeps the LDS twiddle reads inside the item loop (VGPR budget)
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const float2 *tp1 = twp1 + z, *tp2 = twp2 + z;
        // opaque thread index: every lane-dependent address is rebuilt per item instead of
        // being hoisted out of the loop into VGPRs that stay live across the whole item
        int tq;
        asm volatile("v_mov_b32 %0, %1" : "=v"(tq) : "v"(tid));
        const int k2 = tq >> 5;   // step-2 sub-FFT of this half-wave
        const int l32 = tq & 31;  // lane in the half-wave
        const int g = u / (8 * RS), rem = u - g * (8 * RS);
        const int r = rem >> 3, frame = g * 8 + (rem & 7);
        const bool active = frame < a.n_frames;
        const rsrc_t in_rs =
            make_rsrc(a.in + (size_t)(active ? frame : 0) * (size_t)a.frame_stride, active ? (unsigned)(n * BPS) : 0u);
        float2 v[PT];
        if constexpr (STG) {
            // every wave's piece of this item's frame has landed
            if (pending >= 63) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else if (pending >= 32) asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        // ---- pre-stage (DIF residue r) + step 1: v[t] = y[tid + 1024 t]
        using RawT = typename Raw<FMT>::T;
        [&]<int... Rs>(std::integer_sequence<int, Rs...>) {
            ((r == Rs ? prestage<LOGM, PT, RS, FMT, Rs, STG, false, 0, true>(v, a.window_il, a.wide_tw, in_rs, tq,
                                                                             n * 4, reinterpret_cast<const RawT *>(buf))
                      : void()), ...);
        }(std::make_integer_sequence<int, RS>{});
        dft<32>(v);  // z[k2], natural order
        if constexpr (!(RFA_W64_ABL & 1)) {  // * W_M^(tid k2) = A[tid >> 5][k2] * B[tid & 31][k2] (exact tables)
            const float2 *ra = tp2 + (tq >> 5) * G::P2_ROW - 1;
            const float2 *rb = tp2 + G::TW_P2A + (tq & 31) * G::P2_ROW - 1;
            v[1] = cmul(v[1], cmul(ra[1], rb[1]));
#pragma unroll
            for (int t = 2; t < 32; t += 2) {
                float2 w0 = ra[t], w1 = ra[t + 1];
                cmul2(w0, rb[t], w1, rb[t + 1]);
                cmul2(v[t], w0, v[t + 1], w1);
            }
        }
        // ---- exchange 0: buffer [k2][m1 - 512 h] per half-round h (m1 half), 16 K points
        lds_barrier();  // the staged frame and every wave's previous transpose are consumed
        // round 0 lands in tmp (v is still live in waves 8..15), round 1 straight in v
        float2 tmp[16];
        if constexpr (!(RFA_W64_ABL & 2)) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if ((tid >> 9) == h) {  // wave-uniform: waves 8h .. 8h + 7 hold m1 in this half
                    float2 *w = buf + (tq - 512 * h);
#pragma unroll
                    for (int k = 0; k < 32; k++) w[k * 512] = v[k];
                }
                lds_barrier();
                const float2 *rd = buf + k2 * 512 + l32;
#pragma unroll
                for (int bb = 0; bb < 16; bb++) {  // m1 = l32 + 32 (16 h + bb)
                    if (h == 0) tmp[bb] = rd[32 * bb];
                    else v[16 + bb] = rd[32 * bb];
                }
                lds_barrier();
            }
#pragma unroll
            for (int t = 0; t < 16; t++) v[t] = tmp[t];
        }
        // ---- step 2, pass A: DFT32 over b, then * W_1024^(a c) (a = l32; table row a)
        dft<32>(v);
        if constexpr (!(RFA_W64_ABL & 8)) {
            const float2 *row = tp1 + l32 * G::P1_ROW - 1;
            v[1] = cmul(v[1], row[1]);
#pragma unroll
            for (int t = 2; t < 32; t += 2) cmul2(v[t], row[t], v[t + 1], row[t + 1]);
        }
        // ---- transpose inside the wave, two rounds by a half (a = 16 ar + a'): the writers
        // (lanes of that half, EXEC-masked) store T[a'][c] at a' * 33 + c, every lane c then
        // reads its 16 values; the odd pitch keeps both directions conflict free and every
        // address is a lane base plus an immediate
        if constexpr (!(RFA_W64_ABL & 4)) {
            float2 *tw = buf + wave * WREG + ((tq >> 5) & 1) * 528;
#pragma unroll
            for (int ar = 0; ar < 2; ar++) {
                if ((l32 >> 4) == ar) {
                    float2 *w = tw + (l32 - 16 * ar) * 33;
#pragma unroll
                    for (int c = 0; c < 32; c++) w[c] = v[c];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const float2 *rd = tw + l32;
#pragma unroll
                for (int ap = 0; ap < 16; ap++) {
                    if (ar == 0) tmp[ap] = rd[ap * 33];
                    else v[16 + ap] = rd[ap * 33];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
#pragma unroll
            for (int t = 0; t < 16; t++) v[t] = tmp[t];
        }
#ifdef RFA_W64_EARLY_DMA
        // this wave's region is free: stage its piece of the next item's frame
        {
            const int un = u + (int)gridDim.x;
            if (un < items && frame_of(un) < a.n_frames) stage_piece(frame_of(un));
        }
#endif
        // ---- pass B: DFT32 over a -> v[d] = Y[k2 + 32 c + 1024 d], c = l32
        dft<32>(v);
        pending = 0;
        // stage this wave's piece of the next item's frame into its (free) region now,
        // behind the epilogue's stores' issue: no compiler-placed vmcnt wait of the
        // epilogue can then end up waiting for the DMA (in issue order it is younger)
        auto stage_next = [&]() {
#ifndef RFA_W64_EARLY_DMA
            const int un = u + (int)gridDim.x;
            if (un < items && frame_of(un) < a.n_frames) stage_piece(frame_of(un));
#endif
        };
        if (active) {
        // ---- epilogue (nativedsp.cpp:73-78): bin K = r + 2 (k2 + 32 c + 1024 d); fft-shift
        // (nativedsp.cpp:77) turns d into d' = (d + 16) mod 32: natural index r + 2 k2 + 64 c + 2048 d',
        // ring element (r + 2 k2) * 1024 + c + 32 d' (ring_pos, logrs 6)
        constexpr float db_off = -kDbPerLog2 * (float)(2 * 16);
        const bool to_ring = a.ring && frame >= a.ring_first;
        int rr = 0;
        if (to_ring) {
            rr = (a.ring_base - frame) % a.ring_rows;
            if (rr < 0) rr += a.ring_rows;
        }
        const rsrc_t row_rs = make_rsrc(a.rows ? a.rows + (size_t)frame * n + r : nullptr, a.rows ? n * 4 : 0);
        const rsrc_t ring_rs =
            make_rsrc(to_ring ? a.ring + (size_t)rr * n + (size_t)r * 1024 : nullptr, to_ring ? n * 4 : 0);
        const int vo_ring = (2 * k2 * 1024 + l32) * 4, vo_row = (2 * k2 + 64 * l32) * 4;
        auto epilogue = [&](auto row_c, auto ring_c) {
#pragma unroll
            for (int d = 0; d < 32; d++) {
                const int dp = (d + 16) & 31;
                const float db = db_unscaled(v[d], db_off);
                if constexpr (decltype(row_c)::value) buf_store_f32(db, row_rs, vo_row, 2048 * dp * 4);
                if constexpr (decltype(ring_c)::value) buf_store_f32(db, ring_rs, vo_ring, 32 * dp * 4);
            }
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        if constexpr (RFA_W64_ABL & 16) {
            if (to_ring) epilogue(F_{}, T_{});
        } else {
            if (a.rows && to_ring) epilogue(T_{}, T_{});
            else if (a.rows) epilogue(T_{}, F_{});
            else if (to_ring) epilogue(F_{}, T_{});
        }
        }
        stage_next();
#ifdef RFA_W64_EARLY_DMA
        pending = (a.rows ? 32 : 0) + (to_ring ? 32 : 0);
#endif
    }
}

template <int FMT, bool STG>
static hipError_t launch_w64_one(const FftLaunch &a) {
    using G = WGeo<15, 32>;
    auto kern = &fft_w64_kernel<FMT, STG>;
    const size_t lds = (size_t)G::LDS_BYTES;
    if (!a.wide_tw || !a.window_il) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int items = ((a.n_frames + 7) / 8) * 8 * 2;
    if (items <= 0) return hipSuccess;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    }
    // persistent: one 1024-thread workgroup per CU (LDS and registers), items strided by the grid
    const int blocks = std::min(items, cus);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), lds, a.stream, a);
    return hipGetLastError();
}

static hipError_t launch_w64(const FftLaunch &a) {
    const bool stg = a.stage && ((reinterpret_cast<uintptr_t>(a.in) | (uintptr_t)a.frame_stride) & 15) == 0;
    switch (a.fmt) {
    case 0: return stg ? launch_w64_one<0, true>(a) : launch_w64_one<0, false>(a);
    case 1: return stg ? launch_w64_one<1, true>(a) : launch_w64_one<1, false>(a);
    case 2: return launch_w64_one<2, false>(a);
    case 3: return launch_w64_one<3, false>(a);
    case 4: return launch_w64_one<4, false>(a);
    default: return hipErrorInvalidValue;
    }
}

int ring_logrs_for(int logn, int wide_big, int w64) {
    if (logn > 17 && logn <= kMaxLogN) return logn - kDitLogM;  // large-N kernel B: block s of bins S q + s
    if (!wide_supported(logn) || logn <= 14) return 0;
    if (logn == 16 && wide_big == 15 && w64) return 6;
    return logn - wide_logm(logn, wide_big);
}

template <int LOGM, int PT, int RS, bool CO>
static hipError_t wide_by_fmt(const FftLaunch &a) {
    if constexpr (CO) {
        return a.fmt == 3 ? launch_wide_one<LOGM, PT, RS, 3, true>(a) : hipErrorInvalidValue;
    } else {
        using G = WGeo<LOGM, PT>;
        constexpr int M = 1 << LOGM;
        // LDS-staged input: 16-byte aligned frames that fit the exchange buffer
        const bool stg = a.stage && ((reinterpret_cast<uintptr_t>(a.in) | (uintptr_t)a.frame_stride) & 15) == 0;
        constexpr bool stg8 = G::SLOTS == 1 && M * RS * 2 <= G::HALFP * 8;
        constexpr bool stg16 = G::SLOTS == 1 && M * RS * 4 <= G::HALFP * 8;
        if constexpr (stg8) {
            if (stg && a.fmt == 0) return launch_wide_one<LOGM, PT, RS, 0, false, 0, true>(a);
            if (stg && a.fmt == 1) return launch_wide_one<LOGM, PT, RS, 1, false, 0, true>(a);
        }
        if constexpr (stg16) {
            if (stg && a.fmt == 2) return launch_wide_one<LOGM, PT, RS, 2, false, 0, true>(a);
        }
        switch (a.fmt) {
        case 0: return launch_wide_one<LOGM, PT, RS, 0, false>(a);
        case 1: return launch_wide_one<LOGM, PT, RS, 1, false>(a);
        case 2: return launch_wide_one<LOGM, PT, RS, 2, false>(a);
        case 3: return launch_wide_one<LOGM, PT, RS, 3, false>(a);
        case 4: return launch_wide_one<LOGM, PT, RS, 4, false>(a);
        default: return hipErrorInvalidValue;
        }
    }
}

bool wide_supported(int logn) { return logn >= 13 && logn <= 17; }

// Twiddle blob for the wide kernel (layout must match WGeo): pass-1 [32][R1-1],
// pass-2 A [TPF/LO][15], B [LO][15], pre-stage pre_a [RS][M/32], pre_b [RS][32].
std::vector<float2> wide_twiddles(int logn, int pt, int lm) {
    const int m = 1 << lm, n = 1 << logn, rs = n / m;
    const int r1 = lm >= 14 ? 32 : 16, r2 = m / (32 * r1), tpf = m / pt, lo = tpf > 256 ? 32 : 16;
    auto w = [](double num, double den) {  // exp(-2 pi i num/den), correctly rounded from double
        const double a = -2.0 * M_PI * num / den;
        return make_float2((float)std::cos(a), (float)std::sin(a));
    };
    std::vector<float2> blob;
    for (int k = 0; k < 32; k++)
        for (int t = 1; t < r1; t++) blob.push_back(w((double)t * k, 32.0 * r1));
    for (int hi = 0; hi < tpf / lo; hi++)
        for (int t = 1; t < r2; t++) blob.push_back(w((double)t * hi * lo, m));
    for (int l = 0; l < lo; l++)
        for (int t = 1; t < r2; t++) blob.push_back(w((double)t * l, m));
    if (rs > 1) {
        for (int r = 0; r < rs; r++)
            for (int mp = 0; mp < m / 32; mp++) blob.push_back(w((double)mp * r, n));
        for (int r = 0; r < rs; r++)
            for (int t = 0; t < 32; t++) blob.push_back(w((double)(m / 32) * t * r, n));
    }
    return blob;
}

hipError_t launch_fft_wide(const FftLaunch &a) {
    const bool co = a.complex_out != nullptr;
    if (a.diag == 16 && a.logn == 16) {  // staged 64 K kernel without window loads (profiling only)
        if (a.fmt != 0 || co) return hipErrorInvalidValue;
        return launch_wide_one<15, 32, 2, 0, false, 16, true>(a);
    }
#ifdef RFA_DIAG_STG12
    if (a.diag == 12 && a.logn == 16) {  // staged 64 K kernel, streaming part only (A/B builds)
        if (a.fmt != 0 || co) return hipErrorInvalidValue;
        return launch_wide_one<15, 32, 2, 0, false, 12, true>(a);
    }
#endif
    if (a.diag == 32) {  // phase stamps of the staged s8 kernels (profiling only)
        if (a.fmt != 0 || co || !a.stamps) return hipErrorInvalidValue;
        switch (a.logn) {
        case 13: return launch_wide_one<13, 32, 1, 0, false, 32, true>(a);
        case 14: return launch_wide_one<14, 32, 1, 0, false, 32, true>(a);
        case 15: return launch_wide_one<15, 32, 1, 0, false, 32, true>(a);
        case 16: return launch_wide_one<15, 32, 2, 0, false, 32, true>(a);
        default: return hipErrorInvalidValue;
        }
    }
    if (a.diag) {  // ablations: 16K, s8 only
        if (a.logn != 14 || a.fmt != 0 || co) return hipErrorInvalidValue;
        switch (a.diag) {
        case 1: return launch_wide_one<14, 32, 1, 0, false, 1>(a);
        case 2: return launch_wide_one<14, 32, 1, 0, false, 2>(a);
        case 3: return launch_wide_one<14, 32, 1, 0, false, 3>(a);
        case 4: return launch_wide_one<14, 32, 1, 0, false, 4>(a);
        case 8: return launch_wide_one<14, 32, 1, 0, false, 8>(a);
        case 12: return launch_wide_one<14, 32, 1, 0, false, 12>(a);
        case 16: return launch_wide_one<14, 32, 1, 0, false, 16>(a);
        case 19: return launch_wide_one<14, 32, 1, 0, false, 19>(a);
        case 31: return launch_wide_one<14, 32, 1, 0, false, 31>(a);
        default: return hipErrorInvalidValue;
        }
    }
    if (a.fmt == kFmtDif) {  // kernel B of the large-N pair (dB rows / ring, or the ordered spectrum)
        if (a.dif_ss < 8 || a.dif_ss > 32) return hipErrorInvalidValue;
        return co ? launch_wide_one<kDitLogM, 32, 1, kFmtDif, true>(a) : launch_wide_one<kDitLogM, 32, 1, kFmtDif, false>(a);
    }
    if (a.logn >= 15 && a.wide_big == 15) {
        switch (a.logn) {
        case 15: return co ? wide_by_fmt<15, 32, 1, true>(a) : wide_by_fmt<15, 32, 1, false>(a);
        case 16:
            if (!co && a.w64) return launch_w64(a);
            return co ? wide_by_fmt<15, 32, 2, true>(a) : wide_by_fmt<15, 32, 2, false>(a);
        case 17: return co ? wide_by_fmt<15, 32, 4, true>(a) : wide_by_fmt<15, 32, 4, false>(a);
        default: return hipErrorInvalidValue;
        }
    }
    switch (a.logn) {
    case 13: return co ? wide_by_fmt<13, 32, 1, true>(a) : wide_by_fmt<13, 32, 1, false>(a);
    case 14: return co ? wide_by_fmt<14, 32, 1, true>(a) : wide_by_fmt<14, 32, 1, false>(a);
    case 15: return co ? wide_by_fmt<14, 32, 2, true>(a) : wide_by_fmt<14, 32, 2, false>(a);
    case 16: return co ? wide_by_fmt<14, 32, 4, true>(a) : wide_by_fmt<14, 32, 4, false>(a);
    case 17: return co ? wide_by_fmt<14, 32, 8, true>(a) : wide_by_fmt<14, 32, 8, false>(a);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace rfa
