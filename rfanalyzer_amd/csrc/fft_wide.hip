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
#include <cstdlib>
#include <cmath>
#include <type_traits>
#include <vector>

#include "fft_common.h"
#include "fft_kernels.h"
#include "fft_w8.h"

namespace rfa {

// sc1 cache policy of a raw buffer access (gfx950: bit 4 of the aux operand: the line
// bypasses / leaves the CU's L1)
[[maybe_unused]] constexpr int kSc1 = 16;
#ifndef RFA_RING_SC1
#define RFA_RING_SC1 1  // 16-B ring tile stores write-through (profiles/r04/ring_store_sc1_ab.txt; A/B: 0)
#endif
#ifndef RFA_WIN_UPFRONT
#define RFA_WIN_UPFRONT 16  // residue 0's first 16 window pairs loaded into v[] up front (A/B: 0;
                            // profiles/r06/residue_loop_window_ab.txt)
#endif
#ifndef RFA_RES_HOIST
#define RFA_RES_HOIST 1  // the 64 K item loop instantiated per residue (A/B: 0; profiles/r06/residue_loop_window_ab.txt)
#endif
#ifndef RFA_STG_OWNQ
#define RFA_STG_OWNQ 1  // QST's staged cf32 quarters (64 K f32) wave-owned too (A/B: 0; profiles/r06/f32_stage_own_ab.txt)
#endif
#ifndef RFA_STG_OWN
#define RFA_STG_OWN 1  // SPLIT halves staged wave-owned (stage_half_own), no item-start barrier (A/B: 0,
                       // profiles/r06/stage_own_ab.txt)
#endif
#ifndef RFA_WIDE_KR1
#define RFA_WIDE_KR1 0
#endif
template <int LOGM, int PT>
struct WGeo {
    static constexpr int M = 1 << LOGM;
    static constexpr int TPF = M / PT;           // threads per sub-FFT (PT points per thread)
    static constexpr int THREADS = TPF < 256 ? 256 : TPF;
    static constexpr int SLOTS = THREADS / TPF;  // sub-FFTs per workgroup
    // exchange buffer (float2) per slot: M / 2, two rounds per exchange; A/B RFA_WIDE_KR1 (8 K): the
    // whole M, one round (half the barriers, 2 instead of 4 workgroups per CU)
    static constexpr int HALF = (RFA_WIDE_KR1 && LOGM == 13) ? M : M / 2;
    static constexpr int HALFP = HALF + HALF / 32;  // ... with one float2 of padding per 32
    static constexpr int R1 = LOGM >= 14 ? 32 : 16;  // radix of pass 1 (pass 0: 32)
    static constexpr int R2 = M / (32 * R1);          // radix of pass 2: 16 (8 K, 16 K) or 32 (32 K)
    // LDS twiddle tables (float2, t = 1..R-1 only).  Odd row strides (R-1)
    // spread the rows read by one lane group over distinct banks.
    static constexpr int P1_ROW = R1 - 1;        // pass 1: [k = tid & 31][t]
    static constexpr int TW_P1 = 32 * P1_ROW;
    static constexpr int LO = TPF > 256 ? 32 : 16;  // pass 2: tid = hi*LO + lo
    static constexpr int P2_ROW = R2 - 1;
    // 8 K: A[hi][t] = W_8192^{16 t hi} = W_512^{t hi} is row hi of the pass-1 table (same
    // row length 15), so pass 2 reads it there: 1.9 KB less LDS per workgroup, and 4 x 39.6 KB
    // fit a CU -- four resident workgroups (the VGPR limit) instead of three
    static constexpr bool A_ALIAS = LOGM == 13 && R1 == 16 && R2 == 16 && LO == 16 && TPF / LO <= 32;
    static constexpr int TW_P2A = A_ALIAS ? 0 : (TPF / LO) * P2_ROW;  // A[hi][t] = W_M^{t hi LO}
    static constexpr int TW_P2B = LO * P2_ROW;          // B[lo][t] = W_M^{t lo}
    static_assert(!A_ALIAS || (32 * R1 * LO == M && P1_ROW == R2 - 1), "A rows = pass-1 rows");
    static constexpr int TW_LDS = TW_P1 + TW_P2A + TW_P2B;
    static constexpr int LDS_BYTES = (TW_LDS + SLOTS * HALFP) * 8;
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
// pass-1/2 twiddle reads as single ds_read_b64 (hipcc would fuse ds_read2_b64: -2.8 %,
// profiles/r03/round3_changes_ab.txt)
template <typename T>
__device__ __forceinline__ float2 tw_ld(const T *p) { return lds_ld2(p); }

template <int Q, int LOGM, int PT, int KR = 2, bool XST = false>
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
        // XST (staged persistent kernels): the round's write base in a register of its own and
        // one ds_write_b64 per output, so every store carries a small positive immediate (hipcc
        // otherwise folds -h*PARTP into each store's offset, which the unsigned ds offset cannot
        // hold, or fuses pairs into ds_write2_b64, whose 8-bit offsets cannot either, and adds a
        // v_add_u32 per store): -2 .. -3 % at 8 K / 16 K s8 (profiles/r04/vadd2_ab.txt); the
        // one-item-per-workgroup cf32 8 K kernel is 5 % slower with it, so it keeps the plain form
        if constexpr (!XST) {
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
        } else {
            int wb = wbase - h * PARTP;
            asm volatile("" : "+v"(wb));
            if constexpr (W::NB == 1) {
                if (my_part == h) {
#pragma unroll
                    for (int t = 0; t < W::R; t++) lds_st2(buf + wb + padw(t * W::P), v[t]);
                }
            } else {
#pragma unroll
                for (int b = h * W::NB / KR; b < (h + 1) * W::NB / KR; b++) {
#pragma unroll
                    for (int t = 0; t < W::R; t++) lds_st2(buf + wb + padw(W::R * G::TPF * b + t * W::P), v[b * W::R + t]);
                }
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
template <int LOGM, int PT, bool W8>
__device__ __forceinline__ void pass1(float2 (&v)[PT], int tid, const float2 *twp1) {
    using W = WPass<1, LOGM, PT>;
    const float2 *row = twp1 + (tid & 31) * WGeo<LOGM, PT>::P1_ROW - 1;
#pragma unroll
    for (int b = 0; b < W::NB; b++) {
        v[b * W::R + 1] = cmul(v[b * W::R + 1], tw_ld(row + 1));
#pragma unroll
        for (int t = 2; t < W::R; t += 2)
            cmul2(v[b * W::R + t], tw_ld(row + t), v[b * W::R + t + 1], tw_ld(row + t + 1));
    }
#pragma unroll
    for (int b = 0; b < W::NB; b++) dftw<W::R, W8>(&v[b * W::R]);
}

// Pass 2 (last, radix R2): k = i = tid + TPF*b.  W_M^{t i} = W_M^{t tid} * W_PT^{t b}
// (M / TPF = PT); W_M^{t tid} = A[tid/LO][t] * B[tid%LO][t] from two exact
// tables, the b-dependent factor is a compile-time constant.
// W8: butterfly B's factors for t = 4 and 12 are both W_8-type (W_16^{2 or 6}), so
// their sqrt(1/2) is left to the first adds of its DFT-16 (dft16r S0)
template <int PT, int R2, int B, bool W8>
constexpr bool p2_s0() {
    return W8 && R2 == 16 && B > 0 && ((4 * B * (64 / PT)) & 15) == 8 && ((12 * B * (64 / PT)) & 15) == 8;
}
template <int PT, int R2, int T, int B, bool W8>
__device__ __forceinline__ void p2_const(float2 (&v)[PT]) {
    constexpr int q = T * B * (64 / PT);
    if constexpr (p2_s0<PT, R2, B, W8>() && (T == 4 || T == 12)) v[B * R2 + T] = w16_p<q / 4>(v[B * R2 + T]);
    else v[B * R2 + T] = w64<q>(v[B * R2 + T]);
}
template <int PT, int R2, int B, bool W8>
__device__ __forceinline__ void p2_dft(float2 (&v)[PT]) {
    if constexpr (p2_s0<PT, R2, B, W8>()) dft16w<0, true>(&v[B * R2]);
    else dftw<R2, W8>(&v[B * R2]);
}
template <int PT, int R2, int T, bool W8, int... Bs>
__device__ __forceinline__ void p2_const_t(float2 (&v)[PT], std::integer_sequence<int, Bs...>) {
    (p2_const<PT, R2, T, Bs + 1, W8>(v), ...);
}
template <int PT, int R2, bool W8, int... Ts>
__device__ __forceinline__ void p2_const_all(float2 (&v)[PT], std::integer_sequence<int, Ts...>) {
    (p2_const_t<PT, R2, Ts, W8>(v, std::make_integer_sequence<int, PT / R2 - 1>{}), ...);
}

template <int LOGM, int PT, bool W8>
__device__ __forceinline__ void pass2(float2 (&v)[PT], int tid, const float2 *twp2) {
    using G = WGeo<LOGM, PT>;
    using W = WPass<2, LOGM, PT>;
    constexpr int R2 = G::R2;
    const float2 *ra = G::A_ALIAS ? twp2 - G::TW_P1 + (tid / G::LO) * G::P1_ROW - 1  // pass-1 row tid / LO
                                  : twp2 + (tid / G::LO) * G::P2_ROW - 1;
    const float2 *rb = twp2 + G::TW_P2A + (tid % G::LO) * G::P2_ROW - 1;
    {
        const float2 w1 = cmul(tw_ld(ra + 1), tw_ld(rb + 1));
#pragma unroll
        for (int b = 0; b < W::NB; b++) v[b * R2 + 1] = cmul(v[b * R2 + 1], w1);
    }
#pragma unroll
    for (int t = 2; t < R2; t += 2) {  // twiddle pairs built and applied in place (no table in VGPRs)
        float2 w0 = tw_ld(ra + t), w1 = tw_ld(ra + t + 1);
        cmul2(w0, tw_ld(rb + t), w1, tw_ld(rb + t + 1));
#pragma unroll
        for (int b = 0; b < W::NB; b++) cmul2(v[b * R2 + t], w0, v[b * R2 + t + 1], w1);
    }
    if constexpr (W::NB > 1) p2_const_all<PT, R2, W8>(v, std::make_integer_sequence<int, R2>{});
    [&]<int... Bs>(std::integer_sequence<int, Bs...>) { (p2_dft<PT, R2, Bs, W8>(v), ...); }(std::make_integer_sequence<int, W::NB>{});
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
// 64 K, 8-bit input (SPLIT below): the next frame is staged in two halves, the first
// right after the pre-stage into region B (the exchanges then run in four rounds
// through the quarter region A), the second after exchange 1 into region A
// (-1..-4 % kernel time, profiles/r02g/split_stage_ab.txt; the late / direct /
// whole-frame alternatives measured slower and were removed: split_direct_ab.txt,
// split_whole_ab.txt).

// JS != 0: the frame's two halves sit JS raw elements apart in LDS (SPLIT staging).
// CW (N = 64 K, residue 1, 8/16-bit input): the twiddle W_N^m is folded into a complex
// window cw[m] = (w[m] W_N^m, -w[m + M] W_N^m) (exact from double, engine), so a point
// costs two complex multiply-adds (cmac2: 4 packed instructions) instead of two window
// products, a subtraction and two complex multiplies (7).  (f32 input keeps the separate
// twiddle: its 8-B raw samples and the 16-B window pairs in flight would spill.)
template <int LOGM, int PT, int RS, int FMT, int R, bool STG = false, bool NOWIN = false, int JS = 0, bool CW = false,
          int QCH = 0>
__device__ __forceinline__ void prestage(float2 (&v)[PT], const float *window_il, const float2 *wide_tw, rsrc_t in_rs,
                                         int tid, int planar_im, const typename Raw<FMT>::T *lraw = nullptr,
                                         const float4 *cw = nullptr) {
    static_assert(!CW || (RS == 2 && R == 1 && !NOWIN), "complex window: residue 1 of N = 2M");
    using G = WGeo<LOGM, PT>;
    constexpr int M = G::M;
    constexpr int SB = FMT == 4 ? 4 : ((FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8));  // bytes per sample (per plane)
    // points per chunk: two chunks of raw samples + window values in flight must
    // fit beside the PT points in the register budget (64 VGPRs at PT = 32)
    constexpr int C = (PT == 64 ? 16 : 8) / RS > 0 ? (PT == 64 ? 16 : 8) / RS : 1;
    constexpr int NCH = PT / C;
    // SPLIT halves staged wave-owned (stage_half_own): wave w's slice, piece t at 64 t
    // (RFA_STG_OWNQ: QST's two staged cf32 quarters too, QN / 16 samples of each per wave)
    constexpr bool OWN = (RFA_STG_OWN && STG && JS < 0) || (RFA_STG_OWNQ && STG && QCH > 0 && RS == 2);
    static_assert(!OWN || (G::THREADS == 1024 && PT == 32), "OWN: 16 waves, M / 16 samples of each half per wave");
    constexpr int OWN_SLICE = QCH > 0 ? JS / 16 : M / 16;  // samples per wave slice
    const int ltid = OWN ? (tid >> 6) * OWN_SLICE + (tid & 63) : tid;
    auto lraw_t = [&] {  // this thread's samples in the staged frame (opaque base, see lds_opaque)
        if constexpr (STG) return lds_opaque(lraw + ltid);
        else return lraw;
    }();
    // the second sample of a point (x[m + M], region A under SPLIT: a negative element
    // offset) from its own base, so every ds_read_u16 takes an immediate offset
    auto lraw_t1 = [&] {
        if constexpr (STG && RS == 2) return lds_opaque(lraw + ltid + (JS != 0 ? JS : M));
        else return lraw_t;
    }();
    const rsrc_t w_rs = CW ? make_rsrc(cw, M * 16) : make_rsrc(window_il, M * RS * 4);
    const rsrc_t pa_rs = make_rsrc(wide_tw + G::TW_LDS, RS * (M / 32) * 8);
    const float2 *pre_b = wide_tw + G::TW_LDS + RS * (M / 32) + R * 32;
    float2 pa[PT / 32];
    if constexpr (R != 0 && !CW) {
#pragma unroll
        for (int b = 0; b < PT / 32; b++) pa[b] = buf_load_f32x2(pa_rs, (tid + G::TPF * b) * 8, R * (M / 32) * 8);
    }
    // loads run one chunk ahead of the arithmetic (two for 64 K float input: ±1 %,
    // profiles/r04/prestage_distance_f32_ab.txt)
    constexpr int DIST = 1;
    typename Raw<FMT>::T raw[DIST + 1][C][RS];
    float win[DIST + 1][C][CW ? 4 : RS];
    // c is a template parameter throughout: every register array index below is a
    // compile-time constant (a runtime index would move the arrays to scratch)
    auto issue = [&]<int c>() {
        constexpr int s = c % (DIST + 1);
#pragma unroll
        for (int q = 0; q < C; q++) {
            const int idx = c * C + q, b = idx >> 5, t = idx & 31;
            const int mo = G::TPF * b + (M / 32) * t;  // uniform part of m
            const int mol = OWN ? 64 * t : mo;           // its place in the staged slice
#pragma unroll
            for (int j = 0; j < RS; j++) {
                if constexpr (STG && (QCH == 0 || c < QCH)) {  // frame (QCH: its first QCH chunks) staged in LDS
                    if (STG && RS == 2 && j == 1) raw[s][q][j] = lraw_t1[mol];
                    else raw[s][q][j] = lraw_t[mol + j * (JS != 0 ? JS : M)];
                }
                else raw[s][q][j] = buf_load_raw<FMT>(in_rs, tid * SB, (mo + j * M) * SB, planar_im);
            }
            if constexpr (NOWIN) {  // ablation (RFA_DIAG=16): constant window, no window loads
#pragma unroll
                for (int j = 0; j < RS; j++) win[s][q][j] = 1.0f / 128.0f;
            } else if constexpr (CW) {  // complex window pair of point m: one 16-B load
                typedef float f4v __attribute__((ext_vector_type(4)));
                const f4v w = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(w_rs, tid * 16, mo * 16, 0));
                win[s][q][0] = w.x;
                win[s][q][1] = w.y;
                win[s][q][2] = w.z;
                win[s][q][3] = w.w;
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
        if constexpr (CW) {  // y_1[m] = x[m] cw0[m] + x[m + M] cw1[m]   (NativeDsp.kt:55-58 window, DIF twiddle)
            if constexpr (STG && C % 2 == 0) {  // two points' chains interleaved (fft_common.h cmac2x2)
#pragma unroll
                for (int q = 0; q < C; q += 2)
                    cmac2x2(v[c * C + q], convert_raw<FMT>(raw[s][q][0]), make_float2(win[s][q][0], win[s][q][1]),
                            convert_raw<FMT>(raw[s][q][1]), make_float2(win[s][q][2], win[s][q][3]), v[c * C + q + 1],
                            convert_raw<FMT>(raw[s][q + 1][0]), make_float2(win[s][q + 1][0], win[s][q + 1][1]),
                            convert_raw<FMT>(raw[s][q + 1][1]), make_float2(win[s][q + 1][2], win[s][q + 1][3]));
            } else {
#pragma unroll
                for (int q = 0; q < C; q++)
                    v[c * C + q] = cmac2(convert_raw<FMT>(raw[s][q][0]), make_float2(win[s][q][0], win[s][q][1]),
                                         convert_raw<FMT>(raw[s][q][1]), make_float2(win[s][q][2], win[s][q][3]));
            }
            return;
        } else if constexpr (RS == 2 && R == 0 && !NOWIN) {  // y_0[m] = x[m] w[m] + x[m + M] w[m + M] (mul + fma)
#pragma unroll
            for (int q = 0; q < C; q++) {
                const f2v x0 = to_v(convert_raw<FMT>(raw[s][q][0])), x1 = to_v(convert_raw<FMT>(raw[s][q][1]));
                v[c * C + q] = from_v(__builtin_elementwise_fma(x1, (f2v){win[s][q][1], win[s][q][1]},
                                                                x0 * win[s][q][0]));
            }
            return;
        }
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
    // RFA_WIN_UPFRONT: residue 0 of a staged frame loads its first KU window pairs straight into
    // v[] (the pre-stage's own output registers) before any arithmetic, so they are all in flight
    // at once instead of two chunks; the samples come from LDS chunk by chunk, each point is the
    // same mul + fma as below, and the remaining points go through the chunk pipeline (all 32 up
    // front spill: 228 B of scratch)
#if RFA_WIN_UPFRONT
    constexpr int KU = RFA_WIN_UPFRONT >= PT ? PT : RFA_WIN_UPFRONT;
    constexpr bool WUP = STG && RS == 2 && R == 0 && !NOWIN && !CW && QCH == 0 && PT == 32 && KU % C == 0;
    if constexpr (WUP) {
        int zo;  // opaque zero: the scalar offsets are built here, not hoisted out of the item loop
        asm volatile("s_mov_b32 %0, 0" : "=s"(zo));
#pragma unroll
        for (int idx = 0; idx < KU; idx++)
            v[idx] = from_v(__builtin_bit_cast(
                f2v, __builtin_amdgcn_raw_buffer_load_b64(w_rs, tid * 8, zo + (M / 32) * idx * 8, 0)));
        constexpr int NU = KU / C;  // up-front chunks
        if constexpr (NU < NCH) issue.template operator()<NU>();
        typename Raw<FMT>::T rw[2][C][2];
        auto ld = [&]<int c>() {
#pragma unroll
            for (int q = 0; q < C; q++) {
                const int t = c * C + q, mol = OWN ? 64 * t : (M / 32) * t;
                rw[c & 1][q][0] = lraw_t[mol];
                rw[c & 1][q][1] = lraw_t1[mol];
            }
        };
        ld.template operator()<0>();
        [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
            (
                [&] {
                    if constexpr (Cs + 1 < NU) ld.template operator()<Cs + 1>();
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < C; q++) {
                        const int i = Cs * C + q;
                        const f2v x0 = to_v(convert_raw<FMT>(rw[Cs & 1][q][0])), x1 = to_v(convert_raw<FMT>(rw[Cs & 1][q][1]));
                        const float w0 = v[i].x, w1 = v[i].y;
                        v[i] = from_v(__builtin_elementwise_fma(x1, (f2v){w1, w1}, x0 * w0));
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }(),
                ...);
        }(std::make_integer_sequence<int, NU>{});
        [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
            (
                [&] {
                    if constexpr (Cs >= NU) {
                        if constexpr (Cs + 1 < NCH) issue.template operator()<Cs + 1>();
                        __builtin_amdgcn_sched_barrier(0);
                        compute.template operator()<Cs>();
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }(),
                ...);
        }(std::make_integer_sequence<int, NCH>{});
        return;
    }
#endif
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
            "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(base + c * 1024), "v"(lane * 16), "s"(rs), "s"(c * 1024)
            : "memory");
    }
}

// Wave-owned staging of one half of a 64 K 8-bit frame (SPLIT kernels, RFA_STG_OWN) or of one of
// the 64 K cf32 kernel's two staged quarters (QST, RFA_STG_OWNQ): wave w stages exactly the samples
// its own threads read in the pre-stage -- sample 64 w + l + (M/32) t of the piece for lane l, i.e.
// runs of 64 samples, (M/32) samples apart -- into its own contiguous slice of the region (run t at
// t * 64 samples).  Each 16-B lane of an LDS-DMA instruction fetches from its own address, so
// PB / 16 lanes take one run (8 for 8-bit IQ, 32 for cf32).  The item-start wait is then the
// wave's own vmcnt: no barrier.
template <int HALF_BYTES, int THREADS, int BPS, int STRIDE>
__device__ __forceinline__ void stage_half_own(const void *src, float2 *buf) {
    constexpr int NW = THREADS / 64, WB = HALF_BYTES / NW, PB = 64 * BPS, LPP = PB / 16, PPI = 64 / LPP;
    constexpr int PER = WB / 1024;
    static_assert(WB % 1024 == 0 && PB % 16 == 0 && PER * PPI * PB == WB, "whole pieces per instruction");
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const rsrc_t rs = make_rsrc(src, HALF_BYTES);
    const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) uint8_t *)(uint8_t *)buf + w * WB;
    const int vo = (lane / LPP) * STRIDE * BPS + (lane % LPP) * 16;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(base + j * 1024), "v"(vo), "s"(rs), "s"(j * PPI * STRIDE * BPS + w * PB)
            : "memory");
    }
}

// DIAG (profiling-only ablations, RFA_DIAG): 1 synthetic input (no input loads),
// 2 no row stores, 4 no butterflies/twiddles, 8 no LDS exchanges, 16 no window loads.
// STG: raw input staged through LDS by LDS-DMA one work item ahead (8/16-bit
// formats, one sub-FFT per workgroup, frame fits the exchange buffer; the
// host launches a persistent grid and checks 16-byte alignment).
template <int LOGM, int PT, int RS, int FMT, bool COMPLEX_OUT, int DIAG = 0, bool STG = false>
#ifndef RFA_WIDE_WPE
#define RFA_WIDE_WPE 0  // A/B builds: waves per EU the wide kernels are compiled for (0: the launch bound's 4)
#endif
#if RFA_WIDE_WPE
#define RFA_WIDE_ATTR __attribute__((amdgpu_waves_per_eu(RFA_WIDE_WPE, RFA_WIDE_WPE)))
#else
#define RFA_WIDE_ATTR
#endif
__global__ void __launch_bounds__((WGeo<LOGM, PT>::THREADS), (PT == 64 ? 2 : 4)) RFA_WIDE_ATTR fft_wide_kernel(FftLaunch a) {
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
    const int tid0 = threadIdx.x - slot * G::TPF;
    float2 *buf = data + slot * G::HALFP;

    // large-N kernel B (FMT == kFmtDif): S column residues per frame, one work item each
    constexpr bool dif = FMT == kFmtDif;
    // the DFTs' W8 form (fft_common.h pfma_r2) for the kernel's own 8/16-bit frames (not the
    // large-N pair's scratch, not cf32: both sit near the 0.01 dB bar in one test each, §4)
    constexpr bool W8 = !dif && FMT <= 2;
    static_assert(!dif || (RS == 1 && G::SLOTS == 1), "large-N kernel B: one 32 K residue per workgroup");
    const int work = dif ? a.n_frames * a.dif_ss : a.n_frames;
    const int items = RS == 1 ? (work + G::SLOTS - 1) / G::SLOTS : ((a.n_frames + 7) / 8) * 8 * RS;
    __syncthreads();  // twiddle tables in LDS

#ifdef RFA_DIAG_STG12  // A/B builds only: the staged kernel without butterflies / exchanges (DIAG 12),
                       // without stores (2), with dwordx4 ring stores in tile order (64)
    constexpr int STG_DIAG_OK = ~(60 | 2 | 64);
#else
    constexpr int STG_DIAG_OK = ~48;
#endif
    // SPLIT (RS = 2, 8-bit input): the exchanges run in four rounds through the
    // buffer's first M/4 region A, so the next frame's first half is staged into
    // region B right after this item's pre-stage (it flies during both exchanges and
    // passes) and only its second half waits for exchange 1 (into A).
    constexpr bool SPLIT = STG && RS == 2 && LOGM == 15 && BPS == 2 && !COMPLEX_OUT;
    // QST (64 K interleaved cf32): only the first QN points of each half of the next frame
    // (x[0, QN) and x[M, M + QN), 64 KB each) are staged after exchange 1; the pre-stage
    // reads its first QCH chunks from LDS and the rest from memory as before
    constexpr bool QST = STG && FMT == 3 && RS == 2 && LOGM == 15 && !COMPLEX_OUT;
    constexpr int QN = M / 4, QCH = QST ? QN / (M / 32) / ((PT == 64 ? 16 : 8) / RS) : 0;
    constexpr int Q_BYTES = QN * 8;
    // QSTB (one-residue items on 8-byte complex input: large-N kernel B's z_s, or
    // interleaved cf32 frames of 8 K ... 32 K points): the first half of the next item's
    // points (M/2, 4 M bytes) is staged after exchange 1; its pass-0 loads t < 16 read
    // LDS, the rest memory
    constexpr bool QSTB = STG && RS == 1 && (dif || FMT == 3) && !COMPLEX_OUT;
    constexpr int QB_BYTES = (M / 2) * 8;
    constexpr int QP = M / 4 + M / 128;              // region A (padded quarter, float2)
    constexpr int KR = SPLIT ? 4 : ((RFA_WIDE_KR1 && LOGM == 13) ? 1 : 2);  // exchange rounds
    constexpr int HALF_BYTES = M * RS * BPS / 2;
    constexpr int JS = SPLIT ? -(QP * 8) / BPS : 0;  // raw-element offset of the second half (A) from B
    static_assert(!SPLIT || (G::HALFP - QP) * 8 >= HALF_BYTES, "region B holds half a frame");
    static_assert(!STG || (G::SLOTS == 1 && (FMT <= 2 || QST || QSTB) && !COMPLEX_OUT && (DIAG & STG_DIAG_OK) == 0 &&
                           (QST ? 2 * QN <= G::HALFP : QSTB ? M / 2 <= G::HALFP : M * RS * BPS <= G::HALFP * 8)),
                  "STG: one sub-FFT per WG, 8/16-bit input fitting the buffer (or QST's two cf32 quarters)");
    static_assert(!QST || QCH * ((PT == 64 ? 16 : 8) / RS) * (M / 32) == QN, "QST: whole pre-stage chunks");
    auto stage_qb = [&](int u) {  // QSTB: the first half of item u's points (kernel B: of its column block z_s)
        if constexpr (QSTB) {
            if constexpr (dif) {
                const int fr = u / a.dif_ss, sr = u - fr * a.dif_ss;
                stage_frame<QB_BYTES, G::THREADS>(a.in + (size_t)fr * (size_t)a.frame_stride + (size_t)sr * (M * 8), buf);
            } else {
                stage_frame<QB_BYTES, G::THREADS>(a.in + (size_t)u * (size_t)a.frame_stride, buf);
            }
        }
    };
    constexpr bool OWNQ = QST && RFA_STG_OWNQ;
    auto stage_q = [&](int f) {  // QST: the two staged pieces of frame f
        if constexpr (QST) {
            const uint8_t *fb = a.in + (size_t)f * (size_t)a.frame_stride;
            if constexpr (OWNQ) {
                stage_half_own<Q_BYTES, G::THREADS, 8, M / 32>(fb, buf);
                stage_half_own<Q_BYTES, G::THREADS, 8, M / 32>(fb + (size_t)M * 8, buf + QN);
            } else {
                stage_frame<Q_BYTES, G::THREADS>(fb, buf);
                stage_frame<Q_BYTES, G::THREADS>(fb + (size_t)M * 8, buf + QN);
            }
        }
    };
    // frame of work item u (same mapping as body())
    auto frame_of = [&](int u) {
        if constexpr (dif) return u / a.dif_ss;  // kernel B: item = (frame, column block)
        else if constexpr (RS == 1) return u;
        else return (u / (8 * RS)) * 8 + (u & 7);
    };
    // Work distribution: items blockIdx.x, + grid, ... (static: the residues of a frame
    // land on blocks b and b + 8, one XCD, so the second residue re-reads the frame from
    // that XCD's L2; a device-wide work queue measured 7 % slower at 64 K)
    const int u0 = blockIdx.x;  // first item of this workgroup
    auto next_item = [&](int u) { return u + (int)gridDim.x; };
    // SPLIT: half 0 of a frame goes to region B, half 1 to region A
    constexpr bool OWN = SPLIT && RFA_STG_OWN;
    static_assert(!OWN || (PT == 32 && G::TPF == M / 32), "OWN: one pre-stage sample per thread per M/32");
    auto stage_half = [&](int f, int half) {
        if constexpr (OWN)
            stage_half_own<HALF_BYTES, G::THREADS, BPS, M / 32>(
                a.in + (size_t)f * (size_t)a.frame_stride + (half ? HALF_BYTES : 0), half ? buf : buf + QP);
        else if constexpr (SPLIT)
            stage_frame<HALF_BYTES, G::THREADS>(a.in + (size_t)f * (size_t)a.frame_stride + (half ? HALF_BYTES : 0),
                                                half ? buf : buf + QP);
    };
    if constexpr (STG) {
        const int f0 = frame_of(u0);
        if (u0 < items && f0 < a.n_frames) {
            if constexpr (SPLIT) {
                stage_half(f0, 0);
                stage_half(f0, 1);
            } else if constexpr (QST) {
                stage_q(f0);
            } else if constexpr (QSTB) {
                stage_qb(u0);
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
#ifdef RFA_AB_BUILD
    if (STG && a.phase_ticks > 0 && blockIdx.x >= gridDim.x / 2) {  // A/B: phase offset (RFA_PHASE_NS)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)a.phase_ticks) __builtin_amdgcn_s_sleep(2);
    }
#endif
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

#if RFA_RES_HOIST
    auto body = [&]<int RF>(int u, int unext) {  // RF >= 0: every item of this loop is residue RF
#else
    auto body = [&](int u, int unext) {
#endif
        stamp(u, 0);
        // the lane index, opaque per item: the per-thread LDS bases derived from it are then
        // built inside the item, not hoisted out of the item loop (where they spill to scratch,
        // and each reload is followed by a vmcnt(0) that drains the staged loads)
        int tid = tid0;
        asm volatile("" : "+v"(tid));
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
            // blocks b, b+8, b+16, ... share an XCD: put a frame's RS residues there (speed only).
            // A workgroup keeps one residue across its items (rotating it by the round: +0.3 ..
            // +1.2 %, profiles/r04/residue_rotation_ab.txt)
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
        const RawT *lraw = reinterpret_cast<const RawT *>(SPLIT ? buf + QP : buf);
        if constexpr (STG) {
            // this item's frame, staged by LDS-DMA during the previous item: wait for
            // this wave's pieces, then for every wave's (the barrier)
            // operations younger than the frame's LDS-DMA: the epilogue stores
            const int younger = pending_st;
            if constexpr (OWN || OWNQ) {  // the wave's own pieces only: no barrier
                if (younger >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
                else if (younger >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                if (younger >= 63) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                else if (younger >= 32) asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            }
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
                else if constexpr (STG) {
                    if (QSTB && idx >= PT / 2) raw[idx] = buf_load_raw<FMT>(in_rs, tid * SB, so * SB, planar_im);
                    else raw[idx] = lraw[so + tid];
                } else raw[idx] = buf_load_raw<FMT>(in_rs, tid * SB, so * SB, planar_im);
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
#if RFA_RES_HOIST
                (((RF >= 0 ? RF == Rs : r == Rs) ? prestage<LOGM, PT, RS, FMT, Rs, STG, (DIAG & 16) != 0, QST ? QN : JS,
#else
                ((r == Rs ? prestage<LOGM, PT, RS, FMT, Rs, STG, (DIAG & 16) != 0, QST ? QN : JS,
#endif
                                     RS == 2 && Rs == 1 && FMT <= 2 && (DIAG & 16) == 0, QCH>(
                                v, a.window_il, a.wide_tw, in_rs, tid, planar, lraw, a.window_cw)
                          : void()), ...);
            }(std::make_integer_sequence<int, RS>{});
        }

        // ---- FFT: pass 0 (radix 32, no twiddles), exchange, pass 1, exchange, pass 2
    #pragma unroll
        for (int b = 0; b < PT / 32; b++)
            if constexpr (!(DIAG & 4)) dftw<32, W8>(&v[b * 32]);
        stamp(u, 2);
        if constexpr (STG) {
            lds_barrier();  // every wave has read the staged frame before exchange 0 reuses the buffer
            stamp(u, 7);
            if constexpr (SPLIT) {  // region B is free until the next item: its half of the next frame now
                const int fn = frame_of(unext);
                if (unext < items && fn < a.n_frames) stage_half(fn, 0);
            }
        }
        if constexpr (!(DIAG & 8)) exchange<0, LOGM, PT, KR, STG>(v, buf, tid);
        stamp(u, 3);
        if constexpr (!(DIAG & 4)) pass1<LOGM, PT, W8>(v, tid, tp1);
        if constexpr (!(DIAG & 8)) exchange<1, LOGM, PT, KR, STG>(v, buf, tid);
        stamp(u, 4);
        if constexpr (STG) {
            // exchange 1 ended with a barrier after its last reads: the buffer is free
            // until the next item, so stage the next item's frame now
            const int fn = frame_of(unext);
            if (unext < items && fn < a.n_frames) {
                if constexpr (SPLIT) stage_half(fn, 1);
                else if constexpr (QST) stage_q(fn);
                else if constexpr (QSTB) stage_qb(unext);
                else stage_frame<M * RS * BPS, G::THREADS>(a.in + (size_t)fn * (size_t)a.frame_stride, buf);
            }
        }
        if constexpr (!(DIAG & 4)) pass2<LOGM, PT, W8>(v, tid, tp2);
        stamp(u, 5);
        if constexpr ((DIAG & 12) != 0) {
    #pragma unroll
            for (int q = 0; q < PT; q++) asm volatile("" : "+v"(v[q].x), "+v"(v[q].y));
        }

        if (!active) return;
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
            // kRingTile (M = 32 K, fft_kernels.h): the block's elements in this kernel's store
            // tiles -- thread 64 w + l writes its outputs t' = 4j..4j+3 (t' = (t + 16) mod 32
            // after the fft-shift) as one 16-B store at w*2048 + j*256 + l*4
            constexpr bool TILE_OK = LOGM == 15 && PT == 32 && G::TPF == 1024 && !dif;
            const bool tile = TILE_OK && (a.ring_logrs & kRingTile) != 0;
            // kernel B (dif): rows residue-major too, block s (the engine reorders them)
            const rsrc_t row_rs = make_rsrc(a.rows ? a.rows + (size_t)frame * on + (dif ? (size_t)orr * M : 0) : nullptr,
                                            a.rows ? (dif ? M : on) * 4 : 0);
            const rsrc_t ring_rs = make_rsrc(to_ring ? a.ring + (size_t)rr * on + ((rm || tile) ? (size_t)orr * M : 0) : nullptr,
                                             to_ring ? ((rm || tile) ? M : on) * 4 : 0);
            const int vo = (ors * tid + orr) * 4;
            // one uniform branch per item, not per store
            if constexpr ((DIAG & 64) != 0) {  // A/B: the ring's bytes as 8 dwordx4 stores per thread
                if (to_ring) {
                    float db[PT];
    #pragma unroll
                    for (int q = 0; q < PT; q++) db[q] = db_unscaled(v[q], db_off);
                    const int w = tid >> 6, l = tid & 63;
    #pragma unroll
                    for (int j = 0; j < PT / 4; j++)
                        buf_store_f32x4(db[4 * j], db[4 * j + 1], db[4 * j + 2], db[4 * j + 3], ring_rs,
                                        (w * 2048 + l * 4) * 4, j * 256 * 4);
                }
                pending_st = to_ring ? PT / 4 : 0;
                stamp(u, 6);
                return;
            }
            if constexpr (TILE_OK && (DIAG & 2) == 0) {
                if (tile && to_ring) {
                    const int tvo = ((tid >> 6) * 2048 + (tid & 63) * 4) * 4;
                    auto store_tiles = [&](auto rows_c) {
    #pragma unroll
                        for (int j = 0; j < 8; j++) {
                            float d[4];
    #pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const int t = (4 * j + e + 16) & 31;  // register of output t' = 4j + e
                                d[e] = db_unscaled(v[t], db_off);     // nativedsp.cpp:73-78
                                if constexpr (decltype(rows_c)::value)
                                    buf_store_f32(d[e], row_rs, vo,
                                                  ((ors * (t * (M / G::R2)) + on / 2) & (on - 1)) * 4);
                            }
                            if constexpr (RFA_RING_SC1) buf_store_f32x4(d[0], d[1], d[2], d[3], ring_rs, tvo, j * 1024);
                            else buf_store_f32x4_wb(d[0], d[1], d[2], d[3], ring_rs, tvo, j * 1024);
                        }
                    };
                    if (a.rows) store_tiles(std::true_type{});
                    else store_tiles(std::false_type{});
                    pending_st = (a.rows ? PT : 0) + PT / 4;
                    stamp(u, 6);
                    return;
                }
            }
            auto epilogue = [&](auto nat_c, auto ring_c, auto rm_c) {
                if constexpr (dif && (DIAG & 2) == 0) {
                    // large-N kernel B: every store offset is a compile-time constant (residue-major
                    // rows and ring); one s_mov_b32 next to each store instead of 32 offsets hoisted
                    // out of the item loop, spilled to VGPR lanes and read back with v_readlane + s_nop 4
                    [&]<int... Is>(std::integer_sequence<int, Is...>) {
                        (
                            [&] {
                                constexpr int b = Is / G::R2, t = Is % G::R2;
                                constexpr int so_rm = ((G::TPF * b + t * (M / G::R2) + M / 2) & (M - 1)) * 4;
                                const float db = db_unscaled(v[Is], db_off);  // nativedsp.cpp:73-78
                                if constexpr (decltype(nat_c)::value) buf_store_f32_c<so_rm>(db, row_rs, tid * 4);
                                if constexpr (decltype(ring_c)::value) buf_store_f32_c<so_rm>(db, ring_rs, tid * 4);
                            }(),
                            ...);
                    }(std::make_integer_sequence<int, PT>{});
                    return;
                }
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
            pending_st = (DIAG & 2) ? 0 : (a.rows ? PT : 0) + (to_ring ? PT : 0);
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
    };
#if RFA_RES_HOIST
    auto loop = [&]<int RF>() {
        for (int u = u0; u < items; it_count++) {
            const int un = next_item(u);
            body.template operator()<RF>(u, un);
            u = un;
        }
    };
    // RFA_RES_HOIST: with a grid that is a multiple of 8 RS blocks every item of a
    // workgroup has the same residue, so the item loop is instantiated per residue (register
    // allocation per residue path, no per-item residue branch)
    if constexpr (RS == 2 && !dif) {
        if (gridDim.x % (8 * RS) == 0) {
            if (((u0 % (8 * RS)) >> 3) == 0) loop.template operator()<0>();
            else loop.template operator()<1>();
        } else {
            loop.template operator()<-1>();
        }
    } else {
        loop.template operator()<-1>();
    }
#else
    for (int u = u0; u < items; it_count++) {
        const int un = next_item(u);
        body(u, un);
        u = un;
    }
#endif
}

template <int LOGM, int PT, int RS, int FMT, bool CO, int DIAG = 0, bool STG = false>
static hipError_t launch_wide_one(const FftLaunch &a) {
    using G = WGeo<LOGM, PT>;
    auto kern = &fft_wide_kernel<LOGM, PT, RS, FMT, CO, DIAG, STG>;
    const size_t lds = (size_t)G::LDS_BYTES;
    if (!a.wide_tw) return hipErrorInvalidValue;
    if (RS == 2 && FMT <= 2 && (DIAG & 16) == 0 && !a.window_cw) return hipErrorInvalidValue;  // residue 1's table
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
    if (STG) {  // persistent: all resident workgroups
        static int cus = 0, occ = 0;
        if (!cus) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(kern), G::THREADS,
                                                             lds) != hipSuccess || occ < 1)
                occ = 1;
        }
        blocks = std::min(items, (a.cus > 0 ? a.cus : cus) * occ);
#ifdef RFA_AB_BUILD
        if (const char *g = std::getenv("RFA_WIDE_GRID")) blocks = std::min(blocks, std::max(16, std::atoi(g)));  // A/B only
#endif
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(G::THREADS), lds, a.stream, a);
    return hipGetLastError();
}

int ring_logrs_for(int logn, int fmt) {
    if (logn > 17 && logn <= kMaxLogN) return logn - kDitLogM;  // large-N kernel B: block s of bins S q + s
    if (!wide_supported(logn) || logn <= 14) return 0;
    if (logn == 16 && w64_format(fmt)) return 1 | kRingTile2;  // fft_w64.hip store tiles
    // 32 K-point workgroups (N = 32 K .. 128 K): residue blocks in store-tile order
    return (logn - wide_logm(logn)) | kRingTile;
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
        if constexpr (LOGM == 15 && RS == 2 && G::SLOTS == 1) {  // cf32 64 K: quarter staging (QST)
            if (stg && a.fmt == 3) return launch_wide_one<LOGM, PT, RS, 3, false, 0, true>(a);
        }
        // cf32 32 K: half staging (QSTB); at 8 K / 16 K it spills and is slower (profiles/r03/qstage_h_ab.txt)
        if constexpr (LOGM == 15 && RS == 1 && G::SLOTS == 1) {
            if (stg && a.fmt == 3) return launch_wide_one<LOGM, PT, RS, 3, false, 0, true>(a);
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

#ifndef RFA_AB_BUILD
// The wave-decoupled 64 K kernel (scripts/ab/fft_w64.hip, 8-10 % slower: profiles/r04/w64_ab.txt)
// is linked into A/B builds only; product builds run the wide kernel for every 64 K format.
bool w64_format(int) { return false; }
std::vector<float2> w64_twiddles() { return {}; }
hipError_t launch_fft64(const FftLaunch &) { return hipErrorInvalidValue; }
#endif

// Twiddle blob for the wide kernel (layout must match WGeo): pass-1 [32][R1-1],
// pass-2 A [TPF/LO][15] (none at 8 K: WGeo::A_ALIAS), B [LO][15], pre-stage pre_a [RS][M/32], pre_b [RS][32].
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
    const bool a_alias = lm == 13 && pt == 32;  // WGeo::A_ALIAS: A is read from the pass-1 rows
    for (int hi = 0; hi < (a_alias ? 0 : tpf / lo); hi++)
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
#ifdef RFA_AB_BUILD
    if (a.diag == 16 && a.logn == 16) {  // staged 64 K kernel without window loads (profiling only)
        if (a.fmt != 0 || co) return hipErrorInvalidValue;
        return launch_wide_one<15, 32, 2, 0, false, 16, true>(a);
    }
#ifdef RFA_DIAG_STG12
    if (a.logn == 16 && a.diag != 0 && a.diag != 32 && a.diag != 16) {
        // staged 64 K kernel ablations (A/B builds): 2 no stores, 4 no butterflies, 8 no
        // exchanges, 12 streaming part only, 28 streaming part without window loads,
        // 48 stamps without window loads, 64 dwordx4 ring stores in natural tile order
        if (a.fmt != 0 || co) return hipErrorInvalidValue;
        switch (a.diag) {
        case 2: return launch_wide_one<15, 32, 2, 0, false, 2, true>(a);
        case 4: return launch_wide_one<15, 32, 2, 0, false, 4, true>(a);
        case 8: return launch_wide_one<15, 32, 2, 0, false, 8, true>(a);
        case 12: return launch_wide_one<15, 32, 2, 0, false, 12, true>(a);
        case 28: return launch_wide_one<15, 32, 2, 0, false, 28, true>(a);
        case 48: return launch_wide_one<15, 32, 2, 0, false, 48, true>(a);
        case 64: return launch_wide_one<15, 32, 2, 0, false, 64, true>(a);
        default: return hipErrorInvalidValue;
        }
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
#endif
    if (a.fmt == kFmtDif) {  // kernel B of the large-N pair (dB rows / ring, or the ordered spectrum)
        if (a.dif_ss < 8 || a.dif_ss > 32) return hipErrorInvalidValue;
        if (co) return launch_wide_one<kDitLogM, 32, 1, kFmtDif, true>(a);
        // QSTB: half of the next item's z_s staged by LDS-DMA (16-byte aligned scratch)
        if (a.stage && ((reinterpret_cast<uintptr_t>(a.in) | (uintptr_t)a.frame_stride) & 15) == 0)
            return launch_wide_one<kDitLogM, 32, 1, kFmtDif, false, 0, true>(a);
        return launch_wide_one<kDitLogM, 32, 1, kFmtDif, false>(a);
    }
    switch (a.logn) {
    case 13: return co ? wide_by_fmt<13, 32, 1, true>(a) : wide_by_fmt<13, 32, 1, false>(a);
    case 14: return co ? wide_by_fmt<14, 32, 1, true>(a) : wide_by_fmt<14, 32, 1, false>(a);
    case 15: return co ? wide_by_fmt<15, 32, 1, true>(a) : wide_by_fmt<15, 32, 1, false>(a);
    case 16:
#if RFA_RES16K
        if (!co) return wide_by_fmt<14, 32, 4, false>(a);  // A/B: four 16 K residues per frame
#endif
        if (co) return wide_by_fmt<15, 32, 2, true>(a);
        return w64_format(a.fmt) ? launch_fft64(a) : wide_by_fmt<15, 32, 2, false>(a);
    case 17: return co ? wide_by_fmt<15, 32, 4, true>(a) : wide_by_fmt<15, 32, 4, false>(a);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace rfa
