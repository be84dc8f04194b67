// gfx950 64 K-point kernel, wave-decoupled form: A/B builds only (DESIGN.md §6.3 -- measured 8-10 %
// slower than the wide kernel, profiles/r04/w64_ab.txt; product builds keep fft_wide.hip for N = 64 K).
//
// Same per-frame pipeline as the wide kernel (fft_wide.hip): raw IQ -> LUT-exact convert ->
// window (fp32 multiply, NativeDsp.kt:55-58) -> radix-2 decimation-in-frequency pre-stage
// into two 32 K residue items -> FFT (sign -1, unscaled, pffft.h:117) -> 10*log10(|X|/N) +
// fft-shift (nativedsp.cpp:72-79) -> ring / rows.  What differs is how the 16 waves of the
// 1024-thread workgroup that holds one 32 K item are coupled:
//
//   * index bits: m = m0 + 32 m1 + 1024 m2 (5-bit digits).  At pass 0 a thread holds m2 in
//     its 32 registers; lane bits 1-5 carry m0 and lane bit 0 + the 4 wave bits carry m1.
//     Pass 0 (DFT over m2 -> k0), exchange 0, pass 1 (m1 -> k1), exchange 1, pass 2
//     (m0 -> k2): X[k0 + 32 k1 + 1024 k2] (DIT twiddles W_1024^{m1 k0}, W_M^{m0 (k0 + 32 k1)}).
//   * exchange 0 swaps the registers with lane bit 0 + wave bits: the one cross-wave
//     exchange of the item (four rounds through LDS region A, workgroup barriers);
//   * exchange 1 swaps the registers with lane bits 1-5 only, so it is WAVE-LOCAL: register
//     bits 4 / 3 <-> lane bits 5 / 4 by v_permlane32_swap / v_permlane16_swap (one VALU
//     instruction per register pair), register bits 0-2 <-> lane bits 1-3 through the wave's
//     own 4 KiB slice of LDS in four balanced rounds -- no s_barrier;
//   * the 8-bit frame is staged per WAVE: a wave's points of one half of the frame are 32
//     pieces of 64 consecutive samples (128 B), which its own LDS-DMA brings into its own
//     slices (half 0 -> region B right after its pre-stage, half 1 -> its region-A slice right
//     after its exchange 1), so a wave waits for its own DMA only -- no item-start barrier.
//
// Between two passes of exchange 0 the waves run free: one wave's exchange 1 (LDS) and DMA
// waits overlap the other waves' butterflies and dB epilogue on the same SIMD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "../../rfanalyzer_amd/csrc/fft_common.h"
#include "../../rfanalyzer_amd/csrc/fft_kernels.h"

namespace rfa {
namespace {

constexpr int kM = 32768;            // points per residue item (N = 2 M)
constexpr int kN = 65536;
constexpr int kRow = 31;             // TB row: t = 1 .. 31
constexpr int kRow1 = 33;            // T1 row: t = 0 .. 31 (+1 pad: 32 rows read at once, distinct banks)
constexpr int kTw1 = 32 * kRow1;     // T1[a][t] = W_1024^{a t}
constexpr int kTwLds = kTw1 + 32 * kRow;  // + TB[k0][t - 1] = W_M^{t k0}
constexpr int kPreA = kTwLds;        // blob only: W_N^c, c < 1024 (f32 residue 1)
constexpr int kSliceA = 528;         // float2 per wave in region A: exchange-1 rounds (8 x 66) / staged half 1
constexpr int kRegA = 16 * kSliceA;  // 8448: also the four-round exchange 0 (32 x 257 used)
constexpr int kSliceB = 512;         // float2 per wave in region B: staged half 0 (4 KiB)
constexpr int kRegB = 16 * kSliceB;
constexpr int kLdsBytes = (kTwLds + kRegA + kRegB) * 8;  // 148,992 B
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

#ifndef RFA_W64_X0R
#define RFA_W64_X0R 4  // exchange 0: 4 balanced rounds through region A (default); A/B builds: 2 = writer-wave
                       // rounds through A + B, 3 = four writer-wave rounds through A
#endif

// ---- wave-private staging: LDS-DMA of this wave's pieces x[64 w + 1024 t + half M], t < 32
// (64 samples = 128 B of 8-bit IQ each) into its slice, piece t at slice + 128 t bytes.
// Four wave instructions of 1 KiB (16 B per lane, lane-linear in LDS, per-lane source).
// Inline asm like fft_wide.hip stage_frame: the builtin makes hipcc wait vmcnt(0) before
// later LDS reads; completion is waited for explicitly at the start of the next item.
__device__ __forceinline__ void stage_half(const uint8_t *frame, int half, float2 *slice, int w, int l) {
#if defined(__HIP_DEVICE_COMPILE__)
    const rsrc_t rs = make_rsrc(frame, kN * 2);
    const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) uint8_t *)(uint8_t *)slice;
    const int vo = half * (kM * 2) + w * 128 + (l >> 3) * 2048 + (l & 7) * 16;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(base + i * 1024), "v"(vo), "s"(rs), "s"(i * 16384)
            : "memory");
    }
#else
    (void)frame; (void)half; (void)slice; (void)w; (void)l;
#endif
}

// v_permlane32_swap / v_permlane16_swap of both halves of a complex value: lanes 32-63
// (odd 16-lane rows) of a trade places with lanes 0-31 (even rows) of b
template <int BITS>
__device__ __forceinline__ void lane_swap(float2 &a, float2 &b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (BITS == 32) {
        const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
        const auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
        a = make_float2(__uint_as_float(x[0]), __uint_as_float(y[0]));
        b = make_float2(__uint_as_float(x[1]), __uint_as_float(y[1]));
    } else {
        const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
        const auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
        a = make_float2(__uint_as_float(x[0]), __uint_as_float(y[0]));
        b = make_float2(__uint_as_float(x[1]), __uint_as_float(y[1]));
    }
#else
    (void)a; (void)b;
#endif
}

__device__ __forceinline__ void compiler_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::: "memory");
#endif
}

// ---- exchange 0 (cross-wave): registers k0 <-> (lane bit 0, wave bits); lane bits 1-5 (m0)
// stay.  Round h: the WPR writer waves w / WPR == h store all 32 registers (one whole
// k0-row of 64 lanes per instruction, contiguous), then every thread reads its RB registers
// m1 = RB h + b.  Row pitch ROW + 1 float2: the odd / even reading lanes (k0 bit 0) land
// two banks apart, conflict-free.
template <int X0R>
__device__ __forceinline__ void exchange0(float2 (&v)[32], float2 *buf, int l, int w) {
    constexpr int WPR = 16 / X0R, RB = 32 / X0R, ROWP = WPR * 64 + 1;
    const int k0 = (l & 1) | (w << 1);
    auto wb = lds_opaque(buf + (w % WPR) * 64 + l);
    auto rd = lds_opaque(buf + k0 * ROWP + (l & ~1));
    float2 in[X0R][RB];
#pragma unroll
    for (int h = 0; h < X0R; h++) {
        if (w / WPR == h) {
#pragma unroll
            for (int k = 0; k < 32; k++) wb[k * ROWP] = v[k];
        }
        lds_barrier();
#pragma unroll
        for (int b = 0; b < RB; b++) in[h][b] = lds_ld2(rd + (b >> 1) * 64 + (b & 1));  // unfused ds_read_b64
        lds_barrier();
    }
#pragma unroll
    for (int m = 0; m < 32; m++) v[m] = in[m / RB][m % RB];
}

// ---- exchange 0, balanced form (X0R == 4): in round h EVERY wave stores one group of 8
// registers and loads one group of 8, so all 16 waves (4 per SIMD) write at once -- the
// LDS store rate of ds_write_b64 needs about 4 writing waves per SIMD (MI355X_MICROARCH.md,
// LDS), which writer-wave rounds (4 waves per round) do not have.  Round h pairs a writer's
// register group g = (h - hi) & 3 (k0 bits 3-4) with a reader's m1 group (h - hi) & 3, hi =
// wave bits 2-3 (= m1 bits 3-4 of a writer, k0 bits 3-4 of a reader), so a round is 4
// (m1 group, k0 group) pairs x 8 x 8 x 32 m0 = 64 KiB.  The writer's group is wave-uniform
// but not compile-time: each arm of a uniform branch stores its own 8 registers by inline
// asm whose text names the group (hipcc merged plain arms into one sequence with a register
// select, through scratch).  A reader keeps round h's values in register slots 8h .. 8h+7,
// so slot n holds m1 = (n - 8 hi) mod 32: pass 1's input rotated by 8 hi, which multiplies
// its outputs by (-i)^{hi k1}, a phase that factors out of pass 2 and |X|.  (Moving them back
// into m1 order costs 64 register moves or, as four compile-time arms, spills.)
// Element (pair p, k0lo, m1 bits 1-2, m0, m1 bit 0) at p*2048 + k0lo*256 + m1b12*64 + m0*2 +
// m1b0, XOR 1 when k0lo is odd: a store instruction covers 64 consecutive elements, a
// load's odd and even lanes land two banks apart (tests/test_w64_model.py).
__device__ __forceinline__ void exchange0_bal(float2 (&v)[32], float2 *buf, int l, int w) {
    const int hi = w >> 2;  // wave-uniform
    const int k0lo = ((w & 3) << 1) | (l & 1);
    // LDS byte addresses of the two store bases (k0lo even / odd; the stores are inline asm)
    unsigned wb0 = (unsigned)(size_t)(__attribute__((address_space(3))) float2 *)(buf + hi * 2048 + (w & 3) * 64 + l);
    unsigned wb1 = (unsigned)(size_t)(__attribute__((address_space(3))) float2 *)(buf + hi * 2048 + (w & 3) * 64 + (l ^ 1));
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(wb0), "+v"(wb1));
#endif
    auto rd0 = lds_opaque(buf + k0lo * 256 + l);  // load bases (m1 bit 0 even / odd)
    auto rd1 = lds_opaque(buf + k0lo * 256 + (l ^ 1));
    float2 in[4][8];
#pragma unroll
    for (int h = 0; h < 4; h++) {
        const int g = (h - hi) & 3;  // wave-uniform: this round's store group / load pair
        // explicit captures: clang does not capture variables used only as asm operands
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-lambda-capture"
        auto put = [&v, wb0, wb1](auto gc) {
            constexpr int G = decltype(gc)::value;
#if !defined(__HIP_DEVICE_COMPILE__)
            (void)v; (void)wb0; (void)wb1; (void)G;
#else
            asm volatile("; exchange-0 stores, register group %10\n\t"
                         "ds_write_b64 %0, %2\n\t"
                         "ds_write_b64 %1, %3 offset:2048\n\t"
                         "ds_write_b64 %0, %4 offset:4096\n\t"
                         "ds_write_b64 %1, %5 offset:6144\n\t"
                         "ds_write_b64 %0, %6 offset:8192\n\t"
                         "ds_write_b64 %1, %7 offset:10240\n\t"
                         "ds_write_b64 %0, %8 offset:12288\n\t"
                         "ds_write_b64 %1, %9 offset:14336"
                         :
                         : "v"(wb0), "v"(wb1), "v"(to_v(v[8 * G])), "v"(to_v(v[8 * G + 1])), "v"(to_v(v[8 * G + 2])),
                           "v"(to_v(v[8 * G + 3])), "v"(to_v(v[8 * G + 4])), "v"(to_v(v[8 * G + 5])),
                           "v"(to_v(v[8 * G + 6])), "v"(to_v(v[8 * G + 7])), "i"(G)
                         : "memory");
#endif
        };
#pragma clang diagnostic pop
        switch (g) {  // uniform branch: compile-time register indices in each arm
        case 0: put(std::integral_constant<int, 0>{}); break;
        case 1: put(std::integral_constant<int, 1>{}); break;
        case 2: put(std::integral_constant<int, 2>{}); break;
        default: put(std::integral_constant<int, 3>{}); break;
        }
        lds_barrier();
        const int po = g * 2048;  // the pair this wave loads (m1 group g)
#pragma unroll
        for (int j = 0; j < 8; j++) in[h][j] = lds_ld2((j & 1) ? rd1 + po + (j >> 1) * 64 : rd0 + po + (j >> 1) * 64);
        lds_barrier();
    }
#pragma unroll
    for (int n = 0; n < 32; n++) v[n] = in[n >> 3][n & 7];
}

// ---- exchange 1 (wave-local): registers k1 <-> lane bits 1-5 (m0); lane bit 0 and the wave
// bits (k0) stay.  Register bit 4 <-> lane bit 5 and bit 3 <-> lane bit 4 by permlane swaps,
// then bits 0-2 <-> lane bits 1-3 through this wave's slice: round h, lane l stores its
// registers 8h + a at a*66 + l and reads register 8h + b from lane (l & 0x31) | (b << 1),
// slot (l >> 1) & 7.  LDS instructions of one wave execute in order, so the round needs no
// barrier (the compiler fence keeps hipcc from moving the reads above the stores).
__device__ __forceinline__ void exchange1(float2 (&v)[32], float2 *slice, int l) {
#pragma unroll
    for (int j = 0; j < 16; j++) lane_swap<32>(v[j], v[j + 16]);
#pragma unroll
    for (int j = 0; j < 32; j++)
        if ((j & 8) == 0) lane_swap<16>(v[j], v[j + 8]);
    auto wb = lds_opaque(slice + l);
    auto rd = lds_opaque(slice + ((l >> 1) & 7) * 66 + (l & 0x31));
#pragma unroll
    for (int h = 0; h < 4; h++) {
#pragma unroll
        for (int a = 0; a < 8; a++) wb[a * 66] = v[8 * h + a];
        compiler_fence();
#pragma unroll
        for (int b = 0; b < 8; b++) v[8 * h + b] = lds_ld2(rd + 2 * b);
        compiler_fence();
    }
}

// ---- pre-stage (residue R of N = 2M): y_R[m] = W_N^{m R} (x[m] w[m] + (-1)^R x[m + M] w[m + M]),
// m = col + 1024 t, t = register.  8/16-bit residue 1 folds W_N^m into the complex window
// cw[m] = (w[m] W_N^m, -w[m + M] W_N^m) (fft_wide.hip prestage CW); f32 residue 1
// uses W_N^{col} * W_64^t.  Staged input: this wave's samples at l0 / l1 + 64 t (halves 0 / 1).
// Loads run one chunk of four points ahead of the arithmetic.
template <int FMT, int R, bool STG, typename P>
__device__ __forceinline__ void prestage(float2 (&v)[32], const float *window_il, const float4 *cw, float2 pa,
                                         rsrc_t in_rs, int col, P l0, P l1) {
    constexpr bool CW = R == 1 && FMT <= 2;
    constexpr int SB = FMT == 4 ? 4 : ((FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8));
    constexpr int C = 4, NCH = 32 / C;
    const rsrc_t w_rs = CW ? make_rsrc(cw, kM * 16) : make_rsrc(window_il, kM * 8);
    typename Raw<FMT>::T raw[2][C][2];
    float win[2][C][CW ? 4 : 2];
    auto issue = [&]<int c>() {
        constexpr int s = c & 1;
#pragma unroll
        for (int q = 0; q < C; q++) {
            const int t = c * C + q, mo = 1024 * t;
            if constexpr (STG) {
                raw[s][q][0] = l0[64 * t];
                raw[s][q][1] = l1[64 * t];
            } else {
                raw[s][q][0] = buf_load_raw<FMT>(in_rs, col * SB, mo * SB, kN * 4);
                raw[s][q][1] = buf_load_raw<FMT>(in_rs, col * SB, (mo + kM) * SB, kN * 4);
            }
            if constexpr (CW) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                const f4v x = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(w_rs, col * 16, mo * 16, 0));
                win[s][q][0] = x.x;
                win[s][q][1] = x.y;
                win[s][q][2] = x.z;
                win[s][q][3] = x.w;
            } else {
                const f2v x = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(w_rs, col * 8, mo * 8, 0));
                win[s][q][0] = x.x;
                win[s][q][1] = x.y;
            }
        }
    };
    auto compute = [&]<int c>() {
        constexpr int s = c & 1;
        if constexpr (CW) {  // two points' cmac2 chains interleaved (fft_common.h cmac2x2)
#pragma unroll
            for (int q = 0; q < C; q += 2)
                cmac2x2(v[c * C + q], convert_raw<FMT>(raw[s][q][0]), make_float2(win[s][q][0], win[s][q][1]),
                        convert_raw<FMT>(raw[s][q][1]), make_float2(win[s][q][2], win[s][q][3]), v[c * C + q + 1],
                        convert_raw<FMT>(raw[s][q + 1][0]), make_float2(win[s][q + 1][0], win[s][q + 1][1]),
                        convert_raw<FMT>(raw[s][q + 1][1]), make_float2(win[s][q + 1][2], win[s][q + 1][3]));
        } else if constexpr (R == 0) {  // x[m] w[m] + x[m + M] w[m + M]: mul + fma
#pragma unroll
            for (int q = 0; q < C; q++) {
                const f2v x0 = to_v(convert_raw<FMT>(raw[s][q][0])), x1 = to_v(convert_raw<FMT>(raw[s][q][1]));
                v[c * C + q] = from_v(__builtin_elementwise_fma(x1, (f2v){win[s][q][1], win[s][q][1]}, x0 * win[s][q][0]));
            }
        } else {  // (x[m] w[m] - x[m + M] w[m + M]) * W_N^{col} * W_64^t
            [&]<int... Qs>(std::integer_sequence<int, Qs...>) {
                (
                    [&] {
                        constexpr int t = c * C + Qs;
                        const f2v x0 = to_v(convert_raw<FMT>(raw[s][Qs][0])) * win[s][Qs][0];
                        const f2v x1 = to_v(convert_raw<FMT>(raw[s][Qs][1])) * win[s][Qs][1];
                        v[t] = w64<t & 63>(cmul(from_v(x0 - x1), pa));
                    }(),
                    ...);
            }(std::make_integer_sequence<int, C>{});
        }
    };
    issue.template operator()<0>();
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
        (
            [&] {
                if constexpr (Cs + 1 < NCH) issue.template operator()<Cs + 1>();
                __builtin_amdgcn_sched_barrier(0);
                compute.template operator()<Cs>();
                __builtin_amdgcn_sched_barrier(0);
            }(),
            ...);
    }(std::make_integer_sequence<int, NCH>{});
}

// DIAG 32 (A/B builds only): s_memrealtime stamps of every wave's phases, lane 0 of each
// wave into a.stamps[block][item < 4][wave][8] (engine RFA_STAMPS_FILE, scripts/stamps_w64.py):
// 0 item start, 1 own DMA landed, 2 pass 0 done, 3 exchange-0 entry barrier passed,
// 4 exchange 0 done, 5 pass 1 done, 6 exchange 1 (+ DMA issue) done, 7 pass 2 + epilogue done
// Pre-stage with deep window prefetch (8-bit staged input, PREW = 1): at the start of an item the
// 64 VGPRs of v are dead, so all 32 window pairs of residue 0 (8 B per point) are issued at once
// into them and each point's result overwrites its own window pair; residue 1's complex window
// (16 B per point) goes in two waves of 16 loads, the second issued into the registers the
// first frees point by point.  One L2 round trip per item instead of one per 4-point chunk.
template <int FMT, int R, typename P>
__device__ __forceinline__ void prestage_deep(float2 (&v)[32], const float *window_il, const float4 *cw, int col, P l0,
                                              P l1) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    if constexpr (R == 0) {
        const rsrc_t w_rs = make_rsrc(window_il, kM * 8);
        f2v wv[32];
#pragma unroll
        for (int t = 0; t < 32; t++)
            wv[t] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(w_rs, col * 8, 1024 * t * 8, 0));
#pragma unroll
        for (int t = 0; t < 32; t++) {
            const f2v x0 = to_v(convert_raw<FMT>(l0[64 * t])), x1 = to_v(convert_raw<FMT>(l1[64 * t]));
            v[t] = from_v(__builtin_elementwise_fma(x1, (f2v){wv[t].y, wv[t].y}, x0 * wv[t].x));
        }
    } else {
        const rsrc_t w_rs = make_rsrc(cw, kM * 16);
        f4v cv[16];
        auto ld = [&](int t) {
            return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(w_rs, col * 16, 1024 * t * 16, 0));
        };
        auto pt = [&](int t, f4v c) {
            return cmac2(convert_raw<FMT>(l0[64 * t]), make_float2(c.x, c.y), convert_raw<FMT>(l1[64 * t]),
                         make_float2(c.z, c.w));
        };
#pragma unroll
        for (int q = 0; q < 16; q++) cv[q] = ld(q);
#pragma unroll
        for (int q = 0; q < 16; q++) {
            v[q] = pt(q, cv[q]);
            cv[q] = ld(16 + q);
        }
#pragma unroll
        for (int q = 0; q < 16; q++) v[16 + q] = pt(16 + q, cv[q]);
    }
}

template <int FMT, bool STG, int X0R, int DIAG = 0, int PREW = 0>
__global__ void __launch_bounds__(1024, 4) fft64_kernel(FftLaunch a) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    for (int e = threadIdx.x; e < kTwLds; e += 1024) lds[e] = a.w64_tw[e];
    float2 *ra = lds + kTwLds, *rb = ra + kRegA;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float2 *sa = ra + w * kSliceA, *sb = rb + w * kSliceB;  // this wave's slices
    constexpr int BPS = (FMT == 0 || FMT == 1) ? 2 : (FMT == 2 ? 4 : 8);
    using RawT = typename Raw<FMT>::T;
    const int items = ((a.n_frames + 7) / 8) * 16;
    // item u = (frame, residue): the two residues of a frame are items u, u + 8, i.e. blocks
    // b and b + 8 of the persistent grid, one XCD (the second re-reads the frame from L2)
    auto frame_of = [](int u) { return (u >> 4) * 8 + (u & 7); };
    auto frame_ptr = [&](int f) { return a.in + (size_t)f * (size_t)a.frame_stride; };
    __syncthreads();  // twiddle tables
    if constexpr (STG) {
        const int f0 = frame_of(blockIdx.x), l = threadIdx.x & 63;
        if ((int)blockIdx.x < items && f0 < a.n_frames) {
            stage_half(frame_ptr(f0), 0, sb, w, l);
            stage_half(frame_ptr(f0), 1, sa, w, l);
        }
    }
#ifdef RFA_AB_BUILD
    // A/B: static wave priorities (MI355X_MICROARCH.md, two waves per SIMD item 4): 1 = the
    // younger half (waves 8-15) at priority 1; 2 = priority w >> 2 (the youngest wave of each
    // SIMD first); 3 = priority 3 - (w >> 2)
    const int prio = a.prio & 15;
    if (prio == 1 && w >= 8) __builtin_amdgcn_s_setprio(1);
    if (prio == 2) {
        if (w >= 12) __builtin_amdgcn_s_setprio(3);
        else if (w >= 8) __builtin_amdgcn_s_setprio(2);
        else if (w >= 4) __builtin_amdgcn_s_setprio(1);
    }
    if (prio == 3) {
        if (w < 4) __builtin_amdgcn_s_setprio(3);
        else if (w < 8) __builtin_amdgcn_s_setprio(2);
        else if (w < 12) __builtin_amdgcn_s_setprio(1);
    }
#endif
    const float db_off = -kDbPerLog2 * 32.0f;  // 2 log2 N
    int pending_st = 0;  // stores issued after this wave's last staging DMA
    int it = 0;
    auto stamp = [&](int k) {
        if constexpr (DIAG & 32) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            int wi = (int)(threadIdx.x >> 6);  // per-lane (VGPR) index math, kept opaque
            asm volatile("" : "+v"(wi));
            if ((threadIdx.x & 63) == 0 && it < 4) a.stamps[(((size_t)blockIdx.x * 4 + it) * 16 + wi) * 8 + k] = t;
        }
    };
    for (int u = blockIdx.x; u < items; u += gridDim.x, it++) {
        stamp(0);
        const int un = u + gridDim.x, fn = frame_of(un);
        const bool stage_next = STG && un < items && fn < a.n_frames;
        const int frame = frame_of(u), r = (u >> 3) & 1;
        const bool active = frame < a.n_frames;
        int z;  // opaque zero: the per-item table reads are not hoisted out of the item loop
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const float2 *t1 = lds + z, *tb = lds + kTw1 + z;
        // lane index, opaque per item: the per-lane offsets below are rebuilt each item
        // instead of being hoisted out of the item loop (and spilled)
        int l = threadIdx.x & 63;
        asm volatile("" : "+v"(l));
        const int col = (l >> 1) + ((l & 1) << 5) + (w << 6);  // m0 + 32 m1 of this lane at pass 0
        const int k0 = (l & 1) | (w << 1);                      // after exchange 0
        const int k1 = l >> 1;                                  // after exchange 1
        float2 v[32];
        if constexpr (STG) {  // this wave's own pieces of the frame (younger: the epilogue stores)
            if (pending_st >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            else if (pending_st >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        stamp(1);
        {
            const rsrc_t in_rs = make_rsrc(frame_ptr(active ? frame : 0), active ? (unsigned)(kN * BPS) : 0u);
            auto run = [&](auto l0, auto l1) {
                if constexpr (PREW && STG) {
                    if (r == 0) prestage_deep<FMT, 0>(v, a.window_il, a.window_cw, col, l0, l1);
                    else prestage_deep<FMT, 1>(v, a.window_il, a.window_cw, col, l0, l1);
                    return;
                }
                if (r == 0) {
                    prestage<FMT, 0, STG>(v, a.window_il, a.window_cw, make_float2(0.f, 0.f), in_rs, col, l0, l1);
                } else {
                    float2 pa = make_float2(0.f, 0.f);
                    if constexpr (FMT > 2) pa = buf_load_f32x2(make_rsrc(a.w64_tw + kPreA, 1024 * 8), col * 8, 0);
                    prestage<FMT, 1, STG>(v, a.window_il, a.window_cw, pa, in_rs, col, l0, l1);
                }
            };
            if constexpr (STG) {
                const int q = (l >> 1) + ((l & 1) << 5);
                run(lds_opaque(reinterpret_cast<RawT *>(sb) + q), lds_opaque(reinterpret_cast<RawT *>(sa) + q));
            } else {
                run((const RawT *)nullptr, (const RawT *)nullptr);
            }
        }
        dft<32>(v);  // pass 0: m2 -> k0
        stamp(2);
        if constexpr (STG && X0R != 2) {
            if (stage_next) stage_half(frame_ptr(fn), 0, sb, w, l);
        }
        lds_barrier();  // every wave has read its staged pieces before exchange 0 reuses region A
        stamp(3);
        if constexpr (X0R == 4) exchange0_bal(v, ra, l, w);
        else exchange0<X0R == 3 ? 4 : X0R>(v, ra, l, w);
        stamp(4);
        // pass 1: twiddle W_1024^{k0 m1}, DFT over m1 -> k1.  After the balanced exchange slot n
        // holds m1 = (n - 8 hi) mod 32: its twiddle is read at that index, and the DFT of the
        // rotated slots is (-i)^{hi k1} X[k1] -- a phase independent of m0, so it factors out
        // of pass 2 and |X| (the only thing stored) is unchanged
        {
            const float2 *row = t1 + k0 * kRow1;
            if constexpr (X0R == 4) {
                const int hi = w >> 2;
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const float2 *rg = row + ((h - hi) & 3) * 8;
#pragma unroll
                    for (int j = 0; j < 8; j += 2)
                        cmul2(v[8 * h + j], lds_ld2(rg + j), v[8 * h + j + 1], lds_ld2(rg + j + 1));
                }
            } else {
                v[1] = cmul(v[1], lds_ld2(row + 1));
#pragma unroll
                for (int t = 2; t < 32; t += 2) cmul2(v[t], lds_ld2(row + t), v[t + 1], lds_ld2(row + t + 1));
            }
        }
        dft<32>(v);
        stamp(5);
        if constexpr (STG && X0R == 2) {
            if (stage_next) stage_half(frame_ptr(fn), 0, sb, w, l);
        }
        exchange1(v, sa, l);
        if constexpr (STG) {
            if (stage_next) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's slice reads are done
                stage_half(frame_ptr(fn), 1, sa, w, l);
            }
        }
        stamp(6);
        // pass 2: twiddle W_M^{m0 (k0 + 32 k1)} = T1[k1][m0] * TB[k0][m0], DFT over m0 -> k2
        {
            const float2 *pa_ = t1 + k1 * kRow1, *pb_ = tb + k0 * kRow - 1;
            const float2 w1 = cmul(lds_ld2(pa_ + 1), lds_ld2(pb_ + 1));
            v[1] = cmul(v[1], w1);
#pragma unroll
            for (int t = 2; t < 32; t += 2) {
                float2 w0 = lds_ld2(pa_ + t), w2 = lds_ld2(pa_ + t + 1);
                cmul2(w0, lds_ld2(pb_ + t), w2, lds_ld2(pb_ + t + 1));
                cmul2(v[t], w0, v[t + 1], w2);
            }
        }
        dft<32>(v);
        pending_st = 0;
        if (!active) continue;
        // ---- epilogue: register t holds sub-bin k0 + 32 k1 + 1024 t = full bin 2 (...) + r; the
        // fft-shift (nativedsp.cpp:77) flips t's bit 4: t' = t ^ 16
        const bool to_ring = a.ring && frame >= a.ring_first;
        int rr = 0;
        if (to_ring) {
            rr = (a.ring_base - frame) % a.ring_rows;
            if (rr < 0) rr += a.ring_rows;
        }
        const rsrc_t row_rs = make_rsrc(a.rows ? a.rows + (size_t)frame * kN : nullptr, a.rows ? kN * 4 : 0);
        // ring (kRingTile2): block r, thread (w, l)'s registers t' = 4j .. 4j+3 as one 16-B store
        const rsrc_t ring_rs =
            make_rsrc(to_ring ? a.ring + (size_t)rr * kN + (size_t)r * kM : nullptr, to_ring ? kM * 4 : 0);
        const int tvo = (w * 2048 + l * 4) * 4;
        const int rvo = (2 * (k0 + 32 * k1) + r) * 4;  // natural row: bin 2 (k0 + 32 k1 + 1024 t') + r
        auto store = [&](auto rows_c, auto ring_c) {
            [&]<int... Js>(std::integer_sequence<int, Js...>) {
                (
                    [&] {
                        constexpr int j = Js;
                        float d[4];
                        [&]<int... Es>(std::integer_sequence<int, Es...>) {
                            (
                                [&] {
                                    constexpr int tp = 4 * j + Es;
                                    d[Es] = db_unscaled(v[tp ^ 16], db_off);  // nativedsp.cpp:73-78
                                    if constexpr (decltype(rows_c)::value) buf_store_f32_c<2048 * tp * 4>(d[Es], row_rs, rvo);
                                }(),
                                ...);
                        }(std::make_integer_sequence<int, 4>{});
                        if constexpr (decltype(ring_c)::value) buf_store_f32x4(d[0], d[1], d[2], d[3], ring_rs, tvo, j * 1024);
                    }(),
                    ...);
            }(std::make_integer_sequence<int, 8>{});
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        if (a.rows && to_ring) store(T_{}, T_{});
        else if (a.rows) store(T_{}, F_{});
        else if (to_ring) store(F_{}, T_{});
        pending_st = (a.rows ? 32 : 0) + (to_ring ? 8 : 0);
        stamp(7);
    }
}

template <int FMT, bool STG, int X0R, int DIAG = 0, int PREW = 0>
hipError_t launch64_one(const FftLaunch &a) {
    auto kern = &fft64_kernel<FMT, STG, X0R, DIAG, PREW>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int items = ((a.n_frames + 7) / 8) * 16;
    if (items <= 0) return hipSuccess;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    }
    const int blocks = std::min(items, cus);  // persistent: one 1024-thread workgroup per CU
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), kLdsBytes, a.stream, a);
    return hipGetLastError();
}

template <int X0R>
hipError_t launch64_x(const FftLaunch &a) {
    const bool stg = a.stage && ((reinterpret_cast<uintptr_t>(a.in) | (uintptr_t)a.frame_stride) & 15) == 0;
#ifdef RFA_AB_BUILD
    if ((a.diag & 32) && a.stamps) {  // phase stamps (profiling only): staged s8
        if (a.fmt != 0 || !stg) return hipErrorInvalidValue;
        return launch64_one<0, true, X0R, 32>(a);
    }
#endif
#ifdef RFA_AB_BUILD
    if (a.prio >= 16 && stg && a.fmt <= 1) {  // A/B (RFA_W64_PREW=1): deep window prefetch
        return a.fmt == 0 ? launch64_one<0, true, X0R, 0, 1>(a) : launch64_one<1, true, X0R, 0, 1>(a);
    }
#endif
    switch (a.fmt) {
    case 0: return stg ? launch64_one<0, true, X0R>(a) : launch64_one<0, false, X0R>(a);
    case 1: return stg ? launch64_one<1, true, X0R>(a) : launch64_one<1, false, X0R>(a);
    case 2: return launch64_one<2, false, X0R>(a);
    case 3: return launch64_one<3, false, X0R>(a);
    case 4: return launch64_one<4, false, X0R>(a);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// rfa_input_format bits that take this kernel at N = 64 K.  Product builds: none -- the
// round-4 same-call A/B (profiles/r04/w64_ab.txt) measured it 8-10 % slower than the wide
// kernel for every format, so it is compiled into A/B builds only (all formats, or the
// RFA_W64_FORMATS environment mask).
#ifndef RFA_W64_FORMATS
#define RFA_W64_FORMATS 0  // A/B builds too: N = 64 K takes the product's wide kernel unless the
                           // RFA_W64_FORMATS environment mask selects this one
#endif
bool w64_format(int fmt) {
#ifdef RFA_AB_BUILD
    if (const char *x = std::getenv("RFA_W64_FORMATS")) return fmt >= 0 && fmt < 5 && ((std::atoi(x) >> fmt) & 1);
#endif
    return fmt >= 0 && fmt < 5 && ((RFA_W64_FORMATS >> fmt) & 1);
}

// Twiddle blob (exact, correctly rounded from double): T1[a][t] = W_1024^{a t} (t < 33),
// TB[k0][t-1] = W_32768^{t k0} (a, k0 < 32, t = 1..31), then W_65536^c (c < 1024).
std::vector<float2> w64_twiddles() {
    auto w = [](double num, double den) {
        const double ang = -2.0 * M_PI * num / den;
        return make_float2((float)std::cos(ang), (float)std::sin(ang));
    };
    std::vector<float2> blob;
    for (int i = 0; i < 32; i++)
        for (int t = 0; t < kRow1; t++) blob.push_back(w((double)i * t, 1024.0));
    for (int i = 0; i < 32; i++)
        for (int t = 1; t < 32; t++) blob.push_back(w((double)t * i, (double)kM));
    for (int c = 0; c < 1024; c++) blob.push_back(w((double)c, (double)kN));
    return blob;
}

hipError_t launch_fft64(const FftLaunch &a) {
#if RFA_W64_FORMATS == 0 && !defined(RFA_AB_BUILD)
    (void)a;
    return hipErrorInvalidValue;  // not compiled into product builds (w64_format() is false)
#else
    if (a.logn != 16 || a.complex_out || !a.w64_tw || !a.window_il) return hipErrorInvalidValue;
    if (a.fmt <= 2 && !a.window_cw) return hipErrorInvalidValue;
    if (a.ring && (a.ring_logrs != (1 | kRingTile2) || a.ring_rows <= 0)) return hipErrorInvalidValue;
#ifdef RFA_AB_BUILD
    if (const char *x = std::getenv("RFA_W64_PRIO")) const_cast<FftLaunch &>(a).prio = std::atoi(x);
    if (const char *x = std::getenv("RFA_W64_PREW"); x && std::atoi(x) == 1) const_cast<FftLaunch &>(a).prio |= 16;
    if (const char *x = std::getenv("RFA_W64_X0R")) {
        if (std::atoi(x) == 2) return launch64_x<2>(a);
        if (std::atoi(x) == 3) return launch64_x<3>(a);
    }
#endif
    return launch64_x<RFA_W64_X0R>(a);
#endif
}

}  // namespace rfa
