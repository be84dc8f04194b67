// The W8 form of the in-register DFT-16 / DFT-32 (fft_common.h dft<16>, dft<32>) for the wide
// kernel's own 8/16-bit frames (fft_wide.hip): the sqrt(1/2) of every W_8-type twiddle
// x * W_16^q (q = 2 mod 4) is applied by the add that consumes it -- one v_pk_fma_f32 instead of
// a v_pk_mul_f32 and a v_pk_add_f32, rounded once.  -1.5 .. -2 % kernel time at 64 K s8, -0.6 %
// at 8 K (profiles/r04/w8_alias_ab.txt, vadd_ab.txt).  Kept out of fft_common.h so the plain
// DFTs of every other kernel compile exactly as before (the large-N front kernel's two
// alignment paths are bit-identical by construction; a perturbed plain DFT changed hipcc's
// contraction choices in one of them), and not used for cf32 / the large-N scratch, whose
// parity cases sit near the 0.01 dB bar (a 0.0108 / 0.0132 dB bin with this rounding).
#pragma once

#include "fft_common.h"

namespace rfa {

// c + sqrt(1/2) * a * (-i)^Q: a W_8-type factor x * W_16^q (q = 2 mod 4) is sqrt(1/2) * p with
// p = padd<(q-2)/4, (q+2)/4>(x, x); the sqrt(1/2) is applied by the add that consumes it (one
// v_pk_fma_f32 instead of a v_pk_mul_f32 plus a v_pk_add_f32; rounded once instead of twice).
template <int Q_>
RFA_HD float2 pfma_r2(float2 a_, float2 c_) {
    constexpr int Q = Q_ & 3;
#if defined(__HIP_DEVICE_COMPILE__)
    const f2v a = to_v(a_), c = to_v(c_), k = (f2v){kR2, kR2};
    f2v r;
    if constexpr (Q == 0) asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    else if constexpr (Q == 1) asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    else if constexpr (Q == 2) asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    else asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return from_v(r);
#else
    const float2 b = rot<Q>(a_);
    return make_float2(fmaf(b.x, kR2, c_.x), fmaf(b.y, kR2, c_.y));
#endif
}
// the unscaled part p of x * W_16^q, q = 2 mod 4 (x * W_16^q = sqrt(1/2) p)
template <int q_>
RFA_HD float2 w16_p(float2 x) {
    constexpr int q = q_ & 15;
    static_assert((q & 3) == 2, "W_8-type factor");
    return padd<(q - 2) / 4, (q + 2) / 4>(x, x);
}

// dft4r whose x2 (S2) or whose x1 and x3 (S13) arrive as the unscaled parts p of W_8-type
// products (w16_p): the sqrt(1/2) is folded into the adds (pfma_r2)
template <int P1, int P2, int P3, bool S2, bool S13>
RFA_HD void dft4s(float2 &x0, float2 &x1, float2 &x2, float2 &x3) {
    float2 s02, d02;
    if constexpr (S2) {
        s02 = pfma_r2<P2>(x2, x0);
        d02 = pfma_r2<P2 + 2>(x2, x0);
    } else {
        s02 = padd<0, P2>(x0, x2);
        d02 = padd<0, P2 + 2>(x0, x2);
    }
    const float2 s13 = padd<P1, P3>(x1, x3), d13 = padd<P1, P3 + 2>(x1, x3);
    if constexpr (S13) {
        x0 = pfma_r2<0>(s13, s02);
        x2 = pfma_r2<2>(s13, s02);
        x1 = pfma_r2<1>(d13, d02);
        x3 = pfma_r2<3>(d13, d02);
    } else {
        x0 = cadd(s02, s13);
        x2 = csub(s02, s13);
        x1 = padd<0, 1>(d02, d13);
        x3 = padd<0, 3>(d02, d13);
    }
}

// dft16r (fft_common.h) in the W8 form; S0: u[4] and u[12] arrive as the unscaled parts of
// W_8-type products
template <int ROT8, bool S0 = false>
RFA_HD void dft16w(float2 *u) {
    // t = 4*t1 + t2; DFT-4 over t1, twiddle W_16^{t2 q1}, DFT-4 over t2.
    dft4s<0, ROT8, 0, false, S0>(u[0], u[4], u[8], u[12]);
    dft4(u[1], u[5], u[9], u[13]);
    dft4(u[2], u[6], u[10], u[14]);
    dft4(u[3], u[7], u[11], u[15]);
    u[5] = w16<1>(u[5]);
    u[6] = w16_p<2>(u[6]);
    u[7] = w16<3>(u[7]);
    u[9] = w16_p<2>(u[9]);
    u[11] = w16_p<6>(u[11]);
    u[13] = w16<3>(u[13]);
    u[14] = w16_p<6>(u[14]);
    u[15] = w16<9>(u[15]);
    dft4(u[0], u[1], u[2], u[3]);
    dft4s<0, 0, 0, true, false>(u[4], u[5], u[6], u[7]);
    dft4s<0, 1, 0, false, true>(u[8], u[9], u[10], u[11]);  // u[10] * W_16^4 = -i u[10], folded
    dft4s<0, 0, 0, true, false>(u[12], u[13], u[14], u[15]);
    // position 4*q1 + q2 holds Y[q1 + 4 q2]
    float2 y[16];
#pragma unroll
    for (int q = 0; q < 16; q++) y[q] = u[4 * (q & 3) + (q >> 2)];
#pragma unroll
    for (int q = 0; q < 16; q++) u[q] = y[q];
}

// dft<32> (fft_common.h) in the W8 form
RFA_HD void dft32w(float2 *u) {
    // t = 16*t1 + t2 (t1 < 2): DFT-2 over t1, twiddle W_32^{t2 q1} = W_64^{2 t2 q1}, DFT-16 over t2.
#pragma unroll
    for (int t2 = 0; t2 < 16; t2++) dft2(u[t2], u[16 + t2]);
    // W_64^8, W_64^24: sqrt(1/2) folded into dft16w's first adds (S0)
    u[17] = w64<2>(u[17]); u[18] = w64<4>(u[18]); u[19] = w64<6>(u[19]); u[20] = w16_p<2>(u[20]);
    u[21] = w64<10>(u[21]); u[22] = w64<12>(u[22]); u[23] = w64<14>(u[23]);
    u[25] = w64<18>(u[25]); u[26] = w64<20>(u[26]); u[27] = w64<22>(u[27]); u[28] = w16_p<6>(u[28]);
    u[29] = w64<26>(u[29]); u[30] = w64<28>(u[30]); u[31] = w64<30>(u[31]);
    dft16w<0>(u);
    dft16w<1, true>(u + 16);  // u[24] * W_64^16 = -i u[24], folded
    // position 16*q1 + q2 holds Y[q1 + 2 q2]
    float2 y[32];
#pragma unroll
    for (int q = 0; q < 32; q++) y[q] = u[16 * (q & 1) + (q >> 1)];
#pragma unroll
    for (int q = 0; q < 32; q++) u[q] = y[q];
}

// dft<R>, or its W8 form for R = 16 / 32
template <int R, bool W8>
RFA_HD void dftw(float2 *u) {
    if constexpr (W8 && R == 16) dft16w<0>(u);
    else if constexpr (W8 && R == 32) dft32w(u);
    else dft<R>(u);
}

}  // namespace rfa
