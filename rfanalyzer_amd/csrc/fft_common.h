// Shared device helpers of the gfx950 spectrum kernels: complex arithmetic,
// in-register DFTs, twiddle lookup, raw IQ conversion, LDS-only barrier.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <utility>

// Pure-math helpers are host+device so tests/csrc can check them on the CPU.
#define RFA_HD __host__ __device__ __forceinline__

namespace rfa {


// ----------------------------------------------------------------- complex helpers
RFA_HD float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
RFA_HD float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
RFA_HD float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // * (-i)
RFA_HD float2 mul_pi(float2 a) { return make_float2(-a.y, a.x); }  // * (+i)

// ---- packed-fp32 complex arithmetic (gfx950 VOP3P).  A complex value is one
// 64-bit VGPR pair; v_pk_add/mul/fma_f32 operate on both halves at once and
// every source can be half-swapped (op_sel) and negated per half (neg_lo /
// neg_hi) for free.  So a*(-i)^P + b*(-i)^Q is ONE instruction for any
// quarter-turn rotations P, Q, and a complex multiply is two.  hipcc's own
// packing of the float2 code needs extra v_mov for the swaps (checked on
// hardware by scripts/pk_modifiers.hip).
typedef float f2v __attribute__((ext_vector_type(2)));
RFA_HD f2v to_v(float2 a) { return __builtin_bit_cast(f2v, a); }
RFA_HD float2 from_v(f2v a) { return __builtin_bit_cast(float2, a); }

template <int P>
RFA_HD float2 rot(float2 a) {  // a * (-i)^P
    constexpr int q = P & 3;
    if constexpr (q == 0) return a;
    else if constexpr (q == 1) return mul_mi(a);
    else if constexpr (q == 2) return make_float2(-a.x, -a.y);
    else return mul_pi(a);
}

// a * (-i)^P + b * (-i)^Q
template <int P_, int Q_>
RFA_HD float2 padd(float2 a_, float2 b_) {
    constexpr int P = P_ & 3, Q = Q_ & 3;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (P == 0 && (Q == 0 || Q == 2)) {
        return Q == 0 ? cadd(a_, b_) : csub(a_, b_);  // hipcc folds these itself
    } else {
        const f2v a = to_v(a_), b = to_v(b_);
        f2v r;
    if constexpr (P == 0 && Q == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 0 && Q == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 0 && Q == 2) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 0 && Q == 3) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 1 && Q == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 1 && Q == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 1 && Q == 2) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 1 && Q == 3) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 2 && Q == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 2 && Q == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[1,0] neg_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 2 && Q == 2) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,1] neg_lo:[1,1] neg_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 2 && Q == 3) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[1,1] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 3 && Q == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 3 && Q == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 3 && Q == 2) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else if constexpr (P == 3 && Q == 3) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[1,1]" : "=v"(r) : "v"(a), "v"(b));
        return from_v(r);
    }
#else
    return cadd(rot<P>(a_), rot<Q>(b_));
#endif
}

// complex a * w (w in a VGPR pair or an SGPR pair)
RFA_HD float2 cmul(float2 a_, float2 w_) {
#if defined(__HIP_DEVICE_COMPILE__)
    const f2v a = to_v(a_), w = to_v(w_);
    f2v m, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(m) : "v"(a), "v"(w));  // (a.x w.x, a.x w.y)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a), "v"(w), "v"(m));  // (a.y (-w.y) + m.x, a.y w.x + m.y)
    return from_v(r);
#else
    return make_float2(fmaf(a_.x, w_.x, -a_.y * w_.y), fmaf(a_.x, w_.y, a_.y * w_.x));
#endif
}
// two independent complex multiplies a0*w0, a1*w1 interleaved in one block, so
// no multiply is immediately followed by its dependent fma (gfx950 inserts an
// s_nop between a packed write and a dependent packed read)
RFA_HD void cmul2(float2 &a0_, float2 w0_, float2 &a1_, float2 w1_) {
#if defined(__HIP_DEVICE_COMPILE__)
    f2v a0 = to_v(a0_), a1 = to_v(a1_);
    const f2v w0 = to_v(w0_), w1 = to_v(w1_);
    f2v m0, m1;  // early-clobber: written before the other pair's operands are read
    asm("v_pk_mul_f32 %0, %2, %4 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %1, %3, %5 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %2, %2, %4, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %3, %3, %5, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(m0), "=&v"(m1), "+v"(a0), "+v"(a1)
        : "v"(w0), "v"(w1));
    a0_ = from_v(a0);
    a1_ = from_v(a1);
#else
    a0_ = cmul(a0_, w0_);
    a1_ = cmul(a1_, w1_);
#endif
}

// a0 * w0 + a1 * w1 (complex), four packed instructions: the residue-1 pre-stage of
// the 64 K kernel with the twiddle folded into a complex window (fft_wide.hip)
RFA_HD float2 cmac2(float2 a0_, float2 w0_, float2 a1_, float2 w1_) {
#if defined(__HIP_DEVICE_COMPILE__)
    const f2v a0 = to_v(a0_), w0 = to_v(w0_), a1 = to_v(a1_), w1 = to_v(w1_);
    f2v m, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(m) : "v"(a0), "v"(w0));  // (a0.x w0.x, a0.x w0.y)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a0), "v"(w0), "v"(m));  // + (a0.y (-w0.y), a0.y w0.x)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(m) : "v"(a1), "v"(w1), "v"(r));  // + a1.x w1
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a1), "v"(w1), "v"(m));  // + (a1.y (-w1.y), a1.y w1.x)
    return from_v(r);
#else
    return make_float2(a0_.x * w0_.x - a0_.y * w0_.y + a1_.x * w1_.x - a1_.y * w1_.y,
                       a0_.x * w0_.y + a0_.y * w0_.x + a1_.x * w1_.y + a1_.y * w1_.x);
#endif
}

// two independent cmac2 in one block, their chains interleaved (as cmul2): every
// instruction's source was written two instructions earlier, so hipcc has no
// dependent inline-asm pair to pad with s_nop (it padded each link of the single
// cmac2 chain: 3 per point, 96 per residue-1 item)
RFA_HD void cmac2x2(float2 &out0, float2 a0_, float2 w0_, float2 a1_, float2 w1_, float2 &out1, float2 b0_, float2 v0_,
                    float2 b1_, float2 v1_) {
#if defined(__HIP_DEVICE_COMPILE__)
    const f2v a0 = to_v(a0_), w0 = to_v(w0_), a1 = to_v(a1_), w1 = to_v(w1_);
    const f2v b0 = to_v(b0_), v0 = to_v(v0_), b1 = to_v(b1_), v1 = to_v(v1_);
    f2v m, n, r, s;
    asm("v_pk_mul_f32 %0, %4, %5 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %1, %8, %9 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %2, %4, %5, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %3, %8, %9, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %0, %6, %7, %2 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %1, %10, %11, %3 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %2, %6, %7, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %3, %10, %11, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(m), "=&v"(n), "=&v"(r), "=&v"(s)
        : "v"(a0), "v"(w0), "v"(a1), "v"(w1), "v"(b0), "v"(v0), "v"(b1), "v"(v1));
    out0 = from_v(r);
    out1 = from_v(s);
#else
    out0 = cmac2(a0_, w0_, a1_, w1_);
    out1 = cmac2(b0_, v0_, b1_, v1_);
#endif
}

// Large-N front-kernel twiddle for two outputs: v_k *= C_k + C_k * D_k, with the
// wave-uniform C_k in SGPR pairs (scalar loads) and D_k per lane; the two chains are
// interleaved so no packed result is read by the next instruction (as cmul2), and a
// VOP3P instruction reads one SGPR pair at most (constant-bus limit).
RFA_HD void twiddle_cd2(float2 &v0_, float2 d0_, float2 c0_, float2 &v1_, float2 d1_, float2 c1_) {
#if defined(__HIP_DEVICE_COMPILE__)
    f2v v0 = to_v(v0_), v1 = to_v(v1_);
    const f2v d0 = to_v(d0_), d1 = to_v(d1_), c0 = to_v(c0_), c1 = to_v(c1_);
    f2v m0, m1, r0, r1;
    asm("v_pk_mul_f32 %0, %8, %6 op_sel_hi:[0,1]\n\t"  // C * D as cmul(C, D): same products and rounding
        "v_pk_mul_f32 %1, %9, %7 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %2, %8, %6, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %3, %9, %7, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_add_f32 %2, %2, %8\n\t"
        "v_pk_add_f32 %3, %3, %9\n\t"
        "v_pk_mul_f32 %0, %4, %2 op_sel_hi:[0,1]\n\t"
        "v_pk_mul_f32 %1, %5, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %4, %4, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
        "v_pk_fma_f32 %5, %5, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(m0), "=&v"(m1), "=&v"(r0), "=&v"(r1), "+v"(v0), "+v"(v1)
        : "v"(d0), "v"(d1), "s"(c0), "s"(c1));
    v0_ = from_v(v0);
    v1_ = from_v(v1);
#else
    const float2 k0 = cmul(c0_, d0_), k1 = cmul(c1_, d1_);
    const float2 w0 = make_float2(c0_.x + k0.x, c0_.y + k0.y), w1 = make_float2(c1_.x + k1.x, c1_.y + k1.y);
    v0_ = cmul(v0_, w0);
    v1_ = cmul(v1_, w1);
#endif
}

// complex a * (c, s) for a compile-time constant (held in an SGPR pair)
// (plain vector code: both constant pairs live in SGPRs, hipcc emits v_pk_mul +
// v_pk_fma and is free to interleave independent multiplies)
RFA_HD float2 cmulc(float2 a_, float c, float s) {
#if defined(__HIP_DEVICE_COMPILE__)
    const f2v a = to_v(a_);
    const f2v m = (f2v){a.x, a.x} * (f2v){c, s};
    return from_v(__builtin_elementwise_fma((f2v){a.y, a.y}, (f2v){-s, c}, m));
#else
    return make_float2(fmaf(a_.x, c, -a_.y * s), fmaf(a_.x, s, a_.y * c));
#endif
}

// exp(-2*pi*i*m/16), correctly rounded fp32 constants.
constexpr float kC1 = 0.923879532511286756f;  // cos(pi/8)
constexpr float kS1 = 0.382683432365089772f;  // sin(pi/8)
constexpr float kR2 = 0.707106781186547524f;  // sqrt(1/2)

// x * W_16^m (m in 0..15), constant-folded per call site.
template <int m>
RFA_HD float2 w16(float2 x) {
    constexpr int q = m & 15;
    if constexpr ((q & 3) == 0) {
        return rot<q / 4>(x);
    } else if constexpr ((q & 3) == 2) {
        // W_16^q = (-i)^((q-2)/4) * (1 - i)/sqrt(2):  x*(-i)^k + x*(-i)^(k+1), times sqrt(1/2)
        return from_v(to_v(padd<(q - 2) / 4, (q + 2) / 4>(x, x)) * kR2);
    } else {
        constexpr float c[16] = {1, kC1, kR2, kS1, 0, -kS1, -kR2, -kC1, -1, -kC1, -kR2, -kS1, 0, kS1, kR2, kC1};
        constexpr float s[16] = {0, kS1, kR2, kC1, 1, kC1, kR2, kS1, 0, -kS1, -kR2, -kC1, -1, -kC1, -kR2, -kS1};
        return cmulc(x, c[q], -s[q]);
    }
}

// In-register forward DFTs, natural order in and out.
RFA_HD void dft2(float2 &a, float2 &b) {
    float2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}
// radix 2 with b pre-rotated by (-i)^P (folded into the adds)
template <int P>
RFA_HD void dft2r(float2 &a, float2 &b) {
    const float2 t = a;
    a = padd<0, P>(t, b);
    b = padd<0, P + 2>(t, b);
}
// radix 4 with inputs x1, x2, x3 pre-rotated by (-i)^P1, (-i)^P2, (-i)^P3:
// eight v_pk_add_f32 whatever the rotations.
template <int P1, int P2, int P3>
RFA_HD void dft4r(float2 &x0, float2 &x1, float2 &x2, float2 &x3) {
    const float2 s02 = padd<0, P2>(x0, x2), d02 = padd<0, P2 + 2>(x0, x2);
    const float2 s13 = padd<P1, P3>(x1, x3), d13 = padd<P1, P3 + 2>(x1, x3);
    x0 = cadd(s02, s13);
    x2 = csub(s02, s13);
    x1 = padd<0, 1>(d02, d13);  // d02 - i d13
    x3 = padd<0, 3>(d02, d13);  // d02 + i d13
}
RFA_HD void dft4(float2 &x0, float2 &x1, float2 &x2, float2 &x3) { dft4r<0, 0, 0>(x0, x1, x2, x3); }

template <int R>
RFA_HD void dft(float2 *u);

template <>
RFA_HD void dft<2>(float2 *u) { dft2(u[0], u[1]); }
template <>
RFA_HD void dft<4>(float2 *u) { dft4(u[0], u[1], u[2], u[3]); }
template <>
RFA_HD void dft<8>(float2 *u) {
    // t = 2*t1 + t2; DFT-4 over t1, twiddle W_8^{t2 q1} (= W_16^{2 t2 q1}), DFT-2 over t2.
    dft4(u[0], u[2], u[4], u[6]);
    dft4(u[1], u[3], u[5], u[7]);
    u[3] = w16<2>(u[3]);
    u[7] = w16<6>(u[7]);
    dft2(u[0], u[1]);
    dft2(u[2], u[3]);
    dft2r<1>(u[4], u[5]);  // u[5] * W_16^4 = -i u[5], folded
    dft2(u[6], u[7]);
    // position 2*q1 + q2 holds Y[q1 + 4 q2]
    float2 y[8];
#pragma unroll
    for (int q = 0; q < 8; q++) y[q] = u[2 * (q & 3) + (q >> 2)];
#pragma unroll
    for (int q = 0; q < 8; q++) u[q] = y[q];
}
// ROT8: input u[8] arrives pre-rotated by (-i)^ROT8 (folded into the first adds)
template <int ROT8>
RFA_HD void dft16r(float2 *u) {
    // t = 4*t1 + t2; DFT-4 over t1, twiddle W_16^{t2 q1}, DFT-4 over t2.
    dft4r<0, ROT8, 0>(u[0], u[4], u[8], u[12]);
    dft4(u[1], u[5], u[9], u[13]);
    dft4(u[2], u[6], u[10], u[14]);
    dft4(u[3], u[7], u[11], u[15]);
    u[5] = w16<1>(u[5]);
    u[6] = w16<2>(u[6]);
    u[7] = w16<3>(u[7]);
    u[9] = w16<2>(u[9]);
    u[11] = w16<6>(u[11]);
    u[13] = w16<3>(u[13]);
    u[14] = w16<6>(u[14]);
    u[15] = w16<9>(u[15]);
    dft4(u[0], u[1], u[2], u[3]);
    dft4(u[4], u[5], u[6], u[7]);
    dft4r<0, 1, 0>(u[8], u[9], u[10], u[11]);  // u[10] * W_16^4 = -i u[10], folded
    dft4(u[12], u[13], u[14], u[15]);
    // position 4*q1 + q2 holds Y[q1 + 4 q2]
    float2 y[16];
#pragma unroll
    for (int q = 0; q < 16; q++) y[q] = u[4 * (q & 3) + (q >> 2)];
#pragma unroll
    for (int q = 0; q < 16; q++) u[q] = y[q];
}
template <>
RFA_HD void dft<16>(float2 *u) { dft16r<0>(u); }

// cos/sin(2*pi*m/64), correctly rounded fp32 (generated)
constexpr float kCos64[64] = {1.0f, 0.99518472f, 0.980785251f, 0.956940353f, 0.923879504f, 0.881921291f, 0.831469595f, 0.773010433f, 0.707106769f, 0.634393275f, 0.555570245f, 0.471396744f, 0.382683426f, 0.290284663f, 0.195090324f, 0.0980171412f, 0.0f, -0.0980171412f, -0.195090324f, -0.290284663f, -0.382683426f, -0.471396744f, -0.555570245f, -0.634393275f, -0.707106769f, -0.773010433f, -0.831469595f, -0.881921291f, -0.923879504f, -0.956940353f, -0.980785251f, -0.99518472f, -1.0f, -0.99518472f, -0.980785251f, -0.956940353f, -0.923879504f, -0.881921291f, -0.831469595f, -0.773010433f, -0.707106769f, -0.634393275f, -0.555570245f, -0.471396744f, -0.382683426f, -0.290284663f, -0.195090324f, -0.0980171412f, 0.0f, 0.0980171412f, 0.195090324f, 0.290284663f, 0.382683426f, 0.471396744f, 0.555570245f, 0.634393275f, 0.707106769f, 0.773010433f, 0.831469595f, 0.881921291f, 0.923879504f, 0.956940353f, 0.980785251f, 0.99518472f};
constexpr float kSin64[64] = {0.0f, 0.0980171412f, 0.195090324f, 0.290284663f, 0.382683426f, 0.471396744f, 0.555570245f, 0.634393275f, 0.707106769f, 0.773010433f, 0.831469595f, 0.881921291f, 0.923879504f, 0.956940353f, 0.980785251f, 0.99518472f, 1.0f, 0.99518472f, 0.980785251f, 0.956940353f, 0.923879504f, 0.881921291f, 0.831469595f, 0.773010433f, 0.707106769f, 0.634393275f, 0.555570245f, 0.471396744f, 0.382683426f, 0.290284663f, 0.195090324f, 0.0980171412f, 0.0f, -0.0980171412f, -0.195090324f, -0.290284663f, -0.382683426f, -0.471396744f, -0.555570245f, -0.634393275f, -0.707106769f, -0.773010433f, -0.831469595f, -0.881921291f, -0.923879504f, -0.956940353f, -0.980785251f, -0.99518472f, -1.0f, -0.99518472f, -0.980785251f, -0.956940353f, -0.923879504f, -0.881921291f, -0.831469595f, -0.773010433f, -0.707106769f, -0.634393275f, -0.555570245f, -0.471396744f, -0.382683426f, -0.290284663f, -0.195090324f, -0.0980171412f};

// x * W_64^m (m constant), W = exp(-2*pi*i/64); multiples of 4 use the W_16 forms.
template <int m>
RFA_HD float2 w64(float2 x) {
    constexpr int q = m & 63;
    if constexpr ((q & 3) == 0) return w16<q / 4>(x);
    else return cmulc(x, kCos64[q], -kSin64[q]);
}

template <>
RFA_HD void dft<32>(float2 *u) {
    // t = 16*t1 + t2 (t1 < 2): DFT-2 over t1, twiddle W_32^{t2 q1} = W_64^{2 t2 q1}, DFT-16 over t2.
#pragma unroll
    for (int t2 = 0; t2 < 16; t2++) dft2(u[t2], u[16 + t2]);
    u[17] = w64<2>(u[17]); u[18] = w64<4>(u[18]); u[19] = w64<6>(u[19]); u[20] = w64<8>(u[20]);
    u[21] = w64<10>(u[21]); u[22] = w64<12>(u[22]); u[23] = w64<14>(u[23]);
    u[25] = w64<18>(u[25]); u[26] = w64<20>(u[26]); u[27] = w64<22>(u[27]); u[28] = w64<24>(u[28]);
    u[29] = w64<26>(u[29]); u[30] = w64<28>(u[30]); u[31] = w64<30>(u[31]);
    dft<16>(u);
    dft16r<1>(u + 16);  // u[24] * W_64^16 = -i u[24], folded
    // position 16*q1 + q2 holds Y[q1 + 2 q2]
    float2 y[32];
#pragma unroll
    for (int q = 0; q < 32; q++) y[q] = u[16 * (q & 1) + (q >> 1)];
#pragma unroll
    for (int q = 0; q < 32; q++) u[q] = y[q];
}

template <int T2, int Q1>
RFA_HD void tw64_step(float2 *u) {
    u[16 * Q1 + T2] = w64<T2 * Q1>(u[16 * Q1 + T2]);
}
template <int T2>
RFA_HD void tw64_col(float2 *u) {
    tw64_step<T2, 1>(u);
    tw64_step<T2, 2>(u);
    tw64_step<T2, 3>(u);
}
template <int... T2s>
RFA_HD void tw64_all(float2 *u, std::integer_sequence<int, T2s...>) {
    (tw64_col<T2s>(u), ...);
}

template <>
RFA_HD void dft<64>(float2 *u) {
    // t = 16*t1 + t2 (t1 < 4): DFT-4 over t1, twiddle W_64^{t2 q1}, DFT-16 over t2.
#pragma unroll
    for (int t2 = 0; t2 < 16; t2++) dft4(u[t2], u[16 + t2], u[32 + t2], u[48 + t2]);
    tw64_all(u, std::make_integer_sequence<int, 16>{});
    dft<16>(u);
    dft<16>(u + 16);
    dft<16>(u + 32);
    dft<16>(u + 48);
    // position 16*q1 + q2 holds Y[q1 + 4 q2]
    float2 y[64];
#pragma unroll
    for (int q = 0; q < 64; q++) y[q] = u[16 * (q & 3) + (q >> 2)];
#pragma unroll
    for (int q = 0; q < 64; q++) u[q] = y[q];
}

// Twiddle W_N^s from the two-level LDS table.
__device__ __forceinline__ float2 tw(const float2 *twc, const float2 *twf, int s, int shift) {
    return cmul(twc[s >> shift], twf[s & ((1 << shift) - 1)]);
}

// Workgroup-wide barrier for LDS hand-offs only: waits for this wave's LDS
// operations (lgkmcnt) but NOT for its global loads (vmcnt), so the next
// frame's prefetched samples stay in flight across the FFT passes.
// (__syncthreads() would emit vmcnt(0) and drain them.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

// one float2 as its own ds_read_b64: a volatile LDS access keeps hipcc from fusing
// neighbours into ds_read2_b64, which moves half the bytes per LDS cycle on gfx950
// (MI355X_MICROARCH.md, LDS table: 8 cycles per ds_read2_b64 vs 2 per ds_read_b64)
__device__ __forceinline__ float2 lds_ld2(const float2 *p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return from_v(*(const volatile __attribute__((address_space(3))) f2v *)(p));
#else
    return *p;
#endif
}
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float2 lds_ld2(const __attribute__((address_space(3))) float2 *p) {
    return from_v(*(const volatile __attribute__((address_space(3))) f2v *)(p));
}
#endif
// one float2 as its own ds_write_b64 (volatile: not fused into ds_write2_b64, whose two 8-bit
// offsets force a v_add_u32 per store wherever the store's offset exceeds 2 KB)
__device__ __forceinline__ void lds_st2(float2 *p, float2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *(volatile __attribute__((address_space(3))) f2v *)(p) = to_v(v);
#else
    *p = v;
#endif
}


// ----------------------------------------------------------------- input conversion
// Raw sample words as loaded (converted later, so a prefetch holds 1 VGPR per
// sample for 8/16-bit formats).
template <int FMT>
struct Raw {
    using T = float2;
};
template <>
struct Raw<0> { using T = unsigned short; };
template <>
struct Raw<1> { using T = unsigned short; };
template <>
struct Raw<2> { using T = unsigned; };

template <int FMT>
__device__ __forceinline__ typename Raw<FMT>::T load_raw(const uint8_t *fb, int s, int n) {
    if constexpr (FMT == 0 || FMT == 1) return *reinterpret_cast<const unsigned short *>(fb + 2 * (size_t)s);
    else if constexpr (FMT == 2) return *reinterpret_cast<const unsigned *>(fb + 4 * (size_t)s);
    else if constexpr (FMT == 3) return *reinterpret_cast<const float2 *>(fb + 8 * (size_t)s);
    else {
        const float *f = reinterpret_cast<const float *>(fb);
        return make_float2(f[s], f[(size_t)n + s]);
    }
}

// Raw word -> unscaled float pair; the converter scale (1/128, 1/32768) is
// folded into the window table by the engine.  Bit-exact with the reference
// LUTs: s8 b/128 (Signed8BitIQConverter.java:48-50), u8 (b-127.4f)/128
// (Unsigned8BitIQConverter.java:48-50), s16 s/32768 (Signed16BitIQConverter.kt:52-55);
// scaling by a power of two commutes with the fp32 rounding of the window multiply.
// Signed byte / word field of a dword -> float in ONE instruction: SDWA operand
// select with sign extension (hipcc emits a bfe/ashr + convert pair per value).
template <int SEL>  // 0, 1: BYTE_0 / BYTE_1; 4, 5: WORD_0 / WORD_1
__device__ __forceinline__ float cvt_sext(unsigned v) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    if constexpr (SEL == 0)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(r) : "v"(v));
    else if constexpr (SEL == 1)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(r) : "v"(v));
    else if constexpr (SEL == 4)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(r) : "v"(v));
    else
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(r) : "v"(v));
    return r;
#else
    if constexpr (SEL == 0) return (float)(signed char)(v & 0xff);
    else if constexpr (SEL == 1) return (float)(signed char)((v >> 8) & 0xff);
    else if constexpr (SEL == 4) return (float)(short)(v & 0xffff);
    else return (float)(short)(v >> 16);
#endif
}

template <int FMT>
__device__ __forceinline__ float2 convert_raw(typename Raw<FMT>::T v) {
    if constexpr (FMT == 0) return make_float2(cvt_sext<0>(v), cvt_sext<1>(v));
    else if constexpr (FMT == 1) return make_float2((float)(v & 0xff) - 127.4f, (float)(v >> 8) - 127.4f);
    else if constexpr (FMT == 2) return make_float2(cvt_sext<4>(v), cvt_sext<5>(v));
    else return v;
}

template <int FMT>
__device__ __forceinline__ typename Raw<FMT>::T synth_raw(int s) {  // ablation input
    if constexpr (FMT == 0 || FMT == 1) return (unsigned short)(s * 2654435761u >> 16);
    else if constexpr (FMT == 2) return (unsigned)(s * 2654435761u);
    else return make_float2((float)(s & 255) * 0.01f, (float)((s >> 3) & 255) * 0.01f);
}

static __constant__ float2 kW8[8] = {{1.f, 0.f},          {kR2, -kR2}, {0.f, -1.f}, {-kR2, -kR2},
                               {-1.f, 0.f},         {-kR2, kR2}, {0.f, 1.f},  {kR2, kR2}};


// ----------------------------------------------------------------- buffer access
// Raw buffer loads/stores: one 32-bit VGPR offset per lane plus a wave-uniform
// SGPR offset, so the 64+ memory operations of a thread need no 64-bit address
// registers.  Out-of-range accesses (num_records) read 0 / are dropped.
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void *p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float2 buf_load_f32x2(rsrc_t rs, int voff, int soff);

// One raw sample at byte offset voff + soff of the frame (formats as Raw<FMT>).
template <int FMT>
__device__ __forceinline__ typename Raw<FMT>::T buf_load_raw(rsrc_t rs, int voff, int soff, int planar_im_off) {
    if constexpr (FMT == 0 || FMT == 1) return (unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0);
    else if constexpr (FMT == 2) return (unsigned)__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
    else if constexpr (FMT == 3 || FMT == 5) {  // f32 interleaved; 5: the large-N scratch
        return buf_load_f32x2(rs, voff, soff);
    } else {
        const float re = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
        const float im = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff + planar_im_off, 0));
        return make_float2(re, im);
    }
}
__device__ __forceinline__ float buf_load_f32(rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
}
// NOTE: index the b64 result only after bit-casting it to a float vector --
// element access on the builtin's own return type loads a single dword
// (hipcc, ROCm 7.2).
typedef float rfa_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 buf_load_f32x2(rsrc_t rs, int voff, int soff) {
    const rfa_f32x2 v = __builtin_bit_cast(rfa_f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
    return make_float2(v.x, v.y);
}
__device__ __forceinline__ void buf_store_f32(float x, rsrc_t rs, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, x), rs, voff, soff, 0);
}
// dword store at a compile-time byte offset SO: the SGPR offset is set by an s_mov_b32
// next to the store (SALU: no VALU-write-SGPR hazard before the VMEM read), so hipcc
// cannot hoist a kernel's worth of distinct offsets out of a loop and spill them
template <int SO>
__device__ __forceinline__ void buf_store_f32_c(float x, rsrc_t rs, int voff) {
#if defined(__HIP_DEVICE_COMPILE__)
    int so;
    asm volatile("s_mov_b32 %0, %3\n\tbuffer_store_dword %1, %2, %4, %0 offen"
                 : "=&s"(so)
                 : "v"(x), "v"(voff), "i"(SO), "s"(rs)
                 : "memory");
#else
    (void)x; (void)rs; (void)voff;
#endif
}
// 16-B store.  Inline asm with a trailing s_nop: a VALU write to the data VGPRs of a
// just-issued buffer store of more than 64 bits needs a wait state, and hipcc (ROCm
// 7.2, gfx950) let the next v_pk_fma overwrite them back to back -- the last lanes of
// each 16-lane group then stored the new values (measured: ~1/16 of the 64 K ring's
// bins wrong).  The asm block keeps the store and its nop together.
__device__ __forceinline__ void buf_store_f32x4(float a, float b, float c, float d, rsrc_t rs, int voff, int soff) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    i32x4 v = {__builtin_bit_cast(int, a), __builtin_bit_cast(int, b), __builtin_bit_cast(int, c),
               __builtin_bit_cast(int, d)};
#if defined(__HIP_DEVICE_COMPILE__)
    // sc1: write-through, the line leaves the XCD's L2 (MI355X_MICROARCH.md, store flavours), so
    // the ring's 128 KB per 32 K item no longer evicts the window tables and the staged frames:
    // FETCH 91.0 -> 81.7 MB per 64 K launch, 64 K cf32 -2.4 %, 128 K -3 .. -6 %, 64 K s8 +-0
    // (profiles/r04/ring_store_sc1_ab.txt)
    asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen sc1\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs),
                 "s"(soff)
                 : "memory");
#else
    (void)v; (void)rs; (void)voff; (void)soff;
#endif
}
// the same 16-B store without sc1 (write-back in the XCD's L2)
__device__ __forceinline__ void buf_store_f32x4_wb(float a, float b, float c, float d, rsrc_t rs, int voff, int soff) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) int, (f32x4){a, b, c, d}),
                                           rs, voff, soff, 0);
}
__device__ __forceinline__ void buf_store_f32x2(float2 x, rsrc_t rs, int voff, int soff) {
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    i32x2 v = {__builtin_bit_cast(int, x.x), __builtin_bit_cast(int, x.y)};
    __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, soff, 0);
}

// One frame of a chunk's peak / EMA summary (the chunked scan of fft_kernels.hip
// state_partial_kernel: pk = max, emi = the EMA started from -inf, b = the affine offset
// of the EMA started from 0, restart = some frame was -inf).  Peak: FftProcessor.kt:241-242;
// EMA (extension): the avg += alpha (x - avg) idiom of GlobalPerformanceData.kt:44-50.
// Explicit fmaf: every kernel that forms a summary (state_partial / state_fused) rounds
// identically, so the result does not depend on which of them computed a chunk.
RFA_HD void state_step(float &pk, float &emi, float &b, bool &restart, float x, float al) {
    pk = fmaxf(pk, x);
    emi = (emi > -INFINITY) ? fmaf(al, x - emi, emi) : x;
    restart |= x == -INFINITY;
    b = fmaf(al, x - b, b);
}

// Row value 10*log10(sqrt((Re/N)^2 + (Im/N)^2)) (nativedsp.cpp:73-78) from the
// UNSCALED FFT output x.  Scaling by 1/N is exact (power of two), so the power
// is (x.x^2 + x.y^2) * 2^(-2 log2 N) and the dB value is
// (5 log10 2) * (log2(x.x^2 + x.y^2) - 2 log2 N): one fma after the hardware
// log2 (v_log_f32).  db_off = -(5 log10 2) * 2 log2 N.  Working unscaled keeps
// the power 2^(2 log2 N) above the reference's, so it leaves the denormal range
// (where v_log_f32 flushes) only for bins that are exactly or essentially zero
// on both sides (-inf here, <= -380 dB in the reference).  log2(0) = -inf as
// in the reference.
constexpr float kDbPerLog2 = 1.50514997831990598f;  // 5*log10(2)
RFA_HD float db_offset(int logn) { return -kDbPerLog2 * (float)(2 * logn); }
__device__ __forceinline__ float db_unscaled(float2 x, float db_off) {
    const float p = fmaf(x.x, x.x, x.y * x.y);
    return fmaf(__builtin_amdgcn_logf(p), kDbPerLog2, db_off);
}

}  // namespace rfa
