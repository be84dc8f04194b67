#!/usr/bin/env python3
"""float32 emulation of the wave-decoupled 64 K kernel's arithmetic (rfanalyzer_amd/csrc/fft_w64.hip,
fft_common.h), operation by operation, on the CPU: every product, sum and fma rounded to fp32 in
the kernel's order (products of two fp32 are exact in float64; an fma is the float64 a*b + c
rounded once more -- double rounding is rare and only shifts statistics), v_log_f32 as the
correctly rounded log2.  Used to compare precision variants of the kernel against the float64
transform and the reference's pffft on the config-3 batch without GPU time.

usage: w64_precision.py [--frames 500] [--variant plain|rot] [--chunk 25]
  plain: exchange 0 in natural register order; rot: the balanced exchange's rotated pass-1 input
  (slot n holds m1 = (n - 8 hi) mod 32)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

F = np.float32
N, M = 65536, 32768
TW2EXACT = False
EXACT = set()  # stages computed in float64 and rounded to fp32 once: pre, p0, p1, p2, tw1, tw2


def exact_dft32(v):
    z = np.stack([v[t][0].astype(np.float64) + 1j * v[t][1].astype(np.float64) for t in range(32)], 0)
    Z = np.fft.fft(z, axis=0)
    return [(Z[k].real.astype(F), Z[k].imag.astype(F)) for k in range(32)]
R2 = F(0.707106781186547524)
C1, S1 = F(0.923879532511286756), F(0.382683432365089772)
KDB = F(1.50514997831990598)
ang64 = 2 * np.pi * np.arange(64) / 64
COS64, SIN64 = np.cos(ang64).astype(F), np.sin(ang64).astype(F)


def r32(x):
    return np.asarray(x, np.float64).astype(F)


def mul(a, b):
    return r32(np.asarray(a, np.float64) * np.asarray(b, np.float64))


def add(a, b):
    return r32(np.asarray(a, np.float64) + np.asarray(b, np.float64))


def fma(a, b, c):
    return r32(np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64))


# complex value = (re, im) tuple of fp32 arrays
def rot(a, p):
    x, y = a
    p &= 3
    return [(x, y), (y, -x), (-x, -y), (-y, x)][p]


def padd(a, b, p, q):
    ra, rb = rot(a, p), rot(b, q)
    return add(ra[0], rb[0]), add(ra[1], rb[1])


def cmul(a, w):  # fft_common.h cmul: m = (a.x w.x, a.x w.y); r = (fma(a.y, -w.y, m.x), fma(a.y, w.x, m.y))
    mx, my = mul(a[0], w[0]), mul(a[0], w[1])
    return fma(a[1], -w[1], mx), fma(a[1], w[0], my)


def cmulc(a, c, s):  # a * (c, s): m = (a.x c, a.x s); fma((a.y, a.y), (-s, c), m)
    mx, my = mul(a[0], c), mul(a[0], s)
    return fma(a[1], -s, mx), fma(a[1], c, my)


def w16(x, m):
    q = m & 15
    if q & 3 == 0:
        return rot(x, q // 4)
    if q & 3 == 2:
        t = padd(x, x, (q - 2) // 4, (q + 2) // 4)
        return mul(t[0], R2), mul(t[1], R2)
    c = [1, C1, R2, S1, 0, -S1, -R2, -C1, -1, -C1, -R2, -S1, 0, S1, R2, C1]
    s = [0, S1, R2, C1, 1, C1, R2, S1, 0, -S1, -R2, -C1, -1, -C1, -R2, -S1]
    return cmulc(x, F(c[q]), F(-s[q]))


def w64(x, m):
    q = m & 63
    if q & 3 == 0:
        return w16(x, q // 4)
    return cmulc(x, COS64[q], -SIN64[q])


def dft2(a, b):
    return (add(a[0], b[0]), add(a[1], b[1])), (add(a[0], -b[0]), add(a[1], -b[1]))


def dft4r(x0, x1, x2, x3, p1=0, p2=0, p3=0):
    s02, d02 = padd(x0, x2, 0, p2), padd(x0, x2, 0, p2 + 2)
    s13, d13 = padd(x1, x3, p1, p3), padd(x1, x3, p1, p3 + 2)
    return padd(s02, s13, 0, 0), padd(d02, d13, 0, 1), padd(s02, s13, 0, 2), padd(d02, d13, 0, 3)


def dft16r(u, rot8=0):
    u = list(u)
    u[0], u[4], u[8], u[12] = dft4r(u[0], u[4], u[8], u[12], 0, rot8, 0)
    for a in (1, 2, 3):
        u[a], u[a + 4], u[a + 8], u[a + 12] = dft4r(u[a], u[a + 4], u[a + 8], u[a + 12])
    for i, m in ((5, 1), (6, 2), (7, 3), (9, 2), (11, 6), (13, 3), (14, 6), (15, 9)):
        u[i] = w16(u[i], m)
    u[0], u[1], u[2], u[3] = dft4r(u[0], u[1], u[2], u[3])
    u[4], u[5], u[6], u[7] = dft4r(u[4], u[5], u[6], u[7])
    u[8], u[9], u[10], u[11] = dft4r(u[8], u[9], u[10], u[11], 0, 1, 0)
    u[12], u[13], u[14], u[15] = dft4r(u[12], u[13], u[14], u[15])
    return [u[4 * (q & 3) + (q >> 2)] for q in range(16)]


def dft32(u):
    u = list(u)
    for t2 in range(16):
        u[t2], u[16 + t2] = dft2(u[t2], u[16 + t2])
    for i, m in ((17, 2), (18, 4), (19, 6), (20, 8), (21, 10), (22, 12), (23, 14), (25, 18), (26, 20), (27, 22),
                 (28, 24), (29, 26), (30, 28), (31, 30)):
        u[i] = w64(u[i], m)
    a = dft16r(u[:16])
    b = dft16r(u[16:], 1)
    u = a + b
    return [u[16 * (q & 1) + (q >> 1)] for q in range(32)]


def tables():
    def w(num, den):
        ang = -2.0 * np.pi * np.asarray(num, np.float64) / den
        return np.cos(ang).astype(F), np.sin(ang).astype(F)
    a = np.arange(32)[:, None]
    t = np.arange(33)[None, :]
    T1 = w(a * t, 1024.0)             # [a][t]
    TB = w(t * a, 32768.0)            # [k0][t] (t = 0 .. 32; the kernel stores t = 1..31)
    return T1, TB


def frame_rows(x8, wdb, cw, T1, TB, variant):
    """x8: int8 [frames][N][2]; returns dB rows [frames][N] (natural, fft-shifted)."""
    frames = x8.shape[0]
    tid = np.arange(1024)
    l, w = tid & 63, tid >> 6
    col = (l >> 1) + ((l & 1) << 5) + (w << 6)
    k0 = (l & 1) | (w << 1)
    k1 = l >> 1
    hi = w >> 2
    out = np.zeros((frames, N), F)
    xr = x8[..., 0].astype(F)
    xi = x8[..., 1].astype(F)
    for r in range(2):
        m = col[:, None] + 1024 * np.arange(32)[None, :]            # [1024][32]
        a0 = (xr[:, m], xi[:, m])
        a1 = (xr[:, m + M], xi[:, m + M])
        if "pre" in EXACT:
            ang = -2.0 * np.pi * (m * r) / N
            tw = np.exp(1j * ang)
            z0 = a0[0].astype(np.float64) + 1j * a0[1].astype(np.float64)
            z1 = a1[0].astype(np.float64) + 1j * a1[1].astype(np.float64)
            y = (z0 * wdb[m].astype(np.float64) + (1 - 2 * r) * z1 * wdb[m + M].astype(np.float64)) * tw
            v = [(y[..., t].real.astype(F), y[..., t].imag.astype(F)) for t in range(32)]
        elif r == 0:
            w0, w1 = wdb[m], wdb[m + M]
            v = [fma(a1[0][..., t], w1[:, t], mul(a0[0][..., t], w0[:, t])) for t in range(32)], \
                [fma(a1[1][..., t], w1[:, t], mul(a0[1][..., t], w0[:, t])) for t in range(32)]
            v = [(v[0][t], v[1][t]) for t in range(32)]
        else:
            c0 = (cw[0][m], cw[1][m])
            c1 = (cw[2][m], cw[3][m])
            v = []
            for t in range(32):
                A0 = (a0[0][..., t], a0[1][..., t])
                A1 = (a1[0][..., t], a1[1][..., t])
                mx, my = mul(A0[0], c0[0][:, t]), mul(A0[0], c0[1][:, t])
                rx, ry = fma(A0[1], -c0[1][:, t], mx), fma(A0[1], c0[0][:, t], my)
                mx, my = fma(A1[0], c1[0][:, t], rx), fma(A1[0], c1[1][:, t], ry)
                v.append((fma(A1[1], -c1[1][:, t], mx), fma(A1[1], c1[0][:, t], my)))
        v = exact_dft32(v) if "p0" in EXACT else dft32(v)            # pass 0: slot = k0' (regs)
        # exchange 0 (a permutation): thread (m0, k0) takes register k0 of the writer (m0, m1)
        V = np.stack([np.stack(z, 0) for z in v], 0)                 # [32 k0][2][frames][1024 tid]
        W = np.empty_like(V)                                         # [32 slot][2][frames][1024]
        for n in range(32):
            m1 = (n - 8 * hi) % 32 if variant == "rot" else np.full(1024, n)
            src = (m1 >> 1) * 64 + (((l >> 1) << 1) | (m1 & 1))
            g = V[k0, :, :, src].transpose(1, 2, 0)
            if "tw1" in EXACT:
                z = (g[0].astype(np.float64) + 1j * g[1].astype(np.float64)) * np.exp(-2j * np.pi * k0 * m1 / 1024)
                W[n] = np.stack((z.real.astype(F), z.imag.astype(F)), 0)
            else:
                W[n] = np.stack(cmul((g[0], g[1]), (T1[0][k0, m1], T1[1][k0, m1])), 0)
        v = (exact_dft32 if "p1" in EXACT else dft32)([(W[n][0], W[n][1]) for n in range(32)])  # pass 1: slot = k1 (phase (-i)^{hi k1} for rot)
        # exchange 1 (a permutation): thread (k0, k1) takes register k1 of lane (m0, k0 bit 0), same wave
        V = np.stack([np.stack(z, 0) for z in v], 0)                 # [32 k1][2][frames][1024]
        W = np.empty_like(V)
        for j in range(32):                                          # slot j = m0
            src = w * 64 + ((j << 1) | (l & 1))
            W[j] = V[k1, :, :, src].transpose(1, 2, 0)
        v = [(W[j][0], W[j][1]) for j in range(32)]
        for t in range(1, 32):
            if TW2EXACT:  # correctly rounded W_M^{t (k0 + 32 k1)} (a 32 K-entry table)
                ang = -2.0 * np.pi * (t * (k0 + 32 * k1)) / M
                wt = (np.cos(ang).astype(F), np.sin(ang).astype(F))
            else:
                wt = cmul((T1[0][k1, t], T1[1][k1, t]), (TB[0][k0, t], TB[1][k0, t]))
            if "tw2" in EXACT:
                z = (v[t][0].astype(np.float64) + 1j * v[t][1].astype(np.float64)) * np.exp(-2j * np.pi * t * (k0 + 32 * k1) / M)
                v[t] = (z.real.astype(F), z.imag.astype(F))
            else:
                v[t] = cmul(v[t], wt)
        v = exact_dft32(v) if "p2" in EXACT else dft32(v)            # pass 2: slot = k2
        off = F(-KDB * F(32.0))
        for t in range(32):
            p = fma(v[t][0], v[t][0], mul(v[t][1], v[t][1]))
            with np.errstate(divide="ignore"):
                lg = r32(np.log2(p.astype(np.float64)))
            db = fma(lg, KDB, off)
            tp = t ^ 16
            pos = 2 * (k0 + 32 * k1 + 1024 * tp) + r
            out[:, pos] = db
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--chunk", type=int, default=20)
    ap.add_argument("--variant", default="plain")
    ap.add_argument("--tw2exact", action="store_true")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--exact", default="", help="comma list of stages in float64: pre,p0,tw1,p1,tw2,p2")
    args = ap.parse_args()
    global TW2EXACT
    TW2EXACT = args.tw2exact
    EXACT.update(x for x in args.exact.split(",") if x)
    import oracle
    import signals
    import golden_util as gu
    data = signals.frames_bytes(N, args.frames, "s8", args.seed, tones=((0.1234, 0.4), (-0.377, 0.01)), noise=0.05)
    x8 = np.frombuffer(data, np.int8).reshape(args.frames, N, 2)
    wd = np.asarray(oracle.window(N), np.float64)                     # Blackman, double -> float in the kernel
    wf = wd.astype(F).astype(np.float64)
    wdb = (wf * (1.0 / 128.0)).astype(F)
    ang = -2.0 * np.pi * np.arange(M) / N
    w0, w1 = wf[:M] / 128.0, wf[M:] / 128.0
    cw = ((w0 * np.cos(ang)).astype(F), (w0 * np.sin(ang)).astype(F), (-w1 * np.cos(ang)).astype(F),
          (-w1 * np.sin(ang)).astype(F))
    T1, TB = tables()
    rows = np.concatenate([frame_rows(x8[i:i + args.chunk], wdb, cw, T1, TB, args.variant)
                           for i in range(0, args.frames, args.chunk)])
    ref64 = oracle.spectrum_rows(data, oracle.IN_S8, N, args.frames, None, oracle.WIN_BLACKMAN)
    d64 = gu.full_row_diff(rows, ref64, bar=None)
    print(f"variant {args.variant}{' tw2exact' if TW2EXACT else ''} exact={sorted(EXACT)} seed {args.seed}: frames {args.frames}: every-bin max |emul - float64| {d64:.4f} dB, "
          f"share > 0.01 dB {gu.exceed_fraction(rows, ref64):.2e}")
    if oracle.ref_available():
        ref = oracle.ref_spectrum_rows(data, oracle.IN_S8, N, args.frames)
        print(f"  |emul - pffft| {gu.full_row_diff(rows, ref, bar=None):.4f} dB, |pffft - float64| "
              f"{gu.full_row_diff(ref, ref64, bar=None):.4f} dB, beyond pffft's error "
              f"{gu.full_row_bound(rows, ref, ref64):.4f} dB")


if __name__ == "__main__":
    main()
