"""CPU model of the wave-decoupled 64 K kernel's data movement (rfanalyzer_amd/csrc/fft_w64.hip).

Every lane/register/LDS index of the kernel is replayed in numpy -- the per-lane column of the
pre-stage, exchange 0's four writer rounds through region A, exchange 1's v_permlane32_swap /
v_permlane16_swap semantics and its four wave-local LDS rounds, the DIT twiddles and the
kRingTile2 / natural-row store positions -- on complex128 data, and the result is compared
with numpy's FFT of the same frame (fft-shifted, natural bin order).  This pins the index
algebra independently of the GPU; the float32 parity of the kernel itself is tests/test_gpu_*.
"""
import numpy as np
import pytest

M, N = 32768, 65536


def tile2_pos(i):  # fft_kernels.h
    k0, k1, tp = i & 31, (i >> 5) & 31, i >> 10
    return ((k0 >> 1) << 11) | ((tp >> 2) << 8) | (((k0 & 1) | (k1 << 1)) << 2) | (tp & 3)


def tile2_sub(p):
    w, j, l, e = p >> 11, (p >> 8) & 7, (p >> 2) & 63, p & 3
    return ((l & 1) | (w << 1)) | ((l >> 1) << 5) | ((4 * j + e) << 10)


def W(num, den):
    return np.exp(-2j * np.pi * num / den)


def exchange0(V, rounds):
    """V[tid][32] -> V[tid][32]; the kernel's writer rounds, LDS element indices included."""
    wpr, rb = 16 // rounds, 32 // rounds
    rowp = wpr * 64 + 1
    tid = np.arange(1024)
    l, w = tid & 63, tid >> 6
    k0 = (l & 1) | (w << 1)
    wb = (w % wpr) * 64 + l
    rd = k0 * rowp + (l & ~1)
    out = np.zeros_like(V)
    for h in range(rounds):
        buf = np.full(32 * rowp + 64, np.nan, dtype=V.dtype)
        writers = (w // wpr) == h
        for k in range(32):
            idx = wb[writers] + k * rowp
            assert len(np.unique(idx)) == len(idx)
            buf[idx] = V[writers, k]
        for b in range(rb):
            out[:, h * rb + b] = buf[rd + (b >> 1) * 64 + (b & 1)]
    assert not np.isnan(out).any()
    return out


def exchange0_bal(V):
    """The balanced form (fft_w64.hip exchange0_bal): round h, every wave stores register
    group (h - hi) & 3 and loads pair (h - hi) & 3 into slots 8h .. 8h+7."""
    tid = np.arange(1024)
    l, w = tid & 63, tid >> 6
    hi = w >> 2
    k0lo = ((w & 3) << 1) | (l & 1)
    wb = [hi * 2048 + (w & 3) * 64 + l, hi * 2048 + (w & 3) * 64 + (l ^ 1)]
    rd = [k0lo * 256 + l, k0lo * 256 + (l ^ 1)]
    out = np.zeros_like(V)
    for h in range(4):
        buf = np.full(8448, np.nan, dtype=V.dtype)
        g = (h - hi) & 3
        for k in range(8):
            idx = wb[k & 1] + k * 256
            assert len(np.unique(idx)) == len(idx)
            buf[idx] = V[tid, 8 * g + k]
        for j in range(8):
            out[:, 8 * h + j] = buf[rd[j & 1] + g * 2048 + (j >> 1) * 64]
    assert not np.isnan(out).any()
    return out


def lane_swap32(A, B):  # one wave: A, B are [64] lane vectors (vdst, src)
    return np.concatenate([A[:32], B[:32]]), np.concatenate([A[32:], B[32:]])


def lane_swap16(A, B):
    r = lambda X, i: X[16 * i:16 * i + 16]
    return (np.concatenate([r(A, 0), r(B, 0), r(A, 2), r(B, 2)]),
            np.concatenate([r(A, 1), r(B, 1), r(A, 3), r(B, 3)]))


def exchange1(V):
    V = V.copy()
    for w in range(16):
        lanes = slice(64 * w, 64 * w + 64)
        v = [V[lanes, j].copy() for j in range(32)]
        for j in range(16):
            v[j], v[j + 16] = lane_swap32(v[j], v[j + 16])
        for j in range(32):
            if (j & 8) == 0:
                v[j], v[j + 8] = lane_swap16(v[j], v[j + 8])
        l = np.arange(64)
        rd = ((l >> 1) & 7) * 66 + (l & 0x31)
        for h in range(4):
            sl = np.full(528, np.nan, dtype=V.dtype)
            for a in range(8):
                sl[l + a * 66] = v[8 * h + a]
            for b in range(8):
                v[8 * h + b] = sl[rd + 2 * b]
        for j in range(32):
            V[lanes, j] = v[j]
    assert not np.isnan(V).any()
    return V


def model_frame(x, rounds):
    """Ring row (storage order) and natural row of one 64 K frame x (complex, windowed)."""
    tid = np.arange(1024)
    l, w = tid & 63, tid >> 6
    col = (l >> 1) + ((l & 1) << 5) + (w << 6)
    k0 = (l & 1) | (w << 1)
    k1 = l >> 1
    t = np.arange(32)
    ring = np.full(N, np.nan)
    row = np.full(N, np.nan)
    for r in range(2):
        m = col[:, None] + 1024 * t[None, :]
        y = (x[m] + (-1) ** r * x[m + M]) * W(m * r, N)      # pre-stage
        V = np.fft.fft(y, axis=1)                              # pass 0
        if rounds == "bal":
            V = exchange0_bal(V)
            hi = (w >> 2)[:, None]
            m1 = (t[None, :] - 8 * hi) % 32                    # slot n holds m1 = (n - 8 hi) mod 32
            V = V * W(k0[:, None] * m1, 1024)
        else:
            V = exchange0(V, rounds)
            V = V * W(k0[:, None] * t[None, :], 1024)          # W_1024^{k0 m1}
        V = np.fft.fft(V, axis=1)                              # pass 1
        V = exchange1(V)
        V = V * W(t[None, :] * (k0 + 32 * k1)[:, None], M)     # W_M^{m0 (k0 + 32 k1)}
        V = np.fft.fft(V, axis=1)                              # pass 2
        db = 10 * np.log10(np.abs(V) / N)
        for tp in range(32):
            j, e = tp >> 2, tp & 3
            ring[r * M + w * 2048 + j * 256 + l * 4 + e] = db[:, tp ^ 16]
            row[2 * (k0 + 32 * k1 + 1024 * tp) + r] = db[:, tp ^ 16]
    return ring, row


def test_tile2_is_a_bijection():
    i = np.arange(M)
    p = tile2_pos(i)
    assert np.array_equal(np.sort(p), i)
    assert np.array_equal(tile2_sub(p), i)


@pytest.mark.parametrize("rounds", [4, 2, "bal"])
def test_w64_index_algebra_matches_fft(rounds):
    rng = np.random.default_rng(7 + len(str(rounds)))
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    ring, row = model_frame(x, rounds)
    ref = np.fft.fftshift(10 * np.log10(np.abs(np.fft.fft(x)) / N))
    assert np.max(np.abs(row - ref)) < 1e-9
    # ring element p holds natural bin ring_bin(p) = (tile2_sub(p mod M) << 1) | (p >> 15)
    p = np.arange(N)
    nat = (tile2_sub(p & (M - 1)) << 1) | (p >> 15)
    assert np.max(np.abs(ring - ref[nat])) < 1e-9


def _conflicts(elem_idx, kind):
    """Extra LDS cycles of one wave instruction moving 8 B per lane (gfx950 bank model,
    MI355X_MICROARCH.md LDS table): ds_write_b64 in 4 groups of 16 lanes, bank (a/4) mod 32;
    ds_read_b64 in 2 groups of 32 lanes, bank (a/4) mod 64; identical addresses broadcast."""
    size, nb = (16, 32) if kind == "w" else (32, 64)
    extra = 0
    for g in range(0, 64, size):
        e = np.unique(elem_idx[g:g + size])
        banks = np.concatenate([(2 * e) % nb, (2 * e + 1) % nb])
        extra += np.bincount(banks, minlength=nb).max() - 1
    return extra


def test_w64_lds_patterns_are_conflict_free():
    """Every LDS store / load instruction of the balanced exchange 0 and the wave-local
    exchange 1, for every wave: no bank conflicts."""
    l = np.arange(64)
    for w in range(16):
        hi = w >> 2
        wb = [hi * 2048 + (w & 3) * 64 + l, hi * 2048 + (w & 3) * 64 + (l ^ 1)]
        k0lo = ((w & 3) << 1) | (l & 1)
        rd = [k0lo * 256 + l, k0lo * 256 + (l ^ 1)]
        for k in range(8):
            assert _conflicts(wb[k & 1] + k * 256, "w") == 0
        for g in range(4):
            for j in range(8):
                assert _conflicts(rd[j & 1] + g * 2048 + (j >> 1) * 64, "r") == 0
    rd1 = ((l >> 1) & 7) * 66 + (l & 0x31)
    for a in range(8):
        assert _conflicts(l + a * 66, "w") == 0
    for b in range(8):
        assert _conflicts(rd1 + 2 * b, "r") == 0
