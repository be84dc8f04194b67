/*
 * rfa_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of RFAnalyzer's spectrum hot path, used as the parity
 * checker for the HIP path (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Nothing in rfanalyzer_amd/ links or calls this file.
 *
 * Every function cites the reference line(s) it restates (paths relative to
 * the reference root, thomasjoergensen/RFAnalyzer):
 *
 *   converters  app/src/main/java/com/mantz_it/rfanalyzer/source/
 *               Signed8BitIQConverter.java:48-50,80-99
 *               Unsigned8BitIQConverter.java:48-50,80-99
 *               Signed16BitIQConverter.kt:46-57,89-124
 *   window      nativedsp/src/main/java/com/mantz_it/nativedsp/NativeDsp.kt:14-21,55-58
 *   FFT         pffft_transform_ordered (nativedsp.cpp:69) -- restated here as
 *               a plain float64 radix-2 DFT; the real pffft is validated
 *               against it through oracle/_ref (see ref_harness.c).
 *   log-mag     nativedsp/src/main/cpp/nativedsp.cpp:72-79
 *
 * Parity is pinned by golden vectors produced from the reference's own
 * pffft.c compiled into oracle/_ref (tests/golden/gen_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR (-1)

enum { ORC_IN_S8 = 0, ORC_IN_U8 = 1, ORC_IN_S16LE = 2, ORC_IN_F32_INTERLEAVED = 3, ORC_IN_F32_PLANAR = 4 };
enum { ORC_WIN_BLACKMAN = 0, ORC_WIN_HANN = 1, ORC_WIN_NONE = 2 };

/* ---------------------------------------------------------------- converters */

/* Signed8BitIQConverter.java:48-50: lookupTable[i] = (i-128)/128.0f, indexed
 * by packet[i]+128 (:88-94).  Bit-exact: (b)/128 is an exact float. */
void orc_convert_s8(const int8_t *in, size_t n, float *re, float *im) {
    float lut[256];
    for (int i = 0; i < 256; i++) lut[i] = (float)(i - 128) / 128.0f;
    for (size_t k = 0; k < n; k++) {
        re[k] = lut[in[2 * k] + 128];
        im[k] = lut[in[2 * k + 1] + 128];
    }
}

/* Unsigned8BitIQConverter.java:48-50: (i-127.4f)/128.0f, indexed by b & 0xff. */
void orc_convert_u8(const uint8_t *in, size_t n, float *re, float *im) {
    float lut[256];
    for (int i = 0; i < 256; i++) {
        volatile float d = (float)i - 127.4f; /* Java float arithmetic, one rounding */
        lut[i] = d / 128.0f;
    }
    for (size_t k = 0; k < n; k++) {
        re[k] = lut[in[2 * k]];
        im[k] = lut[in[2 * k + 1]];
    }
}

/* Signed16BitIQConverter.kt:46-57 (lut[u] = (short)u / 32768f) and :105-116
 * (little-endian Ilo,Ihi,Qlo,Qhi). */
void orc_convert_s16(const uint8_t *in, size_t n, float *re, float *im) {
    for (size_t k = 0; k < n; k++) {
        int16_t i16 = (int16_t)(uint16_t)(in[4 * k] | (in[4 * k + 1] << 8));
        int16_t q16 = (int16_t)(uint16_t)(in[4 * k + 2] | (in[4 * k + 3] << 8));
        re[k] = (float)i16 / 32768.0f;
        im[k] = (float)q16 / 32768.0f;
    }
}

/* Generic dispatch: converts n samples of one frame to planar float. */
int orc_convert(const void *frame, int fmt, size_t n, float *re, float *im) {
    switch (fmt) {
    case ORC_IN_S8: orc_convert_s8((const int8_t *)frame, n, re, im); return ORC_OK;
    case ORC_IN_U8: orc_convert_u8((const uint8_t *)frame, n, re, im); return ORC_OK;
    case ORC_IN_S16LE: orc_convert_s16((const uint8_t *)frame, n, re, im); return ORC_OK;
    case ORC_IN_F32_INTERLEAVED: {
        const float *f = (const float *)frame;
        for (size_t k = 0; k < n; k++) { re[k] = f[2 * k]; im[k] = f[2 * k + 1]; }
        return ORC_OK;
    }
    case ORC_IN_F32_PLANAR: {
        const float *f = (const float *)frame;
        memcpy(re, f, n * sizeof(float));
        memcpy(im, f + n, n * sizeof(float));
        return ORC_OK;
    }
    default: return ORC_ERR;
    }
}

/* ---------------------------------------------------------------- window */

/* NativeDsp.kt:14-21: Blackman evaluated in double and cast once to float.
 * Hann (north-star extension) uses the same symmetric (N-1) convention. */
int orc_window(int n, int kind, float *w) {
    if (n < 2) return ORC_ERR;
    for (int i = 0; i < n; i++) {
        double x = 2.0 * M_PI * (double)i / (double)(n - 1);
        double v;
        switch (kind) {
        case ORC_WIN_BLACKMAN: v = 0.42 - 0.5 * cos(x) + 0.08 * cos(2.0 * x); break;
        case ORC_WIN_HANN: v = 0.5 - 0.5 * cos(x); break;
        case ORC_WIN_NONE: v = 1.0; break;
        default: return ORC_ERR;
        }
        w[i] = (float)v;
    }
    return ORC_OK;
}

/* ---------------------------------------------------------------- FFT (float64) */

static int ilog2(size_t n) {
    int l = 0;
    while (((size_t)1 << l) < n) l++;
    return ((size_t)1 << l) == n ? l : -1;
}

/* Forward complex DFT, sign -1, unscaled (pffft.h:117, pffft.c:1660), natural
 * bin order.  Iterative radix-2 DIT with exactly-computed double twiddles. */
int orc_fft_f64(double *re, double *im, size_t n) {
    int lg = ilog2(n);
    if (lg < 1) return ORC_ERR;
    for (size_t i = 1, j = 0; i < n; i++) { /* bit reversal */
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    double *tw = (double *)malloc(sizeof(double) * n); /* cos/sin of -2*pi*k/n, k<n/2 */
    if (!tw) return ORC_ERR;
    for (size_t k = 0; k < n / 2; k++) {
        double a = -2.0 * M_PI * (double)k / (double)n;
        tw[2 * k] = cos(a);
        tw[2 * k + 1] = sin(a);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        size_t half = len >> 1, step = n / len;
        for (size_t s = 0; s < n; s += len) {
            for (size_t k = 0; k < half; k++) {
                double wr = tw[2 * k * step], wi = tw[2 * k * step + 1];
                size_t a = s + k, b = a + half;
                double xr = re[b] * wr - im[b] * wi;
                double xi = re[b] * wi + im[b] * wr;
                re[b] = re[a] - xr; im[b] = im[a] - xi;
                re[a] += xr; im[a] += xi;
            }
        }
    }
    free(tw);
    return ORC_OK;
}

/* ---------------------------------------------------------------- log-mag */

/* nativedsp.cpp:72-79: p = (Re/N)^2 + (Im/N)^2, out[(i+N/2)%N] = 10*log10(sqrt(p)). */
void orc_logmag_shift_f64(const double *re, const double *im, size_t n, float *out) {
    for (size_t i = 0; i < n; i++) {
        double r = re[i] / (double)n, q = im[i] / (double)n;
        out[(i + n / 2) % n] = (float)(10.0 * log10(sqrt(r * r + q * q)));
    }
}

/* One full frame: convert -> window (fp32 multiply, NativeDsp.kt:55-58) ->
 * float64 FFT -> log-mag + shift.  `window` may be NULL (= rectangular). */
int orc_spectrum_row(const void *frame, int fmt, size_t n, const float *window, float *out_db) {
    if (ilog2(n) < 1) return ORC_ERR;
    float *fre = (float *)malloc(sizeof(float) * n), *fim = (float *)malloc(sizeof(float) * n);
    double *re = (double *)malloc(sizeof(double) * n), *im = (double *)malloc(sizeof(double) * n);
    int rc = ORC_ERR;
    if (!fre || !fim || !re || !im) goto done;
    if (orc_convert(frame, fmt, n, fre, fim) != ORC_OK) goto done;
    for (size_t i = 0; i < n; i++) {
        float w = window ? window[i] : 1.0f;
        float a = fre[i] * w, b = fim[i] * w; /* fp32 multiply, as the JVM does */
        re[i] = a;
        im[i] = b;
    }
    if (orc_fft_f64(re, im, n) != ORC_OK) goto done;
    orc_logmag_shift_f64(re, im, n, out_db);
    rc = ORC_OK;
done:
    free(fre); free(fim); free(re); free(im);
    return rc;
}

/* Batch of frames at a fixed byte stride (Scheduler framing, Scheduler.kt:252-279). */
int orc_spectrum_rows(const void *base, int fmt, size_t n, size_t n_frames, size_t frame_stride_bytes,
                      const float *window, float *out_rows) {
    const uint8_t *p = (const uint8_t *)base;
    for (size_t f = 0; f < n_frames; f++) {
        int rc = orc_spectrum_row(p + f * frame_stride_bytes, fmt, n, window, out_rows + f * n);
        if (rc != ORC_OK) return rc;
    }
    return ORC_OK;
}

/* ------------------------------------------------- demod front end (§8(f) row 4)
 *
 * mixPacketIntoSamplePacket (source/Signed8BitIQConverter.java:101-130: the
 * table entry lut[b] * cos_t is one float product, formed here per sample with
 * the same rounding; Unsigned8BitIQConverter.java and Signed16BitIQConverter.kt
 * :126-181 alike) followed by FirFilter.filter (dsp/FirFilter.kt:63-107):
 * circular delay line, output when decimationCounter == 0, taps summed in
 * order newest sample first.  One sample at a time, exactly the reference's
 * loop; the CPU baseline of the demod leg (1 thread, scalar).
 * state: dre[T], dim[T] delay lines; counters = {tapCounter, decimationCounter,
 * cosineIndex}.  cos_t == NULL: input is already-mixed interleaved float.
 * Returns the number of outputs written. */
size_t orc_ddc_process(int fmt, const void *raw, size_t n, const float *cos_t, const float *sin_t, int L,
                       const float *taps, int T, int D, float *dre, float *dim, int32_t *counters,
                       float *out_re, float *out_im) {
    int tap = counters[0], dc = counters[1], ci = counters[2];
    size_t k = 0;
    const uint8_t *b = (const uint8_t *)raw;
    for (size_t s = 0; s < n; s++) {
        float re, im;
        if (!cos_t) {
            const float *f = (const float *)raw;
            re = f[2 * s];
            im = f[2 * s + 1];
        } else {
            float i, q;
            if (fmt == ORC_IN_S16LE) {
                i = (float)(int16_t)(b[4 * s] | (b[4 * s + 1] << 8)) / 32768.0f;
                q = (float)(int16_t)(b[4 * s + 2] | (b[4 * s + 3] << 8)) / 32768.0f;
            } else if (fmt == ORC_IN_U8) {
                i = ((float)b[2 * s] - 127.4f) / 128.0f;
                q = ((float)b[2 * s + 1] - 127.4f) / 128.0f;
            } else {
                i = (float)(int8_t)b[2 * s] / 128.0f;
                q = (float)(int8_t)b[2 * s + 1] / 128.0f;
            }
            const float c = cos_t[ci], sn = sin_t[ci];
            const float ic = i * c, qs = q * sn, qc = q * c, is = i * sn;
            re = ic - qs;
            im = qc + is;
            ci = (ci + 1) % L;
        }
        dre[tap] = re;
        dim[tap] = im;
        if (dc == 0) {
            float ar = 0.0f, ai = 0.0f;
            int idx = tap;
            for (int t = 0; t < T; t++) {
                const float pr = taps[t] * dre[idx], pi = taps[t] * dim[idx];
                ar = ar + pr;
                ai = ai + pi;
                if (--idx < 0) idx = T - 1;
            }
            out_re[k] = ar;
            out_im[k] = ai;
            k++;
        }
        if (++dc >= D) dc = 0;
        if (++tap >= T) tap = 0;
    }
    counters[0] = tap;
    counters[1] = dc;
    counters[2] = ci;
    return k;
}
