/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin C harness around the reference's own vendored PFFFT
 * (/root/reference/nativedsp/src/main/cpp/pffft.c, compiled from where it lies
 * by oracle/Makefile into oracle/_ref/libpffft_ref.so; no reference source is
 * copied into this repository).
 *
 * It restates, without JNI, the two native entry points of the reference:
 *   ref_fft_ordered   <- Java_..._NativeDsp_performFFT          nativedsp.cpp:19-42
 *   ref_fft_logmag    <- Java_..._NativeDsp_performFFTAndLogMag nativedsp.cpp:44-81
 * and the reference's single-threaded spectrum loop used as the CPU baseline:
 *   ref_loop_*        <- LUT convert (Signed8BitIQConverter.java:88-94) ->
 *                        Blackman window (NativeDsp.kt:55-58) -> pffft ->
 *                        log-mag (nativedsp.cpp:72-79) -> ring copy +
 *                        peak-hold (FftProcessor.kt:222-242)
 *
 * The log-mag loop is compiled WITHOUT -ffast-math (the reference's
 * CMakeLists.txt:15 puts -O3 -ffast-math into C flags only, i.e. pffft.c).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pffft.h"

typedef struct {
    int n;
    PFFFT_Setup *setup;
    float *scratch, *in, *out;
} ref_ctx;

static ref_ctx g_ctx = {0, 0, 0, 0, 0};

static int ensure(int n) {
    if (g_ctx.n == n) return 0;
    if (g_ctx.setup) {
        pffft_destroy_setup(g_ctx.setup);
        pffft_aligned_free(g_ctx.scratch);
        pffft_aligned_free(g_ctx.in);
        pffft_aligned_free(g_ctx.out);
    }
    g_ctx.setup = pffft_new_setup(n, PFFFT_COMPLEX);
    if (!g_ctx.setup) { g_ctx.n = 0; return -1; }
    g_ctx.scratch = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    g_ctx.in = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    g_ctx.out = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    g_ctx.n = n;
    return 0;
}

int ref_simd_size(void) { return pffft_simd_size(); }

/* nativedsp.cpp:19-42 -- ordered, unscaled forward complex FFT of 2n floats. */
int ref_fft_ordered(const float *in_interleaved, int n, float *out_interleaved) {
    if (ensure(n)) return -1;
    memcpy(g_ctx.in, in_interleaved, 2 * (size_t)n * sizeof(float));
    pffft_transform_ordered(g_ctx.setup, g_ctx.in, g_ctx.out, g_ctx.scratch, PFFFT_FORWARD);
    memcpy(out_interleaved, g_ctx.out, 2 * (size_t)n * sizeof(float));
    return 0;
}

static void logmag_shift(const float *o, int n, float *mag) {
    for (int i = 0; i < n; i++) { /* nativedsp.cpp:72-79 */
        float rp = o[2 * i] / (float)n;
        rp *= rp;
        float ip = o[2 * i + 1] / (float)n;
        ip *= ip;
        int t = (i + n / 2) % n;
        mag[t] = (float)(10 * log10(sqrt(rp + ip)));
    }
}

/* nativedsp.cpp:44-81 -- FFT + 10*log10(sqrt(p)) + fft-shift. */
int ref_fft_logmag(const float *in_interleaved, int n, float *mag_out) {
    if (ensure(n)) return -1;
    memcpy(g_ctx.in, in_interleaved, 2 * (size_t)n * sizeof(float));
    pffft_transform_ordered(g_ctx.setup, g_ctx.in, g_ctx.out, g_ctx.scratch, PFFFT_FORWARD);
    logmag_shift(g_ctx.out, n, mag_out);
    return 0;
}

/* The reference FftProcessor loop for 8-bit signed or f32-interleaved frames,
 * timed as the CPU baseline: per frame LUT/copy -> window -> pffft -> log-mag
 * -> copy into ring row -> peak max.  fmt: 0 = s8, 3 = f32 interleaved.
 * Returns 0 on success.  `ring` holds ring_rows*n floats, `peaks` n floats. */
int ref_loop(const void *frames, int fmt, int n, int n_frames, long frame_stride_bytes, const float *window,
             float *ring, int ring_rows, float *peaks) {
    /* a private context per call (one per FftProcessor thread): the multi-core
     * baseline runs one loop per host thread */
    ref_ctx c;
    c.n = n;
    c.setup = pffft_new_setup(n, PFFFT_COMPLEX);
    if (!c.setup) return -1;
    c.scratch = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    c.in = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    c.out = (float *)pffft_aligned_malloc(2 * (size_t)n * sizeof(float));
    float lut[256];
    for (int i = 0; i < 256; i++) lut[i] = (float)(i - 128) / 128.0f;
    float *re = (float *)malloc(sizeof(float) * n), *im = (float *)malloc(sizeof(float) * n);
    float *mag = (float *)malloc(sizeof(float) * n);
    if (!re || !im || !mag || !c.scratch || !c.in || !c.out) { free(re); free(im); free(mag); return -1; }
    int write_index = 0;
    for (int f = 0; f < n_frames; f++) {
        const uint8_t *p = (const uint8_t *)frames + (size_t)f * frame_stride_bytes;
        if (fmt == 0) {
            const int8_t *s = (const int8_t *)p;
            for (int i = 0; i < n; i++) { re[i] = lut[s[2 * i] + 128]; im[i] = lut[s[2 * i + 1] + 128]; }
        } else {
            const float *s = (const float *)p;
            for (int i = 0; i < n; i++) { re[i] = s[2 * i]; im[i] = s[2 * i + 1]; }
        }
        for (int i = 0; i < n; i++) { c.in[2 * i] = re[i] * window[i]; c.in[2 * i + 1] = im[i] * window[i]; }
        pffft_transform_ordered(c.setup, c.in, c.out, c.scratch, PFFFT_FORWARD);
        logmag_shift(c.out, n, mag);
        float *row = ring + (size_t)write_index * n;
        memcpy(row, mag, sizeof(float) * n);
        write_index = write_index == 0 ? ring_rows - 1 : write_index - 1;
        for (int i = 0; i < n; i++) peaks[i] = fmaxf(peaks[i], row[i]);
    }
    free(re); free(im); free(mag);
    pffft_destroy_setup(c.setup);
    pffft_aligned_free(c.scratch);
    pffft_aligned_free(c.in);
    pffft_aligned_free(c.out);
    return 0;
}
