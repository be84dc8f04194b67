/*
 * rfa_jni.h -- JNI entry points exported by librfa.so as a drop-in for the
 * reference's libnativedsp.so (System.loadLibrary("nativedsp"),
 * nativedsp/src/main/java/com/mantz_it/nativedsp/NativeDsp.kt:33).
 *
 * The JNI types come from rfanalyzer_amd/csrc/jni_min.h, a minimal restatement
 * of the JNI specification's types and JNINativeInterface function-table
 * layout (this image ships no JDK / jni.h).  With a real jni.h the signatures
 * are identical.
 *
 *   symbol                                                   replaces
 *   Java_com_mantz_1it_nativedsp_NativeDsp_performFFT         nativedsp.cpp:19-42
 *   Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag nativedsp.cpp:44-81
 *   Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative
 *        new native for the Kotlin seam NativeDsp.performWindowedFftAndReturnMag
 *        (NativeDsp.kt:43-62): planar re/im in, Blackman + FFT + log-mag fused
 *        on the GPU, returns JNI_FALSE on a length mismatch like the Kotlin code.
 *   Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative
 *        raw IQ packet bytes (IQSourceInterface.getPacket, IQSourceInterface.java:128)
 *        straight to log-mag rows: the converter LUT (fillPacketIntoSamplePacket,
 *        IQSourceInterface.java:159) is fused into the same kernel.
 *
 * Stateful natives (one jlong handle = one rfa_handle / rfa_ddc):
 *   createAnalyzerNative / destroyAnalyzerNative / processPacketNative
 *        FftProcessor's ring, peak-hold and averaging on the device
 *        (FftProcessor.kt:96-257, Scheduler.kt:252-279): rfa_create, rfa_set_tuning
 *        + rfa_process_host
 *   drawPreprocessNative   AnalyzerSurface.drawPreprocessing (AnalyzerSurface.kt:599-743):
 *        rfa_draw_preprocess, colours in the reference's colorBuffer layout
 *   rowWindowStatsNative   the scanner / squelch row reductions
 *        (MainViewModel.kt:861-929, :1391-1540): rfa_row_window_stats
 *   ddcCreate / ddcDestroy / ddcSetFrequencies / ddcProcess
 *        IQConverter.mixPacketIntoSamplePacket + Decimator / Resampler
 *        (Scheduler.kt:237-250, Decimator.java:175-191): rfa_ddc_*
 *   Handle-taking natives return an rfa_status (0 = ok, < 0 = error) or a count
 *   (>= 0) / negative status; create functions return 0 on failure.
 *
 * Threading: like the reference (NativeDsp.kt:23-26) one caller thread per
 * library is expected; the shim additionally serialises the legacy (global
 * setup) calls with a mutex.  A handle must not be used from two threads at once.
 */
#ifndef RFA_JNI_H
#define RFA_JNI_H

#include "../rfanalyzer_amd/csrc/jni_min.h"

#ifdef __cplusplus
extern "C" {
#endif

/* JNI surface version.  2 (round 3): frame_stride 0 of processIqBytesNative /
 * processPacketNative is the reference's packet framing (one frame per completing packet,
 * the rest of that packet dropped); version 1 read 0 as "every whole frame, densely
 * packed" -- callers of that form pass frame_stride = fft_size * bytes per sample. */
#define RFA_JNI_ABI_VERSION 2
JNIEXPORT int rfa_jni_abi_version(void);
/* Status of the last legacy call (performFFT, performFFTAndLogMag,
 * performWindowedFftAndReturnMagNative, processIqBytesNative), whose JNI signatures
 * return nothing (nativedsp.cpp:19-81): RFA_OK, or e.g. RFA_ERR_UNSUPPORTED when the
 * reference's pffft rejects the length too (not a multiple of 16, a factor other than
 * 2, 3, 5, or above 2^26: pffft.c:1236-1277) -- the output array is then left
 * untouched.  Every length pffft takes is served: powers of two 64 .. 2^20 by a cached
 * streaming handle, the others (16, 32, 2^21 .. 2^26, mixed lengths) by a cached
 * rfa_seam plan (rfa.h).  processIqBytesNative takes the handle's lengths only. */
JNIEXPORT int rfa_jni_last_status(void);

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(JNIEnv *env, jobject thiz,
                                                                          jfloatArray input, jfloatArray output);
JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag(JNIEnv *env, jobject thiz,
                                                                                   jfloatArray input,
                                                                                   jfloatArray output);
JNIEXPORT jboolean JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
    JNIEnv *env, jobject thiz, jfloatArray re, jfloatArray im, jfloatArray mag_out);
/* format: rfa_input_format.  frame_stride 0: the reference's framing
 * (Scheduler.kt:252-273) on the cached setup -- the packet fills a partial frame
 * across calls; returns 1 with the completed frame's row in mag_out[0, fft_size)
 * or 0 while the frame is incomplete.  frame_stride > 0: batch mode, every whole
 * frame at frame_stride bytes that packet and mag_out hold; returns the count.
 * -1 on error (mag_out shorter than fft_size, bad format). */
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(
    JNIEnv *env, jobject thiz, jbyteArray packet, jint format, jint fft_size, jint frame_stride,
    jfloatArray mag_out);

/* FftProcessor on the device.  window: rfa_window; avg_mode: rfa_avg_mode. */
JNIEXPORT jlong JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_createAnalyzerNative(
    JNIEnv *env, jobject thiz, jint fft_size, jint input_format, jint window, jint avg_mode, jint avg_length,
    jfloat ema_alpha, jboolean peak_hold, jint ring_rows, jint device);
JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_destroyAnalyzerNative(JNIEnv *env, jobject thiz,
                                                                                     jlong handle);
/* One raw packet into ring + state.  frame_stride 0: the reference's framing
 * (rfa_push_packet: Scheduler.kt:252-273, a partial frame filled across packets,
 * the tuning of the completing packet); returns 1 when a frame was processed,
 * 0 while it is incomplete.  frame_stride > 0: batch mode, every whole frame at
 * that stride after rfa_set_tuning(frequency, sample_rate); returns the count.
 * < 0: rfa_status. */
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processPacketNative(
    JNIEnv *env, jobject thiz, jlong handle, jbyteArray packet, jint frame_stride, jlong frequency,
    jlong sample_rate);
/* colorBuffer holds ringRows*width ARGB ints (colorBuffer[bufferIndex*width + i]);
 * peaksY may be null; autoscale holds 2 floats (min, max).  Returns rfa_status. */
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_drawPreprocessNative(
    JNIEnv *env, jobject thiz, jlong handle, jint width, jint fft_height, jlong viewport_frequency,
    jlong viewport_sample_rate, jfloat min_db, jfloat max_db, jint average_length, jintArray color_map,
    jintArray color_buffer, jfloatArray fft_path_y, jfloatArray peaks_y, jfloatArray autoscale);
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_rowWindowStatsNative(
    JNIEnv *env, jobject thiz, jlong handle, jintArray lo, jintArray hi, jfloatArray peak, jfloatArray avg);
/* Demod front end, one handle per channel; resampler: JNI_TRUE = Resampler.kt mode. */
JNIEXPORT jlong JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcCreate(JNIEnv *env, jobject thiz, jint input_format,
                                                                         jint sample_rate, jint output_rate,
                                                                         jboolean resampler, jint device);
JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcDestroy(JNIEnv *env, jobject thiz, jlong handle);
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcSetFrequencies(JNIEnv *env, jobject thiz,
                                                                                jlong handle, jlong frequency,
                                                                                jlong channel_frequency);
/* Raw packet in (format of the handle), decimated planar samples out; returns the
 * count written (SamplePacket.size) or < 0 (e.g. RFA_ERR_SIZE: re/im too short). */
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcProcess(JNIEnv *env, jobject thiz, jlong handle,
                                                                         jbyteArray packet, jfloatArray re,
                                                                         jfloatArray im);

#ifdef __cplusplus
}
#endif

#endif /* RFA_JNI_H */
