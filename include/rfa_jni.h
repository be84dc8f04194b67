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
 * Threading: like the reference (NativeDsp.kt:23-26) one caller thread per
 * library is expected; the shim additionally serialises calls with a mutex.
 */
#ifndef RFA_JNI_H
#define RFA_JNI_H

#include "../rfanalyzer_amd/csrc/jni_min.h"

#ifdef __cplusplus
extern "C" {
#endif

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(JNIEnv *env, jobject thiz,
                                                                          jfloatArray input, jfloatArray output);
JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag(JNIEnv *env, jobject thiz,
                                                                                   jfloatArray input,
                                                                                   jfloatArray output);
JNIEXPORT jboolean JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
    JNIEnv *env, jobject thiz, jfloatArray re, jfloatArray im, jfloatArray mag_out);
/* format: rfa_input_format; packet holds n_frames*fft frames at frame_stride bytes
 * (0 = dense); mag_out holds n_frames*fft floats.  Returns frames processed or -1. */
JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(
    JNIEnv *env, jobject thiz, jbyteArray packet, jint format, jint fft_size, jint frame_stride,
    jfloatArray mag_out);

#ifdef __cplusplus
}
#endif

#endif /* RFA_JNI_H */
