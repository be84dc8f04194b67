// JNI shim: exports the reference's libnativedsp.so symbols on top of the
// rfa_* C-ABI (include/rfa_jni.h documents the mapping).
//
// Reference behaviour kept: copy-in / copy-out through Get/SetFloatArrayRegion
// (nativedsp.cpp:66,80), a cached per-size setup re-created on a size change
// (nativedsp.cpp:56-64 -- here a handle, freed instead of leaked), no return
// value on the legacy void symbols.  The new planar symbol returns JNI_FALSE on
// a size mismatch like NativeDsp.kt:45-46.
#include <mutex>
#include <vector>

#include "../../include/rfa.h"
#include "../../include/rfa_jni.h"

namespace {

std::mutex g_mu;
rfa_handle *g_handle = nullptr;  // the shim's cached "setup"
int g_n = 0, g_fmt = -1, g_win = -1;

rfa_handle *handle_for(int n, int fmt, int window) {
    if (g_handle && g_n == n && g_fmt == fmt && g_win == window) return g_handle;
    if (g_handle) rfa_destroy(g_handle);
    g_handle = nullptr;
    rfa_config c;
    rfa_default_config(&c);
    c.fft_size = n;
    c.input_format = fmt;
    c.window = window;
    c.ring_rows = 0;
    if (rfa_create(&c, &g_handle) != RFA_OK) {
        g_handle = nullptr;
        g_n = 0;
        return nullptr;
    }
    g_n = n;
    g_fmt = fmt;
    g_win = window;
    return g_handle;
}

}  // namespace

extern "C" {

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(JNIEnv *env, jobject, jfloatArray input,
                                                                          jfloatArray output) {
    const jsize length = (*env)->GetArrayLength(env, input);
    if (length <= 0 || (length & 1)) return;
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_handle *h = handle_for(length / 2, RFA_IN_F32_INTERLEAVED, RFA_WINDOW_NONE);
    if (!h) return;
    std::vector<float> in(length), out(length);
    (*env)->GetFloatArrayRegion(env, input, 0, length, in.data());
    if (rfa_fft_ordered(h, in.data(), out.data(), (size_t)length / 2) != RFA_OK) return;
    (*env)->SetFloatArrayRegion(env, output, 0, length, out.data());
}

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag(JNIEnv *env, jobject,
                                                                                   jfloatArray input,
                                                                                   jfloatArray output) {
    const jsize length = (*env)->GetArrayLength(env, input);
    if (length <= 0 || (length & 1)) return;
    const jsize out_len = length / 2;
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_handle *h = handle_for(out_len, RFA_IN_F32_INTERLEAVED, RFA_WINDOW_NONE);
    if (!h) return;
    std::vector<float> in(length), mag(out_len);
    (*env)->GetFloatArrayRegion(env, input, 0, length, in.data());
    if (rfa_fft_logmag_interleaved(h, in.data(), mag.data(), (size_t)out_len) != RFA_OK) return;
    (*env)->SetFloatArrayRegion(env, output, 0, out_len, mag.data());
}

JNIEXPORT jboolean JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
    JNIEnv *env, jobject, jfloatArray re, jfloatArray im, jfloatArray mag_out) {
    const jsize n = (*env)->GetArrayLength(env, re);
    if ((*env)->GetArrayLength(env, im) != n || (*env)->GetArrayLength(env, mag_out) != n) return JNI_FALSE;
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_handle *h = handle_for(n, RFA_IN_F32_PLANAR, RFA_WINDOW_BLACKMAN);
    if (!h) return JNI_FALSE;
    std::vector<float> r(n), i(n), m(n);
    (*env)->GetFloatArrayRegion(env, re, 0, n, r.data());
    (*env)->GetFloatArrayRegion(env, im, 0, n, i.data());
    if (rfa_windowed_fft_mag_planar(h, r.data(), i.data(), m.data(), (size_t)n) != RFA_OK) return JNI_FALSE;
    (*env)->SetFloatArrayRegion(env, mag_out, 0, n, m.data());
    return JNI_TRUE;
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(
    JNIEnv *env, jobject, jbyteArray packet, jint format, jint fft_size, jint frame_stride, jfloatArray mag_out) {
    const jsize bytes = (*env)->GetArrayLength(env, packet);
    const jsize out_len = (*env)->GetArrayLength(env, mag_out);
    if (fft_size <= 0 || frame_stride < 0 || bytes <= 0) return -1;
    static const int bps_tab[5] = {2, 2, 4, 8, 8};
    if (format < 0 || format > 4) return -1;
    const long long frame_bytes = (long long)fft_size * bps_tab[format];
    const long long stride = frame_stride ? frame_stride : frame_bytes;
    if (bytes < frame_bytes) return 0;
    long long n_frames = (bytes - frame_bytes) / stride + 1;
    if (n_frames * fft_size > out_len) n_frames = out_len / fft_size;
    if (n_frames <= 0) return 0;
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_handle *h = handle_for(fft_size, format, RFA_WINDOW_BLACKMAN);
    if (!h) return -1;
    std::vector<jbyte> in(bytes);
    std::vector<float> rows((size_t)n_frames * fft_size);
    (*env)->GetByteArrayRegion(env, packet, 0, bytes, in.data());
    if (rfa_process_host(h, in.data(), (size_t)n_frames, (size_t)stride, rows.data()) != RFA_OK) return -1;
    (*env)->SetFloatArrayRegion(env, mag_out, 0, (jsize)rows.size(), rows.data());
    return (jint)n_frames;
}

}  // extern "C"
