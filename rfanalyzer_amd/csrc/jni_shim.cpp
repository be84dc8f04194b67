// JNI shim: exports the reference's libnativedsp.so symbols on top of the
// rfa_* C-ABI (include/rfa_jni.h documents the mapping).
//
// Reference behaviour kept: copy-in / copy-out through Get/SetFloatArrayRegion
// (nativedsp.cpp:66,80), a cached per-size setup re-created on a size change
// (nativedsp.cpp:56-64 -- here a handle, freed instead of leaked; a mixed-radix
// plan for the lengths pffft takes and the handle does not), no return value on
// the legacy void symbols.  The new planar symbol returns JNI_FALSE on
// a size mismatch like NativeDsp.kt:45-46.
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/rfa.h"
#include "../../include/rfa_jni.h"

namespace {

// The legacy symbols share a small cache of setups keyed by (N, input format, window),
// least recently used out: alternating performFFT (f32, no window), performFFTAndLogMag and
// processIqBytesNative (raw bytes, Blackman) keeps each one's handle -- no table rebuild,
// and the framing mode's partial frame stays pending on its handle between calls.
constexpr int kCacheSlots = 4;
struct Setup {
    rfa_handle *h = nullptr;
    int n = 0, fmt = -1, win = -1;
    unsigned long long used = 0;
};
std::mutex g_mu;
Setup g_cache[kCacheSlots];
unsigned long long g_tick = 0;
int g_status = RFA_OK;  // status of the last legacy call (rfa_jni_last_status)

rfa_handle *handle_for(int n, int fmt, int window) {
    Setup *victim = &g_cache[0];
    for (Setup &s : g_cache) {
        if (s.h && s.n == n && s.fmt == fmt && s.win == window) {
            s.used = ++g_tick;
            return s.h;
        }
        if (!s.h || (victim->h && s.used < victim->used)) victim = &s;
    }
    // a length or format the handle refuses evicts nothing: a cached setup's pending
    // partial frame survives any call in between
    rfa_config c;
    rfa_default_config(&c);
    c.fft_size = n;
    c.input_format = fmt;
    c.window = window;
    c.ring_rows = 0;
    rfa_handle *h = nullptr;
    g_status = rfa_create(&c, &h);  // e.g. RFA_ERR_UNSUPPORTED for a length only a seam plan takes
    if (g_status != RFA_OK) return nullptr;
    if (victim->h) rfa_destroy(victim->h);
    *victim = Setup();
    victim->h = h;
    victim->n = n;
    victim->fmt = fmt;
    victim->win = window;
    victim->used = ++g_tick;
    return h;
}

// Lengths the handle does not take but pffft does (16, 32, 2^21 .. 2^26, mixed
// 2/3/5 lengths) go to cached plans keyed by N (nativedsp.cpp:26-33 keeps one
// setup; two slots here, so alternating two such lengths does not rebuild).
constexpr int kSeamSlots = 2;
struct SeamSlot {
    rfa_seam *s = nullptr;
    int n = 0;
    unsigned long long used = 0;
};
SeamSlot g_seams[kSeamSlots];

rfa_seam *seam_for(int n) {
    SeamSlot *victim = &g_seams[0];
    for (SeamSlot &e : g_seams) {
        if (e.s && e.n == n) {
            e.used = ++g_tick;
            return e.s;
        }
        if (!e.s || (victim->s && e.used < victim->used)) victim = &e;
    }
    rfa_seam *s = nullptr;
    g_status = rfa_seam_create(n, 0, &s);
    if (g_status != RFA_OK) return nullptr;
    if (victim->s) rfa_seam_destroy(victim->s);
    victim->s = s;
    victim->n = n;
    victim->used = ++g_tick;
    return s;
}

// the streaming handle for (n, fmt, window) when rfa_create takes n, else nullptr
// and, for a length only pffft-style plans take, *seam
rfa_handle *legacy_target(int n, int fmt, int window, rfa_seam **seam) {
    *seam = nullptr;
    if (rfa_handle *h = handle_for(n, fmt, window)) return h;
    if (g_status == RFA_ERR_UNSUPPORTED && rfa_seam_supported(n)) *seam = seam_for(n);
    return nullptr;
}

}  // namespace

extern "C" {

JNIEXPORT int rfa_jni_abi_version(void) { return RFA_JNI_ABI_VERSION; }

JNIEXPORT int rfa_jni_last_status(void) {
    std::lock_guard<std::mutex> lock(g_mu);
    return g_status;
}

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(JNIEnv *env, jobject, jfloatArray input,
                                                                          jfloatArray output) {
    const jsize length = (*env)->GetArrayLength(env, input);
    std::lock_guard<std::mutex> lock(g_mu);
    g_status = RFA_ERR_UNSUPPORTED;
    if (length <= 0 || (length & 1)) return;
    rfa_seam *sp = nullptr;
    rfa_handle *h = legacy_target(length / 2, RFA_IN_F32_INTERLEAVED, RFA_WINDOW_NONE, &sp);
    if (!h && !sp) return;
    std::vector<float> in(length), out(length);
    (*env)->GetFloatArrayRegion(env, input, 0, length, in.data());
    g_status = h ? rfa_fft_ordered(h, in.data(), out.data(), (size_t)length / 2)
                 : rfa_seam_fft_ordered(sp, in.data(), out.data(), (size_t)length / 2);
    if (g_status != RFA_OK) return;
    (*env)->SetFloatArrayRegion(env, output, 0, length, out.data());
}

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag(JNIEnv *env, jobject,
                                                                                   jfloatArray input,
                                                                                   jfloatArray output) {
    const jsize length = (*env)->GetArrayLength(env, input);
    std::lock_guard<std::mutex> lock(g_mu);
    g_status = RFA_ERR_UNSUPPORTED;
    if (length <= 0 || (length & 1)) return;
    const jsize out_len = length / 2;
    rfa_seam *sp = nullptr;
    rfa_handle *h = legacy_target(out_len, RFA_IN_F32_INTERLEAVED, RFA_WINDOW_NONE, &sp);
    if (!h && !sp) return;
    std::vector<float> in(length), mag(out_len);
    (*env)->GetFloatArrayRegion(env, input, 0, length, in.data());
    g_status = h ? rfa_fft_logmag_interleaved(h, in.data(), mag.data(), (size_t)out_len)
                 : rfa_seam_fft_logmag_interleaved(sp, in.data(), mag.data(), (size_t)out_len);
    if (g_status != RFA_OK) return;
    (*env)->SetFloatArrayRegion(env, output, 0, out_len, mag.data());
}

JNIEXPORT jboolean JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
    JNIEnv *env, jobject, jfloatArray re, jfloatArray im, jfloatArray mag_out) {
    const jsize n = (*env)->GetArrayLength(env, re);
    if ((*env)->GetArrayLength(env, im) != n || (*env)->GetArrayLength(env, mag_out) != n) {
        std::lock_guard<std::mutex> lock(g_mu);
        g_status = RFA_ERR_SIZE;
        return JNI_FALSE;
    }
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_seam *sp = nullptr;
    rfa_handle *h = legacy_target(n, RFA_IN_F32_PLANAR, RFA_WINDOW_BLACKMAN, &sp);
    if (!h && !sp) return JNI_FALSE;
    std::vector<float> r(n), i(n), m(n);
    (*env)->GetFloatArrayRegion(env, re, 0, n, r.data());
    (*env)->GetFloatArrayRegion(env, im, 0, n, i.data());
    g_status = h ? rfa_windowed_fft_mag_planar(h, r.data(), i.data(), m.data(), (size_t)n)
                 : rfa_seam_windowed_fft_mag_planar(sp, r.data(), i.data(), m.data(), (size_t)n);
    if (g_status != RFA_OK) return JNI_FALSE;
    (*env)->SetFloatArrayRegion(env, mag_out, 0, n, m.data());
    return JNI_TRUE;
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(
    JNIEnv *env, jobject, jbyteArray packet, jint format, jint fft_size, jint frame_stride, jfloatArray mag_out) {
    if (!packet || !mag_out || fft_size <= 0 || frame_stride < 0) return -1;
    const jsize bytes = (*env)->GetArrayLength(env, packet);
    const jsize out_len = (*env)->GetArrayLength(env, mag_out);
    static const int bps_tab[5] = {2, 2, 4, 8, 8};
    if (format < 0 || format > 4 || bytes < 0 || out_len < fft_size) return -1;
    std::lock_guard<std::mutex> lock(g_mu);
    rfa_handle *h = handle_for(fft_size, format, RFA_WINDOW_BLACKMAN);
    if (!h) return -1;
    g_status = RFA_OK;
    std::vector<jbyte> in((size_t)bytes);
    if (bytes) (*env)->GetByteArrayRegion(env, packet, 0, bytes, in.data());
    if (frame_stride == 0) {
        // the reference's framing (Scheduler.kt:252-273): the packet fills the cached
        // setup's partial frame; a completed frame's row goes to mag_out[0, N)
        if (format == RFA_IN_F32_PLANAR) return -1;
        std::vector<float> row((size_t)fft_size);
        int32_t frames = 0;
        if (rfa_push_packet(h, in.data(), (size_t)bytes, 0, 1, row.data(), &frames) != RFA_OK) return -1;
        if (frames) (*env)->SetFloatArrayRegion(env, mag_out, 0, fft_size, row.data());
        return frames;
    }
    // batch mode: whole frames at frame_stride bytes, as many as packet and mag_out hold
    const long long frame_bytes = (long long)fft_size * bps_tab[format];
    if (bytes < frame_bytes) return 0;
    long long n_frames = (bytes - frame_bytes) / frame_stride + 1;
    if (n_frames * fft_size > out_len) n_frames = out_len / fft_size;
    std::vector<float> rows((size_t)n_frames * fft_size);
    if (rfa_process_host(h, in.data(), (size_t)n_frames, (size_t)frame_stride, rows.data()) != RFA_OK) return -1;
    (*env)->SetFloatArrayRegion(env, mag_out, 0, (jsize)rows.size(), rows.data());
    return (jint)n_frames;
}

// ---------------------------------------------------------------- stateful natives
static rfa_handle *as_h(jlong h) { return reinterpret_cast<rfa_handle *>(static_cast<intptr_t>(h)); }
static rfa_ddc *as_d(jlong h) { return reinterpret_cast<rfa_ddc *>(static_cast<intptr_t>(h)); }

JNIEXPORT jlong JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_createAnalyzerNative(
    JNIEnv *, jobject, jint fft_size, jint input_format, jint window, jint avg_mode, jint avg_length,
    jfloat ema_alpha, jboolean peak_hold, jint ring_rows, jint device) {
    rfa_config c;
    rfa_default_config(&c);
    c.fft_size = fft_size;
    c.input_format = input_format;
    c.window = window;
    c.avg_mode = avg_mode;
    c.avg_length = avg_length;
    c.ema_alpha = ema_alpha;
    c.peak_hold = peak_hold ? 1 : 0;
    c.ring_rows = ring_rows;
    c.device_id = device;
    rfa_handle *h = nullptr;
    if (rfa_create(&c, &h) != RFA_OK) return 0;
    return static_cast<jlong>(reinterpret_cast<intptr_t>(h));
}

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_destroyAnalyzerNative(JNIEnv *, jobject, jlong handle) {
    if (handle) rfa_destroy(as_h(handle));
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_processPacketNative(
    JNIEnv *env, jobject, jlong handle, jbyteArray packet, jint frame_stride, jlong frequency, jlong sample_rate) {
    rfa_handle *h = as_h(handle);
    if (!h || !packet || frame_stride < 0) return RFA_ERR_INVALID;
    rfa_config c;
    if (rfa_get_config(h, &c) != RFA_OK) return RFA_ERR_INVALID;
    static const int bps_tab[5] = {2, 2, 4, 8, 8};
    const jsize bytes = (*env)->GetArrayLength(env, packet);
    if (bytes < 0) return RFA_ERR_INVALID;
    std::vector<jbyte> in((size_t)bytes);
    if (bytes) (*env)->GetByteArrayRegion(env, packet, 0, bytes, in.data());
    if (frame_stride == 0) {
        // Scheduler.kt:252-273: the packet fills the handle's partial frame (across
        // packets when it is shorter than a frame, the rest dropped when longer);
        // returns 1 when a frame was completed and processed, else 0
        int32_t frames = 0;
        const int rc = rfa_push_packet(h, in.data(), (size_t)bytes, frequency, sample_rate, nullptr, &frames);
        return rc != RFA_OK ? rc : frames;
    }
    // batch mode (no reference counterpart): every whole frame at frame_stride bytes;
    // a partial frame of the framing mode is left pending
    const long long frame_bytes = (long long)c.fft_size * bps_tab[c.input_format];
    if (bytes < frame_bytes) return 0;
    const long long n_frames = (bytes - frame_bytes) / frame_stride + 1;
    int rc = rfa_set_tuning(h, frequency, sample_rate);
    if (rc != RFA_OK) return rc;
    rc = rfa_process_host(h, in.data(), (size_t)n_frames, (size_t)frame_stride, nullptr);
    return rc != RFA_OK ? rc : (jint)n_frames;
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_drawPreprocessNative(
    JNIEnv *env, jobject, jlong handle, jint width, jint fft_height, jlong viewport_frequency,
    jlong viewport_sample_rate, jfloat min_db, jfloat max_db, jint average_length, jintArray color_map,
    jintArray color_buffer, jfloatArray fft_path_y, jfloatArray peaks_y, jfloatArray autoscale) {
    rfa_handle *h = as_h(handle);
    if (!h || !color_map || !color_buffer || !fft_path_y || !autoscale || width <= 0) return RFA_ERR_INVALID;
    rfa_config c;
    if (rfa_get_config(h, &c) != RFA_OK) return RFA_ERR_INVALID;
    const jsize cm = (*env)->GetArrayLength(env, color_map);
    if ((*env)->GetArrayLength(env, color_buffer) < (jsize)((long long)c.ring_rows * width) ||
        (*env)->GetArrayLength(env, fft_path_y) < width || (*env)->GetArrayLength(env, autoscale) < 2 ||
        (peaks_y && (*env)->GetArrayLength(env, peaks_y) < width) || cm <= 0)
        return RFA_ERR_SIZE;
    std::vector<jint> cmap(cm);
    (*env)->GetIntArrayRegion(env, color_map, 0, cm, cmap.data());
    rfa_draw_params p;
    std::memset(&p, 0, sizeof(p));
    p.width = width;
    p.fft_height = fft_height;
    p.viewport_frequency = viewport_frequency;
    p.viewport_sample_rate = viewport_sample_rate;
    p.min_db = min_db;
    p.max_db = max_db;
    p.average_length = average_length;
    p.colormap = reinterpret_cast<const uint32_t *>(cmap.data());
    p.colormap_size = cm;
    std::vector<uint32_t> colors((size_t)c.ring_rows * width);
    std::vector<float> path(width), pk(peaks_y ? width : 0);
    float mm[2] = {0, 0};
    const int rc = rfa_draw_preprocess(h, &p, colors.data(), path.data(), peaks_y ? pk.data() : nullptr, mm);
    if (rc != RFA_OK) return rc;
    (*env)->SetIntArrayRegion(env, color_buffer, 0, (jsize)colors.size(), reinterpret_cast<const jint *>(colors.data()));
    (*env)->SetFloatArrayRegion(env, fft_path_y, 0, width, path.data());
    if (peaks_y) (*env)->SetFloatArrayRegion(env, peaks_y, 0, width, pk.data());
    (*env)->SetFloatArrayRegion(env, autoscale, 0, 2, mm);
    return RFA_OK;
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_rowWindowStatsNative(JNIEnv *env, jobject, jlong handle,
                                                                                  jintArray lo, jintArray hi,
                                                                                  jfloatArray peak, jfloatArray avg) {
    rfa_handle *h = as_h(handle);
    if (!h || !lo || !hi || !peak || !avg) return RFA_ERR_INVALID;
    const jsize n = (*env)->GetArrayLength(env, lo);
    if ((*env)->GetArrayLength(env, hi) != n || (*env)->GetArrayLength(env, peak) < n ||
        (*env)->GetArrayLength(env, avg) < n)
        return RFA_ERR_SIZE;
    std::vector<jint> l(n), u(n);
    std::vector<float> pk(n), av(n);
    (*env)->GetIntArrayRegion(env, lo, 0, n, l.data());
    (*env)->GetIntArrayRegion(env, hi, 0, n, u.data());
    const int rc = rfa_row_window_stats(h, l.data(), u.data(), (size_t)n, pk.data(), av.data());
    if (rc != RFA_OK) return rc;
    (*env)->SetFloatArrayRegion(env, peak, 0, n, pk.data());
    (*env)->SetFloatArrayRegion(env, avg, 0, n, av.data());
    return RFA_OK;
}

JNIEXPORT jlong JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcCreate(JNIEnv *, jobject, jint input_format,
                                                                         jint sample_rate, jint output_rate,
                                                                         jboolean resampler, jint device) {
    rfa_ddc *d = nullptr;
    const int rc = resampler ? rfa_ddc_create_resampler(device, input_format, sample_rate, output_rate, &d)
                             : rfa_ddc_create(device, input_format, sample_rate, output_rate, &d);
    return rc == RFA_OK ? static_cast<jlong>(reinterpret_cast<intptr_t>(d)) : 0;
}

JNIEXPORT void JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcDestroy(JNIEnv *, jobject, jlong handle) {
    if (handle) rfa_ddc_destroy(as_d(handle));
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcSetFrequencies(JNIEnv *, jobject, jlong handle,
                                                                                jlong frequency,
                                                                                jlong channel_frequency) {
    rfa_ddc *d = as_d(handle);
    return d ? rfa_ddc_set_frequencies(d, frequency, channel_frequency) : RFA_ERR_INVALID;
}

JNIEXPORT jint JNICALL Java_com_mantz_1it_nativedsp_NativeDsp_ddcProcess(JNIEnv *env, jobject, jlong handle,
                                                                         jbyteArray packet, jfloatArray re,
                                                                         jfloatArray im) {
    rfa_ddc *d = as_d(handle);
    if (!d || !packet || !re || !im) return RFA_ERR_INVALID;
    const jsize bytes = (*env)->GetArrayLength(env, packet);
    const jsize cap = (*env)->GetArrayLength(env, re);
    if ((*env)->GetArrayLength(env, im) < cap) return RFA_ERR_SIZE;
    static const int bps_tab[4] = {2, 2, 4, 8};
    int32_t fmt = 0;  // the handle's input format gives the packet's bytes per sample
    if (rfa_ddc_get_format(d, &fmt) != RFA_OK || fmt < 0 || fmt > 3) return RFA_ERR_INVALID;
    const size_t n_samples = (size_t)bytes / bps_tab[fmt];
    std::vector<jbyte> in(bytes);
    (*env)->GetByteArrayRegion(env, packet, 0, bytes, in.data());
    std::vector<float> r((size_t)cap), q((size_t)cap);
    size_t got = 0;
    const int rc = rfa_ddc_process_host(d, in.data(), n_samples, r.data(), q.data(), (size_t)cap, &got);
    if (rc != RFA_OK) return rc;
    (*env)->SetFloatArrayRegion(env, re, 0, (jsize)got, r.data());
    (*env)->SetFloatArrayRegion(env, im, 0, (jsize)got, q.data());
    return (jint)got;
}

}  // extern "C"
