// Host-side ASan / UBSan driver (SURVEY.md §5 sanitizers; CPU only, no GPU needed).
//
// Built by tests/sanitize/Makefile with clang -fsanitize=address,undefined against
// a librfa whose host code (engine.hip, ddc.hip, jni_shim.cpp) is compiled with the
// same sanitizers, plus the oracle's C restatement (oracle/rfa_oracle.c).  It drives:
//  * the JNI symbols through a C++ mock JNIEnv whose arrays bounds-check every
//    Get/Set*ArrayRegion (a shim that reads or writes past a Java array aborts here,
//    the way the JVM would throw): argument validation and size-mismatch paths
//    (NativeDsp.kt:45-46 returns false), null handles, bad formats, short outputs;
//  * host-only C-ABI helpers: rfa_retune_offset over extreme inputs (Kotlin's
//    saturating Float.toInt), rfa_lowpass_taps / rfa_resampler_design over a rate grid,
//    rfa_create's validation, rfa_status_string, the PacketFramer of rfa_push_packet;
//  * the oracle restatement over every format and size 64 .. 16384.
// Exit 0 = every check passed and no sanitizer report (reports abort: -fno-sanitize-recover).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <vector>

#include "../../include/rfa.h"
#include "../../include/rfa_jni.h"
#include "../../rfanalyzer_amd/csrc/framer.h"

extern "C" {
int orc_window(int n, int kind, float *w);
int orc_spectrum_rows(const void *base, int fmt, size_t n, size_t n_frames, size_t frame_stride_bytes,
                      const float *window, float *out_db);
int orc_convert(const void *frame, int fmt, size_t n, float *re, float *im);
}

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                     \
        }                                                                 \
    } while (0)

// ---------------------------------------------------------------- mock JNIEnv
struct MockArray {
    std::vector<uint8_t> data;
    size_t elem = 1;
    size_t len() const { return data.size() / elem; }
};
static std::map<void *, MockArray *> g_arrays;

static MockArray *arr(void *h) {
    auto it = g_arrays.find(h);
    if (it == g_arrays.end()) {
        std::fprintf(stderr, "JNI: unknown array handle %p\n", h);
        std::abort();
    }
    return it->second;
}
static void region(void *h, jsize start, jsize len, size_t elem) {
    MockArray *a = arr(h);
    if (a->elem != elem || start < 0 || len < 0 || (size_t)start + (size_t)len > a->len()) {
        std::fprintf(stderr, "JNI: ArrayIndexOutOfBounds (start %d len %d size %zu)\n", start, len, a->len());
        std::abort();
    }
}
static jsize JNICALL m_len(JNIEnv *, jarray a) { return (jsize)arr(a)->len(); }
template <typename T>
static void JNICALL m_get(JNIEnv *, jarray a, jsize s, jsize l, T *buf) {
    region(a, s, l, sizeof(T));
    std::memcpy(buf, arr(a)->data.data() + (size_t)s * sizeof(T), (size_t)l * sizeof(T));
}
template <typename T>
static void JNICALL m_set(JNIEnv *, jarray a, jsize s, jsize l, const T *buf) {
    region(a, s, l, sizeof(T));
    std::memcpy(arr(a)->data.data() + (size_t)s * sizeof(T), buf, (size_t)l * sizeof(T));
}
static jboolean JNICALL m_exc(JNIEnv *) { return 0; }

template <typename T>
static void *new_array(size_t n, T fill = T()) {
    MockArray *a = new MockArray;
    a->elem = sizeof(T);
    a->data.resize(n * sizeof(T));
    for (size_t i = 0; i < n; i++) std::memcpy(a->data.data() + i * sizeof(T), &fill, sizeof(T));
    g_arrays[a] = a;
    return a;
}
static void free_arrays() {
    for (auto &kv : g_arrays) delete kv.second;
    g_arrays.clear();
}

static JNINativeInterface_ g_table;
static JNIEnv g_envp = &g_table;

static void jni_checks() {
    std::memset(&g_table, 0, sizeof(g_table));
    g_table.GetArrayLength = m_len;
    g_table.GetByteArrayRegion = m_get<jbyte>;
    g_table.GetIntArrayRegion = m_get<jint>;
    g_table.GetFloatArrayRegion = m_get<jfloat>;
    g_table.SetIntArrayRegion = m_set<jint>;
    g_table.SetFloatArrayRegion = m_set<jfloat>;
    g_table.ExceptionCheck = m_exc;
    JNIEnv *env = &g_envp;
    // NativeDsp.kt:45-46: mismatched lengths -> false, before any device work
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
              env, nullptr, new_array<float>(1024), new_array<float>(1023), new_array<float>(1024)) == JNI_FALSE);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_performWindowedFftAndReturnMagNative(
              env, nullptr, new_array<float>(1024), new_array<float>(1024), new_array<float>(7)) == JNI_FALSE);
    // legacy void symbols: odd / empty inputs return without touching the output
    void *out = new_array<float>(8, 123.0f);
    Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(env, nullptr, new_array<float>(7), out);
    Java_com_mantz_1it_nativedsp_NativeDsp_performFFTAndLogMag(env, nullptr, new_array<float>(0), out);
    for (size_t i = 0; i < 8; i++) CHECK(reinterpret_cast<float *>(arr(out)->data.data())[i] == 123.0f);
    // processIqBytesNative: bad format, negative stride, short mag_out, null arrays -> -1
    void *pkt = new_array<jbyte>(4096, 1);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(env, nullptr, pkt, 7, 1024, 0,
                                                                       new_array<float>(1024)) == -1);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(env, nullptr, pkt, 0, 1024, -2,
                                                                       new_array<float>(1024)) == -1);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(env, nullptr, pkt, 0, 1024, 0,
                                                                       new_array<float>(1023)) == -1);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_processIqBytesNative(env, nullptr, nullptr, 0, 1024, 0,
                                                                       new_array<float>(1024)) == -1);
    // handle-taking natives with a null handle -> RFA_ERR_INVALID, no array access
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_processPacketNative(env, nullptr, 0, pkt, 0, 1, 1) ==
          RFA_ERR_INVALID);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_rowWindowStatsNative(env, nullptr, 0, new_array<jint>(2),
                                                                       new_array<jint>(2), new_array<float>(2),
                                                                       new_array<float>(2)) == RFA_ERR_INVALID);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_drawPreprocessNative(
              env, nullptr, 0, 100, 50, 0, 1, -100.f, 0.f, 1, new_array<jint>(4), new_array<jint>(400),
              new_array<float>(100), nullptr, new_array<float>(2)) == RFA_ERR_INVALID);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_ddcProcess(env, nullptr, 0, pkt, new_array<float>(4),
                                                             new_array<float>(4)) == RFA_ERR_INVALID);
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_ddcSetFrequencies(env, nullptr, 0, 1, 2) == RFA_ERR_INVALID);
    Java_com_mantz_1it_nativedsp_NativeDsp_destroyAnalyzerNative(env, nullptr, 0);
    Java_com_mantz_1it_nativedsp_NativeDsp_ddcDestroy(env, nullptr, 0);
    // creation without a device (or with a bad config) fails cleanly with a 0 handle
    int ndev = 0;
    rfa_device_count(&ndev);
    if (ndev == 0) {
        CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_createAnalyzerNative(env, nullptr, 1024, 0, 0, 0, 0, 0.1f, 1,
                                                                          10, 0) == 0);
        CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_ddcCreate(env, nullptr, 0, 2400000, 96000, 0, 0) == 0);
        // legacy symbols without a device: no output written, no crash
        void *o2 = new_array<float>(2048, 5.0f);
        Java_com_mantz_1it_nativedsp_NativeDsp_performFFT(env, nullptr, new_array<float>(2048), o2);
        CHECK(reinterpret_cast<float *>(arr(o2)->data.data())[0] == 5.0f);
    }
    CHECK(Java_com_mantz_1it_nativedsp_NativeDsp_createAnalyzerNative(env, nullptr, 1000, 0, 0, 0, 0, 0.1f, 1, 10,
                                                                      0) == 0);
    free_arrays();
}

// ---------------------------------------------------------------- host helpers
static void helper_checks() {
    CHECK(rfa_abi_version() == RFA_ABI_VERSION);
    for (int s = -8; s <= 0; s++) CHECK(rfa_status_string(s) != nullptr);
    rfa_config c;
    rfa_default_config(&c);
    CHECK(c.fft_size == 16384 && c.ring_rows == 400);
    rfa_handle *h = nullptr;
    c.fft_size = 1000;
    CHECK(rfa_create(&c, &h) == RFA_ERR_UNSUPPORTED && h == nullptr);
    rfa_default_config(&c);
    c.window = 9;
    CHECK(rfa_create(&c, &h) == RFA_ERR_INVALID);
    rfa_default_config(&c);
    c.avg_mode = RFA_AVG_EMA;
    c.ema_alpha = 0.f;
    CHECK(rfa_create(&c, &h) == RFA_ERR_INVALID);
    CHECK(rfa_create(nullptr, &h) == RFA_ERR_INVALID);
    CHECK(rfa_destroy(nullptr) == RFA_ERR_INVALID);
    int32_t frames = 0;
    CHECK(rfa_push_packet(nullptr, nullptr, 0, 0, 1, nullptr, &frames) == RFA_ERR_INVALID);
    // Kotlin Float.toInt(): truncating and saturating (FftProcessor.kt:143,173,199)
    const int64_t extremes[] = {0, 1, -1, INT64_MAX, INT64_MIN, 123456789, -987654321, (int64_t)1 << 40};
    for (int64_t d : extremes)
        for (int n : {64, 1024, 65536, 1 << 20})
            for (int64_t sr : {(int64_t)1, (int64_t)2000000, (int64_t)250000000, INT64_MAX}) {
                const int64_t off = rfa_retune_offset(d, n, sr);
                CHECK(off >= INT32_MIN && off <= INT32_MAX);
            }
    CHECK(rfa_retune_offset(5, 1024, 0) == 0);
    // filter design over a grid of rates (FirFilter.kt:134-195, RationalResampler.kt:165-235)
    std::vector<float> taps(1 << 16);
    for (float fs : {2.4e6f, 10e6f, 20e6f})
        for (float out : {48e3f, 96e3f, 384e3f}) {
            int32_t nt = 0;
            const int rc = rfa_lowpass_taps(1.f, fs, 0.75f * out, 0.25f * out, 60.f, 1 << 16, taps.data(), taps.size(), &nt);
            CHECK(rc == RFA_OK || rc == RFA_ERR_SIZE);
            CHECK(nt > 0);
            if (rc == RFA_OK)
                for (int i = 0; i < nt; i++) CHECK(std::isfinite(taps[i]));
            int32_t I = 0, D = 0, np = 0;
            const int r2 = rfa_resampler_design((int32_t)out, (int32_t)fs, 10000, 0.4f, 500, &I, &D, taps.data(),
                                                taps.size(), &np);
            CHECK(r2 == RFA_OK || r2 == RFA_ERR_SIZE);
            CHECK(I >= 1 && D >= 1);
        }
    int32_t nt = 0;
    CHECK(rfa_lowpass_taps(1.f, 2.4e6f, 2e6f, 1e5f, 60.f, 100, taps.data(), 4, &nt) != RFA_OK);  // cutoff > fs/2
    // the PacketFramer (Scheduler.kt:252-273): ragged packets, odd byte counts, empty packets
    rfa::PacketFramer fr;
    fr.configure(1000, 2);
    std::mt19937 rng(7);
    std::vector<uint8_t> pkt(5000);
    for (auto &b : pkt) b = (uint8_t)rng();
    size_t total = 0, frames_done = 0;
    for (int i = 0; i < 200; i++) {
        const size_t sz = rng() % 2600;
        const bool done = fr.push(pkt.data(), sz);
        total += sz / 2;
        if (done) {
            CHECK(std::memcmp(fr.data(), fr.data(), 2000) == 0);
            fr.clear();
            frames_done++;
        }
        CHECK(fr.filled() < 1000);
    }
    CHECK(frames_done > 0);
    CHECK(!fr.push(nullptr, 0) || fr.filled() == 1000);
}

// ---------------------------------------------------------------- oracle restatement
static void oracle_checks() {
    std::mt19937 rng(3);
    for (int n = 64; n <= 16384; n *= 4) {
        std::vector<float> w(n);
        CHECK(orc_window(n, 0, w.data()) == 0);
        for (int fmt = 0; fmt <= 4; fmt++) {
            const size_t bps = fmt <= 1 ? 2 : fmt == 2 ? 4 : 8;
            std::vector<uint8_t> raw(3 * n * bps);
            for (auto &b : raw) b = (uint8_t)rng();
            if (fmt >= 3) {  // finite floats only
                float *f = reinterpret_cast<float *>(raw.data());
                for (size_t i = 0; i < raw.size() / 4; i++) f[i] = (float)((int)(rng() % 2001) - 1000) / 1000.f;
            }
            std::vector<float> out(3 * n);
            CHECK(orc_spectrum_rows(raw.data(), fmt, n, 3, n * bps, w.data(), out.data()) == 0);
            for (float x : out) CHECK(!std::isnan(x));
            std::vector<float> re(n), im(n);
            CHECK(orc_convert(raw.data(), fmt, n, re.data(), im.data()) == 0);
        }
    }
}

int main() {
    jni_checks();
    helper_checks();
    oracle_checks();
    if (g_fail) {
        std::fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("sanitizer driver: all checks passed\n");
    return 0;
}
