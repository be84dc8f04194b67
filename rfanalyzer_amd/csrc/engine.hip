// librfa engine: the handle-based C-ABI of include/rfa.h.
//
// A handle is the native counterpart of one reference FftProcessor + NativeDsp
// pair (analyzer/FftProcessor.kt:64-257, nativedsp/.../NativeDsp.kt): it owns a
// HIP stream, the device-resident window and twiddle tables, the waterfall
// ring, peak-hold and EMA state, and the ring bookkeeping (writeIndex /
// readIndex / last frequency and sample rate).  No process-global state.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rfa.h"
#include "fft_kernels.h"
#include "framer.h"

static constexpr size_t kStampWords = (size_t)2048 * 16 * 8;  // RFA_STAMPS_FILE buffer: [blocks][16][8]

using rfa::FftLaunch;

struct rfa_handle {
    rfa_config cfg{};
    int n = 0, logn = 0;
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    float *d_window = nullptr;
    float *d_window_none = nullptr;   // all ones (already-windowed f32 seams)
    float *d_window_black = nullptr;  // unscaled Blackman (NativeDsp.kt seam, f32 planar)
    float *d_window_il = nullptr;     // N > 32768: scaled window as [m][j], m < 32768, j < N/32768
    float4 *d_window_cw = nullptr;    // N = 65536: (w[m] W_N^m, -w[m+M] W_N^m), residue 1 of the pre-stage
    float2 *d_wide_tw = nullptr;      // wide-kernel twiddle blob (N = 2^13..2^17, and kernel A for larger N)
    float2 *d_w64_tw = nullptr;       // N = 64 K: the wave-decoupled kernel's twiddle blob (fft_w64.hip)
    // N = 2^18..2^20 (decimation in frequency, fft_large.hip)
    float2 *d_dit_c = nullptr, *d_dit_d = nullptr;  // W_N^{m s} = C[s][m >> 7] * D[s][m & 127]
    float2 *d_dit_cp = nullptr, *d_dit_dp = nullptr;  // the pipelined 8-bit kernel's split (rfa::dif_lo_points)
    uint8_t *d_dit_in = nullptr;      // misaligned 8-bit frames, copied 16-B aligned for the pipelined kernel
    size_t d_dit_in_cap = 0;
    float2 *d_dit_y = nullptr;        // scratch z [frames][S][M] complex
    size_t d_dit_y_cap = 0;
    float *d_dit_db = nullptr;        // caller rows of a batch, residue-major, before cols_to_rows
    size_t d_dit_db_cap = 0;
    int dit_frames = 1;               // frames per kernel-A/B pair (scratch <= kDitScratch)
    int dif_pipe = 6;                 // frame groups of the pipelined front kernel (8-bit input)
    hipStream_t dif_stream2 = nullptr;  // A/B builds (RFA_DIF_SPLIT): second stream of the split batch
    hipEvent_t *dif_split_ev = nullptr; // [2]: first half's kernel A done, second half done
    int variant = 0;                  // 1: the narrow kernel (A/B builds: RFA_KERNEL=narrow)
    int stage = 1;                    // LDS-DMA staged input in the wide kernel (A/B builds: RFA_STAGE=0 off)
    // profiling / ablation hooks, set only by A/B builds (-DRFA_AB_BUILD, scripts/build_variant.sh);
    // the product library reads no environment and never takes these paths
    std::string stamps_file;          // RFA_STAMPS_FILE: phase stamps appended per launch
    unsigned long long *d_stamps = nullptr;
    int diag = 0;                     // RFA_DIAG ablation variant
    int phase_ticks = 0;              // RFA_PHASE_NS (A/B builds)
    int ring_logrs = 0;               // ring row order (fft_kernels.h ring_pos): residue split of the main kernel
    float2 *d_twc = nullptr, *d_twf = nullptr;
    int tw_shift = 0;
    float *d_ring = nullptr, *d_ring_tmp = nullptr;
    int ring_rows = 0;
    int pending_ring_rows = -1;       // rfa_set_ring_rows: applied when the next frame arrives
    int write_index = 0, read_index = 0;
    bool have_rows = false;  // at least one row pushed since the last reset
    float *d_peaks = nullptr;
    float *d_ema = nullptr;
    float4 *d_state_part = nullptr;   // chunked state update: [state_chunks][n]
    int state_chunks = 1;
    int state_fused = 1;              // single-launch chunked scan (A/B builds: RFA_STATE_FUSED=0 two kernels)
    // pipelined state (rfa_set_pipelined): the state pass on a CU-masked stream,
    // the FFT kernels on two CU-masked streams over the other CUs (alternating per call), so call
    // k's pass runs under call k + 1's FFT
    int pipe_cus = 0;                       // CUs of the state stream (0: off)
    int pipe_fft_cus = 0;                   // CUs of the FFT streams (their persistent grids)
    hipStream_t pipe_fft[2] = {nullptr, nullptr};
    hipStream_t pipe_state = nullptr;
    hipEvent_t pipe_in = nullptr;           // handle stream -> FFT stream: the call's input is ready
    hipEvent_t pipe_fft_done[2] = {nullptr, nullptr};    // by call parity
    hipEvent_t pipe_state_done[2] = {nullptr, nullptr};
    bool pipe_recorded[2] = {false, false};
    long long pipe_k = 0;                   // pipelined calls (parity: FFT stream and ring buffer)
    int pipe_prev_frames = 0;               // frames of the last pipelined call while it is not joined
    bool pipe_pending = false;              // pipelined work the handle stream is not ordered after
    float *d_boxcar = nullptr;
    bool have_tuning = false;
    // channel mean (FftProcessor.kt:143-157)
    bool chan_on = false;
    int64_t chan_start = 0, chan_end = 0;
    float *d_chan = nullptr;
    size_t d_chan_cap = 0;
    void *d_draw = nullptr;           // rfa_draw_preprocess: colormap, averages, outputs, row list
    size_t d_draw_cap = 0;
    // the draw thread's persistent state (AnalyzerSurface.kt:619-640,678-684,735):
    // colour buffer, dirty map (FftProcessorData.waterfallBufferDirtyMap), last viewport
    unsigned *d_colors = nullptr;
    int colors_rows = 0, colors_width = 0;
    std::vector<uint8_t> dirty;
    bool have_view = false;
    int64_t view_frequency = 0, view_sample_rate = 0;
    float view_min_db = 0.f, view_max_db = 0.f;
    size_t chan_count = 0;
    size_t chan_offset = 0;           // first frame of the means rfa_get_channel_means returns (packed batches: the last batch)
    int64_t last_frequency = 0, last_sample_rate = 0;
    // rfa_push_packet: the partial SamplePacket Scheduler.run fills across packets
    rfa::PacketFramer framer;
    int64_t generation = 0;           // rfa_get_state_generation: device state pointers changed
    // staging for host-pointer entry points / state without a row buffer
    void *d_in = nullptr;
    size_t d_in_cap = 0;
    float *d_rows = nullptr;
    size_t d_rows_cap = 0;
    void *h_pinned = nullptr;
    size_t h_pinned_cap = 0;
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    double kernel_ms = 0.0;
    int64_t launches = 0;
    std::string err;
};

namespace {

constexpr float kRingFill = -9999.0f;     // FftProcessor.kt:180
constexpr float kPeakFill = -999999.0f;   // FftProcessor.kt:235

int fail(rfa_handle *h, int code, const std::string &msg) {
    if (h) h->err = msg;
    return code;
}

int hip_fail(rfa_handle *h, hipError_t e, const char *where) {
    return fail(h, RFA_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIPCHK(h, expr)                                      \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail((h), _e, #expr); \
    } while (0)

int ilog2_exact(int n) {
    if (n <= 0) return -1;
    int l = 0;
    while ((1 << l) < n) l++;
    return (1 << l) == n ? l : -1;
}

size_t bytes_per_sample(int fmt) {
    switch (fmt) {
    case RFA_IN_S8:
    case RFA_IN_U8: return 2;
    case RFA_IN_S16LE: return 4;
    case RFA_IN_F32_INTERLEAVED:
    case RFA_IN_F32_PLANAR: return 8;
    default: return 0;
    }
}

size_t load_alignment(int fmt) {
    switch (fmt) {
    case RFA_IN_S8:
    case RFA_IN_U8: return 2;
    case RFA_IN_S16LE: return 4;
    case RFA_IN_F32_INTERLEAVED: return 8;
    default: return 4;
    }
}

// NativeDsp.kt:14-21: Blackman in double, cast once; Hann with the same (N-1) convention.
std::vector<float> make_window(int n, int kind) {
    std::vector<float> w(n);
    for (int i = 0; i < n; i++) {
        const double x = 2.0 * M_PI * (double)i / (double)(n - 1);
        double v = 1.0;
        if (kind == RFA_WINDOW_BLACKMAN) v = 0.42 - 0.5 * std::cos(x) + 0.08 * std::cos(2.0 * x);
        else if (kind == RFA_WINDOW_HANN) v = 0.5 - 0.5 * std::cos(x);
        w[i] = (float)v;
    }
    return w;
}

int ensure_device_buffer(rfa_handle *h, void **p, size_t *cap, size_t bytes) {
    if (*cap >= bytes) return RFA_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) return fail(h, RFA_ERR_NOMEM, "hipMalloc staging");
    *cap = bytes;
    return RFA_OK;
}

int ensure_pinned(rfa_handle *h, size_t bytes) {
    if (h->h_pinned_cap >= bytes) return RFA_OK;
    if (h->h_pinned) hipHostFree(h->h_pinned);
    h->h_pinned = nullptr;
    h->h_pinned_cap = 0;
    if (hipHostMalloc(&h->h_pinned, bytes, hipHostMallocDefault) != hipSuccess)
        return fail(h, RFA_ERR_NOMEM, "hipHostMalloc staging");
    h->h_pinned_cap = bytes;
    return RFA_OK;
}

int set_device(rfa_handle *h) {
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    return RFA_OK;
}

// Collect finished profiling event pairs.
void drain_events(rfa_handle *h, bool wait) {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> keep;
    for (auto &pr : h->ev_pending) {
        if (wait) hipEventSynchronize(pr.second);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
            h->kernel_ms += ms;
            h->launches++;
            h->ev_pool.push_back(pr.first);
            h->ev_pool.push_back(pr.second);
        } else {
            keep.push_back(pr);
        }
    }
    h->ev_pending.swap(keep);
}

hipEvent_t get_event(rfa_handle *h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
}

// N = 2^18..2^20: kernel A (column DFT-S + twiddle, complex scratch z) + kernel B
// (the 32 K-point wide kernel on each z_s: dB rows / ring / complex out), in
// batches of dit_frames frames so the scratch stays cache resident.
static hipError_t launch_large(rfa_handle *h, const FftLaunch &a) {
    const int n = h->n, s = n >> rfa::kDitLogM;
    for (int f0 = 0; f0 < a.n_frames; f0 += h->dit_frames) {
        const int cnt = std::min(h->dit_frames, a.n_frames - f0);
        rfa::DifLaunch A;
        A.in = a.in + (size_t)f0 * (size_t)a.frame_stride;
        A.frame_stride = a.frame_stride;
        A.n_frames = cnt;
        A.fmt = a.fmt;
        A.logn = h->logn;
        A.window = a.window;  // natural order: the scaled window or a seam window
        A.tw_c = h->d_dit_c;
        A.tw_d = h->d_dit_d;
        A.tw_cp = h->d_dit_cp;
        A.tw_dp = h->d_dit_dp;
        A.pipe = h->dif_pipe;  // (the staging below is for the pipelined kernel only)
        if (A.pipe > 0 && A.fmt <= 1 && ((reinterpret_cast<uintptr_t>(A.in) | (uintptr_t)A.frame_stride) & 15) != 0) {
            // misaligned 8-bit frames: an aligned copy, so every 8-bit frame takes the same kernel
            // (and the same rounding) whatever the caller's pointer
            const size_t fb = (size_t)n * 2;
            if (ensure_device_buffer(h, (void **)&h->d_dit_in, &h->d_dit_in_cap, (size_t)h->dit_frames * fb))
                return hipErrorOutOfMemory;
            // (one frame: its stride is not validated against the frame size and is not used)
            const size_t sp = cnt > 1 ? (size_t)A.frame_stride : fb;
            hipError_t e = hipMemcpy2DAsync(h->d_dit_in, fb, A.in, sp, fb, cnt, hipMemcpyDeviceToDevice, a.stream);
            if (e != hipSuccess) return e;
            A.in = h->d_dit_in;
            A.frame_stride = (long long)fb;
        }
        // one kernel pair over frames [g0, g0 + gc) of this batch on stream st (scratch z and the
        // row scratch are frame-major, so disjoint frame ranges use disjoint scratch)
        auto pair = [&](int g0, int gc, hipStream_t st) -> hipError_t {
            rfa::DifLaunch Ah = A;
            Ah.in = A.in + (size_t)g0 * (size_t)A.frame_stride;
            Ah.n_frames = gc;
            Ah.z = h->d_dit_y + (size_t)g0 * n;
            Ah.stream = st;
            hipError_t e = rfa::launch_dif_front(Ah);
            if (e != hipSuccess) return e;
            if (st == a.stream && h->dif_split_ev) {  // (A/B split: the second half's kernel A may start now)
                e = hipEventRecord(h->dif_split_ev[0], st);
                if (e != hipSuccess) return e;
            }
#ifdef RFA_DIT_FLUSH_MB
            {  // A/B builds only: evict the scratch z from the Infinity Cache before kernel B
                static void *flush = nullptr;
                if (!flush && hipMalloc(&flush, (size_t)RFA_DIT_FLUSH_MB << 20) != hipSuccess) return hipErrorOutOfMemory;
                e = hipMemsetAsync(flush, f0 & 0xff, (size_t)RFA_DIT_FLUSH_MB << 20, st);
                if (e != hipSuccess) return e;
            }
#endif
            FftLaunch B = a;
            B.stream = st;
            B.in = reinterpret_cast<const uint8_t *>(h->d_dit_y + (size_t)g0 * n);
            B.frame_stride = (long long)n * (long long)sizeof(float2);
            B.n_frames = gc;
            B.fmt = rfa::kFmtDif;
            B.dif_ss = s;
            B.window = nullptr;
            B.window_il = nullptr;
            B.rows = a.rows ? h->d_dit_db + (size_t)g0 * n : nullptr;
            B.complex_out = a.complex_out ? a.complex_out + (size_t)(f0 + g0) * n : nullptr;
            B.ring_base = a.ring_base - (f0 + g0);  // frame f0 + g0 + f of the call is frame f of this pair
            B.ring_first = a.ring_first - (f0 + g0);
            B.stage = h->stage;  // kernel B stages half of its next item's z_s (fft_wide.hip QSTB)
            B.diag = 0;
            B.stamps = nullptr;
            e = rfa::launch_fft_wide(B);
            if (e != hipSuccess) return e;
            if (a.rows) e = rfa::launch_cols_to_rows(h->d_dit_db + (size_t)g0 * n, a.rows + (size_t)(f0 + g0) * n, gc, h->logn, st);
            return e;
        };
        hipError_t e = hipSuccess;
        if (h->dif_split_ev && cnt >= 2) {
            // A/B builds (RFA_DIF_SPLIT): the batch in two halves, the second on its own stream once
            // the first half's kernel A is done, so its kernel A runs beside the first half's kernel B
            const int h1 = cnt / 2;
            e = pair(0, h1, a.stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(h->dif_stream2, h->dif_split_ev[0], 0);
            if (e == hipSuccess) e = pair(h1, cnt - h1, h->dif_stream2);
            if (e == hipSuccess) e = hipEventRecord(h->dif_split_ev[1], h->dif_stream2);
            if (e == hipSuccess) e = hipStreamWaitEvent(a.stream, h->dif_split_ev[1], 0);
        } else {
            e = pair(0, cnt, a.stream);
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int launch_main(rfa_handle *h, FftLaunch &a, hipStream_t st) {
    a.stream = st;
    a.logn = h->logn;
    a.tw_coarse = h->d_twc;
    a.tw_fine = h->d_twf;
    a.tw_shift = h->tw_shift;
    a.diag = h->diag;
    a.phase_ticks = h->phase_ticks;
    a.stage = h->stage;
    if (h->d_stamps) {
        a.diag |= 32;  // phase stamps (+ RFA_DIAG 16: without window loads)
        a.stamps = h->d_stamps;
    }
    a.wide_tw = h->d_wide_tw;
    a.w64_tw = h->d_w64_tw;
    a.variant = h->variant;
    if (a.window == h->d_window) {
        a.window_il = h->d_window_il;
        a.window_cw = h->d_window_cw;
    }
    else if (h->logn > 14) a.variant = 1;  // seam windows have no interleaved copy: narrow kernel
    // the ring order is a property of the wide kernel's residue split (ring_pos)
    if (a.ring && h->ring_logrs && a.variant == 1 && h->logn <= 17)
        return fail(h, RFA_ERR_INVALID, "ring order needs the wide kernel");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->profile) {
        // collect finished pairs without blocking; block (oldest first) only when far behind
        if (h->ev_pending.size() > 512) drain_events(h, false);
        if (h->ev_pending.size() > 4096) drain_events(h, true);
        e0 = get_event(h);
        e1 = get_event(h);
        hipEventRecord(e0, st);
    }
    hipError_t e = hipSuccess;
    if (h->logn > 17) {
        const size_t need = (size_t)std::min(h->dit_frames, a.n_frames) * h->n * sizeof(float2);
        if (need > h->d_dit_y_cap) {
            hipFree(h->d_dit_y);
            h->d_dit_y = nullptr;
            h->d_dit_y_cap = 0;
            if (hipMalloc(&h->d_dit_y, need) != hipSuccess) return fail(h, RFA_ERR_NOMEM, "large-N scratch");
            h->d_dit_y_cap = need;
        }
        if (a.rows && need / 2 > h->d_dit_db_cap) {
            hipFree(h->d_dit_db);
            h->d_dit_db = nullptr;
            h->d_dit_db_cap = 0;
            if (hipMalloc(&h->d_dit_db, need / 2) != hipSuccess) return fail(h, RFA_ERR_NOMEM, "large-N row scratch");
            h->d_dit_db_cap = need / 2;
        }
        e = launch_large(h, a);
    } else {
        e = rfa::launch_fft(a);
    }
    if (h->profile) {
        hipEventRecord(e1, st);
        h->ev_pending.emplace_back(e0, e1);
    }
    if (e != hipSuccess) return hip_fail(h, e, "launch_fft");
    if (a.stamps) {  // profiling only: synchronous dump of this launch's phase stamps
        std::vector<unsigned long long> sv((size_t)kStampWords);
        if (hipMemcpyAsync(sv.data(), a.stamps, sv.size() * 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            if (FILE *f = std::fopen(h->stamps_file.c_str(), "ab")) {
                std::fwrite(sv.data(), 8, sv.size(), f);
                std::fclose(f);
            }
        }
        hipMemsetAsync(a.stamps, 0, sv.size() * 8, st);
    }
    return RFA_OK;
}

int clear_ring(rfa_handle *h) {
    std::fill(h->dirty.begin(), h->dirty.end(), 1);  // FftProcessor.kt:215,219
    if (!h->d_ring) return RFA_OK;
    HIPCHK(h, rfa::launch_fill(h->d_ring, (long long)h->ring_rows * h->n, kRingFill, h->stream));
    return RFA_OK;
}

int reset_peaks_ema(rfa_handle *h) {
    if (h->d_peaks) HIPCHK(h, rfa::launch_fill(h->d_peaks, h->n, kPeakFill, h->stream));
    if (h->d_ema) HIPCHK(h, rfa::launch_fill(h->d_ema, h->n, -INFINITY, h->stream));
    return RFA_OK;
}

// Order the handle stream after every pipelined kernel so far (rfa_join).  Every entry point
// but a pipelined rfa_process joins first, so only pipelined calls overlap one another.
int join(rfa_handle *h) {
    if (!h->pipe_pending) return RFA_OK;
    for (int p = 0; p < 2; p++) {
        if (!h->pipe_recorded[p]) continue;
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->pipe_fft_done[p], 0));
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->pipe_state_done[p], 0));
    }
    h->pipe_pending = false;
    h->pipe_prev_frames = 0;
    return RFA_OK;
}

void pipe_release(rfa_handle *h) {
    for (hipStream_t *s : {&h->pipe_fft[0], &h->pipe_fft[1], &h->pipe_state}) {
        if (*s) hipStreamSynchronize(*s), hipStreamDestroy(*s);
        *s = nullptr;
    }
    for (hipEvent_t *e : {&h->pipe_in, &h->pipe_fft_done[0], &h->pipe_fft_done[1], &h->pipe_state_done[0],
                          &h->pipe_state_done[1]}) {
        if (*e) hipEventDestroy(*e);
        *e = nullptr;
    }
    h->pipe_recorded[0] = h->pipe_recorded[1] = false;
    h->pipe_cus = h->pipe_fft_cus = 0;
    h->pipe_pending = false;
    h->pipe_prev_frames = 0;
}

}  // namespace

extern "C" {

int rfa_abi_version(void) { return RFA_ABI_VERSION; }

int rfa_device_count(int *count) {
    if (!count) return RFA_ERR_INVALID;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return RFA_OK;
}

const char *rfa_status_string(int status) {
    switch (status) {
    case RFA_OK: return "ok";
    case RFA_ERR_INVALID: return "invalid argument";
    case RFA_ERR_SIZE: return "size mismatch";
    case RFA_ERR_UNSUPPORTED: return "unsupported";
    case RFA_ERR_NODEVICE: return "no HIP device";
    case RFA_ERR_NOMEM: return "out of memory";
    case RFA_ERR_HIP: return "HIP runtime error";
    case RFA_ERR_STATE: return "feature not enabled";
    default: return "unknown status";
    }
}

void rfa_default_config(rfa_config *c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->fft_size = 16384;  // AppStateRepository.kt:196
    c->window = RFA_WINDOW_BLACKMAN;
    c->input_format = RFA_IN_S8;
    c->avg_mode = RFA_AVG_NONE;
    c->avg_length = 0;  // AppStateRepository.kt:197
    c->ema_alpha = 0.1f;
    c->peak_hold = 0;     // AppStateRepository.kt:198
    c->ring_rows = 400;   // waterfallSpeed NORMAL, FftProcessor.kt:103
    c->device_id = 0;
}

int rfa_create(const rfa_config *cfg, rfa_handle **out) {
    if (!cfg || !out) return RFA_ERR_INVALID;
    *out = nullptr;
    const int logn = ilog2_exact(cfg->fft_size);
    if (logn < 0 || cfg->fft_size < RFA_MIN_FFT_SIZE || cfg->fft_size > RFA_MAX_FFT_SIZE) return RFA_ERR_UNSUPPORTED;
    if (logn > rfa::kMaxLogN) return RFA_ERR_UNSUPPORTED;
    if (cfg->window < 0 || cfg->window > RFA_WINDOW_NONE) return RFA_ERR_INVALID;
    if (bytes_per_sample(cfg->input_format) == 0) return RFA_ERR_INVALID;
    if (cfg->avg_mode < RFA_AVG_NONE || cfg->avg_mode > RFA_AVG_EMA) return RFA_ERR_INVALID;
    if (cfg->avg_mode == RFA_AVG_EMA && !(cfg->ema_alpha > 0.f && cfg->ema_alpha <= 1.f)) return RFA_ERR_INVALID;
    if (cfg->ring_rows < 0 || cfg->avg_length < 0) return RFA_ERR_INVALID;
    if (cfg->avg_mode == RFA_AVG_BOXCAR && cfg->avg_length >= std::max(cfg->ring_rows, 1)) return RFA_ERR_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RFA_ERR_NODEVICE;
    if (cfg->device_id < 0 || cfg->device_id >= ndev) return RFA_ERR_NODEVICE;

    rfa_handle *h = new (std::nothrow) rfa_handle();
    if (!h) return RFA_ERR_NOMEM;
    h->cfg = *cfg;
    h->n = cfg->fft_size;
    h->logn = logn;
    h->device = cfg->device_id;
    h->ring_rows = cfg->ring_rows;
    h->framer.configure((size_t)h->n, bytes_per_sample(cfg->input_format));
    int rc = set_device(h);
    if (rc) { delete h; return rc; }
    auto bail = [&](int code) { rfa_destroy(h); return code; };
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) return bail(RFA_ERR_HIP);
    h->stream = h->own_stream;

    const int n = h->n;
    // window tables; the converter's power-of-two scale (1/128 for 8-bit,
    // 1/32768 for 16-bit) is folded in exactly (scaling commutes with rounding)
    std::vector<float> w = make_window(n, cfg->window), ones(n, 1.0f), black = make_window(n, RFA_WINDOW_BLACKMAN);
    const float scale = (cfg->input_format == RFA_IN_S8 || cfg->input_format == RFA_IN_U8) ? 1.0f / 128.0f
                        : cfg->input_format == RFA_IN_S16LE                                ? 1.0f / 32768.0f
                                                                                           : 1.0f;
    for (float &x : w) x *= scale;
    float **tabs[3] = {&h->d_window, &h->d_window_none, &h->d_window_black};
    const float *src[3] = {w.data(), ones.data(), black.data()};
    for (int i = 0; i < 3; i++) {
        if (hipMalloc(tabs[i], n * sizeof(float)) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMemcpy(*tabs[i], src[i], n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return bail(RFA_ERR_HIP);
    }
    const int m_sub = 1 << rfa::wide_logm(logn);
    if (n > m_sub && logn <= 17) {  // interleaved copy for the wide kernel's decimation-in-frequency pre-stage
        const int rs = n / m_sub;
        std::vector<float> il(n);
        for (int m = 0; m < m_sub; m++)
            for (int j = 0; j < rs; j++) il[(size_t)m * rs + j] = w[(size_t)m + (size_t)j * m_sub];
        if (hipMalloc(&h->d_window_il, n * sizeof(float)) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMemcpy(h->d_window_il, il.data(), n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
            return bail(RFA_ERR_HIP);
        if (rs == 2) {  // residue 1's complex window (fft_wide.hip prestage CW): products in double, rounded once
            const std::vector<float> wd = make_window(n, cfg->window);
            std::vector<float4> cw((size_t)m_sub);
            for (int m = 0; m < m_sub; m++) {
                const double sc = (double)scale, ang = -2.0 * M_PI * (double)m / (double)n;
                const double c = std::cos(ang), s = std::sin(ang);
                const double w0 = (double)wd[m] * sc, w1 = (double)wd[(size_t)m + m_sub] * sc;
                cw[m] = make_float4((float)(w0 * c), (float)(w0 * s), (float)(-w1 * c), (float)(-w1 * s));
            }
            if (hipMalloc(&h->d_window_cw, cw.size() * sizeof(float4)) != hipSuccess) return bail(RFA_ERR_NOMEM);
            if (hipMemcpy(h->d_window_cw, cw.data(), cw.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess)
                return bail(RFA_ERR_HIP);
        }
    }
    if (logn > 17) {  // decimation in frequency: S column DFTs, then S sub-FFTs of M = 32768 points
        std::vector<float2> c, d, cp, dp, blob = rfa::wide_twiddles(rfa::kDitLogM, rfa::kWidePT, rfa::kDitLogM);
        rfa::dif_twiddles(logn, rfa::dif_lo_points(false), c, d);
        rfa::dif_twiddles(logn, rfa::dif_lo_points(true), cp, dp);
        struct { void **dst; const void *src; size_t bytes; } up[] = {
            {(void **)&h->d_dit_c, c.data(), c.size() * sizeof(float2)},
            {(void **)&h->d_dit_d, d.data(), d.size() * sizeof(float2)},
            {(void **)&h->d_dit_cp, cp.data(), cp.size() * sizeof(float2)},
            {(void **)&h->d_dit_dp, dp.data(), dp.size() * sizeof(float2)},
            {(void **)&h->d_wide_tw, blob.data(), blob.size() * sizeof(float2)}};
        for (auto &u : up) {
            if (hipMalloc(u.dst, u.bytes) != hipSuccess) return bail(RFA_ERR_NOMEM);
            if (hipMemcpy(*u.dst, u.src, u.bytes, hipMemcpyHostToDevice) != hipSuccess) return bail(RFA_ERR_HIP);
        }
        // scratch per kernel pair <= 128 MB so it stays in the 256 MB Infinity Cache
        const size_t mb = 128;
        h->dit_frames = (int)std::max<size_t>(1, (mb << 20) / ((size_t)n * sizeof(float2)));
    }
    if (logn == 16 && rfa::w64_format(cfg->input_format)) {
        std::vector<float2> blob = rfa::w64_twiddles();
        if (hipMalloc(&h->d_w64_tw, blob.size() * sizeof(float2)) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMemcpy(h->d_w64_tw, blob.data(), blob.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess)
            return bail(RFA_ERR_HIP);
    }
    if (rfa::wide_supported(logn)) {
        std::vector<float2> blob = rfa::wide_twiddles(logn, rfa::kWidePT, rfa::wide_logm(logn));
        if (hipMalloc(&h->d_wide_tw, blob.size() * sizeof(float2)) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMemcpy(h->d_wide_tw, blob.data(), blob.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess)
            return bail(RFA_ERR_HIP);
    }
#ifdef RFA_AB_BUILD
    // A/B and profiling builds only (scripts/build_variant.sh): ablation switches
    if (const char *d = std::getenv("RFA_KERNEL")) h->variant = std::string(d) == "narrow" ? 1 : 0;
    if (const char *d = std::getenv("RFA_DIAG")) h->diag = std::atoi(d);
    if (const char *d = std::getenv("RFA_PHASE_NS")) h->phase_ticks = std::atoi(d) / 10;
    if (const char *d = std::getenv("RFA_DIF_PIPE")) h->dif_pipe = std::max(0, std::atoi(d));
    if (const char *d = std::getenv("RFA_DIF_SPLIT"); d && std::atoi(d) && logn > 17) {
        h->dif_split_ev = new hipEvent_t[2];
        if (hipStreamCreateWithFlags(&h->dif_stream2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&h->dif_split_ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&h->dif_split_ev[1], hipEventDisableTiming) != hipSuccess)
            return bail(RFA_ERR_HIP);
    }
    if (const char *d = std::getenv("RFA_STAGE")) h->stage = std::atoi(d);
    if (const char *d = std::getenv("RFA_STAMPS_FILE")) {
        h->stamps_file = d;
        if (hipMalloc(&h->d_stamps, kStampWords * 8) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMemset(h->d_stamps, 0, kStampWords * 8) != hipSuccess) return bail(RFA_ERR_HIP);
    }
#endif
    // ring row order: residue-major when the main kernel splits N into residue
    // sub-FFTs (whole-line stores per workgroup), natural otherwise
    if (h->variant != 1 || logn > 17) h->ring_logrs = rfa::ring_logrs_for(logn, cfg->input_format);
    // two-level twiddle table W_N^s = C[s >> sh] * F[s & (2^sh - 1)], both correctly
    // rounded from double (no device sin/cos)
    h->tw_shift = (logn + 1) / 2;
    const int nc = n >> h->tw_shift, nf = 1 << h->tw_shift;
    std::vector<float2> tc(nc), tf(nf);
    for (int c = 0; c < nc; c++) {
        const double a = -2.0 * M_PI * (double)((long long)c << h->tw_shift) / (double)n;
        tc[c] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    for (int f = 0; f < nf; f++) {
        const double a = -2.0 * M_PI * (double)f / (double)n;
        tf[f] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    if (hipMalloc(&h->d_twc, nc * sizeof(float2)) != hipSuccess) return bail(RFA_ERR_NOMEM);
    if (hipMalloc(&h->d_twf, nf * sizeof(float2)) != hipSuccess) return bail(RFA_ERR_NOMEM);
    if (hipMemcpy(h->d_twc, tc.data(), nc * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) return bail(RFA_ERR_HIP);
    if (hipMemcpy(h->d_twf, tf.data(), nf * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) return bail(RFA_ERR_HIP);
    // state
    h->dirty.assign((size_t)std::max(h->ring_rows, 0), 1);  // FftProcessor.kt:181
    if (h->ring_rows > 0) {
        const size_t bytes = (size_t)h->ring_rows * n * sizeof(float);
        if (hipMalloc(&h->d_ring, bytes) != hipSuccess) return bail(RFA_ERR_NOMEM);
        if (hipMalloc(&h->d_ring_tmp, bytes) != hipSuccess) return bail(RFA_ERR_NOMEM);
    }
    if (cfg->peak_hold && hipMalloc(&h->d_peaks, n * sizeof(float)) != hipSuccess) return bail(RFA_ERR_NOMEM);
    if (cfg->avg_mode == RFA_AVG_EMA && hipMalloc(&h->d_ema, n * sizeof(float)) != hipSuccess) return bail(RFA_ERR_NOMEM);
    if (h->d_peaks || h->d_ema) {
        // enough (bin, chunk) threads to fill the chip (~2^19) for large batches
        h->state_chunks = (int)std::min<size_t>(32, std::max<size_t>(1, ((size_t)1 << 20) / n));
#ifdef RFA_AB_BUILD
        if (const char *d = std::getenv("RFA_STATE_CHUNKS")) h->state_chunks = std::max(1, std::min(64, std::atoi(d)));
        if (const char *d = std::getenv("RFA_STATE_FUSED")) h->state_fused = std::atoi(d);
#endif
        if (h->state_chunks > 1 &&
            hipMalloc(&h->d_state_part, (size_t)h->state_chunks * n * sizeof(float4)) != hipSuccess)
            return bail(RFA_ERR_NOMEM);
    }
    if (hipMalloc(&h->d_boxcar, n * sizeof(float)) != hipSuccess) return bail(RFA_ERR_NOMEM);
    if (clear_ring(h) || reset_peaks_ema(h)) return bail(RFA_ERR_HIP);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(RFA_ERR_HIP);
    *out = h;
    return RFA_OK;
}

int rfa_destroy(rfa_handle *h) {
    if (!h) return RFA_ERR_INVALID;
    hipSetDevice(h->device);
    pipe_release(h);  // synchronises the pipelined streams
    if (h->dif_split_ev) {
        hipStreamSynchronize(h->dif_stream2);
        hipStreamDestroy(h->dif_stream2);
        hipEventDestroy(h->dif_split_ev[0]);
        hipEventDestroy(h->dif_split_ev[1]);
        delete[] h->dif_split_ev;
    }
    if (h->stream) hipStreamSynchronize(h->stream);
    for (auto &pr : h->ev_pending) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
    for (auto e : h->ev_pool) hipEventDestroy(e);
    hipFree(h->d_stamps);
    hipFree(h->d_window);
    hipFree(h->d_window_none);
    hipFree(h->d_window_black);
    hipFree(h->d_window_il);
    hipFree(h->d_window_cw);
    hipFree(h->d_wide_tw);
    hipFree(h->d_w64_tw);
    hipFree(h->d_dit_c);
    hipFree(h->d_dit_d);
    hipFree(h->d_dit_cp);
    hipFree(h->d_dit_dp);
    hipFree(h->d_dit_in);
    hipFree(h->d_dit_y);
    hipFree(h->d_dit_db);
    hipFree(h->d_twc);
    hipFree(h->d_twf);
    hipFree(h->d_ring);
    hipFree(h->d_ring_tmp);
    hipFree(h->d_peaks);
    hipFree(h->d_ema);
    hipFree(h->d_state_part);
    hipFree(h->d_chan);
    hipFree(h->d_draw);
    hipFree(h->d_colors);
    hipFree(h->d_boxcar);
    hipFree(h->d_in);
    hipFree(h->d_rows);
    if (h->h_pinned) hipHostFree(h->h_pinned);
    if (h->own_stream) hipStreamDestroy(h->own_stream);
    delete h;
    return RFA_OK;
}

int rfa_get_config(const rfa_handle *h, rfa_config *cfg) {
    if (!h || !cfg) return RFA_ERR_INVALID;
    *cfg = h->cfg;
    return RFA_OK;
}

const char *rfa_last_error(const rfa_handle *h) { return h ? h->err.c_str() : "null handle"; }

int rfa_set_stream(rfa_handle *h, void *stream) {
    if (!h) return RFA_ERR_INVALID;
    if (int rc = set_device(h)) return rc;
    if (int rc = join(h)) return rc;  // the old stream is ordered after the pipelined calls
    h->stream = (hipStream_t)stream;
    return RFA_OK;
}

int rfa_use_own_stream(rfa_handle *h) {
    if (!h) return RFA_ERR_INVALID;
    if (int rc = set_device(h)) return rc;
    if (int rc = join(h)) return rc;
    h->stream = h->own_stream;
    return RFA_OK;
}

int rfa_get_stream(const rfa_handle *h, void **stream) {
    if (!h || !stream) return RFA_ERR_INVALID;
    *stream = (void *)h->stream;
    return RFA_OK;
}

int rfa_join(rfa_handle *h) {
    if (!h) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    return join(h);
}

// CU masks (hipExtStreamCreateWithCUMask): the driver maps mask bit i to XCD i mod X, and its
// index j = i / X within the XCD to shader engine j mod SE, CU slot j / SE -- so bits
// [0, state_cus) put state_cus / X CUs on every XCD, each on another shader engine, and the
// complement leaves every XCD the same number of FFT CUs (the FFT kernels' blocks b, b + 8, ...
// share an XCD)
int rfa_set_pipelined(rfa_handle *h, int32_t state_cus) {
    if (!h || state_cus < 0) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    pipe_release(h);
    if (state_cus == 0) return RFA_OK;
    int ncu = 0, nxcc = 1;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || ncu <= 0)
        return fail(h, RFA_ERR_HIP, "CU count");
    if (hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, h->device) != hipSuccess || nxcc <= 0) nxcc = 1;
    if (state_cus % nxcc || state_cus >= ncu)
        return fail(h, RFA_ERR_UNSUPPORTED, "state_cus must be a multiple of the XCD count, below the CU count");
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> ms(words, 0u), mf(words, 0u);
    for (int i = 0; i < ncu; i++) (i < state_cus ? ms : mf)[i / 32] |= 1u << (i % 32);
    auto bail = [&](const char *what) {
        pipe_release(h);
        return fail(h, RFA_ERR_UNSUPPORTED, what);
    };
    bool nomask = false;
#ifdef RFA_AB_BUILD
    // A/B builds (RFA_PIPE_NOMASK=1): no CU masks -- the state pass's workgroups share the FFT's CUs
    // (co-resident beside an FFT workgroup compiled for fewer VGPRs, RFA_WIDE_WPE); the FFT streams
    // get the higher priority
    if (const char *d = std::getenv("RFA_PIPE_NOMASK")) nomask = std::atoi(d) != 0;
#endif
    if (nomask) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (hipStreamCreateWithPriority(&h->pipe_state, hipStreamNonBlocking, lo) != hipSuccess) return bail("state stream");
        for (hipStream_t &fs : h->pipe_fft)
            if (hipStreamCreateWithPriority(&fs, hipStreamNonBlocking, hi) != hipSuccess) return bail("FFT stream");
    } else {
        if (hipExtStreamCreateWithCUMask(&h->pipe_state, (uint32_t)words, ms.data()) != hipSuccess)
            return bail("CU-masked state stream");
        for (hipStream_t &fs : h->pipe_fft)
            if (hipExtStreamCreateWithCUMask(&fs, (uint32_t)words, mf.data()) != hipSuccess)
                return bail("CU-masked FFT stream");
    }
    for (hipEvent_t *e : {&h->pipe_in, &h->pipe_fft_done[0], &h->pipe_fft_done[1], &h->pipe_state_done[0],
                          &h->pipe_state_done[1]})
        if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return bail("pipeline events");
    h->pipe_cus = state_cus;
    h->pipe_fft_cus = nomask ? ncu : ncu - state_cus;
    return RFA_OK;
}

int rfa_synchronize(rfa_handle *h) {
    if (!h) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

// Waterfall-speed resize (FftProcessor.kt:185-195), done where the reference
// does it: with the next frame, before the retune shift and the row write.
static int apply_ring_resize(rfa_handle *h) {
    const int rn = h->pending_ring_rows;
    h->pending_ring_rows = -1;
    if (rn < 0 || rn == h->ring_rows) return RFA_OK;
    if (int rc = join(h)) return rc;
    const size_t bytes = (size_t)rn * h->n * sizeof(float);
    float *nr = nullptr, *nt = nullptr;
    if (hipMalloc(&nr, bytes) != hipSuccess) return fail(h, RFA_ERR_NOMEM, "ring resize");
    if (hipMalloc(&nt, bytes) != hipSuccess) {
        hipFree(nr);
        return fail(h, RFA_ERR_NOMEM, "ring resize");
    }
    hipError_t e = rfa::launch_ring_rotate(h->d_ring, h->ring_rows, nr, rn, h->n, h->write_index, kRingFill, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        hipFree(nr);
        hipFree(nt);
        return hip_fail(h, e, "ring resize");
    }
    hipFree(h->d_ring);
    hipFree(h->d_ring_tmp);
    h->d_ring = nr;
    h->d_ring_tmp = nt;
    h->ring_rows = rn;
    h->cfg.ring_rows = rn;
    h->dirty.assign((size_t)rn, 1);  // FftProcessor.kt:193
    h->write_index = 0;
    if (h->read_index >= rn) h->read_index = 0;  // rewritten by the frame that triggered the resize
    h->generation++;
    return RFA_OK;
}

static int process_impl(rfa_handle *h, const void *in, size_t n_frames, size_t stride, float *rows,
                        const float *window, int fmt) {
    const int n = h->n;
    const size_t bps = bytes_per_sample(fmt);
    if (stride == 0) stride = (size_t)n * bps;
    if (stride < (size_t)n * bps && n_frames > 1) return fail(h, RFA_ERR_INVALID, "frame stride smaller than a frame");
    const size_t al = load_alignment(fmt);
    if ((uintptr_t)in % al || stride % al) return fail(h, RFA_ERR_INVALID, "input pointer/stride misaligned for format");
    if (n_frames > (size_t)0x7fffffff) return fail(h, RFA_ERR_INVALID, "too many frames");
    if (n_frames == 0) return RFA_OK;
    if (h->pending_ring_rows >= 0) {
        int rc = apply_ring_resize(h);
        if (rc) return rc;
    }
    const bool need_state = h->d_peaks || h->d_ema;
    // channel mean bins of this tuning (FftProcessor.kt:143-151)
    int chan_first = 0, chan_last = 0;
    if (h->chan_on && h->have_tuning) {
        const float samples_per_hz = (float)n / (float)h->last_sample_rate;
        const int64_t f0 = h->last_frequency - h->last_sample_rate / 2;
        auto idx = [&](int64_t f) {
            const float x = (float)(f - f0) * samples_per_hz;
            const long long i = std::isnan(x) ? 0 : x >= 2147483647.0f ? 2147483647LL : x <= -2147483648.0f ? -2147483648LL
                                                                                                               : (long long)x;
            return (int)std::min<long long>(std::max<long long>(i, 0), n);  // coerceIn(0, size)
        };
        chan_first = idx(h->chan_start);
        chan_last = idx(h->chan_end);
    }
    const bool need_chan = chan_last > chan_first;
    h->chan_count = 0;
    h->chan_offset = 0;
    // state and channel means need the rows of the whole batch: use the caller's,
    // else the ring when every frame lands there, else a staging buffer
    float *state_rows = rows;
    bool rows_in_ring = false;
    if ((need_state || need_chan) && !rows) {
        if (h->d_ring && n_frames <= (size_t)h->ring_rows) {
            rows_in_ring = true;
        } else {
            int rc = ensure_device_buffer(h, (void **)&h->d_rows, &h->d_rows_cap, n_frames * (size_t)n * sizeof(float));
            if (rc) return rc;
            state_rows = h->d_rows;
        }
    }
    // pipelined state (rfa_set_pipelined): this call's FFT may start while the
    // previous pipelined call's state pass still reads that call's rows, so it writes the ring's
    // second buffer (the call rewrites every ring row) or only rows the previous call did not
    // write; anything else first joins
    const bool flip = (long long)n_frames == (long long)h->ring_rows;
    const bool pipe = h->pipe_cus > 0 && need_state && rows_in_ring &&
                      (flip || (long long)n_frames + h->pipe_prev_frames <= (long long)h->ring_rows);
    if (!pipe) {
        int rc = join(h);
        if (rc) return rc;
    }
    const int par = (int)(h->pipe_k & 1);
    hipStream_t fft_stream = h->stream, state_stream = h->stream;
    if (pipe) {
        // (N > 128 K: the decimation-in-frequency pair shares the handle's scratch z between its
        // two kernels, so consecutive calls stay on one FFT stream)
        fft_stream = h->pipe_fft[h->logn > 17 ? 0 : par];
        state_stream = h->pipe_state;
        // the input (and everything before it) is on the handle stream; the pass of call k - 2
        // (same parity) read the buffer / rows this call writes
        HIPCHK(h, hipEventRecord(h->pipe_in, h->stream));
        HIPCHK(h, hipStreamWaitEvent(fft_stream, h->pipe_in, 0));
        if (h->pipe_recorded[par]) HIPCHK(h, hipStreamWaitEvent(fft_stream, h->pipe_state_done[par], 0));
        if (flip) {  // the other ring buffer: its rows are all rewritten by this call
            std::swap(h->d_ring, h->d_ring_tmp);
            h->generation++;
        }
    }
    FftLaunch a;
    a.in = (const uint8_t *)in;
    a.frame_stride = (long long)stride;
    a.n_frames = (int)n_frames;
    a.fmt = fmt;
    a.window = window;
    a.rows = state_rows;
    if (pipe) a.cus = h->pipe_fft_cus;
    if (h->d_ring) {
        a.ring = h->d_ring;
        a.ring_rows = h->ring_rows;
        a.ring_base = h->write_index;
        a.ring_first = (int)std::max<long long>(0, (long long)n_frames - h->ring_rows);
        a.ring_logrs = h->ring_logrs;
    }
    int rc = launch_main(h, a, fft_stream);
    if (rc) return rc;
    if (pipe) {
        HIPCHK(h, hipEventRecord(h->pipe_fft_done[par], fft_stream));
        HIPCHK(h, hipStreamWaitEvent(state_stream, h->pipe_fft_done[par], 0));
    }
    if (need_state || need_chan) {
        rfa::StateLaunch s;
        s.n = n;
        s.n_frames = (int)n_frames;
        s.peaks = h->d_peaks;
        s.ema = h->d_ema;
        s.ema_alpha = h->cfg.ema_alpha;
        s.part = h->d_state_part;
        s.max_chunks = h->state_chunks;
        s.fused = h->state_fused;
        s.stream = state_stream;
        if (rows_in_ring) {
            s.rows = h->d_ring;
            s.ring_rows = h->ring_rows;
            s.ring_base = h->write_index;
            s.ring_logrs = h->ring_logrs;
        } else {
            s.rows = state_rows;
            s.row_stride = n;
        }
        if (need_state) HIPCHK(h, rfa::launch_state(s));
        if (need_chan) {
            // means, then (channels wider than 16384 bins) the per-span partial sums
            const int spans = rfa::channel_mean_spans(chan_last - chan_first);
            const size_t words = n_frames * (size_t)(spans > 1 ? 1 + spans : 1);
            if (pipe && words * sizeof(float) > h->d_chan_cap)  // the last pass may still write the old buffer
                HIPCHK(h, hipStreamSynchronize(state_stream));
            int rc = ensure_device_buffer(h, (void **)&h->d_chan, &h->d_chan_cap, words * sizeof(float));
            if (rc) return rc;
            HIPCHK(h, rfa::launch_channel_mean(s, chan_first, chan_last, h->d_chan,
                                               spans > 1 ? h->d_chan + n_frames : nullptr));
            h->chan_count = n_frames;
        }
    }
    if (pipe) {
        HIPCHK(h, hipEventRecord(h->pipe_state_done[par], state_stream));
        h->pipe_recorded[par] = true;
        h->pipe_pending = true;
        h->pipe_prev_frames = (int)n_frames;
        h->pipe_k++;
    }
    if (h->d_ring) {
        const long long R = h->ring_rows;
        const long long last = (long long)n_frames - 1;
        // the rows this batch wrote are dirty for the draw thread (FftProcessor.kt:223)
        for (long long f = std::max<long long>(0, (long long)n_frames - R); f < (long long)n_frames; f++)
            h->dirty[(size_t)((((long long)h->write_index - f) % R + R) % R)] = 1;
        h->read_index = (int)((((long long)h->write_index - last) % R + R) % R);
        h->write_index = h->read_index == 0 ? h->ring_rows - 1 : h->read_index - 1;  // FftProcessor.kt:226-227
    }
    h->have_rows = true;
    if (h->profile) drain_events(h, false);
    return RFA_OK;
}

int rfa_process(rfa_handle *h, const void *in, size_t n_frames, size_t frame_stride_bytes, float *rows) {
    if (!h || (!in && n_frames)) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    return process_impl(h, in, n_frames, frame_stride_bytes, rows, h->d_window, h->cfg.input_format);
}

int rfa_process_batches(rfa_handle *h, const void *in, size_t n_batches, size_t batch_stride_bytes,
                        size_t frames_per_batch, size_t frame_stride_bytes, float *rows) {
    if (!h || (!in && n_batches && frames_per_batch)) return RFA_ERR_INVALID;
    if (n_batches == 0 || frames_per_batch == 0) return RFA_OK;
    int rc = set_device(h);
    if (rc) return rc;
    const size_t stride = frame_stride_bytes ? frame_stride_bytes : (size_t)h->n * bytes_per_sample(h->cfg.input_format);
    if (n_batches == 1 || batch_stride_bytes == frames_per_batch * stride) {
        // packed: one batch of n_batches * frames_per_batch frames is the same frame stream
        // (the ring and the peak / EMA recursion see the frames in the same order)
        if (n_batches > (size_t)0x7fffffff / frames_per_batch) return fail(h, RFA_ERR_INVALID, "too many frames");
        rc = process_impl(h, in, n_batches * frames_per_batch, stride, rows, h->d_window, h->cfg.input_format);
        if (!rc && h->chan_count) {  // the channel means of the last batch, as after consecutive calls
            h->chan_offset = (n_batches - 1) * frames_per_batch;
            h->chan_count = frames_per_batch;
        }
        return rc;
    }
    for (size_t b = 0; b < n_batches; b++) {
        rc = process_impl(h, static_cast<const uint8_t *>(in) + b * batch_stride_bytes, frames_per_batch, stride,
                          rows ? rows + b * frames_per_batch * (size_t)h->n : nullptr, h->d_window,
                          h->cfg.input_format);
        if (rc) return rc;
    }
    return RFA_OK;
}

int rfa_process_host(rfa_handle *h, const void *in, size_t n_frames, size_t frame_stride_bytes, float *rows) {
    if (!h || (!in && n_frames)) return RFA_ERR_INVALID;
    if (n_frames == 0) return RFA_OK;
    int rc = set_device(h);
    if (rc) return rc;
    const size_t bps = bytes_per_sample(h->cfg.input_format);
    const size_t stride = frame_stride_bytes ? frame_stride_bytes : (size_t)h->n * bps;
    const size_t in_bytes = (n_frames - 1) * stride + (size_t)h->n * bps;
    rc = ensure_device_buffer(h, &h->d_in, &h->d_in_cap, in_bytes);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(h->d_in, in, in_bytes, hipMemcpyHostToDevice, h->stream));
    float *d_rows = nullptr;
    if (rows) {
        rc = ensure_device_buffer(h, (void **)&h->d_rows, &h->d_rows_cap, n_frames * (size_t)h->n * sizeof(float));
        if (rc) return rc;
        d_rows = h->d_rows;
    }
    rc = process_impl(h, h->d_in, n_frames, stride, d_rows, h->d_window, h->cfg.input_format);
    if (rc) return rc;
    if ((rc = join(h))) return rc;  // synchronous: the next call's copy reuses d_in
    if (rows)
        HIPCHK(h, hipMemcpyAsync(rows, d_rows, n_frames * (size_t)h->n * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_push_packet(rfa_handle *h, const void *packet, size_t packet_bytes, int64_t frequency, int64_t sample_rate,
                    float *row_out, int32_t *frames) {
    if (!h || !frames || (!packet && packet_bytes)) return RFA_ERR_INVALID;
    *frames = 0;
    if (h->cfg.input_format == RFA_IN_F32_PLANAR)
        return fail(h, RFA_ERR_UNSUPPORTED, "packet framing needs an interleaved sample format");
    if (!h->framer.push(packet, packet_bytes)) return RFA_OK;  // the frame waits for more packets
    // only the completing packet's tuning is used (Signed8BitIQConverter.java:95-97), so only
    // its sample rate must be valid; the frame is dropped with it
    if (sample_rate <= 0) {
        h->framer.clear();
        return fail(h, RFA_ERR_INVALID, "rfa_push_packet: sample_rate <= 0 on the packet completing a frame");
    }
    // complete: the tuning of the packet that completed it (Signed8BitIQConverter.java:95-96),
    // then one frame through ring / peaks / EMA / channel mean (FftProcessor.kt:125-245)
    int rc = rfa_set_tuning(h, frequency, sample_rate);
    if (!rc) rc = rfa_process_host(h, h->framer.data(), 1, 0, row_out);
    h->framer.clear();  // the next packet starts a new SamplePacket (Scheduler.kt:266-270)
    if (rc) return rc;
    *frames = 1;
    return RFA_OK;
}

int rfa_pending_samples(const rfa_handle *h, int64_t *samples) {
    if (!h || !samples) return RFA_ERR_INVALID;
    *samples = (int64_t)h->framer.filled();
    return RFA_OK;
}

int64_t rfa_retune_offset(int64_t frequency_diff, int n, int64_t sample_rate) {
    if (sample_rate <= 0) return 0;
    // FftProcessor.kt:143,199: (fdiff * (N / sampleRate.toFloat())).toInt(), float arithmetic
    const float samples_per_hz = (float)n / (float)sample_rate;
    const float prod = (float)frequency_diff * samples_per_hz;
    if (std::isnan(prod)) return 0;
    if (prod >= 2147483647.0f) return 2147483647LL;
    if (prod <= -2147483648.0f) return -2147483648LL;
    return (int64_t)prod;  // truncation toward zero
}

int rfa_set_tuning(rfa_handle *h, int64_t frequency, int64_t sample_rate) {
    if (!h || sample_rate <= 0) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    if (!h->have_tuning) {
        h->have_tuning = true;
        h->last_frequency = frequency;
        h->last_sample_rate = sample_rate;
        return reset_peaks_ema(h);
    }
    const bool fchg = frequency != h->last_frequency;
    const bool schg = sample_rate != h->last_sample_rate;
    if (!fchg && !schg) return RFA_OK;
    const int64_t fdiff = h->last_frequency - frequency;  // FftProcessor.kt:173
    h->last_frequency = frequency;
    h->last_sample_rate = sample_rate;
    if (h->d_ring) {
        if (fdiff != 0) {
            const long long off = rfa_retune_offset(fdiff, h->n, sample_rate);
            if ((off < 0 && -off < h->n) || (off >= 0 && off < h->n)) {
                HIPCHK(h, rfa::launch_ring_shift(h->d_ring, h->d_ring_tmp, h->ring_rows, h->n, h->ring_logrs, (int)off, kRingFill,
                                                 h->stream));
                std::swap(h->d_ring, h->d_ring_tmp);
                h->generation++;
                std::fill(h->dirty.begin(), h->dirty.end(), 1);  // FftProcessor.kt:215
            } else {
                rc = clear_ring(h);
                if (rc) return rc;
            }
        } else {
            rc = clear_ring(h);  // sample-rate change, FftProcessor.kt:216-219
            if (rc) return rc;
        }
    }
    return reset_peaks_ema(h);  // FftProcessor.kt:238-239 (peaks), EMA likewise
}

// Kotlin Double.toInt() / Float.toInt(): truncation toward zero, NaN -> 0, saturating.
static int kt_toint(double x) {
    if (std::isnan(x)) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int)x;
}

int rfa_draw_preprocess(rfa_handle *h, const rfa_draw_params *p, uint32_t *colors, float *fft_path_y, float *peaks_y,
                        float *autoscale) {
    if (!h || !p || !colors || !fft_path_y || !p->colormap) return RFA_ERR_INVALID;
    if (p->width <= 0 || p->fft_height < 0 || p->colormap_size <= 0 || p->average_length < 0) return RFA_ERR_INVALID;
    if (!h->d_ring) return fail(h, RFA_ERR_STATE, "display preprocessing reads the ring (ring_rows > 0)");
    if (!h->have_tuning) return fail(h, RFA_ERR_STATE, "display preprocessing needs rfa_set_tuning (frequency, rate)");
    if (p->average_length >= h->ring_rows) return RFA_ERR_INVALID;
    if (peaks_y && !h->d_peaks) return fail(h, RFA_ERR_STATE, "peak-hold y needs peak_hold");
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    const int n = h->n, R = h->ring_rows, W = p->width, L = p->average_length;
    // AnalyzerSurface.kt:650-672, in the reference's types (Long, Double, Float, Int)
    const float samples_per_hz = (float)n / (float)h->last_sample_rate;
    const int64_t frequency_diff = p->viewport_frequency - h->last_frequency;
    const int64_t sample_rate_diff = p->viewport_sample_rate - h->last_sample_rate;
    const int start = kt_toint(((double)frequency_diff - (double)sample_rate_diff / 2.0) * (double)samples_per_hz);
    const int end = n + kt_toint(((double)frequency_diff + (double)sample_rate_diff / 2.0) * (double)samples_per_hz);
    rfa::DrawLaunch a;
    a.samples_per_px = (float)(end - start) / (float)W;
    const float db_diff = p->max_db - p->min_db;
    a.db_width = (float)p->fft_height / db_diff;
    a.scale = (float)p->colormap_size / db_diff;
    a.first_pixel = start >= 0 ? 0 : kt_toint((double)((float)(start * -1) / a.samples_per_px));
    a.last_pixel = end >= n ? kt_toint((double)((float)(n - start) / a.samples_per_px))
                            : kt_toint((double)((float)(end - start) / a.samples_per_px));
    a.start = start;
    a.min_db = p->min_db;
    a.ring = h->d_ring;
    a.ring_logrs = h->ring_logrs;
    a.peaks = peaks_y ? h->d_peaks : nullptr;
    a.ring_rows = R;
    a.n = n;
    a.read_index = h->read_index;
    a.width = W;
    a.fft_height = p->fft_height;
    a.avg_length = L;
    a.colormap_size = p->colormap_size;
    // persistent colour buffer (AnalyzerSurface.kt:619-626: a new size starts zeroed, all rows dirty)
    if (!h->d_colors || h->colors_rows != R || h->colors_width != W) {
        hipFree(h->d_colors);
        h->d_colors = nullptr;
        if (hipMalloc(&h->d_colors, (size_t)R * W * 4) != hipSuccess) return fail(h, RFA_ERR_NOMEM, "colour buffer");
        HIPCHK(h, hipMemsetAsync(h->d_colors, 0, (size_t)R * W * 4, h->stream));
        h->colors_rows = R;
        h->colors_width = W;
        std::fill(h->dirty.begin(), h->dirty.end(), 1);
    }
    // a new viewport or vertical scale repaints everything (:634-640)
    if (!h->have_view || p->viewport_frequency != h->view_frequency || p->viewport_sample_rate != h->view_sample_rate ||
        p->min_db != h->view_min_db || p->max_db != h->view_max_db) {
        std::fill(h->dirty.begin(), h->dirty.end(), 1);
        h->have_view = true;
        h->view_frequency = p->viewport_frequency;
        h->view_sample_rate = p->viewport_sample_rate;
        h->view_min_db = p->min_db;
        h->view_max_db = p->max_db;
    }
    // the rows this draw refreshes, newest first (:678-684): every dirty row and rows
    // 0..L (the time average), at most L + 6 of them; refreshed rows become clean
    std::vector<int2> sel;
    for (int row_number = 0; row_number < R; row_number++) {
        const int bi = (h->read_index + row_number) % R;
        if (!h->dirty[bi] && row_number > L) continue;
        if ((int)sel.size() > L + 5) break;
        sel.push_back(make_int2(row_number, bi));
    }
    // one device block: colormap | row list | averages [L+1][W] | path y | peaks y | autoscale
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_cmap = al((size_t)p->colormap_size * 4), b_sel = al(sel.size() * sizeof(int2)),
                 b_avg = al((size_t)(L + 1) * W * 4), b_w = al((size_t)W * 4);
    rc = ensure_device_buffer(h, &h->d_draw, &h->d_draw_cap, b_cmap + b_sel + b_avg + 2 * b_w + 256);
    if (rc) return rc;
    char *base = static_cast<char *>(h->d_draw) + b_sel;
    a.colormap = reinterpret_cast<const unsigned *>(base);
    a.rows = reinterpret_cast<const int2 *>(static_cast<char *>(h->d_draw));
    a.n_rows = (int)sel.size();
    a.colors = h->d_colors;
    a.avg_rows = reinterpret_cast<float *>(base + b_cmap);
    a.path_y = reinterpret_cast<float *>(base + b_cmap + b_avg);
    a.peaks_y = peaks_y ? reinterpret_cast<float *>(base + b_cmap + b_avg + b_w) : nullptr;
    a.autoscale = reinterpret_cast<float *>(base + b_cmap + b_avg + 2 * b_w);
    a.stream = h->stream;
    HIPCHK(h, hipMemcpyAsync(base, p->colormap, (size_t)p->colormap_size * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->d_draw, sel.data(), sel.size() * sizeof(int2), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, rfa::launch_draw(a));
    // refreshed rows become clean only once their refresh is enqueued (a failed
    // launch above leaves them dirty for the next draw)
    for (const int2 &r : sel) h->dirty[(size_t)r.y] = 0;
    HIPCHK(h, hipMemcpyAsync(colors, a.colors, (size_t)R * W * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipMemcpyAsync(fft_path_y, a.path_y, (size_t)W * 4, hipMemcpyDeviceToHost, h->stream));
    if (peaks_y) HIPCHK(h, hipMemcpyAsync(peaks_y, a.peaks_y, (size_t)W * 4, hipMemcpyDeviceToHost, h->stream));
    float mm[2];
    HIPCHK(h, hipMemcpyAsync(mm, a.autoscale, 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (autoscale) {
        autoscale[0] = mm[0];
        autoscale[1] = mm[1];
    }
    return RFA_OK;
}

int rfa_row_window_stats(rfa_handle *h, const int32_t *lo, const int32_t *hi, size_t count, float *peak, float *avg) {
    if (!h || (count && (!lo || !hi || !peak || !avg)) || count > (size_t)0x7fffffff) return RFA_ERR_INVALID;
    if (!h->d_ring) return fail(h, RFA_ERR_STATE, "window statistics read the newest ring row (ring_rows > 0)");
    for (size_t i = 0; i < count; i++)
        if (lo[i] < 0 || hi[i] >= h->n || lo[i] > hi[i]) return fail(h, RFA_ERR_INVALID, "window outside the row");
    if (count == 0) return RFA_OK;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    const size_t b = (count * 4 + 255) & ~(size_t)255;
    rc = ensure_device_buffer(h, &h->d_draw, &h->d_draw_cap, 4 * b);
    if (rc) return rc;
    char *base = static_cast<char *>(h->d_draw);
    int *d_lo = reinterpret_cast<int *>(base), *d_hi = reinterpret_cast<int *>(base + b);
    float *d_pk = reinterpret_cast<float *>(base + 2 * b), *d_av = reinterpret_cast<float *>(base + 3 * b);
    HIPCHK(h, hipMemcpyAsync(d_lo, lo, count * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(d_hi, hi, count * 4, hipMemcpyHostToDevice, h->stream));
    const float *row = h->d_ring + (size_t)h->read_index * h->n;  // FftProcessorData.readIndex: newest row
    HIPCHK(h, rfa::launch_row_windows(row, h->ring_logrs, h->n, d_lo, d_hi, (int)count, d_pk, d_av, h->stream));
    HIPCHK(h, hipMemcpyAsync(peak, d_pk, count * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipMemcpyAsync(avg, d_av, count * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_set_channel(rfa_handle *h, int64_t start_frequency, int64_t end_frequency) {
    if (!h) return RFA_ERR_INVALID;
    h->chan_on = start_frequency != end_frequency;
    h->chan_start = start_frequency;
    h->chan_end = end_frequency;
    return RFA_OK;
}

int rfa_get_channel_means(rfa_handle *h, float *out, size_t capacity, size_t *count) {
    if (!h || !count || (!out && capacity)) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    const size_t k = std::min(capacity, h->chan_count);
    if (k) HIPCHK(h, hipMemcpyAsync(out, h->d_chan + h->chan_offset, k * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    *count = h->chan_count;
    return RFA_OK;
}

int rfa_get_peaks(rfa_handle *h, float *out) {
    if (!h || !out) return RFA_ERR_INVALID;
    if (!h->d_peaks) return fail(h, RFA_ERR_STATE, "peak_hold disabled");
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    HIPCHK(h, hipMemcpyAsync(out, h->d_peaks, h->n * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_get_ema(rfa_handle *h, float *out) {
    if (!h || !out) return RFA_ERR_INVALID;
    if (!h->d_ema) return fail(h, RFA_ERR_STATE, "EMA disabled");
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    HIPCHK(h, hipMemcpyAsync(out, h->d_ema, h->n * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_get_boxcar(rfa_handle *h, int32_t length, float *out) {
    if (!h || !out || length < 0) return RFA_ERR_INVALID;
    if (!h->d_ring) return fail(h, RFA_ERR_STATE, "boxcar needs the ring (ring_rows > 0)");
    if (length >= h->ring_rows) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    HIPCHK(h, rfa::launch_boxcar(h->d_ring, h->ring_rows, h->n, h->ring_logrs, h->read_index, length, h->d_boxcar,
                                  h->stream));
    HIPCHK(h, hipMemcpyAsync(out, h->d_boxcar, h->n * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_get_ring(rfa_handle *h, float *out, int32_t *read_index, int32_t *write_index) {
    if (!h) return RFA_ERR_INVALID;
    if (!h->d_ring) return fail(h, RFA_ERR_STATE, "ring disabled");
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    if (out) {
        const float *src = h->d_ring;
        if (h->ring_logrs) {  // residue-major storage -> natural rows (d_ring_tmp is free outside a retune)
            HIPCHK(h, rfa::launch_ring_natural(h->d_ring, h->d_ring_tmp, h->ring_rows, h->n, h->ring_logrs, h->stream));
            src = h->d_ring_tmp;
        }
        HIPCHK(h, hipMemcpyAsync(out, src, (size_t)h->ring_rows * h->n * sizeof(float), hipMemcpyDeviceToHost,
                                 h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (read_index) *read_index = h->read_index;
    if (write_index) *write_index = h->write_index;
    return RFA_OK;
}

int rfa_reset_state(rfa_handle *h) {
    if (!h) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    h->write_index = h->read_index = 0;
    h->have_rows = false;
    h->have_tuning = false;
    h->framer.clear();
    rc = clear_ring(h);
    if (rc) return rc;
    rc = reset_peaks_ema(h);
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return RFA_OK;
}

int rfa_set_ring_rows(rfa_handle *h, int32_t ring_rows) {
    if (!h || ring_rows < 1) return RFA_ERR_INVALID;
    if (h->cfg.avg_mode == RFA_AVG_BOXCAR && h->cfg.avg_length >= ring_rows)
        return fail(h, RFA_ERR_INVALID, "boxcar average_length does not fit the new ring");
    h->pending_ring_rows = ring_rows == h->ring_rows ? -1 : ring_rows;
    return RFA_OK;
}

int rfa_set_fft_size(rfa_handle *h, int32_t fft_size) {
    if (!h) return RFA_ERR_INVALID;
    if (fft_size == h->n) return RFA_OK;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    rfa_config c = h->cfg;
    c.fft_size = fft_size;
    if (h->pending_ring_rows >= 0) c.ring_rows = h->pending_ring_rows;  // the ring is re-created at the new speed
    rfa_handle *nh = nullptr;
    rc = rfa_create(&c, &nh);
    if (rc) return fail(h, rc, "rfa_set_fft_size: rebuilding the handle failed");
    // carried over: tuning, channel range, caller stream, profiling switch (the
    // ring, peaks and EMA of the new handle start cleared: FftProcessor.kt:178-183,233-236)
    nh->have_tuning = h->have_tuning;
    nh->last_frequency = h->last_frequency;
    nh->last_sample_rate = h->last_sample_rate;
    nh->chan_on = h->chan_on;
    nh->chan_start = h->chan_start;
    nh->chan_end = h->chan_end;
    if (h->stream != h->own_stream) nh->stream = h->stream;
    nh->profile = h->profile;
    nh->generation = h->generation + 1;
    const int pipe_cus = h->pipe_cus;
    std::swap(*h, *nh);
    rfa_destroy(nh);  // the old tables and buffers
    if (pipe_cus) return rfa_set_pipelined(h, pipe_cus);
    return RFA_OK;
}

int rfa_get_ring_order(const rfa_handle *h, int32_t *residues) {
    if (!h || !residues) return RFA_ERR_INVALID;
    *residues = 1 << rfa::ring_lr(h->ring_logrs);
    return RFA_OK;
}

int rfa_get_state_generation(const rfa_handle *h, int64_t *generation) {
    if (!h || !generation) return RFA_ERR_INVALID;
    *generation = h->generation;
    return RFA_OK;
}

int rfa_get_ring_positions(const rfa_handle *h, int32_t *positions, size_t count) {
    if (!h || (!positions && count)) return RFA_ERR_INVALID;
    if (count != (size_t)h->n) return fail(const_cast<rfa_handle *>(h), RFA_ERR_SIZE, "positions must hold fft_size entries");
    const int lm = rfa::ring_logm(h->ring_logrs, h->logn);
    for (int t = 0; t < h->n; t++) positions[t] = rfa::ring_pos(t, h->ring_logrs, lm);
    return RFA_OK;
}

int rfa_get_device_state(rfa_handle *h, float **ring, float **peaks, float **ema) {
    if (!h) return RFA_ERR_INVALID;
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;  // device readers on the handle stream see the last call's state
    if (ring) *ring = h->d_ring;
    if (peaks) *peaks = h->d_peaks;
    if (ema) *ema = h->d_ema;
    return RFA_OK;
}

// One frame through the fused kernel from host arrays, no ring/state side effects.
static int single_frame(rfa_handle *h, const void *host_in, size_t in_bytes, int fmt, const float *d_window,
                        float *host_db, float2 *host_cplx) {
    int rc = set_device(h);
    if (rc) return rc;
    if ((rc = join(h))) return rc;
    const size_t n = (size_t)h->n;
    const size_t out_bytes = host_cplx ? n * sizeof(float2) : n * sizeof(float);
    rc = ensure_device_buffer(h, &h->d_in, &h->d_in_cap, in_bytes);
    if (rc) return rc;
    rc = ensure_device_buffer(h, (void **)&h->d_rows, &h->d_rows_cap, out_bytes);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(h->d_in, host_in, in_bytes, hipMemcpyHostToDevice, h->stream));
    FftLaunch a;
    a.in = (const uint8_t *)h->d_in;
    a.frame_stride = (long long)in_bytes;
    a.n_frames = 1;
    a.fmt = fmt;
    a.window = d_window;
    if (host_cplx) a.complex_out = (float2 *)h->d_rows;
    else a.rows = h->d_rows;
    rc = launch_main(h, a, h->stream);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(host_cplx ? (void *)host_cplx : (void *)host_db, h->d_rows, out_bytes,
                             hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->profile) drain_events(h, false);
    return RFA_OK;
}

int rfa_windowed_fft_mag_planar(rfa_handle *h, const float *re, const float *im, float *mag_out, size_t n) {
    if (!h || !re || !im || !mag_out) return RFA_ERR_INVALID;
    if (n != (size_t)h->n) return fail(h, RFA_ERR_SIZE, "array length != fft_size");  // NativeDsp.kt:45-46
    int rc = ensure_pinned(h, 2 * n * sizeof(float));
    if (rc) return rc;
    float *p = (float *)h->h_pinned;
    std::memcpy(p, re, n * sizeof(float));
    std::memcpy(p + n, im, n * sizeof(float));
    // NativeDsp.kt always applies its Blackman window (:48-49,55-58)
    const float *win = h->d_window_black;
    return single_frame(h, p, 2 * n * sizeof(float), RFA_IN_F32_PLANAR, win, mag_out, nullptr);
}

int rfa_fft_logmag_interleaved(rfa_handle *h, const float *in, float *mag_out, size_t n) {
    if (!h || !in || !mag_out) return RFA_ERR_INVALID;
    if (n != (size_t)h->n) return fail(h, RFA_ERR_SIZE, "array length != fft_size");
    return single_frame(h, in, 2 * n * sizeof(float), RFA_IN_F32_INTERLEAVED, h->d_window_none, mag_out, nullptr);
}

int rfa_fft_ordered(rfa_handle *h, const float *in, float *out, size_t n) {
    if (!h || !in || !out) return RFA_ERR_INVALID;
    if (n != (size_t)h->n) return fail(h, RFA_ERR_SIZE, "array length != fft_size");
    return single_frame(h, in, 2 * n * sizeof(float), RFA_IN_F32_INTERLEAVED, h->d_window_none, nullptr, (float2 *)out);
}

int rfa_stream_copy(void *dst, const void *src, size_t bytes, void *stream) {
    if ((!dst || !src) && bytes) return RFA_ERR_INVALID;
    if (bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16) return RFA_ERR_INVALID;
    if (rfa::launch_stream_copy(dst, src, bytes, (hipStream_t)stream) != hipSuccess) return RFA_ERR_HIP;
    return RFA_OK;
}

int rfa_set_profiling(rfa_handle *h, int enable) {
    if (!h) return RFA_ERR_INVALID;
    // no drain here (that would synchronise): pending pairs are collected by the
    // next profiled launch or by rfa_get_kernel_time, so profiling can be toggled
    // around single launches (sampled timing) without stalling the stream
    h->profile = enable != 0;
    return RFA_OK;
}

const char *rfa_main_kernel_name(const rfa_handle *h) {
    if (!h) return "";
    if (h->logn > 17) return "dif_front_kernel+fft_wide_kernel";  // the large-N pair (fft_large.hip)
    const bool wide = h->variant != 1 && rfa::wide_supported(h->logn);
    return wide ? "fft_wide_kernel" : "fft_rows_kernel";
}

int rfa_get_kernel_time(rfa_handle *h, double *total_ms, int64_t *launches) {
    if (!h) return RFA_ERR_INVALID;
    drain_events(h, true);
    if (total_ms) *total_ms = h->kernel_ms;
    if (launches) *launches = h->launches;
    return RFA_OK;
}

}  // extern "C"
