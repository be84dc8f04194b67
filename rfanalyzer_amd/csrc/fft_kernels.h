// Internal launch interface between the engine (engine.hip) and the gfx950
// kernels (fft_kernels.hip).  Not part of the public C-ABI (include/rfa.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace rfa {

// Ring row storage order.  When the main kernel computes an N-point
// frame as RS = 2^logrs residue sub-FFTs of M = N/RS points (the wide kernel at
// N = 64 K / 128 K), residue r's bins are stored as one contiguous block: the
// fft-shifted bin t of a ring row lives at element (t mod RS)*M + t/RS, so every
// residue workgroup writes whole cache lines.  logrs = 0 is natural order.  Only
// the device ring uses this order; caller rows, peaks, EMA and every host copy
// are in natural order (ring consumers gather through ring_pos).
//
// Order code (engine ring_logrs, FftLaunch / StateLaunch / DrawLaunch ring_logrs):
// bits 0-7 logrs; bit 8 (kRingTile, M = 32 K blocks only) additionally permutes the
// M elements of each block into the wide kernel's store tiles, so its epilogue
// writes 16 B per lane (8 x dwordx4 per thread instead of 32 x dword): sub-position
// i' = t'*1024 + w*64 + l (thread 64 w + l of the 1024-thread sub-FFT, its output
// t' = 0..31 after the fft-shift) lives at w*2048 + (t' >> 2)*256 + l*4 + (t' & 3)
// -- a bit permutation, so every consumer below maps with ring_pos / ring_bin.
constexpr int kRingTile = 0x100;
__host__ __device__ __forceinline__ int ring_lr(int code) { return code & 0xff; }
// logm of a ring of 2^logn bins in order `code`
__host__ __device__ __forceinline__ int ring_logm(int code, int logn) { return logn - (code & 0xff); }
__host__ __device__ __forceinline__ int tile_pos(int i) {  // i' -> storage position (M = 32 K)
    return (((i >> 6) & 15) << 11) | ((i >> 12) << 8) | ((i & 63) << 2) | ((i >> 10) & 3);
}
__host__ __device__ __forceinline__ int tile_sub(int p) {  // inverse of tile_pos
    return ((((p >> 8) & 7) << 2 | (p & 3)) << 10) | ((p >> 11) << 6) | ((p >> 2) & 63);
}
// bit 9 (kRingTile2, N = 64 K only): the store tiles of the wave-decoupled 64 K kernel
// (fft_w64.hip).  Its sub-bin i' = k0 + 32 k1 + 1024 t' (k0, k1 < 32: the output digits the
// kernel's exchanges leave in lane bit 0 + wave bits and in lane bits 1-5) is held by lane
// l = (k0 & 1) | (k1 << 1) of wave w = k0 >> 1 in register t'; a thread's four registers
// t' = 4j .. 4j+3 are one 16-B store at w*2048 + j*256 + l*4 -- the same store geometry as
// kRingTile with a different (lane, wave) <-> bin assignment.
constexpr int kRingTile2 = 0x200;
__host__ __device__ __forceinline__ int tile2_pos(int i) {
    const int k0 = i & 31, k1 = (i >> 5) & 31, tp = i >> 10;
    return ((k0 >> 1) << 11) | ((tp >> 2) << 8) | (((k0 & 1) | (k1 << 1)) << 2) | (tp & 3);
}
__host__ __device__ __forceinline__ int tile2_sub(int p) {
    const int w = p >> 11, j = (p >> 8) & 7, l = (p >> 2) & 63, e = p & 3;
    return ((l & 1) | (w << 1)) | ((l >> 1) << 5) | ((4 * j + e) << 10);
}
__host__ __device__ __forceinline__ int ring_pos(int t, int code, int logm) {
    const int lr = code & 0xff, sub = t >> lr;
    return ((t & ((1 << lr) - 1)) << logm) |
           ((code & kRingTile) ? tile_pos(sub) : (code & kRingTile2) ? tile2_pos(sub) : sub);
}
// inverse: the natural (fft-shifted) bin stored at ring element p
__host__ __device__ __forceinline__ int ring_bin(int p, int code, int logm) {
    const int lr = code & 0xff, q = p & ((1 << logm) - 1);
    return (((code & kRingTile) ? tile_sub(q) : (code & kRingTile2) ? tile2_sub(q) : q) << lr) | (p >> logm);
}

// Largest sub-FFT one workgroup keeps resident in LDS (16384 complex fp32 =
// 128 KiB + padding, one workgroup per CU).  Larger N split across
// workgroups (see DESIGN.md "Large N").
constexpr int kMaxLogM = 14;
constexpr int kMaxLogSplit = 3;  // up to 8 workgroups per frame (N <= 2^17) in the fused path

struct FftLaunch {
    // input: n_frames frames, frame f at in + f*frame_stride bytes
    const uint8_t *in = nullptr;
    long long frame_stride = 0;
    int n_frames = 0;
    int fmt = 0;   // rfa_input_format
    int logn = 0;  // N = 1 << logn
    const float *window = nullptr;  // N floats (device); all ones for RFA_WINDOW_NONE
    const float *window_il = nullptr;  // N > M: window[m + j*M] at [m*RS + j] (wide kernel pre-stage)
    // N = 64 K, residue 1 of the pre-stage: the twiddle folded into a complex window,
    // [m] = (w[m] W_N^m, -w[m + M] W_N^m) as float4, m < M (null: separate twiddle)
    const float4 *window_cw = nullptr;
    // wide kernel twiddle blob (exact, from double): pass-1 [32][R1] | pass-2 A,B [16][16] |
    // pre-stage pre_a [RS][512] | pre_b [RS][32]   (DESIGN.md "Twiddles")
    const float2 *wide_tw = nullptr;  // wide_twiddles() blob (layout in fft_wide.hip WGeo)
    const float2 *w64_tw = nullptr;   // N = 64 K: w64_twiddles() blob of the wave-decoupled kernel (fft_w64.hip)
    // twiddle table W_N^s = coarse[s >> tw_shift] * fine[s & ((1<<tw_shift)-1)]
    const float2 *tw_coarse = nullptr;
    const float2 *tw_fine = nullptr;
    int tw_shift = 0;
    // outputs (any may be null)
    float *rows = nullptr;      // n_frames * N, frame order
    float *ring = nullptr;      // ring_rows * N
    int ring_rows = 0;
    int ring_base = 0;          // ring row of frame 0 (reference writeIndex)
    int ring_first = 0;         // first frame that is stored into the ring
    int ring_logrs = 0;         // ring row order (ring_pos); must equal the kernel's residue split or 0
    float2 *complex_out = nullptr;  // ordered unscaled FFT (n_frames * N complex) instead of dB
    // kernel B of the large-N pair (fmt == kFmtDif): S = dif_ss column residues per
    // frame; work item u is (frame u / S, residue s = u % S), input z_s at
    // in + (u * M) complex, outputs bins S q + s of an N = S * M frame; its dB rows
    // target is residue-major (block s), like the ring
    int dif_ss = 0;
    int stage = 1;      // wide kernel: LDS-DMA staged 8/16-bit input when aligned (0 only in A/B builds)
    int variant = 0;    // 0 auto (wide kernel for N = 2^13..2^17), 1 narrow kernel only (seam windows)
    // A/B builds only (RFA_AB_BUILD): ablation variant (1 no loads, 2 no stores, 4 no FFT
    // passes, 32 phase stamps); always 0 in the product library
    int diag = 0;
    unsigned long long *stamps = nullptr;  // diag 32: [blocks][16][8] s_memrealtime phase stamps
    int prio = 0;         // A/B builds (RFA_W64_PRIO): fft_w64.hip static wave priorities (s_setprio)
    int phase_ticks = 0;  // A/B builds (RFA_PHASE_NS): persistent workgroups of the second half of
                          // the grid start this many 10-ns ticks late (phase offset between the
                          // two workgroups of a CU)
    // persistent grids: workgroups per CU x this many CUs (0: every CU of the device; a
    // CU-masked stream's CU count, engine.hip pipelined state)
    int cus = 0;
    hipStream_t stream = nullptr;
};

// Fused convert -> window -> FFT -> log-mag/shift -> rows/ring (or complex out).
hipError_t launch_fft(const FftLaunch &a);
// The wide kernel (32 points per thread, one M-point sub-FFT per workgroup,
// M = 8 K / 16 K / 32 K) for N = 2^13..2^17, and kernel B of the large-N pair.
bool wide_supported(int logn);
// ring order (ring_pos logrs) the main kernel writes for N = 2^logn and input format fmt
int ring_logrs_for(int logn, int fmt);
// N = 64 K: input formats (bit per rfa_input_format) that take the wave-decoupled kernel
// (fft_w64.hip); the others take the wide kernel's two-residue form (fft_wide.hip)
bool w64_format(int fmt);
constexpr int kWidePT = 32;  // wide kernel: points per thread (32 and 64 measured)
// sub-FFT size of the wide kernel: N itself up to 16 K, else 32 K (one
// 32 K-point workgroup per CU) with N / 32 K residues
#ifndef RFA_RES16K
#define RFA_RES16K 0  // A/B builds: N = 64 K as four 16 K residue items (two workgroups per CU) -- the
                      // co-scheduled re-read cluster form of VERDICT r5 item 3 (profiles/r06/)
#endif
inline int wide_logm(int logn) { return logn <= 14 ? logn : (RFA_RES16K && logn == 16 ? 14 : 15); }
std::vector<float2> wide_twiddles(int logn, int pt, int lm);
hipError_t launch_fft_wide(const FftLaunch &a);
// N = 64 K (dB rows / ring; not the complex-out seam): the wave-decoupled kernel, one
// cross-wave exchange per 32 K residue item (fft_w64.hip)
std::vector<float2> w64_twiddles();
hipError_t launch_fft64(const FftLaunch &a);

// N = 2^18 .. 2^20: decimation-in-frequency pair (DESIGN.md "Large N", fft_large.hip).
// Kernel A (dif_front_kernel) converts and windows the S = N / 32768 columns
// x[m + M j] of each frame, DFT-S over j, twiddle W_N^{m s}, and writes scratch
// z[f][s][m]; kernel B is the wide kernel on input format kFmtDif: the 32 K-point
// FFT of each z_s gives bins S q + s (ring block s in residue-major order).
struct DifLaunch {
    const uint8_t *in = nullptr;   // raw frames, frame f at in + f * frame_stride
    long long frame_stride = 0;
    int n_frames = 0;
    int fmt = 0;
    int logn = 0;
    const float *window = nullptr;  // natural order, N floats (scaled or seam window)
    const float2 *tw_c = nullptr;   // [S][M/128]  W_N^{s * 128 * mhi}  (per-tile kernel)
    const float2 *tw_d = nullptr;   // [S][128]    W_N^{s * mlo} - 1
    const float2 *tw_cp = nullptr;  // the pipelined kernel's split: [S][M/LO], [S][LO] (dif_lo_points(true))
    const float2 *tw_dp = nullptr;
    float2 *z = nullptr;            // scratch [n_frames][S][M]
    int pipe = 6;                   // 8-bit, 16-B aligned frames: pipelined kernel with `pipe` frame groups (0: off;
                                    // the engine stages misaligned 8-bit frames to an aligned copy for it)
    hipStream_t stream = nullptr;
};
constexpr int kDitLogM = 15;
constexpr int kMaxLogN = 20;
constexpr int kFmtDif = 5;  // wide-kernel input: kernel A's scratch (complex f32, already windowed)
hipError_t launch_dif_front(const DifLaunch &a);
// kernel B's residue-major dB rows -> natural order (caller rows of the large-N pair)
hipError_t launch_cols_to_rows(const float *cols, float *rows, int n_frames, int logn, hipStream_t st);
// points of the twiddle split's fine table: the pipelined 8-bit kernel's (pipe) or the per-tile kernel's
int dif_lo_points(bool pipe);
void dif_twiddles(int logn, int lo, std::vector<float2> &c, std::vector<float2> &d);

// Sequential EMA / peak-hold over n_frames rows.  Row f is at
// rows + f*row_stride, or, when ring_rows > 0, at rows + ((ring_base - f) mod ring_rows)*n
// (the reference's reverse-ordered ring, FftProcessor.kt:222-227).
struct StateLaunch {
    const float *rows = nullptr;
    long long row_stride = 0;
    int ring_rows = 0;
    int ring_base = 0;
    int ring_logrs = 0;      // ring row order (ring_pos), ring mode only
    int n_frames = 0;
    int n = 0;
    float *peaks = nullptr;  // may be null
    float *ema = nullptr;    // may be null; -inf = uninitialised
    float ema_alpha = 0.f;
    float4 *part = nullptr;  // chunk summaries [max_chunks][n] (null: sequential kernel only)
    int max_chunks = 1;
    int fused = 1;           // single-launch chunked scan (RFA_STATE_FUSED=0: partial + combine kernels)
    hipStream_t stream = nullptr;
};
hipError_t launch_state(const StateLaunch &a);
// The single-launch chunked scan launch_state takes for n_frames rows of n bins (max_chunks
// summaries, fused on): true with its chunk count and chunk length, else false
bool state_fused_plan(int n, int n_frames, int max_chunks, int fused, int *chunks, int *chunk_len);
// Mean of row[first, last) for every frame (rows addressed as in StateLaunch).
// channel mean of every frame (FftProcessor.kt:143-157); channels wider than 16384 bins are
// summed in channel_mean_spans() pieces whose sums go to partial[n_frames][spans] first
int channel_mean_spans(int width);
hipError_t launch_channel_mean(const StateLaunch &a, int first, int last, float *out, float *partial);

// Display preprocessing (AnalyzerSurface.kt:599-743), display.hip.  Scalars are
// computed on the host exactly as the reference does (double / fp32 / Kotlin toInt).
struct DrawLaunch {
    const float *ring = nullptr;   // [ring_rows][n]
    const float *peaks = nullptr;  // [n] or null
    int ring_rows = 0, n = 0, read_index = 0;
    int ring_logrs = 0;            // ring row order (ring_pos)
    int width = 0, fft_height = 0, avg_length = 0;
    int start = 0, first_pixel = 0, last_pixel = 0;
    float samples_per_px = 0.f, min_db = 0.f, db_width = 0.f, scale = 0.f;
    const unsigned *colormap = nullptr;
    int colormap_size = 0;
    unsigned *colors = nullptr;    // [ring_rows][width], ring storage order (persistent between draws)
    const int2 *rows = nullptr;    // the rows to refresh this draw: (rowNumber, bufferIndex), newest first
    int n_rows = 0;
    float *avg_rows = nullptr;     // scratch [avg_length + 1][width]
    float *path_y = nullptr;       // [width]
    float *peaks_y = nullptr;      // [width] or null
    float *autoscale = nullptr;    // [2]
    hipStream_t stream = nullptr;
};
hipError_t launch_draw(const DrawLaunch &a);
// Peak / mean of inclusive bin windows of one row (scanner reductions), display.hip.
hipError_t launch_row_windows(const float *row, int ring_logrs, int n, const int *lo, const int *hi, int count,
                              float *peak, float *avg, hipStream_t s);

// Ring maintenance (FftProcessor.kt:197-220) and boxcar (AnalyzerSurface.kt:710-714).
hipError_t launch_fill(float *p, long long count, float value, hipStream_t s);
hipError_t launch_ring_shift(const float *src, float *dst, int rows, int n, int logrs, int shift, float fill,
                             hipStream_t s);
hipError_t launch_boxcar(const float *ring, int rows, int n, int logrs, int read_index, int length, float *out,
                         hipStream_t s);
// Ring rows in natural order (host read-back): dst[row][t] = src[row][ring_pos(t)].
hipError_t launch_ring_natural(const float *src, float *dst, int rows, int n, int logrs, hipStream_t s);
// Waterfall-speed resize (FftProcessor.kt:185-195): dst[i] = src[(write_index + i) % src_rows]
// for i < src_rows, fill beyond; dst has dst_rows rows.
hipError_t launch_ring_rotate(const float *src, int src_rows, float *dst, int dst_rows, int n, int write_index,
                              float fill, hipStream_t s);

// Streaming float4 copy (bench copy ceiling, rfa_stream_copy).
hipError_t launch_stream_copy(void *dst, const void *src, size_t bytes, hipStream_t s);

}  // namespace rfa
