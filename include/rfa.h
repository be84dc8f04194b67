/*
 * rfa.h -- C-ABI of the MI355X-native RFAnalyzer spectrum pipeline (librfa.so).
 *
 * Replaces the reference's spectrum hot path (thomasjoergensen/RFAnalyzer):
 *
 *   reference interface                                   replaced by
 *   ----------------------------------------------------  -------------------------------------
 *   NativeDsp.performWindowedFftAndReturnMag(re,im,mag)    rfa_windowed_fft_mag_planar()
 *     nativedsp/src/main/java/com/mantz_it/nativedsp/NativeDsp.kt:43-62
 *   JNI performFFTAndLogMag(in[2N], out[N])                rfa_fft_logmag_interleaved()
 *     nativedsp/src/main/cpp/nativedsp.cpp:44-81
 *   JNI performFFT(in[2N], out[2N])                        rfa_fft_ordered()
 *     nativedsp/src/main/cpp/nativedsp.cpp:19-42
 *   IQConverter.fillPacketIntoSamplePacket + window + FFT  rfa_process() / rfa_process_host()
 *     source/Signed8BitIQConverter.java:80-99,                (raw IQ bytes in, fused on device)
 *     Unsigned8BitIQConverter.java:80-99,
 *     Signed16BitIQConverter.kt:89-124, Scheduler.kt:252-279
 *   FftProcessor.run ring write / retune shift / peak-hold rfa_process(), rfa_set_tuning(),
 *     analyzer/FftProcessor.kt:164-245                        rfa_get_ring(), rfa_get_peaks()
 *   AnalyzerSurface boxcar time average                    rfa_get_boxcar()
 *     ui/AnalyzerSurface.kt:657-714
 *   AnalyzerSurface.drawPreprocessing (colour rows, path)  rfa_draw_preprocess()
 *     ui/AnalyzerSurface.kt:599-743
 *   MainViewModel scanner / squelch row reductions          rfa_row_window_stats()
 *     ui/MainViewModel.kt:861-929,1391-1540
 *   IQConverter.mixPacketIntoSamplePacket + Decimator      rfa_ddc_*() (demod front end, below)
 *     source/Signed8BitIQConverter.java:53-131, analyzer/Decimator.java:175-191
 *   Resampler / RationalResampler (live demod path)        rfa_ddc_create_resampler()
 *     analyzer/Resampler.kt:102-110, dsp/RationalResampler.kt:27-127
 *   (north-star extension) exponential average             rfa_get_ema()
 *     idiom of database/GlobalPerformanceData.kt:44-50
 *
 * (app paths are relative to app/src/main/java/com/mantz_it/rfanalyzer/.)
 *
 * Conventions
 *  - Every function returns an int status: RFA_OK (0) or a negative RFA_ERR_*.
 *  - A handle is single-threaded; separate handles are independent (one per
 *    GPU / HIP stream).  There is no process-global state.
 *  - Output rows are 10*log10(|X_k|/N) (nativedsp.cpp:78), fft-shifted so that
 *    out[t] holds bin (t + N/2) mod N (out[0] = -fs/2, out[N/2] = DC).
 *  - N is a power of two, RFA_MIN_FFT_SIZE..RFA_MAX_FFT_SIZE.
 *  - Device pointers are HIP device (or host-coherent) addresses; work is
 *    enqueued on the handle's stream and is asynchronous unless the function
 *    name ends in _host or the doc says it synchronises.
 */
#ifndef RFA_H
#define RFA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef RFA_API
#define RFA_API __attribute__((visibility("default")))
#endif

#define RFA_ABI_VERSION 1
#define RFA_MIN_FFT_SIZE 64
#define RFA_MAX_FFT_SIZE (1 << 20)

enum rfa_status {
    RFA_OK = 0,
    RFA_ERR_INVALID = -1,     /* NULL handle/pointer, bad enum, bad size  */
    RFA_ERR_SIZE = -2,        /* array length mismatch (NativeDsp.kt:45-46) */
    RFA_ERR_UNSUPPORTED = -3, /* fft size / mode not supported             */
    RFA_ERR_NODEVICE = -4,    /* no HIP device visible                     */
    RFA_ERR_NOMEM = -5,       /* device / host allocation failed           */
    RFA_ERR_HIP = -6,         /* HIP runtime error (see rfa_last_error)    */
    RFA_ERR_STATE = -7        /* operation needs a feature not enabled     */
};

enum rfa_window { RFA_WINDOW_BLACKMAN = 0, RFA_WINDOW_HANN = 1, RFA_WINDOW_NONE = 2 };

/* Raw IQ sample formats (IQ_FILE_FORMAT.md / the converters above). */
enum rfa_input_format {
    RFA_IN_S8 = 0,             /* HackRF: int8 I,Q        -> b/128            */
    RFA_IN_U8 = 1,             /* RTL-SDR: uint8 I,Q      -> (b-127.4f)/128   */
    RFA_IN_S16LE = 2,          /* Airspy/HydraSDR: int16  -> s/32768          */
    RFA_IN_F32_INTERLEAVED = 3,/* float I,Q                                   */
    RFA_IN_F32_PLANAR = 4      /* per frame: float re[N] then float im[N]     */
};

enum rfa_avg_mode { RFA_AVG_NONE = 0, RFA_AVG_BOXCAR = 1, RFA_AVG_EMA = 2 };

typedef struct rfa_config {
    int32_t fft_size;      /* N, power of two                                       */
    int32_t window;        /* enum rfa_window                                       */
    int32_t input_format;  /* enum rfa_input_format                                 */
    int32_t avg_mode;      /* enum rfa_avg_mode (boxcar reads the ring)             */
    int32_t avg_length;    /* boxcar: L (average of the newest L+1 rows), 0..ring   */
    float ema_alpha;       /* EMA: avg += alpha*(x-avg), 0 < alpha <= 1             */
    int32_t peak_hold;     /* 0/1 (FftProcessor.kt:229-245)                         */
    int32_t ring_rows;     /* waterfall rows R (500/400/300, FftProcessor.kt:103), 0 = no ring */
    int32_t device_id;     /* HIP device ordinal                                    */
} rfa_config;

typedef struct rfa_handle rfa_handle;

/* Library / device queries (no handle). */
RFA_API int rfa_abi_version(void);
RFA_API int rfa_device_count(int *count);
RFA_API const char *rfa_status_string(int status);
RFA_API void rfa_default_config(rfa_config *cfg); /* N=16384, Blackman, s8, no avg, no peak, 400 rows, dev 0 */

/* Lifetime. */
RFA_API int rfa_create(const rfa_config *cfg, rfa_handle **out);
RFA_API int rfa_destroy(rfa_handle *h);
RFA_API int rfa_get_config(const rfa_handle *h, rfa_config *cfg);
RFA_API const char *rfa_last_error(const rfa_handle *h);

/* Stream control: work is enqueued on exactly `stream` (a hipStream_t; NULL is
 * the HIP null stream) until rfa_use_own_stream() restores the handle's own
 * non-blocking stream. */
RFA_API int rfa_set_stream(rfa_handle *h, void *stream);
RFA_API int rfa_use_own_stream(rfa_handle *h);
RFA_API int rfa_get_stream(const rfa_handle *h, void **stream);
RFA_API int rfa_synchronize(rfa_handle *h);

/* Pipelined state (opt-in, no reference counterpart: FftProcessor.kt:135-245 runs the FFT,
 * the ring write and the peak-hold one after another on one thread).  state_cus > 0 reserves
 * that many CUs (a multiple of the device's XCD count, spread one per shader engine) for a
 * CU-masked state stream that runs each call's peak / EMA / channel-mean pass, while the
 * FFT kernels run on two CU-masked streams over the other CUs, alternating per call.  Call
 * k's state pass then runs under call k + 1's FFT: a call that rewrites the whole ring
 * (n_frames == ring_rows) writes the second ring buffer (the ring and its shift buffer swap
 * per call, so rfa_get_state_generation advances), a call of at most ring_rows / 2 frames
 * writes rows call k's pass does not read, and any other call waits for the previous pass.
 * Pipelined calls are those with rows == NULL, a ring holding the batch, and peak-hold or
 * EMA on; the rest run as before.
 * The handle stream is NOT ordered after a pipelined call: rfa_join(h) enqueues on it a wait
 * for every pipelined kernel so far (the input buffers may be reused and the ring / peaks /
 * EMA read on that stream after it); rfa_synchronize and every other entry point join first.
 * state_cus = 0 turns the mode off (after a join).  RFA_ERR_UNSUPPORTED when the device does
 * not take CU masks or state_cus leaves no CUs for the FFT. */
RFA_API int rfa_set_pipelined(rfa_handle *h, int32_t state_cus);
RFA_API int rfa_join(rfa_handle *h);

/* Batch processing.  `in` holds n_frames frames of N samples in the configured
 * format, frame f starting at byte f*frame_stride_bytes (0 = densely packed).
 * For a headerless file replayed in packets of P bytes with N <= P/bps, the
 * reference's framing (Scheduler.kt:252-279: each packet fills one frame,
 * the rest of the packet is dropped) is frame_stride_bytes = P.
 * Rows go to `rows` (n_frames*N floats, frame order; may be NULL) and, if
 * ring_rows > 0, into the device waterfall ring in the reference's reverse
 * order (frames of this batch that the reference would overwrite within the
 * same batch are not stored).  Peak-hold / EMA state advance frame by frame.
 *   rfa_process      : device pointers, asynchronous on the handle stream.
 *   rfa_process_host : host pointers; copies in/out and synchronises. */
RFA_API int rfa_process(rfa_handle *h, const void *in, size_t n_frames, size_t frame_stride_bytes, float *rows);
RFA_API int rfa_process_host(rfa_handle *h, const void *in, size_t n_frames, size_t frame_stride_bytes, float *rows);

/* Multi-batch enqueue: the result of n_batches consecutive rfa_process calls (ring,
 * peaks, EMA and channel means advance batch after batch; ring rows, peaks and
 * channel means identical, the EMA equal to fp32 rounding -- the packed launch's
 * chunked scan associates the recursion differently), batch b reading
 * frames_per_batch frames at in + b * batch_stride_bytes + f * frame_stride_bytes
 * and writing its rows (if rows != NULL) at rows + b * frames_per_batch * N.
 * When the batches are packed (batch_stride_bytes == frames_per_batch * frame
 * stride) the whole run is ONE kernel launch, so small batches (BASELINE
 * config 4: 256 x 8192 points) stop paying a host call + launch each.
 * Device pointers, asynchronous on the handle stream; rfa_get_channel_means then
 * returns the last batch's frames_per_batch means, in either form. */
RFA_API int rfa_process_batches(rfa_handle *h, const void *in, size_t n_batches, size_t batch_stride_bytes,
                                size_t frames_per_batch, size_t frame_stride_bytes, float *rows);

/* Scheduler.run's FFT branch, one raw packet at a time (Scheduler.kt:252-273
 * with the converters' fillPacketIntoSamplePacket, Signed8BitIQConverter.java:80-98,
 * Unsigned8BitIQConverter.java:80-98, Signed16BitIQConverter.kt:89-124): the
 * packet's whole samples (host bytes in the handle's input format) fill the
 * handle's partial frame from the packet start at startIndex = samples already
 * held; once it holds N samples the frame is processed like rfa_process_host
 * (ring, peaks, EMA, channel mean) after rfa_set_tuning(frequency, sample_rate)
 * of the packet that completed it, and the rest of that packet is dropped.  So
 * P-sample packets give one frame per packet when P >= N and one frame every
 * ceil(N / P) packets when P < N (e.g. RTL-SDR's 16 KiB = 8192-sample packets,
 * RtlsdrSource.java:112, at the default N = 16384).  *frames = 1 when a frame
 * was processed (its row copied to row_out, N floats, unless NULL), else 0.
 * Only the completing packet's frequency / sample_rate are used, so only its
 * sample_rate must be > 0 (else RFA_ERR_INVALID and the frame is dropped); a
 * packet that only partly fills the frame is always accepted.
 * Synchronous.  RFA_ERR_UNSUPPORTED for RFA_IN_F32_PLANAR.  rfa_reset_state and
 * rfa_set_fft_size discard a partial frame (Scheduler.kt:259-260);
 * rfa_pending_samples reports how many samples it holds. */
RFA_API int rfa_push_packet(rfa_handle *h, const void *packet, size_t packet_bytes, int64_t frequency,
                            int64_t sample_rate, float *row_out, int32_t *frames);
RFA_API int rfa_pending_samples(const rfa_handle *h, int64_t *samples);

/* Tuning metadata of the following frames (SamplePacket.frequency/sampleRate).
 * Mirrors FftProcessor.kt:169-220,238-239: a frequency change shifts every ring
 * row by (int)((f_old-f_new)*(N/(float)sr)) bins with -9999 fill (or clears it
 * when |shift| >= N); a sample-rate change clears the ring; either resets the
 * peaks and the EMA.  The first call only records the values (the ring starts
 * cleared). */
RFA_API int rfa_set_tuning(rfa_handle *h, int64_t frequency, int64_t sample_rate);

/* State read-back (synchronise the handle stream; host destination).
 * rfa_get_ring copies ring_rows*N floats in storage order and returns the
 * reference's readIndex (newest row) and writeIndex (FftProcessorData). */
RFA_API int rfa_get_peaks(rfa_handle *h, float *out);
RFA_API int rfa_get_ema(rfa_handle *h, float *out);
RFA_API int rfa_get_boxcar(rfa_handle *h, int32_t length, float *out);
RFA_API int rfa_get_ring(rfa_handle *h, float *out, int32_t *read_index, int32_t *write_index);
RFA_API int rfa_reset_state(rfa_handle *h); /* ring -> -9999, peaks/EMA -> uninitialised */

/* Waterfall speed change (FftProcessor.kt:185-195, waterfallSpeed -> 500/400/300
 * rows, :103).  As in the reference the ring is rebuilt when the next frame
 * arrives (inside rfa_process), keeping the history: new row i = old row
 * (writeIndex + i) % old_rows for i < old_rows, -9999 rows beyond, then
 * writeIndex = 0.  Until then the old ring, readIndex and writeIndex stay
 * valid.  ring_rows >= 1; RFA_ERR_INVALID when a boxcar average_length would
 * not fit.  A ring_rows == 0 handle gains a cleared ring. */
RFA_API int rfa_set_ring_rows(rfa_handle *h, int32_t ring_rows);
/* FFT size change (FftProcessor.kt:178-183 ring re-created at -9999 with
 * writeIndex = 0, :233-236 peaks re-initialised; the EMA restarts): every
 * per-N table and state buffer is rebuilt for fft_size; tuning, channel range,
 * stream and ring_rows carry over.  Synchronises. */
RFA_API int rfa_set_fft_size(rfa_handle *h, int32_t fft_size);

/* Channel signal strength for the squelch (FftProcessor.kt:143-157): for every
 * frame of each rfa_process batch, the mean dB over bins
 * [((start - f0) * (N / sampleRate.toFloat())).toInt(), same for end), each
 * clamped to [0, N], f0 = frequency - sampleRate / 2 (the tuning of
 * rfa_set_tuning).  start_frequency == end_frequency disables it.  The sum is a
 * deterministic parallel reduction: equal to the reference's sequential fp32 loop
 * (:150-152) over the same row to the rounding of the sum -- so a
 * frame whose mean lies within that rounding of the squelch threshold can fall on
 * the other side of it than in the reference.
 * rfa_get_channel_means copies the last batch's means in frame order
 * (synchronises); *count = 0 when the channel range is empty. */
RFA_API int rfa_set_channel(rfa_handle *h, int64_t start_frequency, int64_t end_frequency);
RFA_API int rfa_get_channel_means(rfa_handle *h, float *out, size_t capacity, size_t *count);

/* Display preprocessing: the reference's
 * AnalyzerSurface.drawPreprocessing (app/.../ui/AnalyzerSurface.kt:599-743)
 * computed on the device from the ring, for the tuning of rfa_set_tuning and the
 * newest row rfa_get_ring reports.  The handle keeps the draw thread's state:
 * a persistent colour buffer and the dirty map (waterfallBufferDirtyMap).  Rows
 * written by rfa_process are dirty; a retune, clear, ring resize, new width or
 * new viewport / vertical scale marks every row.  A draw refreshes, newest
 * first, every dirty row and rows 0..average_length, at most
 * average_length + 6 rows (AnalyzerSurface.kt:619-640,678-684); the other rows
 * keep their colours, exactly as in the reference.  Outputs (host, synchronous):
 *   colors      [ring_rows][width] ARGB, ring storage order (colorBuffer[bufferIndex*width + i]):
 *               colormap[clamp(((avg - min_db) * scale).toInt())] of the pixel's mean
 *               bin value, black (0xff000000) outside the drawn range;
 *   fft_path_y  [width]: fftHeight - (timeAverage - min_db) * dbWidth of the boxcar over
 *               the newest average_length + 1 rows (the fftPath points), NaN where the
 *               reference adds no point;
 *   peaks_y     [width] or NULL: peaksYCoordinates (-1 outside), needs peak_hold;
 *   autoscale   [2] or NULL: min / max of the time averages, starting from
 *               (10, -100) = (VERTICAL_SCALE_UPPER_BOUNDARY, _LOWER_BOUNDARY), before
 *               the reference's +-5 dB margin (AnalyzerSurface.kt:731-735).
 * Bit-identical to the JVM's fp32 arithmetic; where the reference would index the
 * row out of bounds (and throw) the bin is skipped. */
typedef struct rfa_draw_params {
    int32_t width;                /* surface width in pixels                           */
    int32_t fft_height;           /* spectrum plot height in pixels                    */
    int64_t viewport_frequency;   /* viewport centre frequency (Hz)                    */
    int64_t viewport_sample_rate; /* viewport span (Hz)                                */
    float min_db, max_db;         /* vertical scale (viewportVerticalScaleMin/Max)     */
    int32_t average_length;       /* fftAverageLength, < ring_rows                     */
    int32_t colormap_size;        /* entries of colormap                               */
    const uint32_t *colormap;     /* ARGB colours, e.g. ColorMaps.kt createGqrxMap()   */
} rfa_draw_params;
RFA_API int rfa_draw_preprocess(rfa_handle *h, const rfa_draw_params *p, uint32_t *colors, float *fft_path_y,
                                float *peaks_y, float *autoscale);

/* Scanner / squelch reductions of the newest ring row:
 * for each inclusive bin window [lo[i], hi[i]] of the fft-shifted newest row
 * (FftProcessorData.readIndex), peak = FloatArray.maxOrNull() (NaN wins) and
 * avg = FloatArray.average().toFloat() (double sum / count).  Replaces the JVM
 * loops of MainViewModel.kt:861-929 (detectIEMChannelsInFFT, window
 * +-max(5, (100000 / resolution).toInt()) bins), :1391-1457 (getAverageSignalLevel,
 * detectSignal: the whole row [0, N-1]) and :1462-1540 (detectSignalsInFFT,
 * +-2 bins per step); the window arithmetic and thresholds stay with the caller
 * (rfanalyzer_amd/scanner.py mirrors them).  Synchronous, host arrays. */
RFA_API int rfa_row_window_stats(rfa_handle *h, const int32_t *lo, const int32_t *hi, size_t count, float *peak,
                                 float *avg);

/* Device-side state pointers, for zero-copy consumers.  peaks and EMA are in
 * natural (fft-shifted) bin order.  The ring's rows are stored in the order
 * rfa_get_ring_order reports.  The pointers (and the ring order) stay valid only
 * while rfa_get_state_generation returns the same value: a retune that shifts
 * the ring (rfa_set_tuning swaps the ring with its shift buffer), a ring resize
 * applied by rfa_process (rfa_set_ring_rows) and rfa_set_fft_size (which rebuilds
 * every buffer and frees the old ones) each advance it; re-query after a change. */
RFA_API int rfa_get_device_state(rfa_handle *h, float **ring, float **peaks, float **ema);
RFA_API int rfa_get_state_generation(const rfa_handle *h, int64_t *generation);

/* Storage order of the device ring rows (no reference counterpart: the JVM
 * waterfallBuffer rows are natural order, FftProcessor.kt:222-227, and
 * rfa_get_ring returns them so).  *residues = RS: the fft-shifted bin t of a
 * device ring row lives in block t mod RS of N/RS elements.  RS = 1 is one block;
 * the N = 64 K / 128 K kernels compute a frame as RS residue sub-FFTs and store
 * each residue's bins as one block (whole cache lines per workgroup); N = 256 K ..
 * 1 M use RS = N / 32768 (the large-N kernel B writes the bins S q + s of column
 * s as block s).  Inside a block, N = 32 K .. 128 K keep the 32 K-point kernel's
 * store tiles (16-B stores per lane); N = 256 K .. 1 M and N <= 16 K natural
 * order (bin t at block offset t / RS).  rfa_get_ring_positions fills the
 * storage position of every fft-shifted bin (positions[N]) for zero-copy
 * consumers; every rfa_* consumer of the ring handles the order internally. */
RFA_API int rfa_get_ring_order(const rfa_handle *h, int32_t *residues);
RFA_API int rfa_get_ring_positions(const rfa_handle *h, int32_t *positions, size_t count);

/* Reference-seam entry points (host arrays, synchronous).  They use the
 * handle's N; the window/format of the handle are ignored where the reference
 * symbol fixes them. */
/* NativeDsp.kt:43-62: Blackman-windowed FFT of planar re/im, log-mag row out.
 * Returns RFA_ERR_SIZE on length mismatch (the Kotlin method returns false). */
RFA_API int rfa_windowed_fft_mag_planar(rfa_handle *h, const float *re, const float *im, float *mag_out, size_t n);
/* nativedsp.cpp:44-81: already-windowed interleaved input (2N floats) -> N dB. */
RFA_API int rfa_fft_logmag_interleaved(rfa_handle *h, const float *in, float *mag_out, size_t n);
/* nativedsp.cpp:19-42: ordered, unscaled, forward complex FFT, 2N floats each. */
RFA_API int rfa_fft_ordered(rfa_handle *h, const float *in, float *out, size_t n);

/* The same three seams at every length the reference's pffft accepts
 * (pffft_new_setup, pffft.c:1231-1280: N a multiple of 16, N / 4 a product of
 * 2, 3, 4 and 5, N <= 2^26), one plan per N like nativedsp.cpp:12-17's cached
 * setup.  rfa_create covers the powers of two 64 .. 2^20 with its fused kernels;
 * a plan serves the rest (16, 32, 2^21 .. 2^26, mixed lengths such as 48 or
 * 3 * 2^20) with a mixed-radix Stockham FFT on the GPU (csrc/fft_seam.hip).
 * rfa_seam_create returns RFA_ERR_UNSUPPORTED for a length pffft rejects.
 * Synchronous, host arrays, RFA_ERR_SIZE on a length mismatch. */
typedef struct rfa_seam rfa_seam;
RFA_API int rfa_seam_supported(int32_t n); /* 1 when pffft accepts N, else 0 */
RFA_API int rfa_seam_create(int32_t n, int32_t device_id, rfa_seam **out);
RFA_API int rfa_seam_destroy(rfa_seam *s);
RFA_API const char *rfa_seam_last_error(const rfa_seam *s);
/* the pass radices (8, 4, 2, 3, 5), first pass first; count = number of passes */
RFA_API int rfa_seam_get_plan(const rfa_seam *s, int32_t *radices, int32_t cap, int32_t *count);
RFA_API int rfa_seam_windowed_fft_mag_planar(rfa_seam *s, const float *re, const float *im, float *mag_out, size_t n);
RFA_API int rfa_seam_fft_logmag_interleaved(rfa_seam *s, const float *in, float *mag_out, size_t n);
RFA_API int rfa_seam_fft_ordered(rfa_seam *s, const float *in, float *out, size_t n);

/* Profiling: while enabled, HIP events bracket every main FFT kernel launch on
 * the handle stream; rfa_get_kernel_time waits for and sums them.  Toggling
 * never synchronises, so a caller may profile a sample of its launches. */
/* Measurement support (no reference counterpart).  rfa_stream_copy: the device
 * stream-copy kernel whose rate is the measured bandwidth ceiling SURVEY.md
 * §8(d) asks the bench to report beside the 8 TB/s spec (float4 loads and
 * stores, several in flight per lane; bytes a multiple of 16, 16-byte aligned
 * device pointers), asynchronous on `stream` (a hipStream_t, NULL = default). */
RFA_API int rfa_stream_copy(void *dst, const void *src, size_t bytes, void *stream);
RFA_API int rfa_set_profiling(rfa_handle *h, int enable);
RFA_API int rfa_get_kernel_time(rfa_handle *h, double *total_ms, int64_t *launches);
/* Host-only helper (no device work): the waterfall shift in bins applied by
 * rfa_set_tuning for a retune by frequency_diff = last_frequency - frequency,
 * ((lastF - f) * (N / sampleRate.toFloat())).toInt() in fp32 with Kotlin's
 * truncating, saturating Float.toInt() (FftProcessor.kt:143,173,199). */
RFA_API int64_t rfa_retune_offset(int64_t frequency_diff, int n, int64_t sample_rate);
/* Name of the HIP kernel rfa_process launches for this handle's configuration
 * ("fft_wide_kernel" or "fft_rows_kernel"), as rocprofv3 reports it. */
RFA_API const char *rfa_main_kernel_name(const rfa_handle *h);

/* ------------------------------------------------------------------------
 * Demod-branch front end: NCO down-mix of raw IQ
 * bytes + decimating low-pass FIR, one handle per demodulated channel.
 * Replaces (app paths as above):
 *   IQConverter.mixPacketIntoSamplePacket        rfa_ddc_set_frequencies() +
 *     source/Signed8BitIQConverter.java:53-131,    rfa_ddc_process()
 *     Unsigned8BitIQConverter.java:53-131,
 *     Signed16BitIQConverter.kt:59-181, IQConverter.java:64-76
 *   Decimator.downsampling / FirFilter.filter    rfa_ddc_process()
 *     analyzer/Decimator.java:175-191, dsp/FirFilter.kt:63-107
 *   FirFilter.createLowPassTaps                  rfa_lowpass_taps()  (host only)
 *     dsp/FirFilter.kt:134-195, dsp/WindowFunctions.kt:44-52
 * The filter state (delay line, decimation counter) and the mixer's cosine
 * index carry over between calls exactly as in the reference, so one call on
 * a long buffer equals the reference run packet by packet.
 * ------------------------------------------------------------------------ */
typedef struct rfa_ddc rfa_ddc;

/* input_format: RFA_IN_S8 / RFA_IN_U8 / RFA_IN_S16LE are mixed then filtered;
 * RFA_IN_F32_INTERLEAVED is taken as already-mixed samples and only filtered
 * (the Decimator on a float SamplePacket).  Decimation = sample_rate /
 * output_sample_rate; taps = createLowPassTaps(decimation, 1, sample_rate,
 * 0.75 * out, 0.25 * out, 60) (Decimator.java:177-181).  RFA_ERR_INVALID where
 * the reference's filter design returns null. */
RFA_API int rfa_ddc_create(int device, int input_format, int32_t sample_rate, int32_t output_sample_rate,
                           rfa_ddc **out);
/* The same front end with the resampler the live app uses instead of the
 * Decimator (analyzer/Resampler.kt:102-110, dsp/RationalResampler.kt): the
 * ratio out/in reduced by limitDenominator(out, in, 10000), polyphase bank
 * from designResamplerTaps (Kaiser beta 7, fractionalBw 0.4, 500 taps per phase
 * at most), outputs in the reference's phase order.  Downsampling only
 * (RFA_ERR_UNSUPPORTED otherwise, as the reference's TODO states).
 * rfa_ddc_get_taps returns the prototype padded to a multiple of the
 * interpolation; rfa_ddc_get_ratio the reduced interpolation/decimation. */
RFA_API int rfa_ddc_create_resampler(int device, int input_format, int32_t sample_rate, int32_t output_sample_rate,
                                     rfa_ddc **out);
/* A FirFilter with the caller's taps and decimation (dsp/FirFilter.kt:34-110,
 * e.g. FirFilter.createLowPass): delay line of num_taps zeros, decimationCounter
 * 1, outputs sum taps[k] * delay[newest - k] with the JVM's separately rounded
 * products and sums.  input_format as in rfa_ddc_create (RFA_IN_F32_INTERLEAVED:
 * samples taken as they are; raw formats are mixed first). */
RFA_API int rfa_ddc_create_fir(int device, int input_format, int32_t sample_rate, const float *taps, int32_t num_taps,
                               int32_t decimation, rfa_ddc **out);
/* Enqueue on exactly `stream` (a hipStream_t; NULL restores the handle's own
 * stream).  Pending work of the previous stream is drained first. */
RFA_API int rfa_ddc_set_stream(rfa_ddc *d, void *stream);
RFA_API int rfa_ddc_get_ratio(const rfa_ddc *d, int32_t *interpolation, int32_t *decimation, int32_t *taps_per_output);
RFA_API int rfa_ddc_get_format(const rfa_ddc *d, int32_t *input_format);  /* rfa_input_format of the handle */
RFA_API int rfa_ddc_destroy(rfa_ddc *d);
RFA_API const char *rfa_ddc_last_error(const rfa_ddc *d);
/* Like IQConverter.setSampleRate + the Decimator's rebuild check: the mixer
 * table is invalidated; the filter is rebuilt (fresh delay line) only when the
 * integer decimation changes (Decimator.java:177-178). */
RFA_API int rfa_ddc_set_sample_rate(rfa_ddc *d, int32_t sample_rate);
/* mixFrequency = (int)(frequency - channel_frequency), folded by +sample_rate
 * when 0 or when sample_rate / |mix| > 500; the table (and the cosine index)
 * is regenerated only when the folded frequency changes. */
RFA_API int rfa_ddc_set_frequencies(rfa_ddc *d, int64_t frequency, int64_t channel_frequency);
/* n_samples complex samples of raw input at device address `in` -> the
 * decimated outputs at device out_re/out_im (planar float).  *n_out is set on
 * return (computed on the host); RFA_ERR_SIZE if it would exceed out_capacity
 * (nothing is consumed then).  Asynchronous on the handle's stream. */
RFA_API int rfa_ddc_process(rfa_ddc *d, const void *in, size_t n_samples, float *out_re, float *out_im,
                            size_t out_capacity, size_t *n_out);
/* Same with host buffers; synchronous. */
RFA_API int rfa_ddc_process_host(rfa_ddc *d, const void *in, size_t n_samples, float *out_re, float *out_im,
                                 size_t out_capacity, size_t *n_out);
RFA_API int rfa_ddc_synchronize(rfa_ddc *d);
RFA_API int rfa_ddc_get_stream(const rfa_ddc *d, void **stream);
/* Current design: taps (capacity floats), mixer cos/sin per time step
 * (capacity floats each, may be NULL), counts and folded mix frequency. */
RFA_API int rfa_ddc_get_taps(const rfa_ddc *d, float *taps, size_t capacity, int32_t *num_taps, int32_t *decimation);
RFA_API int rfa_ddc_get_mixer(const rfa_ddc *d, float *cos_t, float *sin_t, size_t capacity, int32_t *length,
                              int32_t *mix_frequency, int32_t *cosine_index);
/* Host-only filter design, FirFilter.createLowPassTaps with a Blackman window
 * (no device work).  *num_taps is always set; taps written when it fits. */
/* Host-only RationalResampler design: limitDenominator + designResamplerTaps
 * (RationalResampler.kt:165-235); the prototype taps before the polyphase split. */
RFA_API int rfa_resampler_design(int32_t output_rate, int32_t input_rate, int32_t max_denominator, float fractional_bw,
                                 int32_t max_taps, int32_t *interpolation, int32_t *decimation, float *taps,
                                 size_t capacity, int32_t *num_taps);
RFA_API int rfa_lowpass_taps(float gain, float sample_rate, float cutoff, float transition, float attenuation,
                             int32_t max_taps, float *taps, size_t capacity, int32_t *num_taps);

#ifdef __cplusplus
}
#endif

#endif /* RFA_H */
