// Display preprocessing on the device: the reference's
// AnalyzerSurface.drawPreprocessing (app/.../ui/AnalyzerSurface.kt:599-743)
// computed from the waterfall ring where it already lives, so a frame of the UI
// needs width-sized rows back instead of N-float rows.
//
// Per ring row (newest first, rowNumber r -> bufferIndex (readIndex + r) % R) and
// pixel i inside (firstPixel, lastPixel - 1): the mean of the row's bins
// j in [(int)(i*spp), (i+1)*spp) (stopping at N), summed in bin order in fp32
// (AnalyzerSurface.kt:693-705); the colour map index ((avg - minDB) * scale)
// truncated and clamped (:721-722); black outside (:725).  Rows 0..L feed the
// time average, summed newest first per pixel (:710-714), whose spectrum-path y
// and autoscale min/max come from draw_finish_kernel; row 0 also gives the
// peak-hold y (:707).  Every float operation is the reference's single fp32
// operation in the reference's order (no FMA contraction), so the results are
// bit-identical to the JVM's.
#include <hip/hip_runtime.h>

#include <cmath>

#include "fft_kernels.h"
#include "wave.h"

namespace rfa {

#pragma clang fp contract(off)

// Kotlin Float.toInt(): truncation, NaN -> 0, saturating.
__device__ __forceinline__ int kt_toint(float x) {
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x <= -2147483648.0f) return (-2147483647 - 1);
    return (int)x;
}

// java.lang.Math.min / max on floats: NaN wins, -0 < +0.
__device__ __forceinline__ float jmin(float a, float b) {
    if (a != a || b != b) return NAN;
    if (a == b) return signbit(a) ? a : b;
    return a < b ? a : b;
}
__device__ __forceinline__ float jmax(float a, float b) {
    if (a != a || b != b) return NAN;
    if (a == b) return signbit(a) ? b : a;
    return a > b ? a : b;
}

// One block row per refreshed ring row (the host picks them as the reference's
// dirty-row loop does, AnalyzerSurface.kt:678-684); the other rows keep their colours.
__global__ void __launch_bounds__(256) draw_rows_kernel(DrawLaunch a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int2 sel = a.rows[blockIdx.y];
    const int row_number = sel.x;
    if (i >= a.width) return;
    const int buffer_index = sel.y;
    const float *row = a.ring + (size_t)buffer_index * a.n;
    const int lm = ring_logm(a.ring_logrs, 31 - __clz(a.n));  // ring storage order (ring_pos)
    unsigned *out = a.colors + (size_t)buffer_index * a.width + i;
    if (i >= a.first_pixel + 1 && i < a.last_pixel - 1) {
        const bool peaks_here = row_number == 0 && a.peaks_y;
        float avg = 0.0f, peak_avg = 0.0f;
        int counter = 0;
        const float hi = (float)(i + 1) * a.samples_per_px;
        // (the reference reads fftRow[j + start] unchecked; a negative index -- which
        // would throw there -- is skipped here instead of read)
        int j = kt_toint((float)i * a.samples_per_px);
        if (j + a.start < 0) j = -a.start;
        for (; (float)j < hi && j + a.start < a.n; j++) {
            avg += row[ring_pos(j + a.start, a.ring_logrs, lm)];
            if (peaks_here) peak_avg += a.peaks[j + a.start];
            counter++;
        }
        avg = avg / (float)counter;
        if (peaks_here) {
            const float pk = peak_avg / (float)counter;
            a.peaks_y[i] = (float)a.fft_height - (pk - a.min_db) * a.db_width;
        }
        if (row_number <= a.avg_length) a.avg_rows[(size_t)row_number * a.width + i] = avg;
        int ci = kt_toint((avg - a.min_db) * a.scale);
        ci = ci < 0 ? 0 : (ci >= a.colormap_size ? a.colormap_size - 1 : ci);
        *out = a.colormap[ci];
    } else {
        *out = 0xff000000u;  // Color.rgb(0, 0, 0)
        if (row_number == 0 && a.peaks_y) a.peaks_y[i] = -1.0f;
    }
}

// Time average of rows 0..L per pixel (newest first), spectrum-path y, autoscale
// min/max starting from (VERTICAL_SCALE_UPPER_BOUNDARY, _LOWER_BOUNDARY) =
// (10, -100) (AppStateRepository.kt:92-93).  One workgroup; path y is NaN where
// the reference adds no path point.
__global__ void __launch_bounds__(1024) draw_finish_kernel(DrawLaunch a) {
    __shared__ float smin[16], smax[16];
    float mn = 10.0f, mx = -100.0f;
    for (int i = threadIdx.x; i < a.width; i += blockDim.x) {
        if (i >= a.first_pixel + 1 && i < a.last_pixel - 1) {
            float acc = 0.0f;
            for (int r = 0; r <= a.avg_length; r++) acc += a.avg_rows[(size_t)r * a.width + i];
            const float ta = acc / (float)(a.avg_length + 1);
            a.path_y[i] = (float)a.fft_height - (ta - a.min_db) * a.db_width;
            mn = jmin(ta, mn);
            mx = jmax(ta, mx);
        } else {
            a.path_y[i] = NAN;
        }
    }
    // min / max are order independent (NaN propagates either way): per wave by
    // cross-lane moves (wave.h), then the waves' results
    mn = wave_reduce(mn, [](float x, float y) { return jmin(x, y); });
    mx = wave_reduce(mx, [](float x, float y) { return jmax(x, y); });
    const int nw = (blockDim.x + 63) / 64;
    if ((threadIdx.x & 63) == 0) {
        smin[threadIdx.x >> 6] = mn;
        smax[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < nw; k++) {
            mn = jmin(mn, smin[k]);
            mx = jmax(mx, smax[k]);
        }
        a.autoscale[0] = mn;
        a.autoscale[1] = mx;
    }
}

// Newest-row window statistics for the scanners and squelch (SURVEY.md §8(f)
// row 2; MainViewModel.kt:861-929 detectIEMChannelsInFFT, :1391-1457
// getAverageSignalLevel / detectSignal, :1462-1540 detectSignalsInFFT): for every
// window [lo, hi] (inclusive bins of the fft-shifted row) the peak
// (FloatArray.maxOrNull: NaN wins) and FloatArray.average() -- a double sum
// divided by the count, then toFloat().  One workgroup per window; the double
// partial sums meet by wavefront shuffles and then across the four waves (a different
// summation order than the JVM's sequential one, equal after the final rounding to
// float up to one ulp).
__global__ void __launch_bounds__(256) row_window_kernel(const float *row, int logrs, int n, const int *lo,
                                                         const int *hi, int count, float *peak, float *avg) {
    const int w = blockIdx.x;
    if (w >= count) return;
    const int lm = ring_logm(logrs, 31 - __clz(n));  // ring storage order (ring_pos)
    const int a = lo[w], b = hi[w];
    float mx = -INFINITY;
    bool nan = false;
    double s = 0.0;
    for (int j = a + (int)threadIdx.x; j <= b; j += 256) {
        const float x = row[ring_pos(j, logrs, lm)];
        nan |= x != x;
        mx = x > mx ? x : mx;
        s += (double)x;
    }
    // per wave by cross-lane moves (wave.h), then the four waves in order
    s = wave_reduce(s, [](double x, double y) { return x + y; });
    mx = wave_reduce(mx, [](float x, float y) { return fmaxf(x, y); });
    const int anynan = wave_reduce((int)nan, [](int x, int y) { return x | y; });
    __shared__ double ss[4];
    __shared__ float sm[4];
    __shared__ int sn[4];
    if ((threadIdx.x & 63) == 0) {
        ss[threadIdx.x >> 6] = s;
        sm[threadIdx.x >> 6] = mx;
        sn[threadIdx.x >> 6] = anynan;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double sum = ((ss[0] + ss[1]) + ss[2]) + ss[3];
        const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
        peak[w] = (sn[0] | sn[1] | sn[2] | sn[3]) ? NAN : m;
        avg[w] = (float)(sum / (double)(b - a + 1));
    }
}

hipError_t launch_row_windows(const float *row, int ring_logrs, int n, const int *lo, const int *hi, int count,
                              float *peak, float *avg, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(row_window_kernel, dim3(count), dim3(256), 0, s, row, ring_logrs, n, lo, hi, count, peak, avg);
    return hipGetLastError();
}

hipError_t launch_draw(const DrawLaunch &a) {
    if (a.width <= 0 || a.ring_rows <= 0 || a.n_rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(draw_rows_kernel, dim3((a.width + 255) / 256, a.n_rows), dim3(256), 0, a.stream, a);
    hipLaunchKernelGGL(draw_finish_kernel, dim3(1), dim3(1024), 0, a.stream, a);
    return hipGetLastError();
}

}  // namespace rfa
