// N = 2^18 .. 2^20 (BASELINE config 5, 1 M-point FFT): decimation in frequency
// over S = N / M column DFTs, M = 32768.  With n = m + M j (m < M, j < S) and
// k = S q + s (q < M, s < S):
//
//   X[S q + s] = sum_m W_M^{m q} [ W_N^{m s} sum_j x[m + M j] w[m + M j] W_S^{j s} ]
//                                 `------------------ z_s[m] -------------------'
//
// Kernel A (here, dif_front_kernel): one thread per m.  The S samples x[m + M j]
// of a column sit in S contiguous rows of the frame, so every load instruction
// is a run of consecutive samples across the lanes; convert (LUT-exact), window
// (fp32 multiply with the natural window, NativeDsp.kt:55-58), an in-register
// DFT-S, the twiddle W_N^{m s} = C[s][m >> 7] * (1 + D[s][m & 127]) (both tables
// from double; D is the small difference to 1, so the product is nearly as exact
// as C itself), and one coalesced 8-B store per s into scratch z[f][s][m].
//
// Kernel B (fft_wide.hip, input format 5): the 32 K-point workgroup transforms
// z_s (contiguous, already windowed) and writes bins S q + s: into the device
// ring as residue-major block s (ring_pos, logrs = log2 S -- whole lines per
// workgroup); caller rows go residue-major to a scratch and cols_to_rows_kernel
// puts them in natural order; the ordered complex spectrum is stored at stride S.
// Scratch traffic is 16 B per sample (write + read); the engine sizes batches so
// the scratch stays in the 256 MB Infinity Cache.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "fft_common.h"
#include "fft_kernels.h"

namespace rfa {

// Twiddle split m = khi * 2^LO + klo of W_N^{m s} = C[s][khi] (1 + D[s][klo]) (khi is wave-uniform
// for LO >= 6).  The per-tile kernel (16/32-bit input) keeps LO = 7; the pipelined 8-bit kernel
// takes LO = 6: its D table halves to 16 KB of LDS (round 5, profiles/r05/large_n_front_ab.txt).
#ifndef RFA_DIF_LOBITS
#define RFA_DIF_LOBITS 6  // the pipelined kernel's LO (A/B: 7)
#endif
constexpr int kDifLoTile = 128, kDifLoPipe = 1 << RFA_DIF_LOBITS;
#ifndef RFA_DIF_SC1
#define RFA_DIF_SC1 1  // z stores write-through (sc1): the scratch leaves the XCD's L2 for kernel B
#endif
#ifndef RFA_DIF_WPE
#define RFA_DIF_WPE 1  // minimum waves per SIMD the compiler must allow (4: <= 128 VGPRs)
#endif
#ifndef RFA_DIF_DGLOBAL
#define RFA_DIF_DGLOBAL 0  // D factors read through L1 instead of the 32 KB LDS table
#endif
#ifndef RFA_DIF_ST16
#define RFA_DIF_ST16 1  // z stored 16 B per lane: lane pairs swap one value per two rows (A/B: 0)
#endif

// The S rows of column m into z (row s at s * M): 16 B per lane (RFA_DIF_ST16) -- rows s, s + 1 of
// the column pair (m & ~1, m | 1): the even lane stores row s, the odd lane row s + 1, each both
// columns.  Both rows' values cross (DPP quad_perm 1,0,3,2) and each lane picks: a select between
// v[s] and v[s + 1] themselves became a select of addresses and put v[] on the stack (S = 16: 80 B
// of scratch, +35 %).  Write-through (sc1): kernel B reads z from other XCDs.
template <int S>
__device__ __forceinline__ void store_z(const float2 *v, rsrc_t z_rs, int m) {
    constexpr int M = 1 << kDitLogM;
#if RFA_DIF_ST16
    const bool p = (m & 1) != 0;
    auto swap = [](float2 x) {
        return make_float2(
            __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x.x), 0xB1, 0xF, 0xF, false)),
            __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x.y), 0xB1, 0xF, 0xF, false)));
    };
#pragma unroll
    for (int s = 0; s < S; s += 2) {
        const float2 r0 = swap(v[s]), r1 = swap(v[s + 1]);  // the partner's rows s, s + 1
        const float2 lo = p ? r1 : v[s], hi = p ? v[s + 1] : r0;
        if constexpr (RFA_DIF_SC1) buf_store_f32x4(lo.x, lo.y, hi.x, hi.y, z_rs, ((m - p) + p * M) * 8, s * M * 8);
        else buf_store_f32x4_wb(lo.x, lo.y, hi.x, hi.y, z_rs, ((m - p) + p * M) * 8, s * M * 8);
    }
#else
#pragma unroll
    for (int s = 0; s < S; s++) buf_store_f32x2(v[s], z_rs, m * 8, s * M * 8);
#endif
}

template <int S, int FMT>
__global__ void __launch_bounds__(256) dif_front_kernel(DifLaunch a) {
    constexpr int M = 1 << kDitLogM, n = S * M;
    constexpr int SB = (FMT == 0 || FMT == 1) ? 2 : (FMT == 2 || FMT == 4) ? 4 : 8;  // bytes per sample (per plane)
    constexpr int PLANES = FMT == 4 ? 2 : 1;
    // 8/16-bit formats: the block's raw tile (S rows x 256 consecutive samples) is
    // fetched with 16-B loads all in flight at once, then read per thread from LDS.
    // f32 formats load straight into registers (8 B per lane is already a wide
    // access; their 64 KB tile would halve the resident blocks: measured slower).
    constexpr bool TILE = FMT <= 2;
    constexpr int ROWB = 256 * SB, PPR = ROWB / 16, NP = TILE ? S * PPR : 256;
    static_assert(NP % 256 == 0, "whole 16-B pieces per thread");
    __shared__ uint4 tile[NP];
    const int m0 = blockIdx.x * 256, m = m0 + threadIdx.x;
    const int f = blockIdx.y;
    const rsrc_t in_rs = make_rsrc(a.in + (size_t)f * (size_t)a.frame_stride, n * SB * PLANES);
    const rsrc_t w_rs = make_rsrc(a.window, n * 4);
    float2 v[S];
    if constexpr (TILE) {
        {
            uint4 q[NP / 256];
#pragma unroll
            for (int i = 0; i < NP / 256; i++) {
                const int e = i * 256 + threadIdx.x;
                const int j = e / PPR, pc = e % PPR;
                q[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(in_rs, pc * 16, (j * M + m0) * SB, 0));
            }
#pragma unroll
            for (int i = 0; i < NP / 256; i++) tile[i * 256 + threadIdx.x] = q[i];
        }
        float w[S];
#pragma unroll
        for (int j = 0; j < S; j++) w[j] = buf_load_f32(w_rs, m * 4, j * M * 4);
        __syncthreads();
        const uint8_t *tb = reinterpret_cast<const uint8_t *>(tile);
#pragma unroll
        for (int j = 0; j < S; j++) {
            const float2 x = convert_raw<FMT>(*reinterpret_cast<const typename Raw<FMT>::T *>(tb + j * ROWB + threadIdx.x * SB));
            v[j] = make_float2(x.x * w[j], x.y * w[j]);  // NativeDsp.kt:55-58 (fp32 multiply)
        }
    } else {
        // chunks of 8 rows (scheduling barriers): fewer live registers, more waves per SIMD
        constexpr int CH = S < 8 ? S : 8;
#pragma unroll
        for (int j0 = 0; j0 < S; j0 += CH) {
            typename Raw<FMT>::T raw[CH];
            float w[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) {
                raw[j] = buf_load_raw<FMT>(in_rs, m * SB, (j0 + j) * M * SB, n * 4);
                w[j] = buf_load_f32(w_rs, m * 4, (j0 + j) * M * 4);
            }
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const float2 x = convert_raw<FMT>(raw[j]);
                v[j0 + j] = make_float2(x.x * w[j], x.y * w[j]);  // NativeDsp.kt:55-58 (fp32 multiply)
            }
            if (j0 + CH < S) __builtin_amdgcn_sched_barrier(0);
        }
    }
    dft<S>(v);  // v[s] = sum_j x w W_S^{j s}
    // m >> 7 is the same for the 64 lanes of a wave (256-thread blocks of consecutive m):
    // the C factors are scalar loads
    const int khi = __builtin_amdgcn_readfirstlane(m >> 7), klo = m & (kDifLoTile - 1);
    constexpr int mc = M / kDifLoTile;
    // W_N^{m s} = C (1 + delta): the small correction C * delta is added last, so the
    // twiddle carries C's rounding and one add instead of a full product's.  Chunks
    // of 8 (scheduling barriers) keep the delta loads from all being live at once.
#pragma unroll
    for (int s0 = 0; s0 < S; s0 += 8) {
        float2 d[8];
#pragma unroll
        for (int s = s0; s < s0 + 8 && s < S; s++) d[s - s0] = a.tw_d[s * kDifLoTile + klo];
#pragma unroll
        for (int s = (s0 ? s0 : 1); s < s0 + 8 && s < S; s++) {
            const float2 c = a.tw_c[s * mc + khi], corr = cmul(c, d[s - s0]);
            v[s] = cmul(v[s], make_float2(c.x + corr.x, c.y + corr.y));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    store_z<S>(v, make_rsrc(a.z + (size_t)f * n, n * 8), m);
}

// 8-bit formats, persistent and pipelined: block b owns the 256 columns
// (b % 128) * 256 .. + 255 and frames b / 128, + G, + 2G, ... (G = frame groups).
// The window values of its columns stay in registers and the D table in LDS
// across its frames; the next frame's tile is fetched by LDS-DMA (16 B per lane,
// no VGPRs) right after every wave has read the current one, so it lands while
// this frame is transformed and its z stores drain: loads and stores of a block
// overlap instead of every block loading, then storing, in lock step.
// BW columns per block.  512-column blocks (one D table per 8 waves, 4 waves per SIMD) measured
// -1.4 % at 1 M with the ring and +3 % at 256 K / 512 K (profiles/r04/dif_block_width_ab.txt)
template <int S, int FMT, int BW = 256>
__global__ void __launch_bounds__(BW, BW >= 512 ? 2 : RFA_DIF_WPE) dif_front_pipe_kernel(DifLaunch a, int groups) {
    static_assert(FMT <= 1, "8-bit formats");
    constexpr int M = 1 << kDitLogM, n = S * M, mc = M / kDifLoPipe;
    constexpr int SB = 2, NW = BW / 64;
    constexpr int ROWB = BW * SB, TILEB = S * ROWB, NPIECE = TILEB / 1024, PPW = NPIECE / NW;
    constexpr int RPP = ROWB >= 1024 ? 1 : 1024 / ROWB, LPR = 64 / RPP;  // tile rows per 1 KiB piece, lanes per row
    constexpr int PPR = ROWB >= 1024 ? ROWB / 1024 : 1;                   // 1 KiB pieces per tile row
    static_assert(NPIECE % NW == 0 && RPP >= 1, "whole pieces per wave");
    __shared__ __attribute__((aligned(16))) uint8_t tile[TILEB];
#if RFA_DIF_DGLOBAL
    const float2 *dtab = a.tw_dp;
#else
    __shared__ float2 dtab[S * kDifLoPipe];
#endif
    const int bx = blockIdx.x % (M / BW), g0 = blockIdx.x / (M / BW);
    const int m0 = bx * BW, m = m0 + threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const unsigned tbase = (unsigned)(size_t)(__attribute__((address_space(3))) uint8_t *)tile;
    auto stage = [&](int f) {  // this wave's PPW pieces of frame f's tile (inline asm: see stage_frame)
        const rsrc_t rs = make_rsrc(a.in + (size_t)f * (size_t)a.frame_stride, n * SB);
#pragma unroll
        for (int i = 0; i < PPW; i++) {
            const int pc = wave * PPW + i, j = (pc / PPR) * RPP + lane / LPR;
            const int voff = (j * M + m0) * SB + (pc % PPR) * 1024 + (lane % LPR) * 16;
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "s"(tbase + pc * 1024), "v"(voff), "s"(rs)
                : "memory");
        }
    };
#if !RFA_DIF_DGLOBAL
    for (int e = threadIdx.x; e < S * kDifLoPipe; e += BW) dtab[e] = a.tw_dp[e];
#endif
    const rsrc_t w_rs = make_rsrc(a.window, n * 4);
    float w[S];
#pragma unroll
    for (int j = 0; j < S; j++) w[j] = buf_load_f32(w_rs, m * 4, j * M * 4);
    const int khi = __builtin_amdgcn_readfirstlane(m >> RFA_DIF_LOBITS), klo = m & (kDifLoPipe - 1);
    // C factors through the constant address space: the index is wave-uniform, so they
    // are scalar loads (s_load_dwordx2) instead of a uniform-address VMEM load per s
    const auto *tw_c_s = (const __attribute__((address_space(4))) f2v *)(uintptr_t)a.tw_cp;
    auto c_at = [&](int i) { return from_v(tw_c_s[i]); };
    if (g0 < a.n_frames) stage(g0);
    bool first = true;
    for (int f = g0; f < a.n_frames; f += groups) {
        // this frame's tile has landed (younger than its DMA: the previous frame's z stores, S or S / 2)
        if (first) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(RFA_DIF_ST16 ? S / 2 : S) : "memory");
        first = false;
        float2 v[S];
#pragma unroll
        for (int j = 0; j < S; j++) {
            const auto raw = *reinterpret_cast<const typename Raw<FMT>::T *>(tile + j * ROWB + threadIdx.x * SB);
            const float2 x = convert_raw<FMT>(raw);
            v[j] = make_float2(x.x * w[j], x.y * w[j]);  // NativeDsp.kt:55-58 (fp32 multiply)
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave has read the tile
        if (f + groups < a.n_frames) stage(f + groups);
        dft<S>(v);
        {  // W_N^{m s} = C (1 + delta), as dif_front_kernel; C in SGPRs (scalar loads,
           // profiles/r03/dif_front_smem_ab.txt)
            {
                const float2 c = c_at(mc + khi), corr = cmul(c, dtab[kDifLoPipe + klo]);
                v[1] = cmul(v[1], make_float2(c.x + corr.x, c.y + corr.y));
            }
#pragma unroll
            for (int s = 2; s < S; s += 2)
                twiddle_cd2(v[s], dtab[s * kDifLoPipe + klo], c_at(s * mc + khi), v[s + 1], dtab[(s + 1) * kDifLoPipe + klo],
                            c_at((s + 1) * mc + khi));
        }
        const rsrc_t z_rs = make_rsrc(a.z + (size_t)f * n, n * 8);
        store_z<S>(v, z_rs, m);
    }
}

template <int S>
static hipError_t launch_s(const DifLaunch &a) {
    const dim3 grid((1 << kDitLogM) / 256, a.n_frames);
    // pipelined kernel: 8-bit input (16-bit measured slower: its 64 KB of LDS halves the resident blocks)
    if (a.pipe > 0 && a.fmt <= 1 && ((reinterpret_cast<uintptr_t>(a.in) | (uintptr_t)a.frame_stride) & 15) == 0) {
        const int groups = std::min(a.n_frames, a.pipe);  // frame groups: blocks = (M / 256) x groups
        const dim3 pg((1 << kDitLogM) / 256 * groups);
        if (a.fmt == 0) hipLaunchKernelGGL((dif_front_pipe_kernel<S, 0>), pg, dim3(256), 0, a.stream, a, groups);
        else hipLaunchKernelGGL((dif_front_pipe_kernel<S, 1>), pg, dim3(256), 0, a.stream, a, groups);
        return hipGetLastError();
    }
    switch (a.fmt) {
    case 0: hipLaunchKernelGGL((dif_front_kernel<S, 0>), grid, dim3(256), 0, a.stream, a); break;
    case 1: hipLaunchKernelGGL((dif_front_kernel<S, 1>), grid, dim3(256), 0, a.stream, a); break;
    case 2: hipLaunchKernelGGL((dif_front_kernel<S, 2>), grid, dim3(256), 0, a.stream, a); break;
    case 3: hipLaunchKernelGGL((dif_front_kernel<S, 3>), grid, dim3(256), 0, a.stream, a); break;
    case 4: hipLaunchKernelGGL((dif_front_kernel<S, 4>), grid, dim3(256), 0, a.stream, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_dif_front(const DifLaunch &a) {
    if (a.n_frames <= 0) return hipSuccess;
    switch (a.logn - kDitLogM) {
    case 3: return launch_s<8>(a);
    case 4: return launch_s<16>(a);
    case 5: return launch_s<32>(a);
    default: return hipErrorInvalidValue;
    }
}

// Caller rows of the large-N pair: kernel B writes dB rows residue-major (block s
// holds bins S q + s, like the ring); this puts them in natural order,
// rows[f][q S + s] = cols[f][s][q], through a 64-column LDS tile (coalesced both ways).
template <int S>
__global__ void __launch_bounds__(256) cols_to_rows_kernel(const float *cols, float *rows) {
    constexpr int M = 1 << kDitLogM;
    __shared__ float tile[S][65];  // odd pitch: the column-order reads are conflict free
    const int q0 = blockIdx.x * 64;
    const size_t off = (size_t)blockIdx.y * S * M;
    for (int e = threadIdx.x; e < S * 64; e += 256) tile[e >> 6][e & 63] = cols[off + (size_t)(e >> 6) * M + q0 + (e & 63)];
    __syncthreads();
    for (int e = threadIdx.x; e < S * 64; e += 256) rows[off + (size_t)q0 * S + e] = tile[e % S][e / S];
}

hipError_t launch_cols_to_rows(const float *cols, float *rows, int n_frames, int logn, hipStream_t st) {
    if (n_frames <= 0) return hipSuccess;
    const dim3 grid((1 << kDitLogM) / 64, n_frames);
    switch (logn - kDitLogM) {
    case 3: hipLaunchKernelGGL((cols_to_rows_kernel<8>), grid, dim3(256), 0, st, cols, rows); break;
    case 4: hipLaunchKernelGGL((cols_to_rows_kernel<16>), grid, dim3(256), 0, st, cols, rows); break;
    case 5: hipLaunchKernelGGL((cols_to_rows_kernel<32>), grid, dim3(256), 0, st, cols, rows); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int dif_lo_points(bool pipe) { return pipe ? kDifLoPipe : kDifLoTile; }

void dif_twiddles(int logn, int lo, std::vector<float2> &c, std::vector<float2> &d) {
    const int m = 1 << kDitLogM, s = 1 << (logn - kDitLogM), mc = m / lo;
    const double n = (double)(1 << logn);
    auto w = [&](double e) {  // exp(-2 pi i e / N), correctly rounded from double
        const double ang = -2.0 * M_PI * e / n;
        return make_float2((float)std::cos(ang), (float)std::sin(ang));
    };
    c.assign((size_t)s * mc, make_float2(1.f, 0.f));
    d.assign((size_t)s * lo, make_float2(1.f, 0.f));
    for (int r = 0; r < s; r++) {
        for (int h = 0; h < mc; h++) c[(size_t)r * mc + h] = w(std::fmod((double)r * (double)lo * h, n));
        for (int l = 0; l < lo; l++) {  // delta = W_N^{r l} - 1: (-2 sin^2(a/2), sin a) from double
            const double ang = -2.0 * M_PI * (double)r * l / n, h = std::sin(0.5 * ang);
            d[(size_t)r * lo + l] = make_float2((float)(-2.0 * h * h), (float)std::sin(ang));
        }
    }
}

}  // namespace rfa
