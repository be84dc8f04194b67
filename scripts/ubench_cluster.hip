// XCD-cluster exchange cost, measured.
//
// The cluster split of a 64 K frame would put its four 16 K residues on four co-resident
// workgroups of one XCD (block ids b, b + 8, b + 16, b + 24: the dispatcher sends block b to XCD
// b mod 8).  Residue r needs every quarter of the frame (the radix-4 decimation-in-frequency
// pre-stage: y_r[m] = W^{mr} sum_j x[m + jM'] w[m + jM'] W_4^{jr}), which the cluster can get
// (a) by every member re-reading the whole raw frame (three quarters of it from the XCD's L2,
//     co-scheduled), or
// (b) by every member loading only its quarter, windowing it to complex fp32 (8 B per sample)
//     and exchanging those partials with the other three through L2: sc1 16-B stores, every
//     storing wave's vmcnt(0), a workgroup barrier, one lane's sc1 flag store; the consumer polls
//     the flags with sc1 loads, passes a barrier, and loads with sc1 (MI355X_MICROARCH.md,
//     hand-off table, row 1).
// No FFT arithmetic: this is only the data movement each form adds.  Persistent grid of 256
// workgroups of 1024 threads (one per CU by its LDS, like the 64 K kernel), 64 clusters, 500
// frames per launch from a rotating pool past the Infinity Cache.  Modes (s8 frames, 128 KB;
// f32 frames, 512 KB):
//   quarter  every member loads its own quarter only (the floor any split pays)
//   reread   (a): every member loads the whole frame
//   xchg     (b): quarter + window-convert + partial exchange (128 KB written, 384 KB read per member)
// Prints the launch time, the per-frame chip time (launch / 500) and the cost of (a) and (b)
// over `quarter` per frame -- the number VERDICT r5 compares with 0.08 us.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../rfanalyzer_amd/csrc/fft_common.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

using rfa::make_rsrc;
using rfa::rsrc_t;
constexpr int kThreads = 1024, kFrames = 500, kClusters = 64;
constexpr int kQSamples = 16384;  // samples per quarter of a 64 K frame

typedef float f4v __attribute__((ext_vector_type(4)));

template <int AUX = 0>
__device__ __forceinline__ f4v ld16(rsrc_t rs, int off) {
    return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
}

// MODE 0 quarter, 1 reread, 2 xchg; BPS bytes per raw sample (2: s8, 8: f32)
template <int MODE, int BPS>
__global__ void __launch_bounds__(kThreads) cluster_kernel(const uint8_t *pool, float2 *xbuf, unsigned *flags,
                                                            float *out, unsigned gen0, unsigned *timeouts) {
    extern __shared__ float lds_pad[];  // > 80 KB: one workgroup per CU
    const int b = blockIdx.x, x = b % 8, s = b / 8, cl = s / 4, mem = s % 4;
    const int cid = cl * 8 + x;  // 64 clusters, each on one XCD
    constexpr int FB = 65536 * BPS, QB = FB / 4;
    float acc = 0.f;
    if (threadIdx.x == 0) lds_pad[0] = 0.f;
    int k = 0;
    for (int f = cid; f < kFrames; f += kClusters, k++) {
        const rsrc_t fr = make_rsrc(pool + (size_t)f * FB, FB);
        if constexpr (MODE == 0 || MODE == 2) {
            constexpr int PER = QB / 16 / kThreads;  // 16-B loads per thread of the quarter
            f4v r[PER];
#pragma unroll
            for (int i = 0; i < PER; i++) r[i] = ld16(fr, mem * QB + (i * kThreads + threadIdx.x) * 16);
            if constexpr (MODE == 0) {
#pragma unroll
                for (int i = 0; i < PER; i++) acc += r[i].x + r[i].y + r[i].z + r[i].w;
            } else {
                // window-convert this thread's samples to complex fp32 and publish them (sc1)
                const int par = k & 1;
                float2 *mine = xbuf + (((size_t)cid * 2 + par) * 4 + mem) * kQSamples;
                const rsrc_t ws = make_rsrc(mine, kQSamples * 8);
#pragma unroll
                for (int i = 0; i < PER; i++) {
                    const int e0 = (i * kThreads + threadIdx.x) * 16 / BPS;  // first sample of these 16 B
                    if constexpr (BPS == 2) {  // 8 samples -> 4 x 16-B stores
                        const unsigned w[4] = {__builtin_bit_cast(unsigned, r[i].x), __builtin_bit_cast(unsigned, r[i].y),
                                               __builtin_bit_cast(unsigned, r[i].z), __builtin_bit_cast(unsigned, r[i].w)};
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const float a0 = (float)(signed char)(w[q] & 0xff) * 0.0078125f, a1 = (float)(signed char)((w[q] >> 8) & 0xff) * 0.0078125f;
                            const float a2 = (float)(signed char)((w[q] >> 16) & 0xff) * 0.0078125f, a3 = (float)(signed char)(w[q] >> 24) * 0.0078125f;
                            rfa::buf_store_f32x4(a0, a1, a2, a3, ws, (e0 + 2 * q) * 8, 0);
                        }
                    } else {  // 2 samples -> one 16-B store
                        rfa::buf_store_f32x4(r[i].x * 0.5f, r[i].y * 0.5f, r[i].z * 0.5f, r[i].w * 0.5f, ws, e0 * 8, 0);
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
                __syncthreads();
                const unsigned g = gen0 + (unsigned)k;
                if (threadIdx.x == 0) {
                    __hip_atomic_store(&flags[(cid * 4 + mem) * 32], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    for (int o = 1; o < 4; o++) {  // the other members' flags (sc1 loads), bounded
                        const unsigned *fl = &flags[(cid * 4 + (mem + o) % 4) * 32];
                        while (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g) {
                            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {  // 20 ms: give up
                                atomicAdd(timeouts, 1u);
                                break;
                            }
                            __builtin_amdgcn_s_sleep(2);
                        }
                    }
                }
                __syncthreads();
                // the three other quarters' partials, sc1 16-B loads
                constexpr int PER_X = kQSamples * 8 / 16 / kThreads;  // 8 per member
#pragma unroll
                for (int o = 1; o < 4; o++) {
                    const rsrc_t os = make_rsrc(xbuf + (((size_t)cid * 2 + par) * 4 + (mem + o) % 4) * kQSamples, kQSamples * 8);
#pragma unroll
                    for (int i = 0; i < PER_X; i++) {
                        const f4v v = ld16<16>(os, (i * kThreads + threadIdx.x) * 16);
                        acc += v.x + v.y + v.z + v.w;
                    }
                }
            }
        } else {  // reread: the whole frame
            constexpr int PER = FB / 16 / kThreads;
#pragma unroll 8
            for (int i = 0; i < PER; i++) {
                const f4v v = ld16(fr, (i * kThreads + threadIdx.x) * 16);
                acc += v.x + v.y + v.z + v.w;
            }
        }
        __syncthreads();
    }
    if (acc == 1234.5f) out[b] = acc + lds_pad[0];
}

template <int MODE, int BPS>
static float run(const char *name, const uint8_t *pool, size_t pool_frames, float2 *xbuf, unsigned *flags, float *out,
                 unsigned *timeouts, unsigned &gen) {
    auto kern = cluster_kernel<MODE, BPS>;
    const int lds = 100 * 1024;
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t FB = 65536 * (size_t)BPS;
    std::vector<float> t;
    for (int it = 0; it < 12; it++) {
        const uint8_t *p = pool + (size_t)(it % (pool_frames / kFrames)) * kFrames * FB;
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kern, dim3(256), dim3(kThreads), lds, 0, p, xbuf, flags, out, gen, timeouts);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        gen += 8;  // each cluster handles <= 8 frames per launch
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) t.push_back(ms * 1e3f);
    }
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    std::printf("%-8s %s: launch %7.2f us (min %7.2f)  %6.4f us per frame\n", name, BPS == 2 ? "s8 " : "f32", med, t[0],
                med / kFrames);
    return med;
}

int main() {
    unsigned *flags, *timeouts;
    float2 *xbuf;
    float *out;
    CK(hipMalloc(&flags, kClusters * 4 * 32 * 4));
    CK(hipMemset(flags, 0, kClusters * 4 * 32 * 4));
    CK(hipMalloc(&timeouts, 4));
    CK(hipMemset(timeouts, 0, 4));
    CK(hipMalloc(&xbuf, (size_t)kClusters * 2 * 4 * kQSamples * 8));
    CK(hipMalloc(&out, 256 * 4));
    unsigned gen = 1;
    for (int bps : {2, 8}) {
        const size_t FB = 65536 * (size_t)bps, pool_frames = (bps == 2 ? 8 : 3) * (size_t)kFrames;
        uint8_t *pool;
        CK(hipMalloc(&pool, pool_frames * FB));
        CK(hipMemset(pool, 3, pool_frames * FB));
        float t0, ta, tb;
        if (bps == 2) {
            t0 = run<0, 2>("quarter", pool, pool_frames, xbuf, flags, out, timeouts, gen);
            ta = run<1, 2>("reread", pool, pool_frames, xbuf, flags, out, timeouts, gen);
            tb = run<2, 2>("xchg", pool, pool_frames, xbuf, flags, out, timeouts, gen);
        } else {
            t0 = run<0, 8>("quarter", pool, pool_frames, xbuf, flags, out, timeouts, gen);
            ta = run<1, 8>("reread", pool, pool_frames, xbuf, flags, out, timeouts, gen);
            tb = run<2, 8>("xchg", pool, pool_frames, xbuf, flags, out, timeouts, gen);
        }
        std::printf("%s: (a) re-read costs %6.4f us per frame, (b) partial exchange %6.4f us per frame over the quarter floor\n",
                    bps == 2 ? "s8 " : "f32", (ta - t0) / kFrames, (tb - t0) / kFrames);
        CK(hipFree(pool));
    }
    unsigned to = 0;
    CK(hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost));
    std::printf("flag-wait timeouts: %u\n", to);
    return 0;
}
