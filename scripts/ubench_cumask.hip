// CU-masked streams on MI355X (the peak / EMA state pass on reserved CUs).
//
// 1. Census: which physical CU (XCC, SE, CU id from the hardware registers) each bit of a
//    hipExtStreamCreateWithCUMask mask enables -- one-bit masks, 16 workgroups each.
// 2. Read rate of a streaming reduction (the state pass's access: 16-B loads, 4 or 8 in flight
//    per thread) over 131 MB (the 500-row 64 K ring) on k CUs, k spread evenly over the XCDs,
//    with the rows Infinity-Cache resident (just written) and evicted (1 GiB written after).
//    Prints GB/s and GB/s per CU: the CU count a state stream needs to keep pace with the FFT.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void census(unsigned *out) {
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

// every block records its (XCC, HW_ID) after a ~20 us spin, so a block per resident slot is seen
__global__ void census2(unsigned *out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(4);
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

static void census_mask(const char *name, const std::vector<uint32_t> &m, int words) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
    std::vector<uint32_t> got(words, 0u);
    CK(hipExtStreamGetCUMask(s, words, got.data()));
    const int blocks = 2048;
    unsigned *d;
    CK(hipMalloc(&d, blocks * 8));
    hipLaunchKernelGGL(census2, dim3(blocks), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned> h(2 * blocks);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    std::map<unsigned, int> cus;       // (xcc, se, sh, cu) -> blocks
    std::map<unsigned, int> per_xcc;   // xcc -> distinct CUs
    for (int b = 0; b < blocks; b++) {
        const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        cus[(xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)]++;
    }
    for (auto &kv : cus) per_xcc[kv.first >> 16]++;
    std::printf("mask %-12s set bits %3d (readback word0 %08x): %zu distinct CUs; per XCC:", name,
                [&] { int c = 0; for (uint32_t w : m) c += __builtin_popcount(w); return c; }(), got[0], cus.size());
    for (auto &kv : per_xcc) std::printf(" x%u:%d", kv.first, kv.second);
    std::printf("\n");
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
}

__global__ void fill(float4 *p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(v, v + 1.f, v, v);
}

// rows [R][N] floats; thread owns 4 bins, walks all rows (like one chunk of state_fused_kernel)
template <int UNROLL>
__global__ void __launch_bounds__(256) rowscan(const float *rows, int R, int N, int chunk, float *out) {
    const int tpc = N / 4;
    const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const int c = (int)(t / tpc), bin = (int)(t % tpc) * 4;
    const int f0 = c * chunk, f1 = min(R, f0 + chunk);
    if (f0 >= R) return;
    float pk = -1e30f, em = 0.f;
    int f = f0;
    for (; f + UNROLL <= f1; f += UNROLL) {
        float4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) x[u] = *reinterpret_cast<const float4 *>(rows + (size_t)(f + u) * N + bin);
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            pk = fmaxf(pk, fmaxf(fmaxf(x[u].x, x[u].y), fmaxf(x[u].z, x[u].w)));
            em = em + 0.1f * (x[u].x - em);
        }
    }
    for (; f < f1; f++) em += rows[(size_t)f * N + bin];
    if (pk == 12345.f || em == 12345.f) out[0] = pk + em;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("CUs %d\n", ncu);
    unsigned *d_out;
    CK(hipMalloc(&d_out, 64 * 2 * 4));
    const int words = (ncu + 31) / 32;
    // ---- 0. census by mask (all blocks' CUs)
    {
        auto range = [&](int lo, int hi) {
            std::vector<uint32_t> m(words, 0u);
            for (int b = lo; b < hi; b++) m[b / 32] |= 1u << (b % 32);
            return m;
        };
        census_mask("all", range(0, ncu), words);
        census_mask("{0}", range(0, 1), words);
        census_mask("{1}", range(1, 2), words);
        census_mask("[0,8)", range(0, 8), words);
        census_mask("[8,16)", range(8, 16), words);
        census_mask("[0,16)", range(0, 16), words);
        census_mask("[0,32)", range(0, 32), words);
        census_mask("[16,256)", range(16, ncu), words);
        census_mask("[24,256)", range(24, ncu), words);
        census_mask("[32,64)", range(32, 64), words);
    }
    if (std::getenv("CENSUS_ONLY")) return 0;
    // ---- 1. census
    std::map<int, std::vector<int>> xcc_bits;  // xcc -> bits
    std::vector<int> bit_xcc(ncu, -1);
    for (int b = 0; b < ncu; b++) {
        std::vector<uint32_t> m(words, 0u);
        m[b / 32] = 1u << (b % 32);
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
        CK(hipMemset(d_out, 0xff, 64 * 2 * 4));
        hipLaunchKernelGGL(census, dim3(16), dim3(64), 0, s, d_out);
        CK(hipStreamSynchronize(s));
        unsigned h[32];
        CK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
        bool same = true;
        for (int i = 1; i < 16; i++) same &= h[2 * i] >> 8 == h[0] >> 8 && h[2 * i + 1] == h[1];
        const unsigned hw = h[0], xcc = h[1] & 0xf;
        std::printf("bit %3d: xcc %u se %u sh %u cu %2u  all16same %d\n", b, xcc, (hw >> 13) & 7, (hw >> 12) & 1,
                    (hw >> 8) & 15, (int)same);
        bit_xcc[b] = (int)xcc;
        xcc_bits[(int)xcc].push_back(b);
        CK(hipStreamDestroy(s));
    }
    // ---- 2. read rate on k CUs spread over the XCDs
    const int R = 500, N = 65536;
    const size_t bytes = (size_t)R * N * 4, evb = (size_t)1 << 30;
    float *rows, *ev, *o;
    CK(hipMalloc(&rows, bytes));
    CK(hipMalloc(&ev, evb));
    CK(hipMalloc(&o, 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nx = (int)xcc_bits.size();
    for (int k : {8, 16, 24, 32, 48, 64, 128, 256}) {
        if (k > ncu) continue;
        std::vector<uint32_t> m(words, 0u);
        for (auto &kv : xcc_bits)
            for (int i = 0; i < k / nx && i < (int)kv.second.size(); i++) m[kv.second[i] / 32] |= 1u << (kv.second[i] % 32);
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
        for (int chunks : {16, 32}) {
            const int chunk = (R + chunks - 1) / chunks;
            const int threads = chunks * (N / 4), grid = threads / 256;
            for (int unroll : {4, 8}) {
                for (int evict = 0; evict < 2; evict++) {
                    float best = 1e9f;
                    for (int rep = 0; rep < 4; rep++) {
                        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float4 *)rows, bytes / 16, 1.0f);
                        if (evict) hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float4 *)ev, evb / 16, 2.0f);
                        CK(hipDeviceSynchronize());
                        CK(hipEventRecord(e0, s));
                        if (unroll == 4) hipLaunchKernelGGL(rowscan<4>, dim3(grid), dim3(256), 0, s, rows, R, N, chunk, o);
                        else hipLaunchKernelGGL(rowscan<8>, dim3(grid), dim3(256), 0, s, rows, R, N, chunk, o);
                        CK(hipEventRecord(e1, s));
                        CK(hipEventSynchronize(e1));
                        float ms;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        best = std::min(best, ms);
                    }
                    std::printf("k %3d CUs chunks %2d unroll %d %s: %8.1f us %7.0f GB/s %6.1f GB/s per CU\n", k, chunks,
                                unroll, evict ? "evicted " : "resident", best * 1e3, bytes / (best * 1e-3) / 1e9,
                                bytes / (best * 1e-3) / 1e9 / k);
                }
            }
        }
        CK(hipStreamDestroy(s));
    }
    return 0;
}
