// Micro-benchmark: device copy kernel variants (bench copy ceiling, rfa_stream_copy).
// GB/s = (bytes read + bytes written) / time, 1 GiB buffers, best of 3 x 10 launches.
// build: hipcc -O3 --offload-arch=gfx950 -o ubench_copy ubench_copy.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, int T, bool NT>
__global__ __launch_bounds__(T) void copy_gs(f4 *__restrict__ d, const f4 *__restrict__ s, long long n4) {
    const long long stride = (long long)gridDim.x * T * U;
    for (long long b = (long long)blockIdx.x * T * U + threadIdx.x; b < n4; b += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (b + u * T < n4) v[u] = NT ? __builtin_nontemporal_load(s + b + u * T) : s[b + u * T];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (b + u * T < n4) {
                if (NT) __builtin_nontemporal_store(v[u], d + b + u * T);
                else d[b + u * T] = v[u];
            }
    }
}

template <int U, int T, bool NT>
void run(const char *name, f4 *d, const f4 *s, long long n4, long long blocks) {
    if (blocks <= 0) blocks = (n4 + (long long)T * U - 1) / ((long long)T * U);
    hipLaunchKernelGGL((copy_gs<U, T, NT>), dim3((unsigned)blocks), dim3(T), 0, 0, d, s, n4);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; i++)
            hipLaunchKernelGGL((copy_gs<U, T, NT>), dim3((unsigned)blocks), dim3(T), 0, 0, d, s, n4);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("%-40s blocks %8lld: %.1f GB/s\n", name, blocks, 2.0 * n4 * 16 * 10 / (best * 1e-3) / 1e9);
}

int main() {
    const long long bytes = 1ll << 30, n4 = bytes / 16;
    f4 *s, *d;
    (void)hipMalloc(&s, bytes);
    (void)hipMalloc(&d, bytes);
    (void)hipMemset(s, 1, bytes);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<4, 256, false>("U4 T256 grid cus*8", d, s, n4, cus * 8);
    run<4, 256, false>("U4 T256 one pass", d, s, n4, 0);
    run<8, 256, false>("U8 T256 grid cus*8", d, s, n4, cus * 8);
    run<8, 256, false>("U8 T256 one pass", d, s, n4, 0);
    run<2, 256, false>("U2 T256 one pass", d, s, n4, 0);
    run<1, 256, false>("U1 T256 one pass", d, s, n4, 0);
    run<4, 1024, false>("U4 T1024 grid cus*2", d, s, n4, cus * 2);
    run<4, 512, false>("U4 T512 grid cus*4", d, s, n4, cus * 4);
    run<4, 256, true>("U4 T256 nt grid cus*8", d, s, n4, cus * 8);
    run<4, 256, true>("U4 T256 nt one pass", d, s, n4, 0);
    run<8, 256, true>("U8 T256 nt grid cus*16", d, s, n4, cus * 16);
    run<4, 256, false>("U4 T256 grid cus*32", d, s, n4, cus * 32);
    return 0;
}
