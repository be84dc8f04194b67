// Read bandwidth of data the previous kernel just wrote (Infinity-Cache resident) vs
// the same read after a 1 GiB eviction write: is the peak/EMA pass (131 MB of rows read
// back at ~6.1 TB/s) at the cache's read rate?  Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void fill(float4 *p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(v, v, v, v);
}
template <int UNROLL>
__global__ void readsum(const float4 *p, size_t n, float *out) {
    float s = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        float4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) x[u] = p[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) s += x[u].x + x[u].y + x[u].z + x[u].w;
    }
    for (; i < n; i += stride) s += p[i].x;
    if (s == 12345.f) out[0] = s;
}

int main() {
    const size_t bytes = 131072000, n = bytes / 16, evb = (size_t)1 << 30;
    float4 *a, *ev;
    float *o;
    hipMalloc(&a, bytes);
    hipMalloc(&ev, evb);
    hipMalloc(&o, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct V { int grid, block, unroll; };
    std::vector<V> vs = {{1024, 256, 4}, {2048, 256, 4}, {4096, 256, 4}, {2048, 256, 8}, {1024, 1024, 4}, {8192, 256, 2}};
    for (int evict = 0; evict < 2; evict++) {
        for (auto v : vs) {
            float best = 1e9f;
            for (int rep = 0; rep < 5; rep++) {
                hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, n, 1.0f);
                if (evict) hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, ev, evb / 16, 2.0f);
                hipEventRecord(e0, 0);
                if (v.unroll == 2) hipLaunchKernelGGL(readsum<2>, dim3(v.grid), dim3(v.block), 0, 0, a, n, o);
                else if (v.unroll == 4) hipLaunchKernelGGL(readsum<4>, dim3(v.grid), dim3(v.block), 0, 0, a, n, o);
                else hipLaunchKernelGGL(readsum<8>, dim3(v.grid), dim3(v.block), 0, 0, a, n, o);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("%s grid %5d block %4d unroll %d: %7.1f us  %7.0f GB/s\n", evict ? "evicted " : "resident", v.grid,
                   v.block, v.unroll, best * 1e3, bytes / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
