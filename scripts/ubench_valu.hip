// Micro-benchmark: VALU issue cost of the instruction forms the FFT kernels use
// (gfx950).  Every lane runs NI independent chains of one instruction form,
// unrolled; 1024-thread workgroups, one per CU x grid; cycles per wave-instruction
// per SIMD = elapsed clocks * (SIMDs) / (wave-instructions issued per CU).
// build: hipcc -O3 --offload-arch=gfx950 -o ubench_valu ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int ITERS = 2048;

template <int KIND>
__global__ __launch_bounds__(1024) void kern(float *out, float seed) {
    f2v a[8], b = {seed, seed * 0.5f}, c = {0.25f, -0.125f};
    float s[16], t = seed * 0.3f;
    unsigned u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = (f2v){seed + i, seed - i};
        s[2 * i] = seed + i;
        s[2 * i + 1] = seed - i;
        u[i] = threadIdx.x * 2654435761u + i;
    }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (KIND == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            else if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            else if constexpr (KIND == 2) {  // two scalar adds (same work as one pk_add)
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[2 * i]) : "v"(t));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[2 * i + 1]) : "v"(t));
            } else if constexpr (KIND == 3) {  // two scalar fmas
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[2 * i]) : "v"(t));
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(s[2 * i + 1]) : "v"(t));
            } else if constexpr (KIND == 4) {  // signed byte -> float via SDWA sext (one instr per value)
                asm volatile("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1"
                             : "=v"(s[2 * i]) : "v"(u[i]));
                asm volatile("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0"
                             : "=v"(s[2 * i + 1]) : "v"(u[i]));
                u[i] += 0x01010101u;
            } else if constexpr (KIND == 5) {  // v_log_f32
                asm volatile("v_log_f32 %0, %0" : "+v"(s[2 * i]));
                asm volatile("v_log_f32 %0, %0" : "+v"(s[2 * i + 1]));
            } else if constexpr (KIND == 6) {  // pk_mul
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            }
        }
    }
    float r = t;
#pragma unroll
    for (int i = 0; i < 8; i++) r += a[i].x + a[i].y + s[2 * i] + s[2 * i + 1] + (float)u[i];
    if (r == 1234.5f) out[threadIdx.x] = r;
}

template <int KIND>
double run(const char *name, int instr_per_iter, int threads) {
    float *out;
    (void)hipMalloc(&out, 4096 * 4);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    hipLaunchKernelGGL(kern<KIND>, dim3(cus), dim3(threads), 0, 0, out, 1.0f);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern<KIND>, dim3(cus), dim3(threads), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double waves_per_simd = threads / 64 / 4.0;
    const double instr = (double)ITERS * instr_per_iter * waves_per_simd * reps;  // wave-instr per SIMD
    const double cyc = ms * 1e-3 * 2.4e9;  // at the 2.4 GHz max clock
    printf("%-34s threads %4d: %.3f ms, %.2f cyc/wave-instr/SIMD (at 2.4 GHz; rated clock %d kHz)\n", name, threads,
           ms / reps, cyc / instr, clk);
    (void)hipFree(out);
    return cyc / instr;
}

int main() {
    for (int th : {256, 1024}) {
        run<0>("v_pk_add_f32", 8, th);
        run<6>("v_pk_mul_f32", 8, th);
        run<1>("v_pk_fma_f32", 8, th);
        run<2>("v_add_f32", 16, th);
        run<3>("v_fma_f32", 16, th);
        run<4>("v_cvt_f32_i32_sdwa sext byte (+1 add)", 24, th);
        run<5>("v_log_f32", 16, th);
    }
    return 0;
}
