// Hardware check of packed-fp32 VOP3P modifiers on gfx950 (op_sel swaps and
// one-sided neg_lo / neg_hi), used by the FFT butterfly helpers.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const f2 *in, f2 *out) {
    const int t = threadIdx.x;
    f2 a = in[2 * t], b = in[2 * t + 1], r;
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    out[8 * t + 0] = r;  // a + (-i) b = (a.x + b.y, a.y - b.x)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    out[8 * t + 1] = r;  // a + (+i) b = (a.x - b.y, a.y + b.x)
    f2 m;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(m) : "v"(a), "v"(b));
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(m));
    out[8 * t + 2] = r;  // a * b complex
    asm volatile("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    out[8 * t + 3] = r;  // (a.x + b.x, a.y - b.y)
    asm volatile("v_pk_mul_f32 %0, %1, %2 neg_lo:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    out[8 * t + 4] = r;  // (-a.x b.x, a.y b.y)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    out[8 * t + 5] = r;  // (-a.y + b.x, a.x + b.y)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 neg_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(a));
    out[8 * t + 6] = r;  // (a.x b.x + a.x, a.y b.y - a.y)
    out[8 * t + 7] = a;
}
int main() {
    const int T = 64;
    f2 h[2 * T], o[8 * T];
    for (int i = 0; i < 2 * T; i++) h[i] = (f2){1.0f + i * 0.5f, -3.0f + i * 0.25f};
    f2 *din, *dout;
    hipMalloc(&din, sizeof h); hipMalloc(&dout, sizeof o);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(T), 0, 0, din, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < T; t++) {
        f2 a = h[2 * t], b = h[2 * t + 1];
        f2 e[7] = {{a.x + b.y, a.y - b.x}, {a.x - b.y, a.y + b.x},
                   {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}, {a.x + b.x, a.y - b.y},
                   {-a.x * b.x, a.y * b.y}, {-a.y + b.x, a.x + b.y}, {a.x * b.x + a.x, a.y * b.y - a.y}};
        for (int c = 0; c < 7; c++) {
            f2 g = o[8 * t + c];
            if (fabsf(g.x - e[c].x) > 1e-4f * (1 + fabsf(e[c].x)) || fabsf(g.y - e[c].y) > 1e-4f * (1 + fabsf(e[c].y))) {
                if (bad++ < 10) printf("case %d t %d got (%g,%g) want (%g,%g)\n", c, t, g.x, g.y, e[c].x, e[c].y);
            }
        }
    }
    printf("pk modifiers: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
    return bad != 0;
}
