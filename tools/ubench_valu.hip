// ubench_valu.hip — VALU issue-rate microbenchmark for the ICP scan's
// instruction mix on gfx950 (diagnostic tool, not part of the product).
// Each kernel runs ITERS x 8 independent copies of one instruction per lane;
// rate = wave-instructions per second per SIMD, reported relative to v_add_f32.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 4096

#define BODY8(ASM)                                                                         \
    asm volatile(ASM : "+v"(a0) : "v"(b)); asm volatile(ASM : "+v"(a1) : "v"(b));            \
    asm volatile(ASM : "+v"(a2) : "v"(b)); asm volatile(ASM : "+v"(a3) : "v"(b));            \
    asm volatile(ASM : "+v"(a4) : "v"(b)); asm volatile(ASM : "+v"(a5) : "v"(b));            \
    asm volatile(ASM : "+v"(a6) : "v"(b)); asm volatile(ASM : "+v"(a7) : "v"(b));

template <typename T>
__device__ void sink(T* out, T a0, T a1, T a2, T a3, T a4, T a5, T a6, T a7) {
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

#define K32(NAME, ASM)                                                                     \
    __global__ void NAME(float* out, float seed) {                                         \
        float b = seed * threadIdx.x;                                                      \
        float a0 = b, a1 = b + 1, a2 = b + 2, a3 = b + 3, a4 = b + 4, a5 = b + 5, a6 = b + 6, a7 = b + 7; \
        for (int i = 0; i < ITERS; ++i) { BODY8(ASM) }                                     \
        sink(out, a0, a1, a2, a3, a4, a5, a6, a7);                                         \
    }
#define K64(NAME, ASM)                                                                     \
    __global__ void NAME(double* out, double seed) {                                       \
        double b = seed * threadIdx.x;                                                     \
        double a0 = b, a1 = b + 1, a2 = b + 2, a3 = b + 3, a4 = b + 4, a5 = b + 5, a6 = b + 6, a7 = b + 7; \
        for (int i = 0; i < ITERS; ++i) { BODY8(ASM) }                                     \
        sink(out, a0, a1, a2, a3, a4, a5, a6, a7);                                         \
    }

K32(k_add_f32, "v_add_f32 %0, %0, %1")
K32(k_fma_f32, "v_fmac_f32 %0, %1, %1")
K32(k_min_u32, "v_min_u32 %0, %0, %1")
K32(k_med3_u32, "v_med3_u32 %0, %0, %1, %0")
K32(k_and_or_b32, "v_and_or_b32 %0, %0, %1, %0")
K64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
K64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %0")
K64(k_add_f64, "v_add_f64 %0, %0, %1")
K64(k_mul_f64, "v_mul_f64 %0, %0, %1")
K64(k_fma_f64, "v_fma_f64 %0, %0, %1, %0")
K64(k_min_f64, "v_min_f64 %0, %0, %1")

template <typename T, typename K>
float run(K kern, const char* name, T* out, int waves_per_simd, double ref) {
    const int blocks = 256 * waves_per_simd;   // 256-thread blocks: 1 wave per SIMD each
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, (T)1e-7);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, (T)1e-7);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winst = 5.0 * blocks * 4.0 * ITERS * 8.0;   // wave-instructions
    const double per_simd = winst / 1024.0 / (ms * 1e-3);    // per SIMD per second
    printf("%-14s waves/SIMD %d  %8.3f ms  %.3e winst/s/SIMD  cycles@2.4GHz %.2f  rel %.2f\n", name,
           waves_per_simd, ms, per_simd, 2.4e9 / per_simd, ref > 0 ? ref / per_simd : 1.0);
    return (float)per_simd;
}

int main() {
    float* of;
    double* od;
    (void)hipMalloc(&of, 256 * 64 * 256 * sizeof(float));
    (void)hipMalloc(&od, 256 * 64 * 256 * sizeof(double));
    for (int w : {1, 2, 4}) {
        double ref = run(k_add_f32, "v_add_f32", of, w, 0);
        run(k_fma_f32, "v_fmac_f32", of, w, ref);
        run(k_min_u32, "v_min_u32", of, w, ref);
        run(k_med3_u32, "v_med3_u32", of, w, ref);
        run(k_and_or_b32, "v_and_or_b32", of, w, ref);
        run(k_pk_add_f32, "v_pk_add_f32", od, w, ref);
        run(k_pk_fma_f32, "v_pk_fma_f32", od, w, ref);
        run(k_add_f64, "v_add_f64", od, w, ref);
        run(k_mul_f64, "v_mul_f64", od, w, ref);
        run(k_fma_f64, "v_fma_f64", od, w, ref);
        run(k_min_f64, "v_min_f64", od, w, ref);
    }
    return 0;
}
