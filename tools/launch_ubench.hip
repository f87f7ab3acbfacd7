// Dependent-launch latency on one stream: N tiny kernels (each 1 workgroup
// reading the previous kernel's output) launched eagerly and as a captured
// HIP graph; prints microseconds per kernel.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/launch_ubench.hip -o tools/launch_ubench
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void step(double* x, int k) {
    if (threadIdx.x == 0) x[0] = x[0] * 0.5 + k;
}
__global__ void step_wide(double* x, int k) {   // 512 workgroups of 256
    const int i = blockIdx.x * 256 + threadIdx.x;
    x[i + 256] = x[i + 256] * 0.5 + x[0] + k;
}

int main() {
    double* x;
    (void)hipMalloc(&x, sizeof(double) * (512 * 256 + 512));
    (void)hipMemset(x, 0, sizeof(double) * (512 * 256 + 512));
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int N = 200;
    for (int wide = 0; wide < 2; ++wide) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, s);
            for (int k = 0; k < N; ++k) {
                if (wide) hipLaunchKernelGGL(step_wide, dim3(512), dim3(256), 0, s, x, k);
                else hipLaunchKernelGGL(step, dim3(1), dim3(64), 0, s, x, k);
            }
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("eager %s: %.2f us per kernel\n", wide ? "512x256" : "1x64", ms * 1000.0f / N);
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int k = 0; k < N; ++k) {
            if (wide) hipLaunchKernelGGL(step_wide, dim3(512), dim3(256), 0, s, x, k);
            else hipLaunchKernelGGL(step, dim3(1), dim3(64), 0, s, x, k);
        }
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int rep = 0; rep < 4; ++rep) {
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, s);
            (void)hipGraphLaunch(ge, s);
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("graph %s: %.2f us per kernel\n", wide ? "512x256" : "1x64", ms * 1000.0f / N);
        }
    }
    (void)hipFree(x);
    return 0;
}
