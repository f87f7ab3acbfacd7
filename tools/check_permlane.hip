// Semantics check of gfx950 v_permlane16_swap / v_permlane32_swap as used by
// the wave reductions in icp_kernels.hip (run on the GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    const unsigned v = threadIdx.x;
    auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    out[threadIdx.x] = a[0];
    out[64 + threadIdx.x] = a[1];
    out[128 + threadIdx.x] = b[0];
    out[192 + threadIdx.x] = b[1];
}
int main() {
    unsigned* d;
    (void)hipMalloc(&d, 256 * 4);
    k<<<1, 64>>>(d);
    unsigned h[256];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[4] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]"};
    for (int r = 0; r < 4; ++r) {
        printf("%s:", nm[r]);
        for (int l = 0; l < 64; l += 8) printf(" %u", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
