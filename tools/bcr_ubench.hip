// Phase timing of the blocked MFMA elimination (gn_bcr.hip built with
// SLAM_BCR_STAMPS): one top-block solve (one workgroup, NR = 1) and one level
// of odd blocks on random SPD blocks, s_memtime per wave and phase, plus HIP
// event times of the MFMA and register-elimination kernels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSLAM_BCR_STAMPS \
//       -I include tools/bcr_ubench.hip -o tools/bcr_ubench && tools/bcr_ubench
#include "../icp-slam-with-loop-closure_amd/csrc/gn_bcr.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace slamhip;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int T = 5, WB = 16 * T;

static void spd(std::vector<double>& m, std::mt19937_64& g, double diag) {
    std::normal_distribution<double> n(0.0, 1.0);
    std::vector<double> a(WB * WB);
    for (auto& v : a) v = n(g);
    for (int r = 0; r < WB; ++r)
        for (int c = 0; c < WB; ++c) {
            double s = 0;
            for (int k = 0; k < WB; ++k) s += a[r * WB + k] * a[c * WB + k];
            m[r * WB + c] = s / WB + (r == c ? diag : 0.0);
        }
}

static void dump(const char* what) {
    unsigned long long h[4][4];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bcr_stamps), sizeof(h));
    printf("%s stamps (cycles; P1 work, barrier1, P2 work, barrier2):\n", what);
    for (int w = 0; w < 4; ++w) printf("  wave %d: %8llu %8llu %8llu %8llu\n", w, h[w][0], h[w][1], h[w][2], h[w][3]);
    unsigned long long z[4][4] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bcr_stamps), z, sizeof(z));
}

int main() {
    std::mt19937_64 g(1);
    const int nb = 3;   // blocks 0, 1, 2: one odd block (1) at s = 1
    std::vector<double> D(nb * WB * WB), E(nb * WB * WB), bz(nb * WB);
    std::vector<double> blk(WB * WB);
    for (int i = 0; i < nb; ++i) {
        spd(blk, g, 4.0);
        std::copy(blk.begin(), blk.end(), D.begin() + i * WB * WB);
    }
    std::normal_distribution<double> n(0.0, 0.1);
    for (auto& v : E) v = n(g);
    for (auto& v : bz) v = n(g);
    double *dD, *dE, *dC, *dX, *dY, *dbz, *dx;
    int32_t* dst;
    const size_t B = sizeof(double) * nb * WB * WB;
    CK(hipMalloc(&dD, B));
    CK(hipMalloc(&dE, B));
    CK(hipMalloc(&dC, B));
    CK(hipMalloc(&dX, B));
    CK(hipMalloc(&dY, B));
    CK(hipMalloc(&dbz, sizeof(double) * nb * WB));
    CK(hipMalloc(&dx, sizeof(double) * WB));
    CK(hipMalloc(&dst, 4));
    auto reset = [&]() {
        (void)hipMemcpy(dD, D.data(), B, hipMemcpyHostToDevice);
        (void)hipMemcpy(dE, E.data(), B, hipMemcpyHostToDevice);
        (void)hipMemcpy(dbz, bz.data(), sizeof(double) * nb * WB, hipMemcpyHostToDevice);
        (void)hipMemset(dst, 0, 4);
    };
    const size_t lds = BcrMfmaLds<T>::bytes;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(bcr_top_mfma_kernel<T>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(bcr_odd_mfma_kernel<T>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    const size_t lds_back = sizeof(double) * (static_cast<size_t>(WB) * (WB + 1) + 4 * static_cast<size_t>(WB));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(bcr_top_reg_kernel<T>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    // top block
    for (int rep = 0; rep < 3; ++rep) {
        reset();
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(bcr_top_mfma_kernel<T>, dim3(1), dim3(kBcrThreads), lds, 0, dD, dbz, dx, WB, dst);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("top mfma: %.2f us\n", ms * 1e3);
        if (rep < 2) dump("(warm)"); else dump("top mfma");
    }
    std::vector<double> x1(WB), x2(WB);
    CK(hipMemcpy(x1.data(), dx, sizeof(double) * WB, hipMemcpyDeviceToHost));
    for (int rep = 0; rep < 2; ++rep) {
        reset();
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(bcr_top_reg_kernel<T>, dim3(1), dim3(kBcrThreads), lds_back, 0, dD, dbz, dx, WB, dst);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("top reg: %.2f us\n", ms * 1e3);
    }
    CK(hipMemcpy(x2.data(), dx, sizeof(double) * WB, hipMemcpyDeviceToHost));
    double md = 0;
    for (int r = 0; r < WB; ++r) md = std::max(md, std::fabs(x1[r] - x2[r]));
    printf("top |x_mfma - x_reg| = %.3e\n", md);
    dump("(reg)");
    // one odd block at s = 1
    for (int rep = 0; rep < 3; ++rep) {
        reset();
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(bcr_odd_mfma_kernel<T>, dim3(1, 3), dim3(kBcrThreads), lds, 0, dD, dE, dC, dX, dY, dbz, WB,
                           nb, 1, dst);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("odd mfma (1 block x 3 wg): %.2f us\n", ms * 1e3);
        if (rep < 2) dump("(warm)"); else dump("odd mfma q=0");
    }
    for (int rep = 0; rep < 2; ++rep) {
        reset();
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(bcr_odd_reg_kernel<T>, dim3(1, 6), dim3(kBcrThreads), 0, 0, dD, dE, dC, dX, dY, dbz, WB, nb,
                           1, dst, nullptr);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("odd reg (1 block x 6 wg): %.2f us\n", ms * 1e3);
    }
    return 0;
}
