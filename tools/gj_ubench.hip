// Phase timing of the explicit-inverse BCR odd kernel (gn_bcr_gj.hip built with
// SLAM_GJ_STAMPS) on random SPD blocks: one odd block (nb = 3, s = 1) and a
// C4-sized first level (nb = 469, 234 odd blocks at UB_T = 2), HIP event times and s_memtime
// cycles of thread 0 of workgroup (0, 0) per phase.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSLAM_GJ_STAMPS \
//       -I include tools/gj_ubench.hip -o tools/gj_ubench && tools/gj_ubench
#include "../icp-slam-with-loop-closure_amd/csrc/gn_bcr_gj.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace slamhip;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

#ifndef UB_T
#define UB_T 2
#endif
constexpr int T = UB_T, WB = 16 * T;   // 2: C4's band + border plan (32-row blocks); 5: 80-row blocks

int main() {
    std::mt19937_64 g(1);
    std::normal_distribution<double> n(0.0, 1.0);
    for (int nb : {3, 469}) {
        std::vector<double> D(static_cast<size_t>(nb) * WB * WB), E(D.size()), bz(static_cast<size_t>(nb) * WB);
        std::vector<double> a(WB * WB);
        for (int i = 0; i < nb; ++i) {
            for (auto& v : a) v = n(g);
            for (int r = 0; r < WB; ++r)
                for (int c = 0; c < WB; ++c) {
                    double s = 0;
                    for (int k = 0; k < WB; ++k) s += a[r * WB + k] * a[c * WB + k];
                    D[static_cast<size_t>(i) * WB * WB + r * WB + c] = s / WB + (r == c ? 4.0 : 0.0);
                }
        }
        for (auto& v : E) v = 0.1 * n(g);
        for (auto& v : bz) v = 0.1 * n(g);
        const size_t B = sizeof(double) * D.size();
        double* work;
        const int64_t ws = bcr_gj_work_size(nb * WB, WB, 1);
        CK(hipMalloc(&work, ws * sizeof(double)));
        int32_t* st;
        CK(hipMalloc(&st, 4));
        const BcrGjBufs b = bcr_gj_bufs(work, nb * WB, WB, 1);
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(bcrgj::odd_kernel<T>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bcrgj::Lds<T>::bytes)));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int n_odd = (nb - 1 + 1) / 2;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemcpy(b.D, D.data(), B, hipMemcpyHostToDevice));
            CK(hipMemcpy(b.E0, E.data(), B, hipMemcpyHostToDevice));
            CK(hipMemcpy(b.bz, bz.data(), sizeof(double) * bz.size(), hipMemcpyHostToDevice));
            unsigned long long z[8] = {};
            CK(hipMemcpyToSymbol(HIP_SYMBOL(bcrgj::g_gj_stamps), z, sizeof(z)));
            CK(hipEventRecord(e0));
            int cpw = 1;
            while (cpw < T && n_odd * (2 * ((T + cpw - 1) / cpw) + 1) > 512) ++cpw;
            const int ng = (T + cpw - 1) / cpw;
            hipLaunchKernelGGL(bcrgj::odd_kernel<T>, dim3(n_odd, 2 * ng + 1), dim3(bcrgj::kThreads), bcrgj::Lds<T>::bytes,
                               0, b.D, b.E0, b.E1, b.Xs, b.Ys, b.SP, b.SN, b.bz, b.SPb, b.SNb, nb, 1, cpw, n_odd, 1, st);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            unsigned long long h[8];
            CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(bcrgj::g_gj_stamps), sizeof(h)));
            printf("nb %d (%d odd blocks x %d wg, cpw %d): %.2f us; cycles: P %llu R %llu U %llu | stage %llu invert %llu "
                   "prod1 %llu prod2 %llu\n", nb, n_odd, 2 * ng + 1, cpw, ms * 1e3, h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
        }
        if (nb == 3) {   // X_1 = D_1^-1 E_0 against a host Gauss-Jordan solve
            std::vector<double> M(D.begin() + WB * WB, D.begin() + 2 * WB * WB), X(E.begin(), E.begin() + WB * WB);
            for (int k = 0; k < WB; ++k) {
                const double pv = 1.0 / M[k * WB + k];
                for (int c = 0; c < WB; ++c) { M[k * WB + c] *= pv; X[k * WB + c] *= pv; }
                for (int r = 0; r < WB; ++r) {
                    if (r == k) continue;
                    const double f = M[r * WB + k];
                    for (int c = 0; c < WB; ++c) { M[r * WB + c] -= f * M[k * WB + c]; X[r * WB + c] -= f * X[k * WB + c]; }
                }
            }
            std::vector<double> Xg(WB * WB);
            CK(hipMemcpy(Xg.data(), b.Xs + WB * WB, sizeof(double) * WB * WB, hipMemcpyDeviceToHost));
            double md = 0, mx = 0;
            for (int e = 0; e < WB * WB; ++e) { md = std::max(md, std::fabs(Xg[e] - X[e])); mx = std::max(mx, std::fabs(X[e])); }
            printf("X_1 check: max |dX| %.3e (max |X| %.3e)\n", md, mx);
        }
        CK(hipFree(work));
        CK(hipFree(st));
    }
    return 0;
}
