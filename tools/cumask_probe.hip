// Where do the workgroups of a CU-masked stream run?  For a few masks
// (hipExtStreamCreateWithCUMask bit layouts), 2,048 workgroups that each spin
// ~20 us record their XCC and HW_ID; prints the XCCs and (XCC, SE, SH, CU)
// slots used.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>
#include <algorithm>

__global__ void where(unsigned long long* out) {
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));     // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
        out[blockIdx.x] = (static_cast<unsigned long long>(xcc & 0xf) << 32) | hw;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) {   // 20 us at 100 MHz
        }
    }
}

// co-residency: n workgroups, each holding a whole CU's LDS, on a stream whose
// mask gives k CUs per XCD; each arrives at a counter and waits (bounded) for
// all; records its XCC and whether every workgroup had arrived
__global__ void gang(unsigned long long* out, unsigned* cnt, unsigned n) {
    extern __shared__ double lds[];
    if (threadIdx.x == 0) {
        lds[0] = 1.0;
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned seen = 0;
        while ((seen = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < n &&
               __builtin_amdgcn_s_memrealtime() - t0 < 10000000) {   // 0.1 s
        }
        out[blockIdx.x] = (static_cast<unsigned long long>(xcc & 0xf) << 32) | seen | (lds[0] > 0.0 ? 0u : 1u << 31);
    }
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    printf("CUs %d\n", ncu);
    const int nw = (ncu + 31) / 32;
    const int G = 2048;
    unsigned long long* d;
    (void)hipMalloc(&d, G * sizeof(unsigned long long));
    struct M { const char* name; std::vector<uint32_t> m; };
    std::vector<M> masks;
    auto mk = [&](const char* name, auto pred) {
        std::vector<uint32_t> m(nw, 0u);
        for (int i = 0; i < ncu; ++i)
            if (pred(i)) m[i / 32] |= 1u << (i % 32);
        masks.push_back({name, m});
    };
    mk("all", [](int) { return true; });
    mk("bits 0-31", [](int i) { return i < 32; });
    mk("bits 0-7", [](int i) { return i < 8; });
    mk("bits i%8==0", [](int i) { return i % 8 == 0; });
    mk("bits i%32<4", [](int i) { return i % 32 < 4; });
    mk("bits i<64 (first 8 per 32?)", [](int i) { return i < 64; });
    for (auto& m : masks) {
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, nw, m.m.data()) != hipSuccess) {
            printf("%s: create failed\n", m.name);
            continue;
        }
        (void)hipMemset(d, 0xff, G * sizeof(unsigned long long));
        hipLaunchKernelGGL(where, dim3(G), dim3(64), 0, s, d);
        (void)hipStreamSynchronize(s);
        std::vector<unsigned long long> h(G);
        (void)hipMemcpy(h.data(), d, G * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::set<int> xccs;
        std::set<std::tuple<int, int, int, int>> cus;
        std::vector<int> per_xcc(16, 0);
        for (auto v : h) {
            const int xcc = static_cast<int>(v >> 32);
            const unsigned hw = static_cast<unsigned>(v);
            const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            xccs.insert(xcc);
            cus.insert({xcc, se, sh, cu});
            per_xcc[xcc & 15]++;
        }
        printf("%-28s xccs %zu, distinct (xcc,se,sh,cu) %zu; wgs per xcc:", m.name, xccs.size(), cus.size());
        for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
        printf("\n   slots:");
        int k = 0;
        for (auto& c : cus) {
            if (k++ < 40) printf(" %d/%d/%d/%d", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
        }
        printf("\n");
        (void)hipStreamDestroy(s);
    }
    // gangs of WGs holding a full CU's LDS on k CUs per XCD
    unsigned* cnt;
    (void)hipMalloc(&cnt, sizeof(unsigned));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gang), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int k : {17, 9, 4}) {
        for (int lds_kb : {160, 80}) {
            std::vector<uint32_t> m(nw, 0u);
            for (int i = 0; i < 8 * k; ++i) m[i / 32] |= 1u << (i % 32);
            hipStream_t s;
            (void)hipExtStreamCreateWithCUMask(&s, nw, m.data());
            const unsigned n = static_cast<unsigned>(8 * k * (160 / lds_kb));   // exactly the capacity
            (void)hipMemset(cnt, 0, sizeof(unsigned));
            hipLaunchKernelGGL(gang, dim3(n), dim3(256), lds_kb * 1024, s, d, cnt, n);
            (void)hipStreamSynchronize(s);
            std::vector<unsigned long long> h(n);
            (void)hipMemcpy(h.data(), d, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            unsigned minseen = ~0u;
            int stride8_same = 1;
            for (unsigned b = 0; b < n; ++b) {
                minseen = std::min(minseen, static_cast<unsigned>(h[b] & 0x7fffffff));
                if (b + 8 < n && (h[b] >> 32) != (h[b + 8] >> 32)) stride8_same = 0;
            }
            printf("gang k=%d lds %d KB: %u WGs, min arrivals seen %u (all co-resident: %s), b/b+8 same XCC: %d\n", k,
                   lds_kb, n, minseen, minseen >= n ? "yes" : "NO", stride8_same);
            (void)hipStreamDestroy(s);
        }
    }
    return 0;
}
