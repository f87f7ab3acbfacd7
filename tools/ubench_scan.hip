// ubench_scan.hip — candidate formulations of the ICP nearest-neighbour scan
// (diagnostic tool, not the product).  Every variant scans NC LDS-resident
// candidates for QPT queries per lane; prints evals/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/ubench_scan.hip -o tools/ubench_scan
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int NC = 1088;
constexpr int QPT = 8;
constexpr int BLOCK = 256;
constexpr int REPS = 8;

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int V>
__global__ __launch_bounds__(BLOCK) void scan(const double2* __restrict__ pts, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) double2 cand[NC];
    __shared__ __attribute__((aligned(16))) float2 candf[NC];
    const double2* p = pts + (blockIdx.x % 64) * NC;
    for (int j = threadIdx.x; j < NC; j += BLOCK) {
        cand[j] = p[j];
        candf[j] = make_float2((float)p[j].x, (float)p[j].y);
    }
    __syncthreads();
    double qx[QPT], qy[QPT];
    float fx[QPT], fy[QPT];
    for (int k = 0; k < QPT; ++k) {
        const double2 q = p[(threadIdx.x * 7 + k * 131) % NC];
        qx[k] = q.x + 0.003;
        qy[k] = q.y - 0.002;
        fx[k] = (float)qx[k];
        fy[k] = (float)qy[k];
    }
    uint32_t acc = 0;
    uint32_t mask = 0xFFFFF800u;
    asm volatile("" : "+v"(mask));
    for (int r = 0; r < REPS; ++r) {
        if constexpr (V == 0) {   // fp64 exact: cmp + 3 cndmask
            double best[QPT];
            int bi[QPT];
            for (int k = 0; k < QPT; ++k) { best[k] = INFINITY; bi[k] = 0; }
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const double2 c = cand[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const double dx = c.x - qx[k], dy = c.y - qy[k];
                    const double d = dx * dx + dy * dy;
                    const bool lt = d < best[k];
                    best[k] = lt ? d : best[k];
                    bi[k] = lt ? j : bi[k];
                }
            }
            for (int k = 0; k < QPT; ++k) acc += bi[k];
        } else if constexpr (V == 1) {   // fp64 exact: min_f64 + cmp + cndmask(idx)
            double best[QPT];
            int bi[QPT];
            for (int k = 0; k < QPT; ++k) { best[k] = INFINITY; bi[k] = 0; }
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const double2 c = cand[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const double dx = c.x - qx[k], dy = c.y - qy[k];
                    const double d = dx * dx + dy * dy;
                    bi[k] = d < best[k] ? j : bi[k];
                    best[k] = fmin(d, best[k]);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += bi[k];
        } else if constexpr (V == 2 || V == 3) {   // fp32 screen, int keys (2: med3 asm, 3: min/max)
            uint32_t m1[QPT], m2[QPT];
            for (int k = 0; k < QPT; ++k) { m1[k] = ~0u; m2[k] = ~0u; }
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const float2 c = candf[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const float dx = c.x - fx[k], dy = c.y - fy[k];
                    const float d = fmaf(dy, dy, dx * dx);
                    const uint32_t key = (__float_as_uint(d) & mask) | (uint32_t)j;
                    if constexpr (V == 2) m2[k] = umed3(m1[k], m2[k], key);
                    else m2[k] = min(max(m1[k], key), m2[k]);
                    m1[k] = min(m1[k], key);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += m1[k] ^ m2[k];
        } else if constexpr (V == 4) {   // fp32 screen, float keys: v_med3_f32 + v_min_f32
            float m1[QPT], m2[QPT];
            for (int k = 0; k < QPT; ++k) { m1[k] = INFINITY; m2[k] = INFINITY; }
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const float2 c = candf[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const float dx = c.x - fx[k], dy = c.y - fy[k];
                    const float d = fmaf(dy, dy, dx * dx);
                    const float key = __uint_as_float((__float_as_uint(d) & mask) | (uint32_t)j);
                    m2[k] = __builtin_amdgcn_fmed3f(m1[k], m2[k], key);
                    m1[k] = fminf(m1[k], key);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += __float_as_uint(m1[k]) ^ __float_as_uint(m2[k]);
        } else if constexpr (V == 5) {   // fp32 screen, float keys, 2 candidates merged with min3
            float m1[QPT], m2[QPT];
            for (int k = 0; k < QPT; ++k) { m1[k] = INFINITY; m2[k] = INFINITY; }
            for (int j = 0; j < NC; j += 2) {
                const float4 c = *reinterpret_cast<const float4*>(&candf[j]);
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const float ax = c.x - fx[k], ay = c.y - fy[k];
                    const float bx = c.z - fx[k], by = c.w - fy[k];
                    const float da = fmaf(ay, ay, ax * ax);
                    const float db = fmaf(by, by, bx * bx);
                    const float ka = __uint_as_float((__float_as_uint(da) & mask) | (uint32_t)j);
                    const float kb = __uint_as_float((__float_as_uint(db) & mask) | (uint32_t)(j + 1));
                    const float lo = fminf(ka, kb), hi = fmaxf(ka, kb);
                    m2[k] = __builtin_amdgcn_fmed3f(m1[k], lo, fminf(m2[k], hi));
                    m1[k] = fminf(m1[k], lo);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += __float_as_uint(m1[k]) ^ __float_as_uint(m2[k]);
        } else if constexpr (V == 6) {   // fp32 value-only top-2 (no index): lower bound of cost
            float m1[QPT], m2[QPT];
            for (int k = 0; k < QPT; ++k) { m1[k] = INFINITY; m2[k] = INFINITY; }
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const float2 c = candf[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const float dx = c.x - fx[k], dy = c.y - fy[k];
                    const float d = fmaf(dy, dy, dx * dx);
                    m2[k] = __builtin_amdgcn_fmed3f(m1[k], m2[k], d);
                    m1[k] = fminf(m1[k], d);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += __float_as_uint(m1[k]) ^ __float_as_uint(m2[k]);
        } else if constexpr (V == 7) {   // fp64 distance only + v_min_f64 (value-only bound)
            double best[QPT];
            for (int k = 0; k < QPT; ++k) best[k] = INFINITY;
#pragma unroll 2
            for (int j = 0; j < NC; ++j) {
                const double2 c = cand[j];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const double dx = c.x - qx[k], dy = c.y - qy[k];
                    best[k] = fmin(dx * dx + dy * dy, best[k]);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += (uint32_t)__double_as_longlong(best[k]);
        } else if constexpr (V == 8 || V == 9) {   // chunked value-only (8: scalar math, 9: packed math)
            constexpr int C = 32;
            float M1[QPT], M2[QPT];
            int C1[QPT];
            for (int k = 0; k < QPT; ++k) { M1[k] = INFINITY; M2[k] = INFINITY; C1[k] = 0; }
            for (int c0 = 0; c0 < NC; c0 += C) {
                float cm[QPT];
                for (int k = 0; k < QPT; ++k) cm[k] = INFINITY;
                if constexpr (V == 8) {
#pragma unroll 4
                    for (int j = c0; j < c0 + C; ++j) {
                        const float2 c = candf[j];
#pragma unroll
                        for (int k = 0; k < QPT; ++k) {
                            const float dx = c.x - fx[k], dy = c.y - fy[k];
                            cm[k] = fminf(cm[k], fmaf(dy, dy, dx * dx));
                        }
                    }
                } else {
                    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll 4
                    for (int j = c0; j < c0 + C; ++j) {
                        const float2 c = candf[j];
                        const f2 cx = {c.x, c.x}, cy = {c.y, c.y};
#pragma unroll
                        for (int k = 0; k < QPT; k += 2) {
                            const f2 qx2 = {fx[k], fx[k + 1]}, qy2 = {fy[k], fy[k + 1]};
                            const f2 dx = cx - qx2, dy = cy - qy2;
                            const f2 d = __builtin_elementwise_fma(dy, dy, dx * dx);
                            cm[k] = fminf(cm[k], d.x);
                            cm[k + 1] = fminf(cm[k + 1], d.y);
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const bool lt = cm[k] < M1[k];
                    M2[k] = __builtin_amdgcn_fmed3f(M1[k], M2[k], cm[k]);
                    C1[k] = lt ? c0 : C1[k];
                    M1[k] = fminf(M1[k], cm[k]);
                }
            }
            for (int k = 0; k < QPT; ++k) acc += __float_as_uint(M1[k]) ^ __float_as_uint(M2[k]) ^ C1[k];
        }
    }
    out[blockIdx.x * BLOCK + threadIdx.x] = acc;
}

template <int V>
void run(const char* name, const double2* pts, uint32_t* out, int blocks) {
    hipLaunchKernelGGL(scan<V>, dim3(blocks), dim3(BLOCK), 0, 0, pts, out);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(scan<V>, dim3(blocks), dim3(BLOCK), 0, 0, pts, out);
    hipLaunchKernelGGL(scan<V>, dim3(blocks), dim3(BLOCK), 0, 0, pts, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double evals = 2.0 * blocks * BLOCK * QPT * (double)NC * REPS;
    printf("V%d %-34s %8.3f ms  %.3f Teval/s  %.2f ns/wave-eval/SIMD\n", V, name, ms, evals / (ms * 1e-3) / 1e12,
           (ms * 1e6) / (evals / 64.0 / 1024.0));
}

int main() {
    std::vector<double2> h(64 * NC);
    uint64_t s = 88172645463325252ull;
    for (auto& v : h) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        v.x = (double)(s % 100000) * 1e-4 - 5.0;
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        v.y = (double)(s % 100000) * 1e-4 - 5.0;
    }
    double2* d;
    uint32_t* out;
    const int blocks = 256 * 8;
    (void)hipMalloc(&d, h.size() * sizeof(double2));
    (void)hipMalloc(&out, (size_t)blocks * BLOCK * sizeof(uint32_t));
    (void)hipMemcpy(d, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice);
    run<0>("fp64 exact cmp+3cndmask", d, out, blocks);
    run<1>("fp64 exact min_f64+cmp+cndmask", d, out, blocks);
    run<2>("fp32 int keys med3(asm)+min", d, out, blocks);
    run<3>("fp32 int keys max/min+min", d, out, blocks);
    run<4>("fp32 float keys fmed3+fmin", d, out, blocks);
    run<5>("fp32 float keys 2-cand min3 merge", d, out, blocks);
    run<6>("fp32 value-only top2 (bound)", d, out, blocks);
    run<7>("fp64 value-only min (bound)", d, out, blocks);
    run<8>("fp32 chunked(32) value-only", d, out, blocks);
    run<9>("fp32 chunked(32) packed math", d, out, blocks);
    return 0;
}
