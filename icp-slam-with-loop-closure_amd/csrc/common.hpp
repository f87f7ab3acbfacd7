// common.hpp — shared helpers of the slamhip C-ABI (error state, launch checks).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "slamhip.h"

// Timing-only ablation switches remove work from the ICP kernel and give
// WRONG results (DESIGN.md section 3.1 cycle budget).  A product build refuses
// them: only a build that also defines SLAM_TIMING_ONLY (tools/ab_build.sh
// A/B libraries under ab/, never the in-tree libslamhip.so) may set them.
#if !defined(SLAM_TIMING_ONLY) && (defined(SLAM_ABL_SUMS) || defined(SLAM_ABL_GROUP) || defined(SLAM_ABL_CERT) || \
                                   defined(SLAM_ABL_STAGE2X) || defined(SLAM_NO_WINX) || defined(SLAM_KABSCH_ALL))
#error "SLAM_ABL_* / SLAM_NO_WINX / SLAM_KABSCH_ALL are timing-only ablations: define SLAM_TIMING_ONLY as well (A/B builds only)"
#endif
#if defined(SLAM_TIMING_ONLY) && defined(SLAMHIP_PRODUCT_BUILD)
#error "SLAM_TIMING_ONLY in a product build"
#endif

namespace slamhip {

// Thread-local message of the last failing call (slam_last_error()).
inline char* last_error_buf() {
    static thread_local char buf[512] = {0};
    return buf;
}

inline int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(last_error_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline int ok() {
    last_error_buf()[0] = 0;
    return SLAM_OK;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SLAM_EHIP, "%s: %s", what, hipGetErrorString(e));
    return ok();
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// 3x3 SE(2) matrix with the last row implicit [0, 0, 1].
struct SE2 {
    double m00, m01, m02, m10, m11, m12;
};

__device__ __forceinline__ SE2 load_se2(const double* p) {
    SE2 t;
    t.m00 = p[0]; t.m01 = p[1]; t.m02 = p[2];
    t.m10 = p[3]; t.m11 = p[4]; t.m12 = p[5];
    return t;
}

__device__ __forceinline__ void store_se2(double* p, const SE2& t) {
    p[0] = t.m00; p[1] = t.m01; p[2] = t.m02;
    p[3] = t.m10; p[4] = t.m11; p[5] = t.m12;
    // the constant row from registers set here: as a hoisted constant the
    // zero pair was the ICP kernel's only VGPR spill
    double z = 0.0, one = 1.0;
    asm volatile("" : "+v"(z), "+v"(one));
    p[6] = z;     p[7] = z;     p[8] = one;
}

// A @ B for SE(2) matrices with NumPy/OpenBLAS dgemm rounding: every entry is
// the k = 0, 1, 2 FMA chain fma(a2, b2, fma(a1, b1, a0 * b0)) (verified bit
// for bit against numpy 2.2 / OpenBLAS 0.3.29 in the build container).  With
// B's last row [0, 0, 1] the k = 2 term is +0 (columns 0, 1) or a2 (column 2).
__device__ __forceinline__ SE2 se2_mul(const SE2& a, const SE2& b) {
    SE2 c;
    c.m00 = fma(a.m02, 0.0, fma(a.m01, b.m10, a.m00 * b.m00));
    c.m01 = fma(a.m02, 0.0, fma(a.m01, b.m11, a.m00 * b.m01));
    c.m02 = fma(a.m02, 1.0, fma(a.m01, b.m12, a.m00 * b.m02));
    c.m10 = fma(a.m12, 0.0, fma(a.m11, b.m10, a.m10 * b.m00));
    c.m11 = fma(a.m12, 0.0, fma(a.m11, b.m11, a.m10 * b.m01));
    c.m12 = fma(a.m12, 1.0, fma(a.m11, b.m12, a.m10 * b.m02));
    return c;
}

// All-lane sum of a wave64 without LDS: pairs and quads by DPP quad_perm,
// quads of a 16-lane row by DPP row_ror 12 / 8 (lane 0 of each row then holds
// the row sum), the four rows combined as (r0+r1)+(r2+r3) by row swaps.  Lane 0
// holds the result (other lanes may differ in rounding; callers use lane 0).
#define SLAM_DPP_D(v, ctrl)                                                                            \
    __longlong_as_double(                                                                              \
        (static_cast<long long>(__builtin_amdgcn_update_dpp(                                           \
             0, static_cast<int>(__double_as_longlong(v) >> 32), ctrl, 0xF, 0xF, false))                \
         << 32) |                                                                                      \
        static_cast<unsigned int>(__builtin_amdgcn_update_dpp(                                         \
            0, static_cast<int>(__double_as_longlong(v) & 0xffffffff), ctrl, 0xF, 0xF, false)))
// Lane `lane`'s double (lane wave-uniform) through SGPRs.
__device__ __forceinline__ double readlane_d(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffff), lane);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), lane);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ double wave_sum(double v) {
    v += SLAM_DPP_D(v, 0xB1);    // xor 1
    v += SLAM_DPP_D(v, 0x4E);    // xor 2
    v += SLAM_DPP_D(v, 0x12C);   // row_ror 12
    v += SLAM_DPP_D(v, 0x128);   // row_ror 8
    // rows: (r0 + r1) in rows 0-1, (r2 + r3) in rows 2-3 (gfx950 v_permlane16_swap),
    // then the halves (v_permlane32_swap): lane 0 holds (r0 + r1) + (r2 + r3)
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(b), static_cast<unsigned>(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(b >> 32), static_cast<unsigned>(b >> 32),
                                                     false, false);
    v = __longlong_as_double((static_cast<long long>(hi[0]) << 32) | lo[0]) +
        __longlong_as_double((static_cast<long long>(hi[1]) << 32) | lo[1]);
    const long long c = __double_as_longlong(v);
    const auto lo2 = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(c), static_cast<unsigned>(c), false, false);
    const auto hi2 = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(c >> 32), static_cast<unsigned>(c >> 32),
                                                      false, false);
    return __longlong_as_double((static_cast<long long>(hi2[0]) << 32) | lo2[0]) +
           __longlong_as_double((static_cast<long long>(hi2[1]) << 32) | lo2[1]);
}
#undef SLAM_DPP_D

// Deterministic block all-reduce of NV doubles; `red` is LDS scratch of
// WAVES * NV doubles.  Every thread returns identical bits (fixed wave order).
template <int NV, int WAVES>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[wave * NV + k] = v[k];
    }
    __syncthreads();
    if constexpr (WAVES <= 8) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double s = red[k];
#pragma unroll
            for (int w = 1; w < WAVES; ++w) s += red[w * NV + k];
            v[k] = s;
        }
    } else {
        // 16-wave workgroups: lane w reads wave w's partials and the wave sums
        // them with the DPP tree (fixed order; NV registers instead of WAVES*NV)
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = lane < WAVES ? red[lane * NV + k] : 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = readlane_d(wave_sum(v[k]), 0);
    }
}

// ---------------------------------------------------------------------------
// Order-free sums.  A term x with |x| <= B (one of n terms) is split onto two
// fixed grids chosen from (B, n) alone: h1 = (x + M1) - M1 is x rounded to a
// multiple of u1 = ulp(M1) (exact: x + M1 stays inside M1's binade), the
// remainder r = x - h1 is exact, and h2 = (r + M2) - M2 rounds r to u2 =
// ulp(M2).  Every partial sum of h1 values (multiples of u1, bounded by
// 2^53 u1) and of h2 values is exact, so the two totals are the same bits for
// ANY summation order: any workgroup shape, query layout or split of a pair
// over workgroups.  The dropped remainder is <= u2 / 2 per term, ~2^-70 of n B
// (far below a naive fp64 sum's rounding).  Valid while n B < 2^900.
// ---------------------------------------------------------------------------
struct RsumGrid {
    double m1, m2;
};

__device__ __forceinline__ RsumGrid rsum_grid(double bound, int n) {
    int e;
    (void)frexp(fmin(fmax(bound, 0x1p-900), 0x1p+900) * static_cast<double>(n), &e);   // n B < 2^e
    e += 2;                                                                           // |x| <= 2^(e-2) / n
    const int lg = 32 - __clz(max(n - 1, 1));                                         // n <= 2^lg
    RsumGrid g;
    g.m1 = ldexp(1.5, e);
    g.m2 = ldexp(1.5, e - 53 + lg + 2);   // |r| <= 2^(e-53) <= 2^(e2-2) / n
    return g;
}

__device__ __forceinline__ void rsum_add(double x, const RsumGrid& g, double& s1, double& s2) {
#ifdef SLAM_ABL_SUMS
    s1 += x;   // ablation build (timing only): plain sums
    return;
#endif
    const double h1 = (x + g.m1) - g.m1;
    const double r = x - h1;
    const double h2 = (r + g.m2) - g.m2;
    s1 += h1;
    s2 += h2;
}

// v_permlane{16,32}_swap on doubles (both 32-bit halves): for a pair (a, b)
// a + b afterwards is a's sum over the two swapped lane sets in one half (rows)
// and b's in the other.
__device__ __forceinline__ void swap32_d(double& a, double& b) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(x), static_cast<unsigned>(y), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<unsigned>(x >> 32), static_cast<unsigned>(y >> 32),
                                                     false, false);
    a = __longlong_as_double((static_cast<long long>(hi[0]) << 32) | lo[0]);
    b = __longlong_as_double((static_cast<long long>(hi[1]) << 32) | lo[1]);
}
__device__ __forceinline__ void swap16_d(double& a, double& b) {
    const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(x), static_cast<unsigned>(y), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<unsigned>(x >> 32), static_cast<unsigned>(y >> 32),
                                                     false, false);
    a = __longlong_as_double((static_cast<long long>(hi[0]) << 32) | lo[0]);
    b = __longlong_as_double((static_cast<long long>(hi[1]) << 32) | lo[1]);
}

// Sum over the 16 lanes of each row; every lane of the row gets it.
__device__ __forceinline__ double row_sum_d(double v) {
#define SLAM_DPP_D(v, ctrl)                                                                            \
    __longlong_as_double(                                                                              \
        (static_cast<long long>(__builtin_amdgcn_update_dpp(                                           \
             0, static_cast<int>(__double_as_longlong(v) >> 32), ctrl, 0xF, 0xF, false))                \
         << 32) |                                                                                      \
        static_cast<unsigned int>(__builtin_amdgcn_update_dpp(                                         \
            0, static_cast<int>(__double_as_longlong(v) & 0xffffffff), ctrl, 0xF, 0xF, false)))
    v += SLAM_DPP_D(v, 0xB1);    // xor 1
    v += SLAM_DPP_D(v, 0x4E);    // xor 2
    v += SLAM_DPP_D(v, 0x12C);   // row_ror 12
    v += SLAM_DPP_D(v, 0x128);   // row_ror 8
#undef SLAM_DPP_D
    return v;
}

// Block all-reduce of 16 per-thread values whose partial sums are all EXACT
// (rsum_add grids), so the reduction order is free and chosen for cost: a
// reduce-scatter over the wave halves and row pairs (permlane swaps: 16 -> 8
// -> 4 values per lane), row sums of the remaining 4, one LDS slot per value
// and wave, and lane q (< 16) of every wave sums value q over the waves.
// `slab` is LDS of WAVES * 16 doubles; one barrier.  Returns value q in lane
// q (readlane_d(ret, q) makes it uniform).
template <int WAVES>
__device__ __forceinline__ double block_sum_exact16(double (&v)[16], double* slab) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // lanes 0-31: v[2j] summed over l, l+32; lanes 32-63: v[2j+1]
        swap32_d(v[2 * j], v[2 * j + 1]);
        v[j] = v[2 * j] + v[2 * j + 1];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // row r holds v[4i + {0, 2, 1, 3}[r]] summed over l, l+16, l+32, l+48
        swap16_d(v[2 * i], v[2 * i + 1]);
        v[i] = v[2 * i] + v[2 * i + 1];
    }
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int row = lane >> 4;
    const int q0 = ((row & 1) << 1) | (row >> 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double s = row_sum_d(v[i]);
        if ((lane & 15) == 0) slab[wave * 16 + 4 * i + q0] = s;
    }
    __syncthreads();
    double t = 0.0;
    if (lane < 16) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) t += slab[w * 16 + lane];
    }
    return t;
}

// The wave-level form of block_sum_exact16: the 16 values summed over this
// wave's 64 lanes (exact partial sums, so the order is free), value q returned
// in lane q < 16 — no LDS, no barrier.
__device__ __forceinline__ double wave_sum_exact16(double (&v)[16]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        swap32_d(v[2 * j], v[2 * j + 1]);
        v[j] = v[2 * j] + v[2 * j + 1];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        swap16_d(v[2 * i], v[2 * i + 1]);
        v[i] = v[2 * i] + v[2 * i + 1];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = row_sum_d(v[i]);   // row r, register i: value 4 i + q0(r)
    const int lane = threadIdx.x & 63;
    const int q = lane & 15, q0 = q & 3;
    const int src = 16 * (((q0 & 1) << 1) | (q0 >> 1));   // the row holding value q (q0 is an involution)
    const double t0 = __shfl(v[0], src, 64), t1 = __shfl(v[1], src, 64);
    const double t2 = __shfl(v[2], src, 64), t3 = __shfl(v[3], src, 64);
    const int i = q >> 2;
    return i == 0 ? t0 : i == 1 ? t1 : i == 2 ? t2 : t3;
}

}  // namespace slamhip
