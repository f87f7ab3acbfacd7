// grid_kernels.hip — occupancy-grid mapping for gfx950 (MI355X).
//
// Rebuilds src/produce_occupancy_grid.py of the reference (cohnt/ICP-SLAM-
// with-Loop-Closure): every lidar beam walks its integer Bresenham line from
// the robot's cell to the point's cell, a "miss" (odds -k_miss) on every cell
// the loop visits, a "hit" (+k_hit) where it stops (:89-121), in beam order.
//
// The reference's int8 arithmetic makes the per-cell result depend on the
// ORDER of its updates only through the last one: a miss on a positive cell
// and a hit on a negative cell saturate (its `-128 - g` / `127 - g` tests wrap
// in int8), so for a cell with initial value g0, m misses and h hits
//   m = h = 0       -> g0
//   h = 0           -> g0 > 0 ? -128 : max(g0 - m k_miss, -128)
//   m = 0           -> g0 < 0 ?  127 : min(g0 + h k_hit, 127)
//   both            -> the last update was a hit ? 127 : -128
// (k_hit, k_miss >= 1; checked exhaustively against the sequential rule in
// tests/test_occupancy.py).  So beams run fully in parallel: one thread per
// beam adds to per-cell miss/hit counters and raises a per-cell "last event"
// key (beam index, step along the beam, hit bit) with 64-bit atomic max; one
// pass per cell then applies the closed form.  No sort, no ordering.
//
// Kernels: grid_points_kernel (global points, one block per scan, + per-block
// bounds), grid_bounds_kernel (min/max of the block bounds), grid_zero_kernel,
// grid_rays_kernel (one thread per beam), grid_finalize_kernel (one per cell).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace slamhip {

constexpr int kGridBlock = 256;

// pose4[s] = (cos theta, sin theta, x, y) of scan s (cos/sin from the host's
// np.cos/np.sin, exactly the reference's odom_change_to_mat values).
__global__ __launch_bounds__(kGridBlock) void grid_points_kernel(const double2* __restrict__ pts,
                                                                 const int64_t* __restrict__ scan_off,
                                                                 const double* __restrict__ pose4,
                                                                 double2* __restrict__ gpts,
                                                                 double* __restrict__ blk_bounds) {
    const int s = blockIdx.x;
    const double c = pose4[4 * s], sn = pose4[4 * s + 1], px = pose4[4 * s + 2], py = pose4[4 * s + 3];
    double bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
    for (int64_t j = scan_off[s] + threadIdx.x; j < scan_off[s + 1]; j += kGridBlock) {
        const double2 p = pts[j];
        // [c -s x; s c y] [p; 1] exactly as NumPy's 3x3 @ 3x1 product rounds it on
        // the build host (OpenBLAS: fma(a0, x0, a1 x1) + a2 x2, found by brute force
        // over every association and fusion; tests/golden/grid_ref.npz pins it)
        const double gx = fma(c, p.x, -sn * p.y) + px;
        const double gy = fma(sn, p.x, c * p.y) + py;
        gpts[j] = make_double2(gx, gy);
        bx0 = fmin(bx0, gx);
        bx1 = fmax(bx1, gx);
        by0 = fmin(by0, gy);
        by1 = fmax(by1, gy);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        bx0 = fmin(bx0, __shfl_xor(bx0, off, 64));
        bx1 = fmax(bx1, __shfl_xor(bx1, off, 64));
        by0 = fmin(by0, __shfl_xor(by0, off, 64));
        by1 = fmax(by1, __shfl_xor(by1, off, 64));
    }
    __shared__ double red[kGridBlock / 64][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave][0] = bx0;
        red[wave][1] = bx1;
        red[wave][2] = by0;
        red[wave][3] = by1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kGridBlock / 64; ++w) {
            red[0][0] = fmin(red[0][0], red[w][0]);
            red[0][1] = fmax(red[0][1], red[w][1]);
            red[0][2] = fmin(red[0][2], red[w][2]);
            red[0][3] = fmax(red[0][3], red[w][3]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) blk_bounds[4 * s + q] = red[0][q];
    }
}

// (min x, max x, min y, max y) over the S block results; one block.
__global__ __launch_bounds__(kGridBlock) void grid_bounds_kernel(const double* __restrict__ blk, int32_t S,
                                                                 double* __restrict__ out) {
    double v[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    for (int s = threadIdx.x; s < S; s += kGridBlock) {
        v[0] = fmin(v[0], blk[4 * s]);
        v[1] = fmax(v[1], blk[4 * s + 1]);
        v[2] = fmin(v[2], blk[4 * s + 2]);
        v[3] = fmax(v[3], blk[4 * s + 3]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        v[0] = fmin(v[0], __shfl_xor(v[0], off, 64));
        v[1] = fmax(v[1], __shfl_xor(v[1], off, 64));
        v[2] = fmin(v[2], __shfl_xor(v[2], off, 64));
        v[3] = fmax(v[3], __shfl_xor(v[3], off, 64));
    }
    __shared__ double red[kGridBlock / 64][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
        for (int q = 0; q < 4; ++q) red[wave][q] = v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kGridBlock / 64; ++w) {
            red[0][0] = fmin(red[0][0], red[w][0]);
            red[0][1] = fmax(red[0][1], red[w][1]);
            red[0][2] = fmin(red[0][2], red[w][2]);
            red[0][3] = fmax(red[0][3], red[w][3]);
        }
        for (int q = 0; q < 4; ++q) out[q] = red[0][q];
    }
}

__global__ void grid_zero_kernel(uint32_t* __restrict__ cnt, unsigned long long* __restrict__ last, int64_t cells) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= cells) return;
    cnt[2 * i] = 0;
    cnt[2 * i + 1] = 0;
    last[i] = 0;
}

// global_position_to_grid_cell (:123-128): floor((p - min) / w)
__device__ __forceinline__ int64_t grid_cell(double p, double mn, double w) {
    return static_cast<int64_t>(floor((p - mn) / w));
}

// One thread per beam (global point index g, in the reference's scan-major
// order): the reference's Bresenham loop, recording events instead of values.
__global__ __launch_bounds__(kGridBlock) void grid_rays_kernel(const double2* __restrict__ gpts,
                                                               const int64_t* __restrict__ scan_off, int32_t S,
                                                               const double* __restrict__ pose4, int64_t P,
                                                               double min_x, double min_y, double w, int32_t H,
                                                               int32_t W, uint32_t* __restrict__ cnt,
                                                               unsigned long long* __restrict__ last) {
    const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= P) return;
    int lo = 0, hi = S - 1;   // scan of beam g: last s with scan_off[s] <= g
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (scan_off[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    const double2 q = gpts[g];
    int64_t x0 = grid_cell(pose4[4 * lo + 2], min_x, w), y0 = grid_cell(pose4[4 * lo + 3], min_y, w);
    const int64_t x1 = grid_cell(q.x, min_x, w), y1 = grid_cell(q.y, min_y, w);
    const int64_t dx = x1 > x0 ? x1 - x0 : x0 - x1;
    const int64_t dy = -(y1 > y0 ? y1 - y0 : y0 - y1);
    const int64_t sx = x1 > x0 ? 1 : -1, sy = y1 > y0 ? 1 : -1;
    int64_t err = dx + dy;
    const unsigned long long base = static_cast<unsigned long long>(g) << 24;
    unsigned long long step = 0;
    while (x0 >= 0 && x0 < W && y0 >= 0 && y0 < H) {
        const int64_t c = y0 * W + x0;
        atomicAdd(&cnt[2 * c], 1u);                                   // miss
        atomicMax(&last[c], base | (step << 1));
        ++step;
        const int64_t e2 = err * 2;
        if (e2 >= dy) {
            if (x0 == x1) break;
            err += dy;
            x0 += sx;
        }
        if (e2 <= dx) {
            if (y0 == y1) break;
            err += dx;
            y0 += sy;
        }
    }
    if (x0 >= 0 && x0 < W && y0 >= 0 && y0 < H) {
        const int64_t c = y0 * W + x0;
        atomicAdd(&cnt[2 * c + 1], 1u);                               // hit
        atomicMax(&last[c], base | (step << 1) | 1ull);
    }
}

__global__ void grid_finalize_kernel(int8_t* __restrict__ grid, const uint32_t* __restrict__ cnt,
                                     const unsigned long long* __restrict__ last, int64_t cells, int32_t k_hit,
                                     int32_t k_miss) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= cells) return;
    const int64_t m = cnt[2 * i], h = cnt[2 * i + 1];
    const int64_t g0 = grid[i];
    int64_t v = g0;
    if (m > 0 && h > 0) v = (last[i] & 1ull) ? 127 : -128;
    else if (m > 0) v = g0 > 0 ? -128 : max(g0 - m * k_miss, static_cast<int64_t>(-128));
    else if (h > 0) v = g0 < 0 ? 127 : min(g0 + h * k_hit, static_cast<int64_t>(127));
    grid[i] = static_cast<int8_t>(v);
}

}  // namespace slamhip

using namespace slamhip;

extern "C" {

int64_t slam_grid_work_size(int32_t S, int32_t H, int32_t W) {
    // bytes: block bounds (4 S doubles) | counters (2 u32 / cell) | last keys (u64 / cell)
    const int64_t cells = static_cast<int64_t>(H) * W;
    return 32 * static_cast<int64_t>(S) + 8 * cells + 8 * cells + 64;
}

int slam_grid_global_points_f64(const double* pts, const int64_t* scan_off, int32_t S, const double* pose4,
                                double* gpts, double* bounds, void* work, void* stream) {
    if (S < 1) return fail(SLAM_EINVAL, "grid: S = %d < 1", S);
    if (!pts || !scan_off || !pose4 || !gpts || !bounds || !work) return fail(SLAM_EINVAL, "grid: null array");
    hipStream_t st = as_stream(stream);
    double* blk = reinterpret_cast<double*>(work);
    hipLaunchKernelGGL(grid_points_kernel, dim3(S), dim3(kGridBlock), 0, st, reinterpret_cast<const double2*>(pts),
                       scan_off, pose4, reinterpret_cast<double2*>(gpts), blk);
    hipLaunchKernelGGL(grid_bounds_kernel, dim3(1), dim3(kGridBlock), 0, st, blk, S, bounds);
    return check_launch("grid points kernels");
}

int slam_grid_update_i8(const double* gpts, const int64_t* scan_off, int32_t S, const double* pose4, int64_t P,
                        double min_x, double min_y, double cell_width, int32_t H, int32_t W, int32_t k_hit,
                        int32_t k_miss, int8_t* grid, void* work, void* stream) {
    if (S < 1 || P < 0 || H < 1 || W < 1) return fail(SLAM_EINVAL, "grid: S=%d P=%lld H=%d W=%d", S,
                                                      static_cast<long long>(P), H, W);
    if (!(cell_width > 0.0)) return fail(SLAM_EINVAL, "grid: cell_width must be > 0");
    if (k_hit < 1 || k_miss < 1 || k_hit > 127 || k_miss > 127)
        return fail(SLAM_EINVAL, "grid: hit/miss odds must be in [1, 127] (got %d, %d)", k_hit, k_miss);
    if (P >= (1ll << 40) || H + static_cast<int64_t>(W) >= (1ll << 22))
        return fail(SLAM_ETOOBIG, "grid: %lld beams / %d x %d cells exceed the event-key range",
                    static_cast<long long>(P), H, W);
    if (!gpts || !scan_off || !pose4 || !grid || !work) return fail(SLAM_EINVAL, "grid: null array");
    hipStream_t st = as_stream(stream);
    const int64_t cells = static_cast<int64_t>(H) * W;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(work) + 32 * static_cast<int64_t>(S));
    unsigned long long* last = reinterpret_cast<unsigned long long*>(cnt + 2 * cells);
    const unsigned gz = static_cast<unsigned>((cells + 255) / 256);
    hipLaunchKernelGGL(grid_zero_kernel, dim3(gz), dim3(256), 0, st, cnt, last, cells);
    if (P > 0)
        hipLaunchKernelGGL(grid_rays_kernel, dim3(static_cast<unsigned>((P + kGridBlock - 1) / kGridBlock)),
                           dim3(kGridBlock), 0, st, reinterpret_cast<const double2*>(gpts), scan_off, S, pose4, P,
                           min_x, min_y, cell_width, H, W, cnt, last);
    hipLaunchKernelGGL(grid_finalize_kernel, dim3(gz), dim3(256), 0, st, grid, cnt, last, cells, k_hit, k_miss);
    return check_launch("grid update kernels");
}

}  // extern "C"
