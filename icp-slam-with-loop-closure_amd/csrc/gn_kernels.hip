// gn_kernels.hip — SE(2) pose-graph Gauss-Newton for gfx950 (MI355X).
//
// The reference (cohnt/ICP-SLAM-with-Loop-Closure) optimises its pose graph by
// SGD relaxation only (src/pose_graph_optimization.py:7-49); the north star
// asks for a Gauss-Newton solve with sparse-block J^T J assembly + Cholesky.
// It is defined on the graph exactly as the reference exports it to g2o
// (src/pose_graph.py:61-73): edge a->b with tf is the relative measurement
// z = (tf02, tf12, atan2(tf10, tf00)), information w I (w = 2 odometry, 5
// loop), node `fixed` held constant.  CPU oracle: oracle/gn_oracle.py.
//
// One iteration = five launches on one stream:
//   gn_linearize_kernel   one thread per edge: e, A = de/dxi, B = de/dxj and
//                         the five weighted products A'WA, A'WB, B'WB, A'We,
//                         B'We (34 doubles per edge, with w|e|^2)
//   gn_assemble_kernel    one thread per H block slot (free node diagonal or
//                         connected node pair), summing its edge list in a
//                         fixed order -> deterministic, no atomics; writes the
//                         lower band of H (nodes in reverse Cuthill-McKee order,
//                         half-bandwidth W scalars) and the right-hand side
//   gn_factor_kernel      ONE workgroup: blocked right-looking band Cholesky,
//                         the active (W + S) x (W + S) window resident in LDS,
//                         L overwrites H in place
//   gn_solve_kernel       ONE workgroup: blocked forward / backward substitution
//   gn_update_kernel      x <- x + dx, headings wrapped to [-pi, pi)
// Band work is latency-bound (a chain of 3 (N-1) / S dependent block steps);
// the roofline is not the lever at C4 size.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace slamhip {

constexpr int kGnContrib = 34;   // per-edge: 9 AtWA, 9 AtWB, 9 BtWB, 3 AtWe, 3 BtWe, 1 chi2
constexpr int kGnBlock = 512;    // threads of the factor / solve workgroup
constexpr int kGnS = 16;         // Cholesky block size (scalar columns per step)

__device__ __forceinline__ double wrap_pi(double a) {
    return a - 2.0 * M_PI * floor((a + M_PI) / (2.0 * M_PI));
}

__global__ void gn_linearize_kernel(const double* __restrict__ poses, const int32_t* __restrict__ ea,
                                    const int32_t* __restrict__ eb, const double* __restrict__ tf,
                                    const double* __restrict__ w, int32_t E, double* __restrict__ contrib) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int i = ea[e], j = eb[e];
    const double* t = tf + 9 * static_cast<int64_t>(e);
    const double zx = t[2], zy = t[5], zt = atan2(t[3], t[0]);
    const double xi = poses[3 * i], yi = poses[3 * i + 1], ti = poses[3 * i + 2];
    const double xj = poses[3 * j], yj = poses[3 * j + 1], tj = poses[3 * j + 2];
    double si, ci, sz, cz;
    sincos(ti, &si, &ci);
    sincos(zt, &sz, &cz);
    const double dx = xj - xi, dy = yj - yi;
    const double ux = ci * dx + si * dy, uy = -si * dx + ci * dy;   // Ri^T (tj - ti)
    const double vx = ux - zx, vy = uy - zy;
    double ev[3];
    ev[0] = cz * vx + sz * vy;
    ev[1] = -sz * vx + cz * vy;
    ev[2] = wrap_pi(tj - ti - zt);
    // M = Rz^T Ri^T; g = d(Ri^T)/dthi (tj - ti)
    const double m00 = cz * ci - sz * si, m01 = cz * si + sz * ci;
    const double m10 = -sz * ci - cz * si, m11 = -sz * si + cz * ci;
    const double gx = -si * dx + ci * dy, gy = -ci * dx - si * dy;
    const double A[3][3] = {{-m00, -m01, cz * gx + sz * gy}, {-m10, -m11, -sz * gx + cz * gy}, {0.0, 0.0, -1.0}};
    const double B[3][3] = {{m00, m01, 0.0}, {m10, m11, 0.0}, {0.0, 0.0, 1.0}};
    const double we = w[e];
    double* o = contrib + static_cast<int64_t>(e) * kGnContrib;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double aa = 0.0, ab = 0.0, bb = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                aa += A[k][r] * A[k][c];
                ab += A[k][r] * B[k][c];
                bb += B[k][r] * B[k][c];
            }
            o[r * 3 + c] = we * aa;
            o[9 + r * 3 + c] = we * ab;
            o[18 + r * 3 + c] = we * bb;
        }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double ga = 0.0, gb = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            ga += A[k][r] * ev[k];
            gb += B[k][r] * ev[k];
        }
        o[27 + r] = we * ga;
        o[30 + r] = we * gb;
    }
    o[33] = we * (ev[0] * ev[0] + ev[1] * ev[1] + ev[2] * ev[2]);
}

// Slot s: rows start at scalar r0 = slot_rc[2s], columns at c0 = slot_rc[2s+1].
// Diagonal slots (r0 == c0) list items 2e + side (side 0: node is e's source,
// use A'WA / A'We; side 1: target, B'WB / B'We).  Pair slots (r0 > c0) list
// items 2e + o: o = 0 when e's source is the ROW node (block = A'WB), o = 1
// when e's target is the row node (block = (A'WB)^T).
__global__ void gn_assemble_kernel(const double* __restrict__ contrib, const int32_t* __restrict__ slot_rc,
                                   const int32_t* __restrict__ slot_ptr, const int32_t* __restrict__ slot_items,
                                   int32_t n_slots, int32_t W, double* __restrict__ Hb, double* __restrict__ rhs) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int r0 = slot_rc[2 * s], c0 = slot_rc[2 * s + 1];
    double blk[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    double g[3] = {0, 0, 0};
    const bool diag = r0 == c0;
    for (int p = slot_ptr[s]; p < slot_ptr[s + 1]; ++p) {
        const int it = slot_items[p];
        const double* o = contrib + static_cast<int64_t>(it >> 1) * kGnContrib;
        if (diag) {
            const int off = (it & 1) ? 18 : 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) blk[k] += o[off + k];
            const int go = (it & 1) ? 30 : 27;
#pragma unroll
            for (int k = 0; k < 3; ++k) g[k] += o[go + k];
        } else if (it & 1) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) blk[r * 3 + c] += o[9 + c * 3 + r];
        } else {
#pragma unroll
            for (int k = 0; k < 9; ++k) blk[k] += o[9 + k];
        }
    }
    const int ld = W + 1;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int R = r0 + r, C = c0 + c;
            if (C <= R) Hb[static_cast<int64_t>(R) * ld + (R - C)] = blk[r * 3 + c];
        }
    if (diag) {
#pragma unroll
        for (int k = 0; k < 3; ++k) rhs[r0 + k] = -g[k];
    }
}

// Blocked band Cholesky, one workgroup.  Window: rows/cols [k0, k0 + M),
// M = W + S, stored cyclically (index mod M) in `win` (LDS or global scratch).
// Only lower-triangle band entries are ever read; every row is zeroed when it
// enters the window so structural zeros stay zero.
template <bool LDS_WIN>
__global__ __launch_bounds__(kGnBlock) void gn_factor_kernel(double* __restrict__ Hb, int32_t nv, int32_t W,
                                                             double* __restrict__ gwin,
                                                             int32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int M = W + kGnS;
    double* win = LDS_WIN ? lds : gwin;
    const int ld = W + 1;
    const int tid = threadIdx.x;

    // rows [ra, rb) enter the window: zero their slots, then copy their band
    auto load_rows = [&](int ra, int rb) {
        for (int idx = tid; idx < (rb - ra) * M; idx += kGnBlock) win[((ra + idx / M) % M) * M + idx % M] = 0.0;
        __syncthreads();
        for (int idx = tid; idx < (rb - ra) * ld; idx += kGnBlock) {
            const int r = ra + idx / ld, d = idx % ld;
            if (d <= r) win[(r % M) * M + (r - d) % M] = Hb[static_cast<int64_t>(r) * ld + d];
        }
    };
    load_rows(0, min(M, nv));
    __syncthreads();

    for (int k0 = 0; k0 < nv; k0 += kGnS) {
        const int sb = min(kGnS, nv - k0);
        // (a) dense Cholesky of the sb x sb diagonal block by wave 0, rows in registers
        if (tid < 64) {
            const int lane = tid;
            double row[kGnS];
#pragma unroll
            for (int c = 0; c < kGnS; ++c)
                row[c] = (lane < sb && c <= lane) ? win[((k0 + lane) % M) * M + (k0 + c) % M] : 0.0;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < kGnS; ++j) {
                if (j < sb) {
                    const double piv = __shfl(row[j], j, 64);
                    bad |= !(piv > 0.0);
                    const double d = sqrt(piv);
                    if (lane == j) row[j] = d;
                    if (lane > j) row[j] = row[j] / d;
                    const double lij = row[j];
#pragma unroll
                    for (int c = j + 1; c < kGnS; ++c) {
                        const double lcj = __shfl(row[j], c, 64);
                        if (lane > j && c <= lane) row[c] -= lij * lcj;
                    }
                }
            }
            if (lane < sb) {
#pragma unroll
                for (int c = 0; c < kGnS; ++c)
                    if (c <= lane) win[((k0 + lane) % M) * M + (k0 + c) % M] = row[c];
            }
            if (bad && lane == 0) *status = 1;
        }
        __syncthreads();
        // (b) panel rows r in [k0 + sb, min(nv, k0 + sb + W)): L[r][k0..] = A[r][k0..] L_D^-T
        const int rend = min(nv, k0 + sb + W);
        for (int r = k0 + sb + tid; r < rend; r += kGnBlock) {
            double* wr = win + (r % M) * M;
            double l[kGnS];
#pragma unroll
            for (int t = 0; t < kGnS; ++t) {
                if (t < sb) {
                    double v = wr[(k0 + t) % M];
                    const double* dt = win + ((k0 + t) % M) * M;
#pragma unroll
                    for (int q = 0; q < t; ++q) v -= l[q] * dt[(k0 + q) % M];
                    l[t] = v / dt[(k0 + t) % M];
                    wr[(k0 + t) % M] = l[t];
                }
            }
        }
        __syncthreads();
        // (c) write the finished block column (diag block + panel) back as L
        for (int idx = tid; idx < (rend - k0) * sb; idx += kGnBlock) {
            const int r = k0 + idx / sb, t = idx % sb;
            const int c = k0 + t;
            if (c <= r && r - c <= W) Hb[static_cast<int64_t>(r) * ld + (r - c)] = win[(r % M) * M + c % M];
        }
        // (d) trailing update of the band below the block: (r, c), k0+sb <= c <= r < rend
        const int n = rend - (k0 + sb);
        for (int idx = tid; idx < n * n; idx += kGnBlock) {
            const int r = k0 + sb + idx / n, c = k0 + sb + idx % n;
            if (c > r || r - c > W) continue;
            const double* wr = win + (r % M) * M;
            const double* wc = win + (c % M) * M;
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < kGnS; ++t)
                if (t < sb) acc = fma(wr[(k0 + t) % M], wc[(k0 + t) % M], acc);
            win[(r % M) * M + c % M] -= acc;
        }
        __syncthreads();
        // (e) rows entering the window take the slots of rows k0 .. k0 + sb
        if (k0 + M < nv) load_rows(k0 + M, min(nv, k0 + M + sb));
        __syncthreads();
    }
}

// Solve L L^T dx = rhs in place (rhs -> dx), one workgroup, blocks of S rows.
// x is staged in LDS when it fits (LDS_X); L rows are read contiguously in
// both sweeps (the backward sweep is column-oriented: each finished block
// subtracts its contribution from the rows above).
template <bool LDS_X>
__global__ __launch_bounds__(kGnBlock) void gn_solve_kernel(const double* __restrict__ Lb, int32_t nv, int32_t W,
                                                            double* __restrict__ gx) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double blk[kGnS][kGnS + 1];
    double* x = LDS_X ? lds : gx;
    const int ld = W + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int WAVES = kGnBlock / 64;
    if (LDS_X) {
        for (int i = tid; i < nv; i += kGnBlock) x[i] = gx[i];
        __syncthreads();
    }
    // forward: y[r] = (b[r] - sum_{c < r} L[r][c] y[c]) / L[r][r]
    for (int k0 = 0; k0 < nv; k0 += kGnS) {
        const int sb = min(kGnS, nv - k0);
        for (int t = wave; t < sb; t += WAVES) {   // off-block part: columns [r - W, k0)
            const int r = k0 + t;
            const double* Lr = Lb + static_cast<int64_t>(r) * ld;
            double acc = 0.0;
            for (int c = max(0, r - W) + lane; c < k0; c += 64) acc = fma(Lr[r - c], x[c], acc);
            acc = wave_sum(acc);
            if (lane == 0) x[r] -= acc;
        }
        for (int idx = tid; idx < sb * sb; idx += kGnBlock) {
            const int t = idx / sb, q = idx % sb;
            blk[t][q] = q <= t ? Lb[static_cast<int64_t>(k0 + t) * ld + (t - q)] : 0.0;
        }
        __syncthreads();
        if (tid < 64) {   // in-block lower-triangular solve, column oriented, one wave
            double v = lane < sb ? x[k0 + lane] : 0.0;
            for (int t = 0; t < sb; ++t) {
                const double xt = __shfl(v, t, 64) / blk[t][t];
                if (lane == t) v = xt;
                if (lane > t && lane < sb) v -= blk[lane][t] * xt;
            }
            if (lane < sb) x[k0 + lane] = v;
        }
        __syncthreads();
    }
    // backward: dx[r] = (y[r] - sum_{c > r} L[c][r] dx[c]) / L[r][r]
    for (int kend = nv; kend > 0; kend -= kGnS) {
        const int k0 = max(0, kend - kGnS);
        const int sb = kend - k0;
        for (int idx = tid; idx < sb * sb; idx += kGnBlock) {
            const int t = idx / sb, q = idx % sb;
            blk[t][q] = q <= t ? Lb[static_cast<int64_t>(k0 + t) * ld + (t - q)] : 0.0;
        }
        __syncthreads();
        if (tid < 64) {   // in-block upper-triangular (L^T) solve, one wave
            double v = lane < sb ? x[k0 + lane] : 0.0;
            for (int t = sb - 1; t >= 0; --t) {
                const double xt = __shfl(v, t, 64) / blk[t][t];
                if (lane == t) v = xt;
                if (lane < t) v -= blk[t][lane] * xt;
            }
            if (lane < sb) x[k0 + lane] = v;
        }
        __syncthreads();
        // subtract this block's contribution from rows c in [k0 - W, k0): x[c] -= sum_t L[k0+t][c] x[k0+t]
        for (int c = max(0, k0 - W - kGnS) + tid; c < k0; c += kGnBlock) {
            double acc = 0.0;
            for (int t = 0; t < sb; ++t) {
                const int r = k0 + t;
                if (r - c <= W) acc = fma(Lb[static_cast<int64_t>(r) * ld + (r - c)], x[r], acc);
            }
            x[c] -= acc;
        }
        __syncthreads();
    }
    if (LDS_X) {
        for (int i = tid; i < nv; i += kGnBlock) gx[i] = x[i];
    }
}

__global__ void gn_update_kernel(double* __restrict__ poses, int32_t N, const int32_t* __restrict__ node_col,
                                 const double* __restrict__ dx) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const int c = node_col[n];
    if (c < 0) return;
    poses[3 * n] += dx[c];
    poses[3 * n + 1] += dx[c + 1];
    poses[3 * n + 2] = wrap_pi(poses[3 * n + 2] + dx[c + 2]);
}

// chi2 = sum_e w_e |e_e|^2, deterministic single-block reduction.
__global__ __launch_bounds__(256) void gn_chi2_kernel(const double* __restrict__ contrib, int32_t E,
                                                      double* __restrict__ out) {
    __shared__ double red[4];
    double v[1] = {0.0};
    for (int e = threadIdx.x; e < E; e += 256) v[0] += contrib[static_cast<int64_t>(e) * kGnContrib + 33];
    block_sum<1, 4>(v, red);
    if (threadIdx.x == 0) *out = v[0];
}

}  // namespace slamhip

using namespace slamhip;

extern "C" {

int64_t slam_gn_work_size(int32_t N, int32_t E, int32_t W) {
    const int64_t nv = 3 * static_cast<int64_t>(N);
    const int64_t M = W + kGnS;
    return static_cast<int64_t>(E) * kGnContrib + nv * (W + 1) + nv + M * M + 8;
}

int slam_gn_max_lds_band(void) {
    // largest W whose (W + S)^2 window fits the 160 KiB LDS
    int W = 0;
    while ((W + 1 + kGnS) * (W + 1 + kGnS) * 8 <= 160 * 1024) ++W;
    return W;
}

int slam_gn_iteration_f64(double* poses, int32_t N, const int32_t* ea, const int32_t* eb, const double* tf,
                          const double* w, int32_t E, const int32_t* node_col, const int32_t* slot_rc,
                          const int32_t* slot_ptr, const int32_t* slot_items, int32_t n_slots, int32_t nv,
                          int32_t W, double* work, double* out_chi2, int32_t* status, void* stream) {
    if (N < 1 || E < 0 || nv < 0 || W < 2) return fail(SLAM_EINVAL, "gn: N=%d E=%d nv=%d W=%d", N, E, nv, W);
    if (!poses || !ea || !eb || !tf || !w || !node_col || !slot_rc || !slot_ptr || !work || !out_chi2 || !status)
        return fail(SLAM_EINVAL, "gn: null array argument");
    hipStream_t s = as_stream(stream);
    double* contrib = work;
    double* Hb = contrib + static_cast<int64_t>(E) * kGnContrib;
    double* rhs = Hb + static_cast<int64_t>(nv) * (W + 1);
    double* gwin = rhs + nv;
    if (E > 0)
        hipLaunchKernelGGL(gn_linearize_kernel, dim3((E + 255) / 256), dim3(256), 0, s, poses, ea, eb, tf, w, E,
                           contrib);
    hipLaunchKernelGGL(gn_chi2_kernel, dim3(1), dim3(256), 0, s, contrib, E, out_chi2);
    if (nv == 0) return check_launch("gn kernels");
    if (hipMemsetAsync(Hb, 0, sizeof(double) * static_cast<size_t>(nv) * (W + 1), s) != hipSuccess)
        return fail(SLAM_EHIP, "gn: memset failed");
    if (n_slots > 0)
        hipLaunchKernelGGL(gn_assemble_kernel, dim3((n_slots + 127) / 128), dim3(128), 0, s, contrib, slot_rc,
                           slot_ptr, slot_items, n_slots, W, Hb, rhs);
    const int M = W + kGnS;
    const size_t win_bytes = sizeof(double) * static_cast<size_t>(M) * M;
    if (W <= slam_gn_max_lds_band()) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gn_factor_kernel<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(win_bytes));
        hipLaunchKernelGGL(gn_factor_kernel<true>, dim3(1), dim3(kGnBlock), win_bytes, s, Hb, nv, W, gwin, status);
    } else {
        hipLaunchKernelGGL(gn_factor_kernel<false>, dim3(1), dim3(kGnBlock), 0, s, Hb, nv, W, gwin, status);
    }
    const size_t x_bytes = sizeof(double) * static_cast<size_t>(nv);
    if (x_bytes <= 150 * 1024) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gn_solve_kernel<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(x_bytes));
        hipLaunchKernelGGL(gn_solve_kernel<true>, dim3(1), dim3(kGnBlock), x_bytes, s, Hb, nv, W, rhs);
    } else {
        hipLaunchKernelGGL(gn_solve_kernel<false>, dim3(1), dim3(kGnBlock), 0, s, Hb, nv, W, rhs);
    }
    hipLaunchKernelGGL(gn_update_kernel, dim3((N + 255) / 256), dim3(256), 0, s, poses, N, node_col, rhs);
    return check_launch("gn kernels");
}

}  // extern "C"
