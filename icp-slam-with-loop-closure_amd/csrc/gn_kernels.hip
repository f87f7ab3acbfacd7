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
//                         lower band of H (nodes in the plan's order,
//                         half-bandwidth W scalars) and the right-hand side —
//                         or, for the default explicit-inverse cyclic
//                         reduction (gn_bcr_gj.hip), H's blocks in that
//                         solver's layout directly
//   gn_factor_kernel      ONE workgroup: blocked right-looking band Cholesky,
//                         the active (W + S) x (W + S) window resident in LDS,
//                         L overwrites H in place
//   gn_factor_kernel also runs the forward substitution; gn_backsolve_kernel
//                         (ONE workgroup) the backward one from the panel store
//   gn_update_kernel      x <- x + dx, headings wrapped to [-pi, pi)
// Band work is latency-bound (a chain of 3 (N-1) / S dependent block steps);
// the roofline is not the lever at C4 size.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "common.hpp"
#include "gn_bcr.hpp"

namespace slamhip {

constexpr int kGnContrib = 34;   // per-edge: 9 AtWA, 9 AtWB, 9 BtWB, 3 AtWe, 3 BtWe, 1 chi2
constexpr int kGnBlock = 512;    // threads of the factor / solve workgroup
constexpr int kGnS = 16;         // Cholesky block size (scalar columns per step)

__device__ __forceinline__ double wrap_pi(double a) {
    return a - 2.0 * M_PI * floor((a + M_PI) / (2.0 * M_PI));
}


// n doubles at z <- 0 by grid-stride double2 stores (a head / tail double by
// thread 0 when z is not 16-byte aligned or the count is odd)
__device__ __forceinline__ void zero_doubles(double* __restrict__ z, int64_t n, int64_t t, int64_t stride) {
    if (n <= 0) return;
    const int64_t head = (reinterpret_cast<uintptr_t>(z) & 15) ? 1 : 0;
    const int64_t np = (n - head) / 2;
    double2* __restrict__ z2 = reinterpret_cast<double2*>(z + head);
    const double2 zero = make_double2(0.0, 0.0);
    for (int64_t q = t; q < np; q += stride) z2[q] = zero;
    if (t == 0) {
        if (head) z[0] = 0.0;
        if ((n - head) & 1) z[n - 1] = 0.0;
    }
}

// Edge e's residual, Jacobian products (contrib) and chi2 term (returned).
__device__ __forceinline__ double linearize_edge(const double* __restrict__ poses, const int32_t* __restrict__ ea,
                                                 const int32_t* __restrict__ eb, const double* __restrict__ tf,
                                                 const double* __restrict__ w, double* __restrict__ contrib, int e) {
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
    return o[33];
}

constexpr int kGnLinBlock = 256;   // linearisation threads per workgroup (one chi2 partial each)

// One thread per edge.  The same launch zeroes the band (and the border rows)
// the assembly fills next, instead of separate memset launches (a memset of
// an odd number of doubles is two fill kernels), and sums its edges' chi2
// terms into chi2p[blockIdx.x] (fixed order; the assembly or gn_chi2_kernel
// adds the partials).
__global__ __launch_bounds__(kGnLinBlock) void gn_linearize_kernel(
    const double* __restrict__ poses, const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
    const double* __restrict__ tf, const double* __restrict__ w, int32_t E, double* __restrict__ contrib,
    double* __restrict__ chi2p, double* __restrict__ z0, int64_t nz0, double* __restrict__ z1, int64_t nz1,
    double* __restrict__ z2, int64_t nz2, double* __restrict__ z3, int64_t nz3) {
    __shared__ double red[kGnLinBlock / 64];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    {
        const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
        zero_doubles(z0, nz0, e, stride);
        zero_doubles(z1, nz1, e, stride);
        zero_doubles(z2, nz2, e, stride);
        zero_doubles(z3, nz3, e, stride);
    }
    // workgroups past the edges only zero (the grid is sized for the zeroing)
    if (static_cast<int64_t>(blockIdx.x) * blockDim.x >= E) return;   // uniform
    double v[1] = {e < E ? linearize_edge(poses, ea, eb, tf, w, contrib, e) : 0.0};
    block_sum<1, kGnLinBlock / 64>(v, red);
    if (threadIdx.x == 0) chi2p[blockIdx.x] = v[0];
}

// Slot s: rows start at scalar r0 = slot_rc[2s], columns at c0 = slot_rc[2s+1].
// Diagonal slots (r0 == c0) list items 2e + side (side 0: node is e's source,
// use A'WA / A'We; side 1: target, B'WB / B'We).  Pair slots (r0 > c0) list
// items 2e + o: o = 0 when e's source is the ROW node (block = A'WB), o = 1
// when e's target is the row node (block = (A'WB)^T).
// Bordered plans: rows R >= nv_band (the border's scalars, ordered last) go to
// the dense border rows BR[(R - nv_band) * nvt + C] (C <= R) instead of the band.
// chi2 of the partials of gn_linearize_kernel, summed in a fixed order by one
// workgroup of NT threads
template <int NT>
__device__ __forceinline__ void chi2_total(const double* __restrict__ chi2p, int32_t np, double* __restrict__ out,
                                           double* red) {
    double q[2] = {0.0, 0.0};
    int k = threadIdx.x;
    for (; k + NT < np; k += 2 * NT) {
        q[0] += chi2p[k];
        q[1] += chi2p[k + NT];
    }
    if (k < np) q[0] += chi2p[k];
    double v[1] = {q[0] + q[1]};
    block_sum<1, NT / 64>(v, red);
    if (threadIdx.x == 0) *out = v[0];
}

// Block layout of the explicit-inverse cyclic reduction (gn_bcr_gj.hip), filled
// by the assembly itself when D is set: D_i (Wb x Wb, both triangles, identity
// past nv_band), E_i = H[i+1, i], and the right-hand sides bz (row stride mc:
// column 0 the rhs, column 1 + k border column k) — what bcr_load_kernel makes
// from the band, without its launch.
struct BcrDirect {
    double* D;
    double* E;
    double* bz;
    int32_t Wb, mc, nb;
};

// The launch has one workgroup more than the slots need when out_chi2 is set:
// it adds the linearisation's chi2 partials beside the assembly (and writes
// the identity rows past nv_band of a direct block layout).
__global__ __launch_bounds__(128) void gn_assemble_kernel(
    const double* __restrict__ contrib, const int32_t* __restrict__ slot_rc, const int32_t* __restrict__ slot_ptr,
    const int32_t* __restrict__ slot_items, int32_t n_slots, int32_t W, double* __restrict__ Hb,
    double* __restrict__ rhs, int32_t nv_band, int32_t nvt, double* __restrict__ BR, const double* __restrict__ chi2p,
    int32_t n_chi2p, double* __restrict__ out_chi2, BcrDirect bd) {
    if (out_chi2 && blockIdx.x == gridDim.x - 1) {   // uniform
        __shared__ double red[2];
        chi2_total<128>(chi2p, n_chi2p, out_chi2, red);
        if (bd.D) {
            const int64_t B2 = static_cast<int64_t>(bd.Wb) * bd.Wb;
            for (int R = nv_band + threadIdx.x; R < bd.nb * bd.Wb; R += blockDim.x)
                bd.D[(R / bd.Wb) * B2 + static_cast<int64_t>(R % bd.Wb) * (bd.Wb + 1)] = 1.0;
        }
        return;
    }
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int r0 = slot_rc[2 * s], c0 = slot_rc[2 * s + 1];
    double blk[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    double g[3] = {0, 0, 0};
    const bool diag = r0 == c0;
    int p = slot_ptr[s];
    const int pe = slot_ptr[s + 1];
    // items four at a time: their indices, then all their contributions in
    // flight, then the sums in item order (the same order as one at a time);
    // the rest one at a time (a masked last batch measured slower)
    constexpr int kU = 4;
    for (; p + kU <= pe; p += kU) {
        int it[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) it[u] = slot_items[p + u];
        double q[kU][9], q3[kU][3];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const double* o = contrib + static_cast<int64_t>(it[u] >> 1) * kGnContrib;
            const int base = diag ? ((it[u] & 1) ? 18 : 0) : 9;
            const int go = (it[u] & 1) ? 30 : 27;
#pragma unroll
            for (int k = 0; k < 9; ++k) q[u][k] = o[base + k];
#pragma unroll
            for (int k = 0; k < 3; ++k) q3[u][k] = diag ? o[go + k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (diag) {
#pragma unroll
                for (int k = 0; k < 9; ++k) blk[k] += q[u][k];
#pragma unroll
                for (int k = 0; k < 3; ++k) g[k] += q3[u][k];
            } else if (it[u] & 1) {
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) blk[r * 3 + c] += q[u][c * 3 + r];
            } else {
#pragma unroll
                for (int k = 0; k < 9; ++k) blk[k] += q[u][k];
            }
        }
    }
    for (; p < pe; ++p) {
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
    const int64_t B2 = static_cast<int64_t>(bd.Wb) * bd.Wb;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int R = r0 + r, C = c0 + c;
            if (C <= R) {
                const double v = blk[r * 3 + c];
                if (R < nv_band) {
                    if (bd.D) {   // R - C <= W <= Wb: the same block or the next one
                        const int bi = R / bd.Wb, rr = R - bi * bd.Wb, bj = C / bd.Wb, cc = C - bj * bd.Wb;
                        if (bi == bj) {
                            bd.D[bi * B2 + rr * bd.Wb + cc] = v;
                            bd.D[bi * B2 + cc * bd.Wb + rr] = v;
                        } else {
                            bd.E[bj * B2 + rr * bd.Wb + cc] = v;
                        }
                    } else {
                        Hb[static_cast<int64_t>(R) * ld + (R - C)] = v;
                    }
                } else {
                    BR[static_cast<int64_t>(R - nv_band) * nvt + C] = v;
                    if (bd.D && C < nv_band) bd.bz[static_cast<int64_t>(C) * bd.mc + 1 + (R - nv_band)] = v;
                }
            }
        }
    if (diag) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            rhs[r0 + k] = -g[k];
            if (bd.D && r0 + k < nv_band) bd.bz[static_cast<int64_t>(r0 + k) * bd.mc] = -g[k];
        }
    }
}

// Blocked band Cholesky + forward substitution, one workgroup.
// Window: rows/cols [k0, k0 + MP), MP a power of two >= W + S, stored
// cyclically (index & (MP-1)) in `win` (LDS, or global scratch when W is
// large).  Only lower-triangle band entries are read; a row's slots are zeroed
// before it enters.  Every finished block column is written to the panel store
// PS as [S x S diagonal factor | W x S panel] (row-major, fixed stride per
// step) for the backward sweep, and y = L^-1 rhs overwrites rhs.
// Per step: (a) wave 0 factors the diagonal block in registers and solves its
// part of y; (b) one thread per panel row forms L[r][block] and updates y[r];
// (c) rank-S update of the trailing band from a compact LDS copy of the panel,
// retiring rows' slots zeroed; (d) entering rows (prefetched at the start of
// the step) are written.  Three barriers per step.
constexpr int kGnFBlock = 256;   // factor workgroup: one wave per SIMD -> up to 512 VGPRs, no spills
constexpr int kGnPf = 11;  // prefetch registers per worker thread: S*MP <= kGnPf*(kGnFBlock-64)
// Compact panel, TRANSPOSED: LpT[t][i] = L[k0+sb+i][k0+t]; row length lpw(W)
// (multiple of 4): a lane reading 4 consecutive i is one conflict-free 32-B chunk.
__host__ __device__ constexpr int lpw(int W) { return ((W + 3) / 4) * 4 + 4; }

template <bool LDS_WIN>
__global__ __launch_bounds__(kGnFBlock) void gn_factor_kernel(const double* __restrict__ Hb, double* __restrict__ rhs,
                                                             int32_t nv, int32_t W, int32_t MP,
                                                             double* __restrict__ gwin, double* __restrict__ gLp,
                                                             double* __restrict__ PS, int32_t* __restrict__ status,
                                                             unsigned long long* __restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double Ld[kGnS][kGnS + 1];
    // diagnostic phase timers (thread 0, s_memtime ticks), only when `stamps`
    unsigned long long tph[5] = {0, 0, 0, 0, 0}, tprev = 0;
    auto stamp = [&](int ph) {
        if (stamps && threadIdx.x == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph >= 0) tph[ph] += t - tprev;
            tprev = t;
        }
    };
    __shared__ double yb[kGnS];
    __shared__ double rdiag[kGnS];
    const int mask = MP - 1;
    const int MS = MP + 1;   // padded row stride: column walks hit distinct LDS banks
    double* win = LDS_WIN ? lds : gwin;
    const int LPW = lpw(W);
    double* Lp = LDS_WIN ? lds + static_cast<size_t>(MP) * MS : gLp;        // [S][LPW] transposed panel
    double* yw = Lp + static_cast<size_t>(kGnS) * LPW;                       // [MP]
    const int ld = W + 1;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int64_t ps_stride = static_cast<int64_t>(kGnS + W) * kGnS;
    auto WIN = [&](int r, int c) -> double& { return win[(r & mask) * MS + (c & mask)]; };

    // initial window: rows [0, min(MP, nv))
    const int r_init = min(MP, nv);
    for (int idx = tid; idx < r_init * MS; idx += kGnFBlock) win[idx] = 0.0;
    __syncthreads();
    for (int idx = tid; idx < r_init * ld; idx += kGnFBlock) {
        const int r = idx / ld, d = idx % ld;
        if (d <= r) WIN(r, r - d) = Hb[static_cast<int64_t>(r) * ld + d];
    }
    for (int r = tid; r < r_init; r += kGnFBlock) yw[r & mask] = rhs[r];
    __syncthreads();

    const int wave = tid >> 6;
    constexpr int kWorkers = kGnFBlock - 64;        // waves 1.. : trailing update + entering rows
    const bool can_pf = kGnS * MP <= kGnPf * kWorkers;

    // Wave 0: factor the sb x sb diagonal block at k0 (lane i holds row i,
    // column values broadcast with v_readlane) and solve its part of y.
    auto diag_factor = [&](int k0, int sb, int step) {
        double* ps = PS + step * ps_stride;
        double row[kGnS], rdv[kGnS];
#pragma unroll
        for (int c = 0; c < kGnS; ++c) {
            row[c] = (lane < sb && c <= lane) ? WIN(k0 + lane, k0 + c) : 0.0;
            rdv[c] = 0.0;
        }
        bool bad = false;
#pragma unroll
        for (int j = 0; j < kGnS; ++j) {
            if (j < sb) {
                const double piv = readlane_d(row[j], j);
                bad |= !(piv > 0.0);
                const double rd = rsqrt(piv);
                const double d = piv * rd;
                rdv[j] = rd;
                if (lane == j) row[j] = d;
                if (lane > j) row[j] = row[j] * rd;
#pragma unroll
                for (int c = j + 1; c < kGnS; ++c) {
                    const double lcj = readlane_d(row[j], c);
                    if (lane > j && c <= lane) row[c] = fma(-row[j], lcj, row[c]);
                }
            }
        }
        double y = lane < sb ? yw[(k0 + lane) & mask] : 0.0;
#pragma unroll
        for (int t = 0; t < kGnS; ++t) {
            if (t < sb) {
                const double yt = readlane_d(y, t) * rdv[t];
                if (lane == t) y = yt;
                if (lane > t) y = fma(-row[t], yt, y);
            }
        }
        if (lane < sb) {
#pragma unroll
            for (int c = 0; c < kGnS; ++c) {
                const double v = c <= lane ? row[c] : 0.0;
                Ld[lane][c] = v;
                ps[lane * kGnS + c] = v;
            }
            rdiag[lane] = rdv[0];
#pragma unroll
            for (int c = 1; c < kGnS; ++c)
                if (lane == c) rdiag[lane] = rdv[c];
            yb[lane] = y;
            rhs[k0 + lane] = y;
        }
        if (bad && lane == 0) *status = 1;
    };

    stamp(-1);
    if (wave == 0) diag_factor(0, min(kGnS, nv), 0);
    __syncthreads();
    stamp(0);
    for (int k0 = 0, step = 0; k0 < nv; k0 += kGnS, ++step) {
        const int sb = min(kGnS, nv - k0);
        const int rend = min(nv, k0 + sb + W);
        const int n = rend - (k0 + sb);
        double* ps = PS + step * ps_stride;
        const int k1 = k0 + sb;                       // next block
        const int sb2 = k1 < nv ? min(kGnS, nv - k1) : 0;
        // rows entering the window at the end of this step (prefetched by the workers)
        const int ra = k0 + MP, rb = min(nv, k0 + MP + sb);
        double pf[kGnPf];
        if (can_pf && wave > 0) {
            const int wt = tid - 64;
#pragma unroll
            for (int q = 0; q < kGnPf; ++q) {
                const int idx = wt + q * kWorkers;
                const int r = ra + idx / MP, d = idx % MP;   // slot of column r - d
                pf[q] = (r < rb && d <= W && d <= r) ? Hb[static_cast<int64_t>(r) * ld + d] : 0.0;
            }
        }
        // (b) panel rows: L[r][k0+t] = (A[r][k0+t] - sum_q L[r][k0+q] Ld[t][q]) / Ld[t][t]
        for (int i = tid; i < n; i += kGnFBlock) {
            asm volatile("" ::: "memory");   // keep the Ld reads inside the loop (no LICM into registers)
            const int r = k0 + sb + i;
            double l[kGnS];
            double ydot = 0.0;
#pragma unroll
            for (int t = 0; t < kGnS; ++t) {
                double v = 0.0;
                if (t < sb) {
                    v = WIN(r, k0 + t);
#pragma unroll
                    for (int q = 0; q < t; ++q) v = fma(-l[q], Ld[t][q], v);
                    v = v * rdiag[t];
                    ydot = fma(v, yb[t], ydot);
                }
                l[t] = v;
            }
#pragma unroll
            for (int t = 0; t < kGnS; ++t) {
                Lp[t * LPW + i] = l[t];
                ps[(kGnS + i) * kGnS + t] = l[t];
            }
            yw[r & mask] -= ydot;
        }
        __syncthreads();
        stamp(1);
        if (wave == 0) {
            // (c1) look-ahead: update the NEXT diagonal block first, then factor it
            if (sb2 > 0) {
                for (int e = lane; e < kGnS * kGnS; e += 64) {
                    const int i = e >> 4, j = e & (kGnS - 1);
                    if (i < sb2 && i < n && j <= i) {   // rows >= n have no coupling to this block (W < S)
                        double acc = 0.0;
#pragma unroll
                        for (int t = 0; t < kGnS; ++t) acc = fma(Lp[t * LPW + i], Lp[t * LPW + j], acc);
                        WIN(k1 + i, k1 + j) -= acc;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                diag_factor(k1, sb2, step + 1);
            }
        } else {
            // (c2) rank-sb update of the rest of the trailing band (panel rows
            // i >= sb2), 4 x 4 register tiles over the lower triangle
            const int wt = tid - 64;
            const int nt = (n + 3) / 4;
            const int t0 = sb2 / 4;                   // first tile row that has rows >= sb2
            const int ntiles = nt * (nt + 1) / 2 - t0 * (t0 + 1) / 2;
            for (int q = wt; q < ntiles; q += kWorkers) {
                // lower-triangle tile q (rows ti >= t0) -> (ti, tj)
                const int qq = q + t0 * (t0 + 1) / 2;
                int ti = static_cast<int>((sqrtf(8.0f * qq + 1.0f) - 1.0f) * 0.5f);
                while ((ti + 1) * (ti + 2) / 2 <= qq) ++ti;
                while (ti * (ti + 1) / 2 > qq) --ti;
                const int tj = qq - ti * (ti + 1) / 2;
                double acc[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
#pragma unroll 4
                for (int t = 0; t < kGnS; ++t) {
                    const double2* row = reinterpret_cast<const double2*>(Lp + t * LPW);
                    const double2 a0 = row[2 * ti], a1 = row[2 * ti + 1];
                    const double2 b0 = row[2 * tj], b1 = row[2 * tj + 1];
                    const double li[4] = {a0.x, a0.y, a1.x, a1.y};
                    const double lj[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 4; ++v) acc[u][v] = fma(li[u], lj[v], acc[u][v]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int i = 4 * ti + u, j = 4 * tj + v;
                        if (i < n && i >= sb2 && j <= i) WIN(k1 + i, k1 + j) -= acc[u][v];
                    }
            }
            // rows [ra, rb) enter the slots of the retired rows [k0, k0+sb):
            // every slot of an entering row is written (band value or 0), so
            // no separate zeroing pass and no extra barrier are needed
            if (ra < rb) {
                if (can_pf) {
#pragma unroll
                    for (int q = 0; q < kGnPf; ++q) {
                        const int idx = wt + q * kWorkers;
                        const int r = ra + idx / MP, d = idx % MP;
                        if (r < rb) WIN(r, r - d) = pf[q];
                    }
                } else {
                    for (int idx = wt; idx < (rb - ra) * MP; idx += kWorkers) {
                        const int r = ra + idx / MP, d = idx % MP;
                        WIN(r, r - d) = (d <= W && d <= r) ? Hb[static_cast<int64_t>(r) * ld + d] : 0.0;
                    }
                }
                for (int r = ra + wt; r < rb; r += kWorkers) yw[r & mask] = rhs[r];
            }
        }
        __syncthreads();
        stamp(2);
        stamp(3);
    }
    if (stamps && tid == 0) {
        for (int q = 0; q < 5; ++q) stamps[q] = tph[q];
    }
}

// Backward substitution L^T x = y (y in x on entry), one workgroup, block
// steps in reverse, reading the panel store PS contiguously; the next step's
// block is prefetched into registers while the current one is reduced.
template <bool LDS_X>
__global__ __launch_bounds__(kGnBlock) void gn_backsolve_kernel(const double* __restrict__ PS, int32_t nv, int32_t W,
                                                                double* __restrict__ gx) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double part[kGnBlock / 64][kGnS];
    double* x = LDS_X ? lds : gx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int WAVES = kGnBlock / 64;
    const int t = tid & (kGnS - 1);       // column of the block
    const int g = tid / kGnS;             // row group
    constexpr int G = kGnBlock / kGnS;    // 32 row groups
    const int64_t ps_stride = static_cast<int64_t>(kGnS + W) * kGnS;
    if (LDS_X) {
        for (int i = tid; i < nv; i += kGnBlock) x[i] = gx[i];
        __syncthreads();
    }
    const int nsteps = (nv + kGnS - 1) / kGnS;
    for (int step = nsteps - 1; step >= 0; --step) {
        const int k0 = step * kGnS;
        const int sb = min(kGnS, nv - k0);
        const int n = min(nv, k0 + sb + W) - (k0 + sb);
        const double* ps = PS + step * ps_stride;
        // wave 0: column `lane` of the diagonal factor, loaded before the reduction
        double lc[kGnS];
        if (tid < 64) {
#pragma unroll
            for (int q = 0; q < kGnS; ++q) lc[q] = (lane < sb && q < sb) ? ps[q * kGnS + lane] : 0.0;
        }
        // v[t] = sum_r L[k0+sb+r][k0+t] x[k0+sb+r]
        double acc = 0.0;
        for (int r = g; r < n; r += G) acc = fma(ps[(kGnS + r) * kGnS + t], x[k0 + sb + r], acc);
        acc += __shfl_xor(acc, 16, 64);
        acc += __shfl_xor(acc, 32, 64);
        if (lane < kGnS) part[wave][lane] = acc;
        __syncthreads();
        if (tid < 64) {
            double v = 0.0;
            if (lane < sb) {
                double sum = 0.0;
#pragma unroll
                for (int w = 0; w < WAVES; ++w) sum += part[w][lane];
                v = x[k0 + lane] - sum;
            }
            // L_D^T solve: x_t = (v_t - sum_{q>t} L[q][t] x_q) / L[t][t]
#pragma unroll
            for (int tt = kGnS - 1; tt >= 0; --tt) {
                if (tt < sb) {
                    const double xt = __shfl(v, tt, 64) / __shfl(lc[tt], tt, 64);
                    if (lane == tt) v = xt;
                    if (lane < tt) v -= lc[tt] * xt;
                }
            }
            if (lane < sb) x[k0 + lane] = v;
        }
        __syncthreads();
    }
    if (LDS_X) {
        for (int i = tid; i < nv; i += kGnBlock) gx[i] = x[i];
    }
}

// Band + border: H = [A B; B^T C] with A the band
// (nv_band scalars, solved by the BCR with mc = 16 ceil((1 + nbd) / 16)
// right-hand-side columns Z = A^-1 [r_a | B]) and a border of nbd <= 31
// scalars (x_b by bcr_border_solve, gn_bcr_gj.hip).
constexpr int kGnBorderMax = 31;

// The pose update of a bordered solve: dx = [Z_r - Z_B x_b ; x_b], one thread
// per scalar (its Z row loaded with every load in flight), applied in place.
template <int MC>
__global__ void gn_border_update_kernel(double* __restrict__ poses, int32_t N, const int32_t* __restrict__ node_col,
                                        const double* __restrict__ Z, const double* __restrict__ xb, int32_t nv_band,
                                        int32_t nbd) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = t / 3, q = t - 3 * n;
    if (n >= N) return;
    const double p0 = poses[3 * n + q];   // in flight beside the node_col -> Z chain
    const int c = node_col[n];
    if (c < 0) return;
    const int R = c + q;
    double d;
    if (R < nv_band) {
        const double2* z = reinterpret_cast<const double2*>(Z + static_cast<int64_t>(R) * MC);
        double2 zr[MC / 2];
#pragma unroll
        for (int k = 0; k < MC / 2; ++k) zr[k] = z[k];
        double acc = 0.0;
#pragma unroll
        for (int k = 1; k < MC; ++k) {
            const double zk = (k & 1) ? zr[k / 2].y : zr[k / 2].x;
            if (k <= nbd) acc = fma(zk, xb[k - 1], acc);
        }
        d = zr[0].x - acc;
    } else {
        d = xb[R - nv_band];
    }
    poses[3 * n + q] = q == 2 ? wrap_pi(p0 + d) : p0 + d;
}

// The pose update of a Schur-accumulating bordered solve: dx = [x_a ; x_b]
// (x_a the band's one-column solution, x_b the border's).
__global__ void gn_schur_update_kernel(double* __restrict__ poses, int32_t N, const int32_t* __restrict__ node_col,
                                       const double* __restrict__ xa, const double* __restrict__ xb, int32_t nv_band) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = t / 3, q = t - 3 * n;
    if (n >= N) return;
    const double p0 = poses[3 * n + q];   // in flight beside the node_col -> dx chain
    const int c = node_col[n];
    if (c < 0) return;
    const int R = c + q;
    const double d = R < nv_band ? xa[R] : xb[R - nv_band];
    poses[3 * n + q] = q == 2 ? wrap_pi(p0 + d) : p0 + d;
}

__global__ void gn_update_kernel(double* __restrict__ poses, int32_t N, const int32_t* __restrict__ node_col,
                                 const double* __restrict__ dx) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const double p0 = poses[3 * n], p1 = poses[3 * n + 1], p2 = poses[3 * n + 2];   // beside the node_col -> dx chain
    const int c = node_col[n];
    if (c < 0) return;
    poses[3 * n] = p0 + dx[c];
    poses[3 * n + 1] = p1 + dx[c + 1];
    poses[3 * n + 2] = wrap_pi(p2 + dx[c + 2]);
}

// chi2 when no assembly runs (no variables or no slots): the partials alone.
__global__ __launch_bounds__(256) void gn_chi2_kernel(const double* __restrict__ chi2p, int32_t np,
                                                      double* __restrict__ out) {
    __shared__ double red[4];
    chi2_total<256>(chi2p, np, out, red);
}

}  // namespace slamhip

namespace slamhip {
int bcr_block_rows(int32_t nv, int32_t W);
int64_t bcr_work_size(int32_t nv, int32_t W, int32_t mc);
int bcr_solve(const double* Hb, const double* rhs, int32_t nv, int32_t W, int32_t Wb, double* work,
              double** dx_out, int32_t* status, hipStream_t st, unsigned long long* stamps, int32_t mc,
              const double* BR, int32_t nbd, int32_t nvt, bool preloaded, const BcrSchur* sc);
bool bcr_gj_default();
int bcr_border_solve(const double* Z, const double* BR, const double* rhs, const int32_t* nbr_rows, int32_t n_nbr,
                     int32_t nv_band, int32_t nbd, int32_t nvt, int32_t mc, double* xb, int32_t* status,
                     hipStream_t st);
}  // namespace slamhip

using namespace slamhip;

static thread_local unsigned long long* g_gn_stamps = nullptr;
static thread_local int g_gn_solver = 0;   // 0 auto, 1 band Cholesky, 2 block cyclic reduction

extern "C" {

// Diagnostics: device buffer of 5 uint64 receiving the factor kernel's
// per-phase s_memtime totals (NULL disables).
int slam_gn_set_stamps(void* dev_buf) {
    g_gn_stamps = reinterpret_cast<unsigned long long*>(dev_buf);
    return ok();
}

int slam_gn_bcr_block_rows(int32_t nv, int32_t W) { return bcr_block_rows(nv, W); }

// Diagnostics: force the linear solver (0 auto, 1 band Cholesky, 2 block
// cyclic reduction when the band allows it).
int slam_gn_set_solver(int mode) {
    if (mode < 0 || mode > 2) return fail(SLAM_EINVAL, "gn solver %d not in {0, 1, 2}", mode);
    g_gn_solver = mode;
    return ok();
}

int slam_gn_get_solver(void) { return g_gn_solver; }

// The Schur path's back-substitution as ONE XCD-local launch (1, default) or
// one launch per level (0); slamhip.gn falls back to 0 for the rest of the
// process when a fused wait timed out (status bit 2).
int slam_gn_set_fused_back(int on) {
    bcr_gj_set_fused(on);
    return ok();
}
int slam_gn_get_fused_back(void) { return bcr_gj_get_fused(); }
// Diagnostics: the fused back-substitution's longest wait (s_memrealtime
// ticks, 0: the default 0.2 s) — a tiny wait forces the timeout path.
int slam_gn_set_fused_wait(uint32_t ticks) {
    bcr_gj_set_fused_wait(ticks ? ticks : 20000000u);
    return ok();
}

static int64_t window_dim(int32_t W) {
    int64_t MP = 32;
    while (MP < W + kGnS) MP <<= 1;
    return MP;
}

static int gn_border_mc(int32_t nbd) { return nbd > 0 ? 16 * ((nbd + 16) / 16) : 1; }

static int64_t gn_work_size(int32_t N, int32_t E, int32_t W, int32_t nbd) {
    const int64_t nv = 3 * static_cast<int64_t>(N);
    const int64_t MP = window_dim(W);
    const int64_t steps = (nv + kGnS - 1) / kGnS;
    return static_cast<int64_t>(E) * kGnContrib + nv * (W + 1) + nv + MP * (MP + 1) +
           static_cast<int64_t>(kGnS) * lpw(W) + MP + steps * (kGnS + W) * kGnS + 8 +
           bcr_work_size(static_cast<int32_t>(nv), W, gn_border_mc(nbd)) +
           (nbd > 0 ? nbd * nv + 32 + nv : 0) + E;   // border rows, x_b, dx; last E: per-edge chi2 terms
}

int64_t slam_gn_work_size(int32_t N, int32_t E, int32_t W) { return gn_work_size(N, E, W, 0); }

int64_t slam_gn_work_size_bordered(int32_t N, int32_t E, int32_t W, int32_t n_border) {
    return gn_work_size(N, E, W, n_border);
}

int slam_gn_max_lds_band(void) {
    // largest W whose power-of-two window + compact panel fit the LDS budget
    int W = 2;
    while (true) {
        const int64_t MP = window_dim(W + 1);
        if (sizeof(double) * (MP * (MP + 1) + static_cast<int64_t>(kGnS) * lpw(W + 1) + MP) + 4096 > 160 * 1024) break;
        ++W;
    }
    return W;
}

}  // extern "C"

// One GN iteration; nv_band < nv: the last nv - nv_band scalars are a border
// (bordered BCR + Schur complement, gn_border_*_kernel).
static int gn_iteration(double* poses, int32_t N, const int32_t* ea, const int32_t* eb, const double* tf,
                        const double* w, int32_t E, const int32_t* node_col, const int32_t* slot_rc,
                        const int32_t* slot_ptr, const int32_t* slot_items, int32_t n_slots, int32_t nv, int32_t W,
                        int32_t nv_band, const int32_t* nbr_rows, int32_t n_nbr, double* work, double* out_chi2,
                        int32_t* status, void* stream, const int32_t* pslot = nullptr, int32_t n_pslot = 0,
                        double* pwork = nullptr) {
    if (N < 1 || E < 0 || nv < 0 || W < 2) return fail(SLAM_EINVAL, "gn: N=%d E=%d nv=%d W=%d", N, E, nv, W);
    if (!poses || !ea || !eb || !tf || !w || !node_col || !slot_rc || !slot_ptr || !work || !out_chi2 || !status)
        return fail(SLAM_EINVAL, "gn: null array argument");
    const int32_t nbd = nv - nv_band;
    if (nbd < 0 || nbd > kGnBorderMax || (nbd > 0 && n_nbr > 0 && !nbr_rows) || n_nbr < 0)
        return fail(SLAM_EINVAL, "gn: border of %d scalars (at most %d)", nbd, kGnBorderMax);
    hipStream_t s = as_stream(stream);
    double* contrib = work;
    double* Hb = contrib + static_cast<int64_t>(E) * kGnContrib;
    double* rhs = Hb + static_cast<int64_t>(nv) * (W + 1);
    double* gwin = rhs + nv;
    double* chi2e = work + gn_work_size(N, E, W, nbd) - E;
    const int64_t MPw = window_dim(W);
    const int64_t steps = (static_cast<int64_t>(nv) + kGnS - 1) / kGnS;
    double* bwork = gwin + MPw * (MPw + 1) + static_cast<int64_t>(kGnS) * lpw(W) + MPw + steps * (kGnS + W) * kGnS + 8;
    const int mc = gn_border_mc(nbd);
    double* BR = bwork + bcr_work_size(3 * N, W, mc);
    double* xb = BR + static_cast<int64_t>(nbd) * 3 * N;
    const int Wb = g_gn_solver == 1 ? 0 : bcr_block_rows(nv_band, W);
    if (nbd > 0 && Wb == 0)
        return fail(SLAM_EINVAL, "gn: a bordered plan needs the cyclic-reduction solver (band %d, %d scalars)", W, nv_band);
    // explicit-inverse reduction with edges and slots: the assembly writes its
    // block layout directly (no band, no load launch)
    BcrDirect bd{nullptr, nullptr, nullptr, Wb, mc, Wb > 0 ? (nv_band + Wb - 1) / Wb : 0};
    if (Wb > 0 && nv_band > 0 && E > 0 && n_slots > 0 && bcr_gj_default()) {
        const BcrGjBufs g = bcr_gj_bufs(bwork, nv_band, Wb, mc);
        bd.D = g.D;
        bd.E = g.E0;
        bd.bz = g.bz;
    }
    // the Schur path (pslot given) needs the direct block layout: without it the
    // border solve below would run with no coupled rows and drop B entirely
    if (nbd > 0 && pslot && !bd.D)
        return fail(SLAM_EINVAL, "gn schur: no block layout (E=%d, %d slots, band %d scalars)", E, n_slots, nv_band);
    // the band (or the blocks) and the border rows are zeroed by the linearisation launch
    const int64_t B2 = static_cast<int64_t>(Wb) * Wb;
    double* z0 = bd.D ? bd.D : Hb;   // D and E0 are adjacent in the block workspace
    const int64_t nz0 = bd.D ? 2 * bd.nb * B2 : static_cast<int64_t>(nv_band) * (W + 1);
    const int64_t nz1 = bd.D ? static_cast<int64_t>(bd.nb) * Wb * mc : 0;
    const int64_t nBR = static_cast<int64_t>(nbd) * nv;
    // the Schur path's back-substitution granules (gn_bcr_gj.hip back_schur_xcd_kernel), zeroed every iteration
    double* z3 = nullptr;
    int64_t nz3 = 0;
    if (nbd > 0 && pslot && bd.D) {
        const BcrGjBufs g = bcr_gj_bufs(bwork, nv_band, Wb, mc);
        z3 = reinterpret_cast<double*>(g.xg);
        nz3 = 2 * static_cast<int64_t>(bd.nb) * Wb;
    }
    const bool fold = E > 0;
    const int n_chi2p = (E + kGnLinBlock - 1) / kGnLinBlock;   // chi2 partials (in chi2e: n_chi2p <= E)
    // enough workgroups for the zeroing too (about 16 double2 stores per thread)
    const int64_t nzero = (nz0 + nz1 + nBR + nz3) / 2;
    const int lin_grid = static_cast<int>(std::max<int64_t>(n_chi2p, std::min<int64_t>((nzero / 16 + kGnLinBlock - 1) / kGnLinBlock, 2048)));
    if (E > 0)
        hipLaunchKernelGGL(gn_linearize_kernel, dim3(lin_grid), dim3(kGnLinBlock), 0, s, poses, ea, eb, tf, w, E,
                           contrib, chi2e, z0, nz0, bd.bz, nz1, BR, nBR, z3, nz3);
    if (nv == 0 || n_slots <= 0) hipLaunchKernelGGL(gn_chi2_kernel, dim3(1), dim3(256), 0, s, chi2e, n_chi2p, out_chi2);
    if (nv == 0) return check_launch("gn kernels");
    if (!fold && hipMemsetAsync(z0, 0, sizeof(double) * static_cast<size_t>(nz0), s) != hipSuccess)
        return fail(SLAM_EHIP, "gn: memset failed");
    if (!fold && nbd > 0 && hipMemsetAsync(BR, 0, sizeof(double) * static_cast<size_t>(nBR), s) != hipSuccess)
        return fail(SLAM_EHIP, "gn: memset failed");
    if (n_slots > 0)
        hipLaunchKernelGGL(gn_assemble_kernel, dim3((n_slots + 127) / 128 + 1), dim3(128), 0, s, contrib, slot_rc,
                           slot_ptr, slot_items, n_slots, W, Hb, rhs, nv_band, nv, BR, chi2e, n_chi2p, out_chi2, bd);
    if (Wb > 0) {   // block cyclic reduction: log2(nv / Wb) parallel levels
        double* dx = nullptr;
        // the border's Schur complement accumulated during the elimination (needs
        // the assembly's direct block layout; slam_gn_iteration_schur_f64)
        const bool schur = nbd > 0 && pslot && bd.D;
        const BcrSchur sc{pslot, pwork, n_pslot, BR, rhs, nv_band, nbd, nv, xb, status};
        const int rc = bcr_solve(Hb, rhs, nv_band, W, Wb, bwork, &dx, status, s, g_gn_stamps, mc, BR, nbd, nv,
                                 bd.D != nullptr, schur ? &sc : nullptr);
        if (rc != 0) return rc;
        if (schur) {
            hipLaunchKernelGGL(gn_schur_update_kernel, dim3((3 * N + 255) / 256), dim3(256), 0, s, poses, N, node_col,
                               dx, xb, nv_band);
            return check_launch("gn kernels");
        }
        if (nbd > 0) {
            const int rb = bcr_border_solve(dx, BR, rhs, nbr_rows, n_nbr, nv_band, nbd, nv, mc, xb, status, s);
            if (rb != 0) return rb;
            if (mc == 16)
                hipLaunchKernelGGL(gn_border_update_kernel<16>, dim3((3 * N + 255) / 256), dim3(256), 0, s, poses, N,
                                   node_col, dx, xb, nv_band, nbd);
            else
                hipLaunchKernelGGL(gn_border_update_kernel<32>, dim3((3 * N + 255) / 256), dim3(256), 0, s, poses, N,
                                   node_col, dx, xb, nv_band, nbd);
            return check_launch("gn kernels");
        }
        hipLaunchKernelGGL(gn_update_kernel, dim3((N + 255) / 256), dim3(256), 0, s, poses, N, node_col, dx);
        return check_launch("gn kernels");
    }
    int MP = 32;
    while (MP < W + kGnS) MP <<= 1;
    const size_t lds_need = sizeof(double) * (static_cast<size_t>(MP) * (MP + 1) + static_cast<size_t>(kGnS) * lpw(W) + MP);
    double* PS = gwin + static_cast<int64_t>(MP) * (MP + 1) + static_cast<int64_t>(kGnS) * lpw(W) + MP;
    if (lds_need + 4096 <= 160 * 1024) {
        static bool attr_f = false;   // once: keeps the launch sequence graph-capturable
        if (!attr_f) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gn_factor_kernel<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096);
            attr_f = true;
        }
        hipLaunchKernelGGL(gn_factor_kernel<true>, dim3(1), dim3(kGnFBlock), lds_need, s, Hb, rhs, nv, W, MP, gwin,
                           gwin, PS, status, g_gn_stamps);
    } else {
        hipLaunchKernelGGL(gn_factor_kernel<false>, dim3(1), dim3(kGnFBlock), 0, s, Hb, rhs, nv, W, MP, gwin,
                           gwin + static_cast<int64_t>(MP) * (MP + 1), PS, status, g_gn_stamps);
    }
    const size_t x_bytes = sizeof(double) * static_cast<size_t>(nv);
    if (x_bytes <= 150 * 1024) {
        static bool attr_b = false;
        if (!attr_b) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gn_backsolve_kernel<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096);
            attr_b = true;
        }
        hipLaunchKernelGGL(gn_backsolve_kernel<true>, dim3(1), dim3(kGnBlock), x_bytes, s, PS, nv, W, rhs);
    } else {
        hipLaunchKernelGGL(gn_backsolve_kernel<false>, dim3(1), dim3(kGnBlock), 0, s, PS, nv, W, rhs);
    }
    hipLaunchKernelGGL(gn_update_kernel, dim3((N + 255) / 256), dim3(256), 0, s, poses, N, node_col, rhs);
    return check_launch("gn kernels");
}

extern "C" {

int slam_gn_schur_supported(void) { return g_gn_solver != 1 && bcr_gj_default() ? 1 : 0; }

int slam_gn_iteration_f64(double* poses, int32_t N, const int32_t* ea, const int32_t* eb, const double* tf,
                          const double* w, int32_t E, const int32_t* node_col, const int32_t* slot_rc,
                          const int32_t* slot_ptr, const int32_t* slot_items, int32_t n_slots, int32_t nv,
                          int32_t W, double* work, double* out_chi2, int32_t* status, void* stream) {
    return gn_iteration(poses, N, ea, eb, tf, w, E, node_col, slot_rc, slot_ptr, slot_items, n_slots, nv, W, nv,
                        nullptr, 0, work, out_chi2, status, stream);
}

int slam_gn_iteration_schur_f64(double* poses, int32_t N, const int32_t* ea, const int32_t* eb, const double* tf,
                                const double* w, int32_t E, const int32_t* node_col, const int32_t* slot_rc,
                                const int32_t* slot_ptr, const int32_t* slot_items, int32_t n_slots, int32_t nv,
                                int32_t W, int32_t nv_band, const int32_t* pslot, int32_t n_pslot, double* pwork,
                                double* work, double* out_chi2, int32_t* status, void* stream) {
    if (nv - nv_band < 1 || !pslot || n_pslot < 0 || (n_pslot > 0 && !pwork))
        return fail(SLAM_EINVAL, "gn schur: border %d, pslot %p, %d slots", nv - nv_band, pslot, n_pslot);
    if (!slam_gn_schur_supported())
        return fail(SLAM_EINVAL, "gn schur: needs the explicit-inverse cyclic reduction (solver mode %d)", g_gn_solver);
    return gn_iteration(poses, N, ea, eb, tf, w, E, node_col, slot_rc, slot_ptr, slot_items, n_slots, nv, W, nv_band,
                        nullptr, 0, work, out_chi2, status, stream, pslot, n_pslot, pwork);
}

int slam_gn_iteration_bordered_f64(double* poses, int32_t N, const int32_t* ea, const int32_t* eb, const double* tf,
                                   const double* w, int32_t E, const int32_t* node_col, const int32_t* slot_rc,
                                   const int32_t* slot_ptr, const int32_t* slot_items, int32_t n_slots, int32_t nv,
                                   int32_t W, int32_t nv_band, const int32_t* nbr_rows, int32_t n_nbr, double* work,
                                   double* out_chi2, int32_t* status, void* stream) {
    return gn_iteration(poses, N, ea, eb, tf, w, E, node_col, slot_rc, slot_ptr, slot_items, n_slots, nv, W, nv_band,
                        nbr_rows, n_nbr, work, out_chi2, status, stream);
}

}  // extern "C"
