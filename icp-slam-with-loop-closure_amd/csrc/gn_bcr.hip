// gn_bcr.hip — parallel solve of the Gauss-Newton normal equations by block
// cyclic reduction (BCR) for gfx950 (MI355X).
//
// H is the lower band of half-bandwidth W written by gn_assemble_kernel (nodes
// in reverse Cuthill-McKee order).  Cut into blocks of Wb >= W rows it is block
// TRIDIAGONAL: D_i = H[i,i], E_i = H[i+1,i] (every other block is zero).  Level
// by level (stride s = 1, 2, 4, ...) the "odd" blocks i = s, 3s, 5s, ... are
// eliminated in parallel — one workgroup each — and their Schur complements
// update the "even" neighbours:
//   C_i C_i^T = D_i,  X_i = C_i^-1 E_p,  Y_i = C_i^-1 E_i^T,  z_i = C_i^-1 b_i
//   D_p -= X_i^T X_i,  D_n -= Y_i^T Y_i,  E'_p = -Y_i^T X_i,
//   b_p -= X_i^T z_i,  b_n -= Y_i^T z_i                      (p = i - s, n = i + s)
// until only block 0 remains; back-substitution walks the levels in reverse:
//   x_i = C_i^-T (z_i - X_i x_p - Y_i x_n).
// log2(nv / Wb) dependent levels of dense Wb x Wb work instead of nv / 16
// dependent band steps (C4: 8 levels vs 938 steps).  The elimination order
// differs from the band Cholesky, so results agree to rounding (tests: 1e-8
// against oracle/gn_oracle.py).  Used when Wb <= kBcrMaxWb and nv / Wb >= 4.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <type_traits>

#include "common.hpp"
#include "gn_bcr.hpp"

namespace slamhip {

constexpr int kBcrThreads = 256;
#ifndef SLAM_ELIM_UNROLL
#define SLAM_ELIM_UNROLL 2   // pivots per unrolled step of the register elimination (A/B)
#endif
constexpr int kBcrMaxWb = 96;


__host__ __device__ inline int64_t bcr_blk(int Wb) { return static_cast<int64_t>(Wb) * Wb; }

// e -> (e / Wb, e % Wb) for e < Wb^2 <= 96^2 without an integer division: the
// float quotient's fraction stays below 1 - 1/Wb + 1e-3.
__device__ inline void bcr_rc(int e, int Wb, float inv, int& r, int& c) {
    r = static_cast<int>(static_cast<float>(e) * inv);
    c = e - r * Wb;
}

// Band (row r holds (r, r-d), d = 0..W) -> D_i (full symmetric), E_i, b_i;
// rows past nv are padded with the identity.
// Bordered solves (mc > 1): the right-hand side of block row i is Wb x mc,
// column 0 the rhs and column 1 + k the border column k of H (BR row k: H's
// row nv + k, row stride nvt), zero padded.
__global__ void bcr_load_kernel(const double* __restrict__ Hb, const double* __restrict__ rhs, int32_t nv,
                                int32_t W, int32_t Wb, int32_t nb, double* __restrict__ D, double* __restrict__ E,
                                double* __restrict__ bz, int32_t mc, const double* __restrict__ BR, int32_t nbd,
                                int32_t nvt) {
    const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= nb * bcr_blk(Wb)) return;
    const int i = static_cast<int>(idx / bcr_blk(Wb));
    const int r = static_cast<int>((idx / Wb) % Wb), c = static_cast<int>(idx % Wb);
    const int64_t ld = W + 1;
    const int R = i * Wb + r, Cc = i * Wb + c;
    const int lo = max(R, Cc), d = abs(R - Cc);
    double v = 0.0;
    if (lo < nv) {
        if (d <= W) v = Hb[lo * ld + d];
    } else if (R == Cc) {
        v = 1.0;
    }
    D[idx] = v;
    if (i + 1 < nb) {
        const int R2 = R + Wb, d2 = R2 - Cc;
        E[idx] = (R2 < nv && d2 <= W) ? Hb[R2 * ld + d2] : 0.0;
    }
    if (mc == 1) {
        if (c == 0) bz[static_cast<int64_t>(i) * Wb + r] = R < nv ? rhs[R] : 0.0;
    } else {
        for (int cc = c; cc < mc; cc += Wb) {   // mc may exceed Wb
            double v = 0.0;
            if (R < nv) v = cc == 0 ? rhs[R] : cc <= nbd ? BR[static_cast<int64_t>(cc - 1) * nvt + R] : 0.0;
            bz[static_cast<int64_t>(R) * mc + cc] = v;
        }
    }
}

// The augmented elimination of a register-tiled [D | R] (16 x 16 threads,
// thread (tr, tc) owns rows tr + 16u, columns tc + 16v / tc + 16w): after it,
// a holds the Cholesky factor C (lower; upper entries are garbage) and r holds
// C^-1 R.  One barrier per pivot (double-buffered LDS broadcast of column k of
// D and row k of R); rdg (optional, LDS) receives 1 / C[k][k].
template <int T, int NW>
__device__ __forceinline__ void bcr_reg_elim(double (&a)[T][T], double (&r)[T][NW], double (*colb)[16 * T],
                                             double (*rowb)[16 * NW], int tr, int tc, bool& bad, double* rdg) {
#pragma unroll
    for (int kv = 0; kv < T; ++kv) {
#pragma unroll SLAM_ELIM_UNROLL
        for (int kk = 0; kk < 16; ++kk) {
            const int k = 16 * kv + kk, kb = k & 1;
            if (tc == kk) {   // column k of D_i (all rows; rows < k are never read)
#pragma unroll
                for (int u = 0; u < T; ++u) colb[kb][tr + 16 * u] = a[u][kv];
            }
            if (tr == kk) {   // row k of R
#pragma unroll
                for (int w = 0; w < NW; ++w) rowb[kb][tc + 16 * w] = r[kv][w];
            }
            __syncthreads();
            // every broadcast value is read at once, unconditionally (one LDS
            // latency), then the pivot's reciprocal square root
            const double piv = colb[kb][k];
            double cr[T], cc[T], cz[NW];
#pragma unroll
            for (int u = 0; u < T; ++u) {
                cr[u] = colb[kb][tr + 16 * u];
                cc[u] = colb[kb][tc + 16 * u];
            }
#pragma unroll
            for (int w = 0; w < NW; ++w) cz[w] = rowb[kb][tc + 16 * w];
            bad |= !(piv > 0.0);
            const double rd = rsqrt(piv);   // reciprocal pivot: no fp64 division on the chain
            if (rdg && tr == kk && tc == kk) rdg[k] = rd;
            const double dg = piv * rd;     // L[k][k]
            double lr[T], lc[T], z[NW];
#pragma unroll
            for (int u = 0; u < T; ++u) {
                lr[u] = cr[u] * rd;                                  // L[R][k] for R > k
                lc[u] = tc + 16 * u > k ? cc[u] * rd : 0.0;          // L[C][k], columns still to update
            }
#pragma unroll
            for (int w = 0; w < NW; ++w) z[w] = cz[w] * rd;   // z_k
#pragma unroll
            for (int u = 0; u < T; ++u) {
                const int R = tr + 16 * u;
                const double l = R > k ? lr[u] : 0.0;
#pragma unroll
                for (int v = 0; v < T; ++v) a[u][v] = fma(-l, lc[v], a[u][v]);
#pragma unroll
                for (int w = 0; w < NW; ++w) r[u][w] = fma(-l, z[w], r[u][w]);
                if (tc == kk) a[u][kv] = R > k ? lr[u] : (R == k ? dg : a[u][kv]);
            }
            if (tr == kk) {
#pragma unroll
                for (int w = 0; w < NW; ++w) r[kv][w] = z[w];
            }
        }
    }
}

// Odd blocks: the Cholesky of D_i and the
// forward substitution of its right-hand sides run as ONE unblocked
// right-looking elimination of the augmented tile [D_i | R] held in registers —
// 16 x 16 threads, thread (tr, tc) owns rows tr + 16u and columns tc + 16v of D_i
// (T x T) and of R (T x (T+1)).  Pivot k: the owners of column k of D_i and
// row k of R publish them in LDS (double-buffered, ONE barrier per pivot);
// every thread scales them by 1/sqrt(piv) and applies the rank-1 update to its
// entries with c > k (D_i) and r > k (R).  Column k of the registers becomes
// L[:, k], row k of R becomes z_k: after Wb pivots the registers hold C_i and
// C_i^-1 R.  (It replaced an LDS-blocked Cholesky + TRSM with 3 barriers per
// 16-column panel: 57 -> 46 us per C4 level)
template <int T>
__global__ __launch_bounds__(kBcrThreads) void bcr_odd_reg_kernel(const double* __restrict__ D,
                                                                  const double* __restrict__ E,
                                                                  double* __restrict__ Cs, double* __restrict__ Xs,
                                                                  double* __restrict__ Ys, double* __restrict__ bz,
                                                                  int32_t Wb, int32_t nb, int32_t s,
                                                                  int32_t* __restrict__ status,
                                                                  unsigned long long* __restrict__ stamps) {
    // six workgroups per odd block (blockIdx.y = q): each eliminates D_i and carries
    // NW of the right-hand-side column tiles — q 0, 1: tiles [0, NW), [NW, T) of
    // E_p (-> X_i); q 2, 3: tiles [0, NW), [NW, T + 1) of [E_i^T | b_i] (-> Y_i, z_i);
    // q 4, 5: tiles [0, NW), [NW, T) of the identity (-> C_i^-1, for the back
    // kernel).  Fewer tiles per workgroup = less work per pivot on the dependent chain.
    constexpr int NW = (T + 2) / 2;
    __shared__ double colb[2][16 * T];
    __shared__ double rowb[2][16 * NW];
    const int q = blockIdx.y;
    const bool iv = q >= 4;                    // C_i^-1: the identity as right-hand side (-> Cs)
    const bool ys = q == 2 || q == 3;          // Y side (E_i^T | b_i)
    const int w0 = (q & 1) ? NW : 0;           // first global column tile
    const int wend = (q & 1) ? (ys ? T + 1 : T) : NW;
    const bool owner = q == 2;                 // writes the status
    const bool stamping = stamps && blockIdx.x == 0 && owner && threadIdx.x == 0;
    unsigned long long t0 = stamping ? __builtin_amdgcn_s_memtime() : 0;
    auto lap = [&](int qq) {
        if (stamping) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            stamps[qq] += t1 - t0;
            t0 = t1;
        }
    };
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const int64_t B2 = bcr_blk(Wb);
    const double* Di = D + i * B2;
    const double* Ep = E + p * B2;   // A[i, p]
    const double* Ei = E + i * B2;   // A[n, i]; A[i, n] = its transpose
    double a[T][T], r[T][NW];
#pragma unroll
    for (int u = 0; u < T; ++u) {
        const int R = tr + 16 * u;
#pragma unroll
        for (int v = 0; v < T; ++v) a[u][v] = Di[R * Wb + tc + 16 * v];
#pragma unroll
        for (int wl = 0; wl < NW; ++wl) {
            const int w = w0 + wl, C = tc + 16 * w;
            double x = 0.0;
            if (w < wend) {
                if (iv) x = R == C ? 1.0 : 0.0;
                else if (!ys) x = Ep[R * Wb + C];
                else if (w < T) x = n < nb ? Ei[C * Wb + R] : 0.0;
                else x = tc == 0 ? bz[static_cast<int64_t>(i) * Wb + R] : 0.0;
            }
            r[u][wl] = x;
        }
    }
    lap(0);
    bool bad = false;
    bcr_reg_elim<T, NW>(a, r, colb, rowb, tr, tc, bad, nullptr);
    lap(1);
    if (bad && owner && tid == 0) *status = 1;
    double* Out = (iv ? Cs : ys ? Ys : Xs) + i * B2;
#pragma unroll
    for (int u = 0; u < T; ++u) {
        const int R = tr + 16 * u;
#pragma unroll
        for (int wl = 0; wl < NW; ++wl) {
            const int w = w0 + wl;
            if (w < wend && w < T) Out[R * Wb + tc + 16 * w] = r[u][wl];
            if (w < wend && w == T && tc == 0) bz[static_cast<int64_t>(i) * Wb + R] = r[u][wl];
        }
    }
    lap(3);
}

// Even blocks of level s: Schur updates from the odd neighbours i1 = j - s
// (its n is j) and i2 = j + s (its p is j), and the new coupling to j + 2s.
// 16 x 16 threads, each a (Wb/16) x (Wb/16) register tile; the factors are
// staged in LDS (A^T B products read columns k of both).
template <int T>   // T = Wb / 16: register tile edge
__global__ __launch_bounds__(kBcrThreads) void bcr_even_kernel(double* __restrict__ D, double* __restrict__ E,
                                                               const double* __restrict__ Xs,
                                                               const double* __restrict__ Ys,
                                                               double* __restrict__ bz, int32_t Wb, int32_t nb,
                                                               int32_t s) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int ld = Wb + 1;
    double* L1 = lds;                                   // [Wb][Wb + 1]
    double* L2 = lds + static_cast<int64_t>(Wb) * ld;   // [Wb][Wb + 1]
    double* zv = L2 + static_cast<int64_t>(Wb) * ld;    // [2][Wb]
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    const int j = 2 * s * blockIdx.x;
    const int i1 = j - s, i2 = j + s;
    // blockIdx.y splits the work by row tiles u of the outputs: part 0 (D_j, b_j updates:
    // two products) over y = 0, 2, 3 -> u in [0, A), [A, B), [B, T); part 1 (new coupling
    // E'_j: one product) over y = 1, 4 -> u in [0, C), [C, T)
    constexpr int A = (T + 2) / 3, B = (2 * T + 2) / 3, C = (T + 1) / 2;
    const int y = blockIdx.y;
    const int part = (y == 1 || y == 4) ? 1 : 0;
    const bool upper = y != 0 && y != 1;   // not the workgroup that owns the rhs update
    const int ulo = y == 0 ? 0 : y == 1 ? 0 : y == 2 ? A : y == 3 ? B : C;
    const int uhi = y == 0 ? A : y == 1 ? C : y == 2 ? B : T;
    if (ulo >= uhi) return;   // empty row range (small T)
    const bool hE = part == 1 && i2 < nb && j + 2 * s < nb;
    const bool h1 = part == 0 && i1 >= 0, h2 = (part == 0 && i2 < nb) || hE;
    if (!h1 && !h2) return;
    const int64_t B2 = bcr_blk(Wb);
    double acc[T][T], accE[T][T];
#pragma unroll
    for (int u = 0; u < T; ++u)
#pragma unroll
        for (int v = 0; v < T; ++v) {
            acc[u][v] = 0.0;
            accE[u][v] = 0.0;
        }
    double bacc = 0.0;   // thread tid < Wb: row tid of the rhs update
    // both operands staged at once, one barrier, one fused k loop:
    //   part 0: L1 = Y1 (h1), L2 = X2 (h2): D_j -= Y1^T Y1 + X2^T X2, b_j -= Y1^T z1 + X2^T z2
    //   part 1: L1 = X2, L2 = Y2:           E'_j = -Y2^T X2
    {
        const double* S1 = part == 0 ? (h1 ? Ys + i1 * B2 : nullptr) : Xs + i2 * B2;
        const double* S2 = part == 0 ? (h2 ? Xs + i2 * B2 : nullptr) : Ys + i2 * B2;
        // compile-time trip count ((16T)^2 / 256 = T^2 per thread): every global
        // load is issued before the first LDS store (one memory latency, not T^2)
        constexpr int WB = 16 * T;
        double g1[T * T], g2[T * T];
#pragma unroll
        for (int q = 0; q < T * T; ++q) {
            const int e = tid + kBcrThreads * q;
            g1[q] = S1 ? S1[e] : 0.0;
            g2[q] = S2 ? S2[e] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < T * T; ++q) {
            const int e = tid + kBcrThreads * q, r = e / WB, c = e % WB;
            L1[r * ld + c] = g1[q];
            L2[r * ld + c] = g2[q];
        }
        if (part == 0)
            for (int r = tid; r < Wb; r += kBcrThreads) {
                zv[r] = h1 ? bz[static_cast<int64_t>(i1) * Wb + r] : 0.0;
                zv[Wb + r] = h2 ? bz[static_cast<int64_t>(i2) * Wb + r] : 0.0;
            }
        __syncthreads();
        if (part == 0) {
            auto rows = [&](auto lo_c, auto hi_c) {   // compile-time row-tile range [lo, hi)
                constexpr int lo = decltype(lo_c)::value, hi = decltype(hi_c)::value;
                for (int k = 0; k < Wb; ++k) {
                    double a1[T], b1[T], a2[T], b2[T];
#pragma unroll
                    for (int u = 0; u < T; ++u) {
                        if (u >= lo && u < hi) {
                            a1[u] = L1[k * ld + tr + 16 * u];
                            a2[u] = L2[k * ld + tr + 16 * u];
                        }
                        b1[u] = L1[k * ld + tc + 16 * u];
                        b2[u] = L2[k * ld + tc + 16 * u];
                    }
#pragma unroll
                    for (int u = lo; u < hi; ++u)
#pragma unroll
                        for (int v = 0; v < T; ++v) acc[u][v] = fma(a2[u], b2[v], fma(a1[u], b1[v], acc[u][v]));
                }
            };
            if (y == 0) rows(std::integral_constant<int, 0>{}, std::integral_constant<int, A>{});
            else if (y == 2) rows(std::integral_constant<int, A>{}, std::integral_constant<int, B>{});
            else rows(std::integral_constant<int, B>{}, std::integral_constant<int, T>{});
            if (!upper && tid < Wb) {
                double b2acc = 0.0;
                for (int k = 0; k < Wb; ++k) {
                    bacc = fma(L1[k * ld + tid], zv[k], bacc);
                    b2acc = fma(L2[k * ld + tid], zv[Wb + k], b2acc);
                }
                bacc += b2acc;
            }
        } else {
            auto rowsE = [&](auto lo_c, auto hi_c) {
                constexpr int lo = decltype(lo_c)::value, hi = decltype(hi_c)::value;
                for (int k = 0; k < Wb; ++k) {
                    double yv[T], b[T];
#pragma unroll
                    for (int u = 0; u < T; ++u) {
                        if (u >= lo && u < hi) yv[u] = L2[k * ld + tr + 16 * u];
                        b[u] = L1[k * ld + tc + 16 * u];
                    }
#pragma unroll
                    for (int u = lo; u < hi; ++u)
#pragma unroll
                        for (int v = 0; v < T; ++v) accE[u][v] = fma(yv[u], b[v], accE[u][v]);
                }
            };
            if (y == 1) rowsE(std::integral_constant<int, 0>{}, std::integral_constant<int, C>{});
            else rowsE(std::integral_constant<int, C>{}, std::integral_constant<int, T>{});
        }
    }
    double* Dj = D + j * B2;
    double* Ej = E + j * B2;
    constexpr int WB = 16 * T;   // compile-time row stride: provably distinct addresses
    if (hE) {
#pragma unroll
        for (int u = 0; u < T; ++u)
#pragma unroll
            for (int v = 0; v < T; ++v)
                if (u >= ulo && u < uhi) Ej[(tr + 16 * u) * WB + tc + 16 * v] = -accE[u][v];
    } else {
        // every D_j load issued before the first store (no load/store chain); this
        // workgroup's row tiles only
        double dv[T][T];
#pragma unroll
        for (int u = 0; u < T; ++u)
#pragma unroll
            for (int v = 0; v < T; ++v)
                if (u >= ulo && u < uhi) dv[u][v] = Dj[(tr + 16 * u) * WB + tc + 16 * v];
#pragma unroll
        for (int u = 0; u < T; ++u)
#pragma unroll
            for (int v = 0; v < T; ++v)
                if (u >= ulo && u < uhi) Dj[(tr + 16 * u) * WB + tc + 16 * v] = dv[u][v] - acc[u][v];
    }
    if (part == 0 && !upper && tid < Wb) bz[static_cast<int64_t>(j) * Wb + tid] -= bacc;
}

// Backward substitution C^T x = v by one wave, C lower in LDS (stride ldc);
// v in lanes (rows lane, lane + 64); returns x in the same layout.
__device__ inline void bcr_backsub_wave(const double* Cm, int ldc, const double* rdg, int Wb, double& v0, double& v1) {
    // lane j holds 1 / C[j][j] (and j + 64): x_k = v_k / C_kk is formed in lane
    // k and broadcast by one v_readlane — no LDS read on the dependent chain;
    // rows >= 64 first, so every branch below is wave-uniform
    const int lane = threadIdx.x & 63;
    const double r0 = lane < Wb ? rdg[lane] : 0.0, r1 = lane + 64 < Wb ? rdg[lane + 64] : 0.0;
    for (int k = Wb - 1; k >= 64; --k) {
        const double xk = readlane_d(v1 * r1, k - 64);
        const double c0 = Cm[k * ldc + lane], c1 = Cm[k * ldc + lane + 64];
        if (lane + 64 == k) v1 = xk;
        if (lane + 64 < k) v1 = fma(-c1, xk, v1);
        v0 = fma(-c0, xk, v0);
    }
    for (int k = min(Wb, 64) - 1; k >= 0; --k) {
        const double xk = readlane_d(v0 * r0, k);
        const double c0 = Cm[k * ldc + lane];
        if (lane == k) v0 = xk;
        if (lane < k) v0 = fma(-c0, xk, v0);
    }
}

// Last block, register-tiled: the elimination of [D_0 | b_0] (bcr_reg_elim with
// one right-hand-side column), C_0 to LDS, then C_0^-T z by one wave.
template <int T>
__global__ __launch_bounds__(kBcrThreads) void bcr_top_reg_kernel(double* __restrict__ D,
                                                                  const double* __restrict__ bz,
                                                                  double* __restrict__ x, int32_t Wb,
                                                                  int32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ double colb[2][16 * T];
    __shared__ double rowb[2][16];
    const int ldc = Wb + 1;
    double* Cm = lds;
    double* y = lds + static_cast<int64_t>(Wb) * ldc;
    double* rdg = y + Wb;
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    double a[T][T], r[T][1];
#pragma unroll
    for (int u = 0; u < T; ++u) {
#pragma unroll
        for (int v = 0; v < T; ++v) a[u][v] = D[(tr + 16 * u) * Wb + tc + 16 * v];
        r[u][0] = tc == 0 ? bz[tr + 16 * u] : 0.0;
    }
    bool bad = false;
    bcr_reg_elim<T, 1>(a, r, colb, rowb, tr, tc, bad, rdg);
    if (bad && tid == 0) *status = 1;
#pragma unroll
    for (int u = 0; u < T; ++u) {
        const int R = tr + 16 * u;
#pragma unroll
        for (int v = 0; v < T; ++v) {
            const int C = tc + 16 * v;
            if (C <= R) Cm[R * ldc + C] = a[u][v];
        }
        if (tc == 0) y[R] = r[u][0];
    }
    __syncthreads();
    if (tid < 64) {
        double v0 = tid < Wb ? y[tid] : 0.0, v1 = tid + 64 < Wb ? y[tid + 64] : 0.0;
        bcr_backsub_wave(Cm, ldc, rdg, Wb, v0, v1);
        if (tid < Wb) x[tid] = v0;
        if (tid + 64 < Wb) x[tid + 64] = v1;
    }
}

// A double moved between lanes of a 16-lane row by DPP (both halves).
template <int CTRL>
__device__ __forceinline__ double dpp_row(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b & 0xffffffff), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Back-substitution of the odd blocks of level s: v = z - X x_p - Y x_n
// (x_p / x_n staged in LDS, X / Y read in 128 B row segments, DPP row sums),
// then x_i = C_i^-T v as the mat-vec (C_i^-1)^T v over the whole workgroup:
// the odd kernel's two extra workgroups eliminated [D_i | I] into C_i^-1, so
// no 80-step triangular solve sits on this level's dependent chain (C4:
// 10.5 -> ~3 us per level, 1,560 -> 1,623 it/s).
template <int T>   // T = Wb / 16
__global__ __launch_bounds__(kBcrThreads) void bcr_back_kernel(const double* __restrict__ Cs,
                                                               const double* __restrict__ Xs,
                                                               const double* __restrict__ Ys,
                                                               const double* __restrict__ bz, double* __restrict__ x,
                                                               int32_t Wb, int32_t nb, int32_t s) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int ldc = Wb + 1;
    double* Cm = lds;
    double* vv = lds + static_cast<int64_t>(Wb) * ldc;     // [Wb]
    double* xpn = vv + Wb;                                  // [2][Wb]
    const int tid = threadIdx.x;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const int64_t B2 = bcr_blk(Wb);
    const double* Ci = Cs + i * B2;
    {
        constexpr int WB = 16 * T;   // compile-time trip count: all loads in flight at once
        double g[T * T];
#pragma unroll
        for (int q = 0; q < T * T; ++q) g[q] = Ci[tid + kBcrThreads * q];
#pragma unroll
        for (int q = 0; q < T * T; ++q) {
            const int e = tid + kBcrThreads * q;
            Cm[(e / WB) * ldc + e % WB] = g[q];
        }
    }
    for (int k = tid; k < Wb; k += kBcrThreads) {
        xpn[k] = x[static_cast<int64_t>(p) * Wb + k];
        xpn[Wb + k] = n < nb ? x[static_cast<int64_t>(n) * Wb + k] : 0.0;
    }
    __syncthreads();
    {
        // 16 x 16 threads: thread (tr, tc) sums columns tc + 16 w of rows tr + 16 u
        // (coalesced 128 B row segments straight from X_i, Y_i); the 16 lanes of a
        // DPP row (tc = lane & 15) then add up with row butterflies
        const int tr = tid >> 4, tc = tid & 15;
        const double* X = Xs + i * B2;
        const double* Y = Ys + i * B2;
        double v[T];
#pragma unroll
        for (int u = 0; u < T; ++u) {
            const int r = tr + 16 * u;
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int w = 0; w < T; ++w) {
                const int k = tc + 16 * w;
                a0 = fma(X[r * Wb + k], xpn[k], a0);
                a1 = fma(Y[r * Wb + k], xpn[Wb + k], a1);
            }
            v[u] = a0 + a1;
        }
#pragma unroll
        for (int u = 0; u < T; ++u) {
            v[u] += dpp_row<0xB1>(v[u]);    // quad_perm [1,0,3,2]
            v[u] += dpp_row<0x4E>(v[u]);    // quad_perm [2,3,0,1]
            v[u] += dpp_row<0x124>(v[u]);   // row_ror 4
            v[u] += dpp_row<0x128>(v[u]);   // row_ror 8
        }
        if (tc == 0) {
#pragma unroll
            for (int u = 0; u < T; ++u) vv[tr + 16 * u] = bz[static_cast<int64_t>(i) * Wb + tr + 16 * u] - v[u];
        }
    }
    __syncthreads();
    {
        // x_i = (C_i^-1)^T v: thread (c16 = tid >> 4, r16 = tid & 15) sums rows
        // r16 + 16 u of columns c16 + 16 w; the 16 lanes of a DPP row add up
        const int r16 = tid & 15, c16 = tid >> 4;
        double a[T];
#pragma unroll
        for (int w = 0; w < T; ++w) {
            const int c = c16 + 16 * w;
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < T; ++u) {
                const int r = r16 + 16 * u;
                acc = fma(Cm[r * ldc + c], vv[r], acc);
            }
            a[w] = acc;
        }
#pragma unroll
        for (int w = 0; w < T; ++w) {
            a[w] += dpp_row<0xB1>(a[w]);
            a[w] += dpp_row<0x4E>(a[w]);
            a[w] += dpp_row<0x124>(a[w]);
            a[w] += dpp_row<0x128>(a[w]);
        }
        if (r16 == 0) {
            double* xi = x + static_cast<int64_t>(i) * Wb;
#pragma unroll
            for (int w = 0; w < T; ++w) xi[c16 + 16 * w] = a[w];
        }
    }
}

// ---------------------------------------------------------------------------
// MFMA path (default): blocked right-looking elimination in 16-column panels,
// the dense trailing and right-hand-side updates and the even blocks' Schur
// products on v_mfma_f64_16x16x4_f64.
// ---------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));

// gfx950 v_mfma_f64_16x16x4_f64 (cdna_hip_programming.md, MFMA fragment
// layout): lane l holds A[row l & 15][k l >> 4] and B[k l >> 4][col l & 15];
// element g of the C/D tile is (row (l >> 4) + 4 g, col l & 15).
__device__ __forceinline__ f64x4 mfma16(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int T>
struct BcrMfmaLds {
    static constexpr int WB = 16 * T;
    static constexpr int LDA = WB + 1;              // A: [WB][LDA] (odd stride: spread banks)
    static constexpr int LDZ = 16 * (T + 1) + 1;    // panel rows of the right-hand side, x2 buffers
    static constexpr size_t doubles = static_cast<size_t>(WB) * LDA + 2 * 16 * LDZ + 2 * WB + 32;   // + rdg, y, 2 columns
    static constexpr size_t bytes = doubles * sizeof(double);
};

// D_i (WB x WB, global, row-major) -> A (LDS): every load in flight at once.
template <int T>
__device__ __forceinline__ void bcr_stage_block(const double* __restrict__ src, double* A) {
    constexpr int WB = 16 * T, LDA = WB + 1, PER = WB * WB / kBcrThreads;
    double g[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) g[q] = src[threadIdx.x + kBcrThreads * q];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + kBcrThreads * q;
        A[(e / WB) * LDA + e % WB] = g[q];
    }
}

// Cholesky D = C C^T of the block in LDS (A; lower triangle read) and the
// forward substitution Z = C^-1 R of NR (<= T + 1) 16-column right-hand-side
// tiles, blocked in T panels of 16 columns.  Per panel p:
//   F(p)   wave 0: rows 16p.. x 16 columns factored in registers, the pivot
//          and L[c][k] broadcast by v_readlane: no barrier inside the panel;
//   UR(p-1) waves 1-3, beside F(p): R_i -= L_i,p-1 Z_p-1 on their register-
//          resident R tiles (MFMA), the tiles of panel p's rows then to LDS;
//   --- barrier ---
//   S(p)   waves 1-2: Z_p = L_pp^-1 R_p, one thread per right-hand-side column;
//   UA(p)  waves 0, 3: A_ij -= L_ip L_jp^T on the lower tiles (MFMA);
//   --- barrier ---
// 2T barriers per block instead of one per pivot (16T).  rinit(row, col) is R,
// out(row, col, z) receives Z; rdg[k] = 1 / C[k][k].  Returns "a pivot was not
// positive" (wave-uniform in wave 0).
#ifdef SLAM_BCR_STAMPS
// tools/bcr_ubench.hip: per wave, cycles in [P1 work, barrier 1, P2 work, barrier 2]
__device__ unsigned long long g_bcr_stamps[4][4];
#define BCR_STAMP(q)                                                                     \
    do {                                                                                 \
        const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                    \
        if (blockIdx.x == 0 && blockIdx.y == 0 && lane == 0) g_bcr_stamps[wave][q] += t1_ - t0_; \
        t0_ = t1_;                                                                       \
    } while (0)
#else
#define BCR_STAMP(q) (void)0
#endif

template <int T, typename RInit, typename Out>
__device__ bool bcr_blocked_elim(double* A, double* Zb, double* rdg, int NR, RInit rinit, Out out) {
    constexpr int WB = 16 * T, LDA = WB + 1, LDZ = 16 * (T + 1) + 1;
    constexpr int MAXS = (T * (T + 1) + 2) / 3;   // R tiles per wave (waves 1-3)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lk = lane >> 4;
#ifdef SLAM_BCR_STAMPS
    unsigned long long t0_ = __builtin_amdgcn_s_memtime();
#endif
    f64x4 racc[MAXS];
    if (wave > 0) {
#pragma unroll
        for (int s = 0; s < MAXS; ++s) {
            const int t = 3 * s + wave - 1;
            if (t < T * NR) {
                const int ti = t / NR, w = t % NR;
#pragma unroll
                for (int g = 0; g < 4; ++g) racc[s][g] = rinit(16 * ti + lk + 4 * g, 16 * w + lr);
                if (ti == 0) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) Zb[(lk + 4 * g) * LDZ + 16 * w + lr] = racc[s][g];
                }
            }
        }
    }
    __syncthreads();   // A staged by the caller, R_0 in Zb[0]
#ifdef SLAM_BCR_STAMPS
    t0_ = __builtin_amdgcn_s_memtime();
#endif
    bool bad = false;
#pragma unroll
    for (int p = 0; p < T; ++p) {
        double* Zc = Zb + (p & 1) * 16 * LDZ;          // R_p (then Z_p)
        double* Zp = Zb + ((p + 1) & 1) * 16 * LDZ;    // Z_p-1
        if (wave == 0) {
            // ---- F(p) --------------------------------------------------------
            const int r0 = 16 * p + lane, r1 = 16 * p + 64 + lane;
            const bool v0 = r0 < WB, v1 = (WB - 16 * p > 64) && r1 < WB;
            double a[16], b[16];
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                a[c] = v0 ? A[r0 * LDA + 16 * p + c] : 0.0;
                b[c] = v1 ? A[r1 * LDA + 16 * p + c] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const double piv = readlane_d(a[k], k);
                bad |= !(piv > 0.0);
#ifdef SLAM_F_FAST
                // v_rsq_f64 and one Newton step (relative error ~2^-57)
                const double y0 = __builtin_amdgcn_rsq(piv);
                const double rd = fma(0.5 * y0, fma(-piv * y0, y0, 1.0), y0);
#else
                const double rd = rsqrt(piv);   // reciprocal pivot: no fp64 division on the chain
#endif
                const double lk0 = a[k] * rd, lk1 = b[k] * rd;
#ifdef SLAM_F_LDS
                // column k of the diagonal block through LDS (one write, broadcast reads)
                double* colk = Zb + 2 * 16 * LDZ + 2 * WB + (k & 1) * 16;
                if (lane < 16) colk[lane] = lk0;
#pragma unroll
                for (int c = k + 1; c < 16; ++c) {
                    const double lc = colk[c];
                    a[c] = fma(-lk0, lc, a[c]);
                    b[c] = fma(-lk1, lc, b[c]);
                }
#else
#pragma unroll
                for (int c = k + 1; c < 16; ++c) {
                    const double lc = readlane_d(lk0, c);   // L[16p + c][16p + k]
                    a[c] = fma(-lk0, lc, a[c]);
                    b[c] = fma(-lk1, lc, b[c]);
                }
#endif
                a[k] = lane > k ? lk0 : (lane == k ? piv * rd : a[k]);
                b[k] = lk1;
                if (lane == k) rdg[16 * p + k] = rd;
            }
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                if (v0) A[r0 * LDA + 16 * p + c] = a[c];
                if (v1) A[r1 * LDA + 16 * p + c] = b[c];
            }
        } else if (p > 0) {
            // ---- UR(p-1) -----------------------------------------------------
#pragma unroll
            for (int s = 0; s < MAXS; ++s) {
                const int t = 3 * s + wave - 1;
                if (t < T * NR) {
                    const int ti = t / NR, w = t % NR;
                    if (ti >= p) {
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) {
                            const double av = -A[(16 * ti + lr) * LDA + 16 * (p - 1) + 4 * kk + lk];
                            const double bv = Zp[(4 * kk + lk) * LDZ + 16 * w + lr];
                            racc[s] = mfma16(av, bv, racc[s]);
                        }
                        if (ti == p) {
#pragma unroll
                            for (int g = 0; g < 4; ++g) Zc[(lk + 4 * g) * LDZ + 16 * w + lr] = racc[s][g];
                        }
                    }
                }
            }
        }
        BCR_STAMP(0);
        __syncthreads();
        BCR_STAMP(1);
        if (wave == 1 || wave == 2) {
            // ---- S(p): one right-hand-side column per thread ----------------------
            const int c = tid - 64;
            if (c < 16 * NR) {
                double z[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) z[r] = Zc[r * LDZ + c];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const double zk = z[k] * rdg[16 * p + k];
                    z[k] = zk;
#pragma unroll
                    for (int r = k + 1; r < 16; ++r) z[r] = fma(-A[(16 * p + r) * LDA + 16 * p + k], zk, z[r]);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    Zc[r * LDZ + c] = z[r];
                    out(16 * p + r, c, z[r]);
                }
            }
        } else {
            // ---- UA(p): lower tiles (ti, tj), p < tj <= ti, alternating waves 0 / 3
            int idx = 0;
#pragma unroll
            for (int ti = p + 1; ti < T; ++ti) {
#pragma unroll
                for (int tj = p + 1; tj <= ti; ++tj, ++idx) {
                    if ((idx & 1) != (wave == 3 ? 1 : 0)) continue;
                    f64x4 cc;
#pragma unroll
                    for (int g = 0; g < 4; ++g) cc[g] = A[(16 * ti + lk + 4 * g) * LDA + 16 * tj + lr];
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) {
                        const double av = -A[(16 * ti + lr) * LDA + 16 * p + 4 * kk + lk];
                        const double bv = A[(16 * tj + lr) * LDA + 16 * p + 4 * kk + lk];
                        cc = mfma16(av, bv, cc);
                    }
#pragma unroll
                    for (int g = 0; g < 4; ++g) A[(16 * ti + lk + 4 * g) * LDA + 16 * tj + lr] = cc[g];
                }
            }
        }
        BCR_STAMP(2);
        __syncthreads();
        BCR_STAMP(3);
    }
    return bad;
}

// Odd blocks of level s, three workgroups per block (blockIdx.y = q), each
// eliminating D_i with one set of right-hand sides: q 0: E_p (-> X_i),
// q 1: [E_i^T | b_i] (-> Y_i, z_i), q 2: the identity (-> C_i^-1, for the
// back-substitution).
template <int T>
__global__ __launch_bounds__(kBcrThreads) void bcr_odd_mfma_kernel(const double* __restrict__ D,
                                                                   const double* __restrict__ E,
                                                                   double* __restrict__ Cs, double* __restrict__ Xs,
                                                                   double* __restrict__ Ys, double* __restrict__ bz,
                                                                   int32_t Wb, int32_t nb, int32_t s,
                                                                   int32_t* __restrict__ status) {
    using L = BcrMfmaLds<T>;
    constexpr int WB = L::WB;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;
    double* Zb = A + WB * L::LDA;
    double* rdg = Zb + 2 * 16 * L::LDZ;
    const int q = blockIdx.y;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const int64_t B2 = bcr_blk(WB);
    const double* Ep = E + p * B2;   // A[i, p]
    const double* Ei = E + i * B2;   // A[n, i]; A[i, n] = its transpose
    const bool hn = n < nb;
    bcr_stage_block<T>(D + i * B2, A);
    double* Out = (q == 0 ? Xs : q == 1 ? Ys : Cs) + i * B2;
    double* bzi = bz + static_cast<int64_t>(i) * WB;
    auto rinit = [&](int row, int col) -> double {
        if (q == 0) return Ep[row * WB + col];
        if (q == 2) return row == col ? 1.0 : 0.0;
        if (col < WB) return hn ? Ei[col * WB + row] : 0.0;
        return col == WB ? bzi[row] : 0.0;
    };
    auto out = [&](int row, int col, double v) {
        if (col < WB) Out[row * WB + col] = v;
        else if (col == WB) bzi[row] = v;
    };
    const bool bad = bcr_blocked_elim<T>(A, Zb, rdg, q == 1 ? T + 1 : T, rinit, out);
    if (bad && q == 1 && threadIdx.x == 0) *status = 1;
}

// Even blocks of level s: the two factors a workgroup needs are staged in LDS
// once (coalesced, every load in flight), then each wave computes one 16 x 16
// output tile with K = WB on MFMA, its operands read from LDS up front:
//   D workgroups (y < nD):  lower tiles of D_j -= Y1^T Y1 + X2^T X2, and the
//                           wave after the last tile b_j -= Y1^T z1 + X2^T z2
//                           (i1 = j - s, i2 = j + s);
//   E workgroups (y >= nD): E'_j = -Y2^T X2 (the new coupling to j + 2s).
// (Only D_j's lower triangle is kept current: every reader uses that half.)
template <int T>
__device__ __forceinline__ f64x4 bcr_tile_atb(const double* La, const double* Lb, int ti, int tj, f64x4 c) {
    // c += (La^T Lb)[16ti.., 16tj..] for La, Lb [WB][WB + 1] in LDS
    constexpr int WB = 16 * T, LD = WB + 1;
    const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    double av[WB / 4], bv[WB / 4];
#pragma unroll
    for (int k4 = 0; k4 < WB / 4; ++k4) {
        av[k4] = La[(4 * k4 + lk) * LD + 16 * ti + lr];
        bv[k4] = Lb[(4 * k4 + lk) * LD + 16 * tj + lr];
    }
#pragma unroll
    for (int k4 = 0; k4 < WB / 4; ++k4) c = mfma16(av[k4], bv[k4], c);
    return c;
}

template <int T>
__device__ __forceinline__ void bcr_stage_pair(const double* __restrict__ s1, const double* __restrict__ s2,
                                               double* L1, double* L2) {
    constexpr int WB = 16 * T, LD = WB + 1, PER = WB * WB / kBcrThreads;
    double g1[PER], g2[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + kBcrThreads * q;
        g1[q] = s1 ? s1[e] : 0.0;
        g2[q] = s2 ? s2[e] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + kBcrThreads * q;
        L1[(e / WB) * LD + e % WB] = g1[q];
        L2[(e / WB) * LD + e % WB] = g2[q];
    }
}

#ifndef SLAM_EVEN_D
#define SLAM_EVEN_D 4
#endif
#ifndef SLAM_EVEN_E
#define SLAM_EVEN_E 7
#endif
// workgroups per even block for the D / E roles (T = 5: one output tile per
// wave; fewer workgroups looping over tiles, 1/2 and 2/3 and 3/4, measured slower)
constexpr int kBcrEvenD = SLAM_EVEN_D, kBcrEvenE = SLAM_EVEN_E;

template <int T>
__global__ __launch_bounds__(kBcrThreads) void bcr_even_mfma_kernel(double* __restrict__ D, double* __restrict__ E,
                                                                    const double* __restrict__ Xs,
                                                                    const double* __restrict__ Ys,
                                                                    double* __restrict__ bz, int32_t Wb, int32_t nb,
                                                                    int32_t s) {
    constexpr int WB = 16 * T, LD = WB + 1, NTD = T * (T + 1) / 2, NTE = T * T;
    constexpr int nD = kBcrEvenD, nE = kBcrEvenE;   // workgroups per even block for each role
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* L1 = lds;
    double* L2 = lds + WB * LD;
    const int j = 2 * s * blockIdx.x;
    const int i1 = j - s, i2 = j + s;
    const bool h1 = i1 >= 0, h2 = i2 < nb, hE = h2 && j + 2 * s < nb;
    const int y = blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    const int64_t B2 = bcr_blk(WB);
    if (y < nD) {
        if (!h1 && !h2) return;
        bcr_stage_pair<T>(h1 ? Ys + i1 * B2 : nullptr, h2 ? Xs + i2 * B2 : nullptr, L1, L2);   // Y1, X2
        __syncthreads();
        for (int task = 4 * y + wave; task <= NTD; task += 4 * nD) {   // the staged factors serve several tiles
        if (task < NTD) {
            int ti = 0, t = task;
            while (t > ti) {   // lower tile t -> (ti, tj), tj <= ti
                t -= ti + 1;
                ++ti;
            }
            const int tj = t;
            double* Dj = D + j * B2;
            f64x4 c;   // -(D_j tile): accumulate the products, store the negation
#pragma unroll
            for (int g = 0; g < 4; ++g) c[g] = -Dj[(16 * ti + lk + 4 * g) * WB + 16 * tj + lr];
            if (h1) c = bcr_tile_atb<T>(L1, L1, ti, tj, c);
            if (h2) c = bcr_tile_atb<T>(L2, L2, ti, tj, c);
#pragma unroll
            for (int g = 0; g < 4; ++g) Dj[(16 * ti + lk + 4 * g) * WB + 16 * tj + lr] = -c[g];
        } else if (task == NTD) {
            const double* z1 = bz + static_cast<int64_t>(h1 ? i1 : 0) * WB;
            const double* z2 = bz + static_cast<int64_t>(h2 ? i2 : 0) * WB;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int r = lane + 64 * half;
                if (r >= WB) continue;
                double a1 = 0.0, a2 = 0.0;
#pragma unroll 8
                for (int k = 0; k < WB; ++k) {
                    a1 = fma(L1[k * LD + r], h1 ? z1[k] : 0.0, a1);
                    a2 = fma(L2[k * LD + r], h2 ? z2[k] : 0.0, a2);
                }
                bz[static_cast<int64_t>(j) * WB + r] -= a1 + a2;
            }
        }
        }
    } else {
        if (!hE) return;
        bcr_stage_pair<T>(Ys + i2 * B2, Xs + i2 * B2, L1, L2);   // Y2, X2
        __syncthreads();
        for (int t = 4 * (y - nD) + wave; t < NTE; t += 4 * nE) {
            const int ti = t / T, tj = t % T;
            f64x4 c = {0.0, 0.0, 0.0, 0.0};
            c = bcr_tile_atb<T>(L1, L2, ti, tj, c);
            double* Ej = E + j * B2;
#pragma unroll
            for (int g = 0; g < 4; ++g) Ej[(16 * ti + lk + 4 * g) * WB + 16 * tj + lr] = -c[g];
        }
    }
}

// Last block: the blocked elimination of [D_0 | b_0], then C_0^T x = z by one
// wave (C_0 in LDS from the elimination).
template <int T>
__global__ __launch_bounds__(kBcrThreads) void bcr_top_mfma_kernel(double* __restrict__ D,
                                                                   const double* __restrict__ bz,
                                                                   double* __restrict__ x, int32_t Wb,
                                                                   int32_t* __restrict__ status) {
    using L = BcrMfmaLds<T>;
    constexpr int WB = L::WB;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;
    double* Zb = A + WB * L::LDA;
    double* rdg = Zb + 2 * 16 * L::LDZ;
    double* y = rdg + WB;
    bcr_stage_block<T>(D, A);
    auto rinit = [&](int row, int col) -> double { return col == 0 ? bz[row] : 0.0; };
    auto out = [&](int row, int col, double v) {
        if (col == 0) y[row] = v;
    };
    const bool bad = bcr_blocked_elim<T>(A, Zb, rdg, 1, rinit, out);
    if (bad && threadIdx.x == 0) *status = 1;
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < 64) {
        double v0 = tid < WB ? y[tid] : 0.0, v1 = tid + 64 < WB ? y[tid + 64] : 0.0;
        bcr_backsub_wave(A, L::LDA, rdg, WB, v0, v1);
        if (tid < WB) x[tid] = v0;
        if (tid + 64 < WB) x[tid + 64] = v1;
    }
}

// ---- host ------------------------------------------------------------------

int bcr_block_rows(int32_t nv, int32_t W) {
    const int Wb = ((max(W, 1) + 15) / 16) * 16;
    if (Wb > kBcrMaxWb) return 0;
    if ((nv + Wb - 1) / Wb < 4) return 0;
    return Wb;
}

int64_t bcr_work_size(int32_t nv, int32_t W, int32_t mc) {
    const int Wb = ((max(W, 1) + 15) / 16) * 16;
    const int64_t nb = (nv + Wb - 1) / Wb;
    return max(5 * nb * bcr_blk(Wb) + 2 * nb * Wb, bcr_gj_work_size(nv, Wb, mc));
}

// Solve H dx = rhs (H in band storage, work of bcr_work_size doubles); *dx_out
// points at the solution inside `work` (first nv entries).
// Bordered (mc > 1, explicit-inverse path only): the mc right-hand sides of
// bcr_load_kernel; *dx_out is then the nv x mc solution block (row stride mc).
// default: the explicit-inverse levels (gn_bcr_gj.hip); the Cholesky paths
// below stay selectable for A/B (SLAMHIP_BCR_CHOL=1, SLAMHIP_BCR_LEGACY=1)
bool bcr_gj_default() {
    static const bool chol = [] {
        const char* e = getenv("SLAMHIP_BCR_CHOL");
        const char* l = getenv("SLAMHIP_BCR_LEGACY");
        return (e && e[0] == '1') || (l && l[0] == '1');
    }();
    return !chol;
}

// preloaded: the caller's assembly already wrote the explicit-inverse path's
// D, E0 and bz (gn_assemble_kernel with a block layout): no load launch.
int bcr_solve(const double* Hb, const double* rhs, int32_t nv, int32_t W, int32_t Wb, double* work,
              double** dx_out, int32_t* status, hipStream_t st, unsigned long long* stamps, int32_t mc,
              const double* BR, int32_t nbd, int32_t nvt, bool preloaded, const BcrSchur* sc) {
    const int nb = (nv + Wb - 1) / Wb;
    const int64_t B2 = bcr_blk(Wb);
    if (bcr_gj_default() || mc > 1 || preloaded) {
        const BcrGjBufs g = bcr_gj_bufs(work, nv, Wb, mc);
        const int64_t tot = nb * B2;
        if (!preloaded)
            hipLaunchKernelGGL(bcr_load_kernel, dim3(static_cast<unsigned>((tot + 255) / 256)), dim3(256), 0, st, Hb,
                               rhs, nv, W, Wb, nb, g.D, g.E0, g.bz, mc, BR, nbd, nvt);
        int rc = bcr_gj_levels(g, nv, Wb, mc, status, st, sc);   // levels + block 0 (+ the Schur border)
        if (rc != 0) return rc;
        rc = bcr_gj_back(g, nv, Wb, mc, st, sc);
        *dx_out = g.x;
        return rc;
    }
    double* D = work;
    double* E = D + nb * B2;
    double* Xs = E + nb * B2;
    double* Ys = Xs + nb * B2;
    double* Cs = Ys + nb * B2;
    double* bz = Cs + nb * B2;
    double* dx = bz + static_cast<int64_t>(nb) * Wb;
    *dx_out = dx;
    const int64_t tot = nb * B2;
    hipLaunchKernelGGL(bcr_load_kernel, dim3(static_cast<unsigned>((tot + 255) / 256)), dim3(256), 0, st, Hb, rhs, nv,
                       W, Wb, nb, D, E, bz, 1, nullptr, 0, nv);
    const size_t lds_even = sizeof(double) * (2 * static_cast<size_t>(Wb) * (Wb + 1) + 2 * static_cast<size_t>(Wb));
    const size_t lds_back = sizeof(double) * (static_cast<size_t>(Wb) * (Wb + 1) + 4 * static_cast<size_t>(Wb));
    using EvenFn = void (*)(double*, double*, const double*, const double*, double*, int32_t, int32_t, int32_t);
    static const EvenFn evens[6] = {bcr_even_kernel<1>, bcr_even_kernel<2>, bcr_even_kernel<3>,
                                    bcr_even_kernel<4>, bcr_even_kernel<5>, bcr_even_kernel<6>};
    const EvenFn even = evens[Wb / 16 - 1];
    using OddFn = void (*)(const double*, const double*, double*, double*, double*, double*, int32_t, int32_t, int32_t,
                           int32_t*, unsigned long long*);
    static const OddFn odds[6] = {bcr_odd_reg_kernel<1>, bcr_odd_reg_kernel<2>, bcr_odd_reg_kernel<3>,
                                  bcr_odd_reg_kernel<4>, bcr_odd_reg_kernel<5>, bcr_odd_reg_kernel<6>};
    const OddFn odd = odds[Wb / 16 - 1];
    using BackFn = void (*)(const double*, const double*, const double*, const double*, double*, int32_t, int32_t,
                            int32_t);
    static const BackFn backs[6] = {bcr_back_kernel<1>, bcr_back_kernel<2>, bcr_back_kernel<3>,
                                    bcr_back_kernel<4>, bcr_back_kernel<5>, bcr_back_kernel<6>};
    const BackFn back = backs[Wb / 16 - 1];
    using TopFn = void (*)(double*, const double*, double*, int32_t, int32_t*);
    static const TopFn tops[6] = {bcr_top_reg_kernel<1>, bcr_top_reg_kernel<2>, bcr_top_reg_kernel<3>,
                                  bcr_top_reg_kernel<4>, bcr_top_reg_kernel<5>, bcr_top_reg_kernel<6>};
    const TopFn top = tops[Wb / 16 - 1];
    // dynamic-LDS limits are raised once (not a stream operation: keeps the
    // launch sequence capturable into a hipGraph)
    static bool attrs = false;
    if (!attrs) {
        const int lim = 160 * 1024;
        for (const TopFn f : tops)   // these also hold 1.5 KB of static LDS
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      lim - 4096);
        for (const BackFn f : backs)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, lim);
        for (const EvenFn f : evens)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, lim);
        attrs = true;
    }
    // MFMA path (default) or the register elimination (SLAMHIP_BCR_LEGACY=1, A/B)
    static const bool legacy = [] {
        const char* e = getenv("SLAMHIP_BCR_LEGACY");
        return e && e[0] == '1';
    }();
    using OddMFn = void (*)(const double*, const double*, double*, double*, double*, double*, int32_t, int32_t,
                            int32_t, int32_t*);
    static const OddMFn odds_m[6] = {bcr_odd_mfma_kernel<1>, bcr_odd_mfma_kernel<2>, bcr_odd_mfma_kernel<3>,
                                     bcr_odd_mfma_kernel<4>, bcr_odd_mfma_kernel<5>, bcr_odd_mfma_kernel<6>};
    static const EvenFn evens_m[6] = {bcr_even_mfma_kernel<1>, bcr_even_mfma_kernel<2>, bcr_even_mfma_kernel<3>,
                                      bcr_even_mfma_kernel<4>, bcr_even_mfma_kernel<5>, bcr_even_mfma_kernel<6>};
    static const TopFn tops_m[6] = {bcr_top_mfma_kernel<1>, bcr_top_mfma_kernel<2>, bcr_top_mfma_kernel<3>,
                                    bcr_top_mfma_kernel<4>, bcr_top_mfma_kernel<5>, bcr_top_mfma_kernel<6>};
    static const size_t lds_m[6] = {BcrMfmaLds<1>::bytes, BcrMfmaLds<2>::bytes, BcrMfmaLds<3>::bytes,
                                    BcrMfmaLds<4>::bytes, BcrMfmaLds<5>::bytes, BcrMfmaLds<6>::bytes};
    // the odd blocks' blocked MFMA elimination (SLAMHIP_BCR_ODD_MFMA=1) is kept
    // for A/B: its single-wave panel factorization is slower than the register
    // elimination today
    static const bool odd_mfma = [] {
        const char* e = getenv("SLAMHIP_BCR_ODD_MFMA");
        return e && e[0] == '1';
    }();
    static bool attrs_m = false;
    if (!attrs_m) {
        for (int t = 0; t < 6; ++t) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(odds_m[t]),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_m[t]));
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tops_m[t]),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_m[t]));
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(evens_m[t]),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        }
        attrs_m = true;
    }
    const int T = Wb / 16;
    // one wave per output tile: D tiles + the rhs wave, then the E' tiles
    const int even_groups = kBcrEvenD + kBcrEvenE;
    int s = 1;
    for (; s < nb; s *= 2) {
        const int n_odd = (nb - s + 2 * s - 1) / (2 * s);        // i = s, 3s, ... < nb
        const int n_even = (nb + 2 * s - 1) / (2 * s);           // j = 0, 2s, ... < nb
        if (legacy) {
            hipLaunchKernelGGL(odd, dim3(n_odd, 6), dim3(kBcrThreads), 0, st, D, E, Cs, Xs, Ys, bz, Wb, nb, s, status,
                               stamps);
            hipLaunchKernelGGL(even, dim3(n_even, 5), dim3(kBcrThreads), lds_even, st, D, E, Xs, Ys, bz, Wb, nb, s);
        } else {
            if (odd_mfma)
                hipLaunchKernelGGL(odds_m[T - 1], dim3(n_odd, 3), dim3(kBcrThreads), lds_m[T - 1], st, D, E, Cs, Xs,
                                   Ys, bz, Wb, nb, s, status);
            else
                hipLaunchKernelGGL(odd, dim3(n_odd, 6), dim3(kBcrThreads), 0, st, D, E, Cs, Xs, Ys, bz, Wb, nb, s,
                                   status, stamps);
            hipLaunchKernelGGL(evens_m[T - 1], dim3(n_even, even_groups), dim3(kBcrThreads), lds_even, st, D, E, Xs,
                               Ys, bz, Wb, nb, s);
        }
    }
    if (legacy) hipLaunchKernelGGL(top, dim3(1), dim3(kBcrThreads), lds_back, st, D, bz, dx, Wb, status);
    else hipLaunchKernelGGL(tops_m[T - 1], dim3(1), dim3(kBcrThreads), lds_m[T - 1], st, D, bz, dx, Wb, status);
    for (s /= 2; s >= 1; s /= 2) {
        const int n_odd = (nb - s + 2 * s - 1) / (2 * s);
        hipLaunchKernelGGL(back, dim3(n_odd), dim3(kBcrThreads), lds_back, st, Cs, Xs, Ys, bz, dx, Wb, nb, s);
    }
    return check_launch("gn bcr kernels");
}

}  // namespace slamhip
