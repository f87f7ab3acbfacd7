// gn_bcr_gj.hip — block cyclic reduction of the Gauss-Newton normal equations
// on explicit block inverses (gfx950 / MI355X; the default BCR path).
//
// The band of H cut into blocks of Wb rows is block tridiagonal (gn_bcr.hip:
// D_i = H[i,i], E_i = H[i+1,i]).  Level s eliminates the odd blocks
// i = s, 3s, ... in parallel.  Where gn_bcr.hip factors D_i = C C^T and carries
// C^-1 through triangular solves (80 barrier-separated pivots per level on the
// dependent chain), this path inverts D_i outright — blocked Gauss-Jordan with
// 16-column steps: one wave inverts the 16 x 16 diagonal tile, the row, trailing
// and column tiles are MFMA products (v_mfma_f64_16x16x4_f64), 3 barriers per
// step, 3 T barriers per block — and every product that follows is a GEMM:
//   G = D_i^-1,  X_i = G A[i,p],  Y_i = G A[i,n],  z_i = G b_i
//   Sp_i = A[p,i] X_i   (-> D_p),   Sn_i = A[n,i] Y_i   (-> D_n)
//   E'_p = -A[n,i] X_i  (the new coupling p <-> n, next level's E)
// with A[i,p] = E_p, A[n,i] = E_i (block rows of H).  The even blocks' updates
// D_j -= Sn_{j-s} + Sp_{j+s}, b_j -= A[j,i] z_i are applied lazily, in level
// order (deterministic), by the kernel that next reads D_j: the odd kernel of
// the level at which j is odd, or the block-0 combine; the back-substitution
// is two mat-vecs,
// x_i = z_i - X_i x_p - Y_i x_n.  Block 0 is solved last (top_kernel).  Each odd block runs on 2 ng + 1 workgroups (blockIdx.y): X side and
// Y side column-tile groups and one for z; every one inverts D_i itself (the
// inversion is the chain, the redundancy costs CU time only).  Gauss-Jordan
// without pivoting is stable for the SPD blocks here; results agree with the
// Cholesky paths to rounding (tests: 1e-8 against oracle/gn_oracle.py).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"
#include "gn_bcr.hpp"

namespace slamhip {

namespace bcrgj {

constexpr int kThreads = 256;
constexpr int kCombineSplit = 4;   // workgroups per block of a combine
#ifdef SLAM_GJ_STAMPS
// tools/gj_ubench.hip: s_memtime per phase, thread 0 of workgroup (0, 0)
__device__ unsigned long long g_gj_stamps[8];
#define GJ_T0() unsigned long long t0_ = __builtin_amdgcn_s_memtime()
#define GJ_STAMP(q)                                                                            \
    do {                                                                                       \
        const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                          \
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) g_gj_stamps[q] += t1_ - t0_; \
        t0_ = t1_;                                                                             \
    } while (0)
#else
#define GJ_T0() (void)0
#define GJ_STAMP(q) (void)0
#endif
typedef double f64x4 __attribute__((ext_vector_type(4)));

// v_mfma_f64_16x16x4_f64: lane l holds A[l & 15][l >> 4] and B[l >> 4][l & 15];
// C/D element g of lane l is (row (l >> 4) + 4 g, col l & 15)
// (cdna_hip_programming.md, fragment layout: f64).
__device__ __forceinline__ f64x4 mma(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int T>
struct Lds {
    static constexpr int WB = 16 * T;
    static constexpr int LDA = WB + 1;   // block / its inverse: [WB][LDA] (odd stride spreads banks)
    static constexpr int LDC = 17;       // one column tile: [WB][LDC]
    static constexpr size_t doubles = static_cast<size_t>(WB) * LDA + static_cast<size_t>(WB) * LDC + 2 * WB;
    static constexpr size_t bytes = doubles * sizeof(double);
    // bordered solves (several right-hand-side columns): + one RHS column tile
    static constexpr size_t bytes_multi = bytes + static_cast<size_t>(WB) * LDC * sizeof(double);
    // Schur-accumulating bordered solves: + the whole RHS block [WB][mc + 1], mc <= 32
    static constexpr size_t bytes_schur = bytes_multi + static_cast<size_t>(WB) * 33 * sizeof(double);
};

// D_i (WB x WB, global, row-major) -> A (LDS): every load in flight at once.
template <int T>
__device__ __forceinline__ void stage(const double* __restrict__ src, double* A) {
    constexpr int WB = 16 * T, LDA = WB + 1, PER = T * T;   // (16T)^2 / 256
    double g[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) g[q] = src[threadIdx.x + kThreads * q];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + kThreads * q;
        A[(e / WB) * LDA + e % WB] = g[q];
    }
}

// Lane `src`'s double in every lane (src may differ per lane): ds_bpermute.
__device__ __forceinline__ double bperm_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src * 4, static_cast<int>(b & 0xffffffff));
    const int hi = __builtin_amdgcn_ds_bpermute(src * 4, static_cast<int>(b >> 32));
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
// Element kq (0..3, a constant after unrolling) of each quad, in every lane of the quad (DPP).
__device__ __forceinline__ double quad_bcast(double v, int kq) {
    const long long b = __double_as_longlong(v);
    int lo = static_cast<int>(b & 0xffffffff), hi = static_cast<int>(b >> 32);
    switch (kq) {
        case 0: lo = __builtin_amdgcn_update_dpp(0, lo, 0x00, 0xF, 0xF, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x00, 0xF, 0xF, false); break;
        case 1: lo = __builtin_amdgcn_update_dpp(0, lo, 0x55, 0xF, 0xF, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x55, 0xF, 0xF, false); break;
        case 2: lo = __builtin_amdgcn_update_dpp(0, lo, 0xAA, 0xF, 0xF, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0xAA, 0xF, 0xF, false); break;
        default: lo = __builtin_amdgcn_update_dpp(0, lo, 0xFF, 0xF, 0xF, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0xFF, 0xF, 0xF, false); break;
    }
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// The 16 x 16 tile at P (row stride LDA) -> its inverse, by ONE wave: a
// register Gauss-Jordan (lane l: row r = l >> 2, columns c0..c0+3, c0 = 4 (l & 3));
// per pivot the row-k values come by ds_bpermute from lane 4k + (l & 3), a[r][k]
// by a DPP quad broadcast, the pivot by v_readlane: no LDS round trip and no
// barrier on the chain.  Returns "a pivot was not positive".
template <int LDA>
__device__ __forceinline__ bool tile_inv16(double* P, int lane) {
    const int r = lane >> 2, cq = lane & 3, c0 = 4 * cq;
    bool bad = false;
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = P[r * LDA + c0 + q];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int kq = k >> 2, kr = k & 3;
        const double ark = quad_bcast(v[kr], kq);
        const double akk = readlane_d(v[kr], 4 * k + kq);
        double akc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) akc[q] = bperm_d(v[q], 4 * k + cq);
        bad |= !(akk > 0.0);
        // reciprocal pivot: v_rcp_f64 and two Newton steps (a few ulp; no fp64
        // division sequence on the chain)
        double pv = __builtin_amdgcn_rcp(akk);
        pv = fma(pv, fma(-akk, pv, 1.0), pv);
        pv = fma(pv, fma(-akk, pv, 1.0), pv);
        // one rank-1 update for every entry: with column k's pivot entry taken
        // as a_kk - 1 and row k's as a_kk + 1, a - u v^T / a_kk gives row k / a_kk,
        // -column k / a_kk and 1 / a_kk at the pivot (2 selects per pivot instead
        // of 8; relative rounding ~a_kk eps on row k)
        const double u = r == k ? akk - 1.0 : ark;
        akc[kr] = cq == kq ? akk + 1.0 : akc[kr];
        const double m = u * pv;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fma(-m, akc[q], v[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) P[r * LDA + c0 + q] = v[q];
    return bad;
}

// In-place inverse of the SPD block in A by blocked Gauss-Jordan.  Step kb:
//   R  (MFMA)    row tiles A[kb,j] <- Pinv A[kb,j]; column tiles A[i,kb] -> C
//   U  (MFMA)    A[i,j] -= C_i A[kb,j] (i, j != kb);  A[i,kb] = -C_i Pinv
// with look-ahead: in U, wave 0 updates the next diagonal tile first and
// inverts it (tile_inv16) while waves 1-3 update every other tile, so the
// pivot chain of step kb + 1 runs beside step kb's trailing update.  Two
// barriers per step.  C: [WB][17] LDS scratch.  Returns "a pivot was not
// positive" (wave 0).
template <int T>
__device__ __forceinline__ bool gj_invert(double* A, double* C) {
    constexpr int WB = 16 * T, LDA = WB + 1, LDC = 17;
    constexpr int NTU = T * (T - 1);                         // U tiles: rows != kb
    constexpr int NPW = NTU > 0 ? (NTU + 2) / 3 : 1;         // per wave of waves 1-3
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lk = lane >> 4;
    bool bad = false;
    GJ_T0();
    if (wave == 0) bad |= tile_inv16<LDA>(A, lane);
    __syncthreads();
    GJ_STAMP(0);
    for (int kb = 0; kb < T; ++kb) {
        double* P = A + 16 * kb * LDA + 16 * kb;
        // R: row tiles (one per wave), the old column tiles to C
        for (int t = wave; t < T; t += 4) {
            if (t == kb) continue;
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
            double a[4], b[4];
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                a[k4] = P[lr * LDA + 4 * k4 + lk];
                b[k4] = A[(16 * kb + 4 * k4 + lk) * LDA + 16 * t + lr];
            }
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) acc = mma(a[k4], b[k4], acc);
#pragma unroll
            for (int g = 0; g < 4; ++g) A[(16 * kb + lk + 4 * g) * LDA + 16 * t + lr] = acc[g];
        }
#pragma unroll
        for (int q = 0; q < WB * 16 / kThreads; ++q) {
            const int e = tid + kThreads * q, rr = e >> 4, cc = e & 15;
            C[rr * LDC + cc] = A[rr * LDA + 16 * kb + cc];
        }
        __syncthreads();
        GJ_STAMP(1);
        const int nx = kb + 1;   // the next diagonal tile (if nx < T)
        // one U tile (ti, tj): A[ti,tj] -= C_ti A[kb,tj]  (tj == kb: A[ti,kb] = -C_ti Pinv)
        auto load_tile = [&](int ti, int tj, f64x4& acc, double (&a)[4], double (&b)[4]) {
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = tj == kb ? 0.0 : A[(16 * ti + lk + 4 * g) * LDA + 16 * tj + lr];
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                a[k4] = -C[(16 * ti + lr) * LDC + 4 * k4 + lk];
                b[k4] = A[(16 * kb + 4 * k4 + lk) * LDA + 16 * tj + lr];
            }
        };
        if (wave == 0) {
            if (nx < T) {
                f64x4 acc;
                double a[4], b[4];
                load_tile(nx, nx, acc, a, b);
#pragma unroll
                for (int k4 = 0; k4 < 4; ++k4) acc = mma(a[k4], b[k4], acc);
#pragma unroll
                for (int g = 0; g < 4; ++g) A[(16 * nx + lk + 4 * g) * LDA + 16 * nx + lr] = acc[g];
                bad |= tile_inv16<LDA>(A + 16 * nx * LDA + 16 * nx, lane);   // this wave's writes precede its reads
            }
        } else {
            // waves 1-3: tiles t = (wave - 1) + 3 u, in chunks of 4 with their
            // operands loaded first and the MFMA chains interleaved
#pragma unroll
            for (int u0 = 0; u0 < NPW; u0 += 4) {
                constexpr int CH = 4;
                f64x4 acc[CH];
                double a[CH][4], b[CH][4];
                int off[CH];
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    const int t = (wave - 1) + 3 * (u0 + c);
                    const int tt = t < NTU ? t : 0;
                    const int ti0 = tt / T, tj = tt % T;
                    const int ti = ti0 + (ti0 >= kb ? 1 : 0);
                    const bool ok = u0 + c < NPW && t < NTU && !(ti == nx && tj == nx);
                    off[c] = ok ? (16 * ti + lk) * LDA + 16 * tj + lr : -1;
                    load_tile(ti, tj, acc[c], a[c], b[c]);
                }
#pragma unroll
                for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
                    for (int c = 0; c < CH; ++c) acc[c] = mma(a[c][k4], b[c][k4], acc[c]);
#pragma unroll
                for (int c = 0; c < CH; ++c)
                    if (off[c] >= 0) {
#pragma unroll
                        for (int g = 0; g < 4; ++g) A[off[c] + 4 * g * LDA] = acc[c][g];
                    }
            }
        }
        __syncthreads();
        GJ_STAMP(2);
    }
    return bad;
}

// Wide levels (many odd blocks): ONE workgroup per odd block folds the previous
// level's updates into D_i, inverts it (the same gj_invert) and writes G_i over
// D_i (an eliminated block's D is not read again); the level's odd kernel then
// stages G_i (preinv) instead of every one of its 2 ng + mct workgroups
// inverting D_i again.  The same operations in the same order: bit-identical.
template <int T>
__global__ __launch_bounds__(kThreads, 2) void inv_kernel(double* __restrict__ D, const double* __restrict__ SP,
                                                      const double* __restrict__ SN, int32_t nb, int32_t s,
                                                      int32_t* __restrict__ status) {
    using L = Lds<T>;
    constexpr int WB = L::WB, LDA = L::LDA, PER = T * T;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;
    double* C = A + WB * LDA;
    const int i = s + 2 * s * blockIdx.x;
    const int sp = s / 2;
    const int tid = threadIdx.x;
    const int64_t B2 = static_cast<int64_t>(WB) * WB;
    {   // the odd kernel's staging with the fold, verbatim
        const double* Di = D + i * B2;
        const double* sn = SN + (i - sp) * B2;
        const double* spp = SP + (i + sp) * B2;
        const bool h1 = sp > 0, h2 = sp > 0 && i + sp < nb;
        double g[PER];
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) g[qq] = Di[tid + kThreads * qq];
        if (h1) {
            double a1[PER];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) a1[qq] = sn[tid + kThreads * qq];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) g[qq] -= a1[qq];
        }
        if (h2) {
            double a2[PER];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) a2[qq] = spp[tid + kThreads * qq];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) g[qq] -= a2[qq];
        }
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            const int e = tid + kThreads * qq;
            A[(e / WB) * LDA + e % WB] = g[qq];
        }
    }
    __syncthreads();
    const bool bad = gj_invert<T>(A, C);   // ends with a barrier
    if (bad && tid == 0) *status = 1;
    double* Gi = D + i * B2;
#pragma unroll
    for (int qq = 0; qq < PER; ++qq) {
        const int e = tid + kThreads * qq;
        Gi[e] = A[(e / WB) * LDA + e % WB];
    }
}

// Odd blocks of level s: grid (n_odd [+ combine workgroups], 2 ng + 1) with
// ng = ceil(T / cpw) column-tile groups of cpw tiles (the host picks cpw per
// level so its workgroups fit the chip).  Every workgroup inverts D_i itself,
// then, per column tile of its group:
//   q < ng   X_i = G E_p (-> Xs_i, LDS), Sp_i = E_p^T X_i (-> SP_i),
//            E'_p = -E_i X_i (-> En_p);
//   q < 2ng  Y_i = G E_i^T (-> Ys_i), Sn_i = E_i Y_i (-> SN_i);
//   q = 2ng  z_i = G b_i (-> bz_i), E_p^T z_i (-> SPb_i), E_i z_i (-> SNb_i).
template <int T>
__global__ __launch_bounds__(kThreads, 2) void odd_kernel(double* __restrict__ D, const double* __restrict__ Ec,
                                                      double* __restrict__ En, double* __restrict__ Xs,
                                                      double* __restrict__ Ys, double* __restrict__ SP,
                                                      double* __restrict__ SN, double* __restrict__ bz,
                                                      double* __restrict__ SPb, double* __restrict__ SNb, int32_t nb,
                                                      int32_t s, int32_t cpw, int32_t n_odd, int32_t mc,
                                                      int32_t* __restrict__ status, double* __restrict__ bzo,
                                                      const int32_t* __restrict__ pslot, double* __restrict__ Pw,
                                                      int32_t preinv) {
    using L = Lds<T>;
    constexpr int WB = L::WB, LDA = L::LDA, LDC = L::LDC, K4 = WB / 4;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;
    double* C = A + WB * LDA;
    double* vz = C + WB * LDC;   // [2][WB]: b_i, z_i
    double* Rt = vz + 2 * WB;    // mc > 1: the workgroup's RHS column tile [WB][LDC]
    double* Ry = Rt + WB * LDC;  // Schur solves: the whole reduced RHS block Y_i [WB][mc + 1]
    const int ng = (T + cpw - 1) / cpw;
    // mc > 1 (bordered solve): the right-hand side is a
    // WB x mc block per block row (row stride mc) in mc / 16 column tiles, one
    // workgroup per tile (q = 2 ng + tile) instead of the mat-vec workgroup
    const int mct = mc > 1 ? mc / 16 : 0;
    const int q = blockIdx.y;
    const int sp = s / 2;   // the previous level (0: none)
    const int tid = threadIdx.x;
    const int64_t B2 = static_cast<int64_t>(WB) * WB;
    if (static_cast<int>(blockIdx.x) >= n_odd) {
        // combine workgroups: block j = 2s x' stays even at this level and takes
        // the previous level's updates D_j -= Sn_{j-sp} + Sp_{j+sp} (b_j likewise)
        const int j = 2 * s * (blockIdx.x - n_odd);
        if (j >= nb || q >= kCombineSplit || sp == 0) return;
        const bool h1 = j - sp >= 0, h2 = j + sp < nb;
        double* Dj = D + j * B2;
        for (int64_t e = q * kThreads + tid; e < B2; e += kCombineSplit * kThreads) {
            double v = Dj[e];
            if (h1) v -= SN[(j - sp) * B2 + e];
            if (h2) v -= SP[(j + sp) * B2 + e];
            Dj[e] = v;
        }
        const int64_t RB = static_cast<int64_t>(WB) * mc;   // RHS doubles per block
        for (int64_t e = q * kThreads + tid; e < RB; e += kCombineSplit * kThreads) {
            double v = bz[j * RB + e];
            if (h1) v -= SNb[(j - sp) * RB + e];
            if (h2) v -= SPb[(j + sp) * RB + e];
            bz[j * RB + e] = v;
        }
        return;
    }
    if (q > 2 * ng + (mct > 0 ? mct - 1 : 0)) return;   // grid.y padded for the combine workgroups
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const bool hn = n < nb;
    // side 0: X / Sp / E', 2: Y / Sn, 3: z (mat-vecs), 4: RHS column tile q - 2 ng
    const int side = q >= 2 * ng ? (mct > 0 ? 4 : 3) : (q < ng ? 0 : 2);
    const bool zwg = side == 3;
    const bool rwg = side == 4;
    const bool xside = side == 0;
    if (side == 2 && !hn) return;   // the last block has no right neighbour
    const int g0 = (q % ng) * cpw;
    const int tj0 = zwg ? 0 : rwg ? q - 2 * ng : g0, tj1 = zwg ? 0 : rwg ? q - 2 * ng + 1 : min(T, g0 + cpw);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lk = lane >> 4;
    const double* Ep = Ec + p * B2;   // A[i, p]
    const double* Ei = Ec + i * B2;   // A[n, i]
    GJ_T0();
    // D_i and b_i with the previous level's Schur updates folded in while
    // staging: D_i -= Sn_{i-sp} + Sp_{i+sp} (older levels reached D_i through
    // the combine workgroups of their next level: every block is at most one
    // level behind, and the subtraction order is the per-level sequence).
    // preinv: inv_kernel already folded and inverted D_i in place (G_i).
    if (preinv) {
        stage<T>(D + i * B2, A);
    } else {
        constexpr int PER = T * T;
        const double* Di = D + i * B2;
        const double* sn = SN + (i - sp) * B2;
        const double* spp = SP + (i + sp) * B2;
        const bool h1 = sp > 0, h2 = sp > 0 && i + sp < nb;
        // three passes (D_i, then - Sn, then - Sp), each with its loads in flight
        // together: at most 2 x PER doubles live (the kernel's register budget)
        double g[PER];
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) g[qq] = Di[tid + kThreads * qq];
        if (h1) {
            double a1[PER];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) a1[qq] = sn[tid + kThreads * qq];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) g[qq] -= a1[qq];
        }
        if (h2) {
            double a2[PER];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) a2[qq] = spp[tid + kThreads * qq];
#pragma unroll
            for (int qq = 0; qq < PER; ++qq) g[qq] -= a2[qq];
        }
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            const int e = tid + kThreads * qq;
            A[(e / WB) * LDA + e % WB] = g[qq];
        }
    }
    // Schur solve: this block's P_i slot (every RHS tile workgroup needs all of Y_i)
    const int pk = (rwg && pslot) ? pslot[i] : -1;
    if (rwg) {
        // RHS tile with the previous level's updates folded in (as D_i)
        const int64_t RB = static_cast<int64_t>(WB) * mc;
        for (int e = tid; e < WB * 16; e += kThreads) {
            const int r = e >> 4, c = 16 * tj0 + (e & 15);
            double v = bz[i * RB + r * mc + c];
            if (sp > 0) {
                v -= SNb[(i - sp) * RB + r * mc + c];
                if (i + sp < nb) v -= SPb[(i + sp) * RB + r * mc + c];
            }
            Rt[r * LDC + (e & 15)] = v;
        }
        if (pk >= 0) {   // the whole Y_i, the same subtraction order
            for (int e = tid; e < WB * mc; e += kThreads) {
                const int r = e / mc, c = e - r * mc;
                double v = bz[i * RB + e];
                if (sp > 0) {
                    v -= SNb[(i - sp) * RB + e];
                    if (i + sp < nb) v -= SPb[(i + sp) * RB + e];
                }
                Ry[r * (mc + 1) + c] = v;
            }
        }
    }
    if (zwg && tid < WB) {
        double v = bz[static_cast<int64_t>(i) * WB + tid];
        if (sp > 0) {
            v -= SNb[static_cast<int64_t>(i - sp) * WB + tid];
            if (i + sp < nb) v -= SPb[static_cast<int64_t>(i + sp) * WB + tid];
        }
        vz[tid] = v;
    }
    __syncthreads();
    GJ_STAMP(3);
    if (!preinv) {
        const bool bad = gj_invert<T>(A, C);   // A = G (ends with a barrier)
        if (bad && q == 0 && tid == 0) *status = 1;
    }
    GJ_STAMP(4);
    for (int tj = tj0; tj < tj1; ++tj) {
        // first product: column tile tj of X_i = G E_p or Y_i = G E_i^T: the
        // tile of E (the B operand, shared by every output tile) is loaded once,
        // all K4 fragments in flight; a wave's output tiles run interleaved
        // RHS tile: z_i's columns 16 tj.. (bz, row stride mc), then E_p^T z (SPb)
        // and E_i z (SNb) as the X side's Sp and E' (sign +)
        const int64_t RB = static_cast<int64_t>(WB) * mc;
        double* Out1 = rwg ? (bzo ? bzo : bz) + i * RB + 16 * tj : (xside ? Xs : Ys) + i * B2 + 16 * tj;
        const int ld1 = rwg ? mc : WB;
        {
            constexpr int N1 = (T + 3) / 4;
            double bf[K4];
#pragma unroll
            for (int k4 = 0; k4 < K4; ++k4)
                bf[k4] = rwg ? Rt[(4 * k4 + lk) * LDC + lr]
                             : xside ? Ep[(4 * k4 + lk) * WB + 16 * tj + lr] : Ei[(16 * tj + lr) * WB + 4 * k4 + lk];
            f64x4 acc[N1];
#pragma unroll
            for (int u = 0; u < N1; ++u) acc[u] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k4 = 0; k4 < K4; ++k4)
#pragma unroll
                for (int u = 0; u < N1; ++u) {
                    const int ti = min(wave + 4 * u, T - 1);
                    acc[u] = mma(A[(16 * ti + lr) * LDA + 4 * k4 + lk], bf[k4], acc[u]);
                }
#pragma unroll
            for (int u = 0; u < N1; ++u) {
                const int ti = wave + 4 * u;
                if (ti < T) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int row = 16 * ti + lk + 4 * g;
                        Out1[row * ld1 + lr] = acc[u][g];
                        C[row * LDC + lr] = acc[u][g];
                    }
                }
            }
        }
        __syncthreads();
        GJ_STAMP(5);
        // second products on that column tile (in C, the B operand):
        // Sp = E_p^T X, E' = -E_i X  |  Sn = E_i Y; each task's K4 A fragments
        // in flight at once
        {
            constexpr int N2 = (2 * T + 3) / 4;
            const int ntask = ((xside || rwg) && hn) ? 2 * T : T;
            double bf[K4];
#pragma unroll
            for (int k4 = 0; k4 < K4; ++k4) bf[k4] = C[(4 * k4 + lk) * LDC + lr];
#pragma unroll
            for (int u = 0; u < N2; ++u) {
                const int t = wave + 4 * u;
                if (t < ntask) {   // wave-uniform
                    const int ti = t % T;
                    const bool e = t >= T;   // X side: the new coupling; RHS tile: E_i z
                    double af[K4];
#pragma unroll
                    for (int k4 = 0; k4 < K4; ++k4)
                        af[k4] = ((xside || rwg) && !e) ? Ep[(4 * k4 + lk) * WB + 16 * ti + lr]
                                                        : Ei[(16 * ti + lr) * WB + 4 * k4 + lk];
                    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int k4 = 0; k4 < K4; ++k4) acc = mma(af[k4], bf[k4], acc);
                    double* Out2 = rwg ? (e ? SNb : SPb) + i * RB + 16 * tj
                                       : (e ? En + p * B2 : xside ? SP + i * B2 : SN + i * B2) + 16 * tj;
                    const double sg = (e && !rwg) ? -1.0 : 1.0;
#pragma unroll
                    for (int g = 0; g < 4; ++g) Out2[(16 * ti + lk + 4 * g) * ld1 + lr] = sg * acc[g];
                }
            }
        }
        __syncthreads();   // C is rewritten by the next column tile
        GJ_STAMP(6);
    }
    if (pk >= 0) {
        // P_i[:, tile] = Y_i^T Z_i[:, tile]: Y_i in Ry, this tile of Z_i = G_i Y_i
        // still in C (rwg: one column tile, its loop body ran once)
        const int ti = wave;
        if (ti < mc / 16) {
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
            double af[K4], bf[K4];
#pragma unroll
            for (int k4 = 0; k4 < K4; ++k4) {
                af[k4] = Ry[(4 * k4 + lk) * (mc + 1) + 16 * ti + lr];
                bf[k4] = C[(4 * k4 + lk) * LDC + lr];
            }
#pragma unroll
            for (int k4 = 0; k4 < K4; ++k4) acc = mma(af[k4], bf[k4], acc);
            double* P = Pw + static_cast<int64_t>(pk) * mc * mc;
#pragma unroll
            for (int g = 0; g < 4; ++g) P[(16 * ti + lk + 4 * g) * mc + 16 * tj0 + lr] = acc[g];
        }
    }
    if (zwg) {
        // three mat-vecs, each over the whole workgroup: rows r = lane, lane + 64
        // of wave w sum k in [w WB/4, (w+1) WB/4), the quarters meet in LDS (C)
        constexpr int KQ = WB / 4;
        double* red = C;   // [4][WB]
        const int k0 = wave * KQ;
        auto quarters = [&](auto term) {   // red[wave][r] = sum_k term(r, k) over the wave's quarter
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = lane + 64 * h;
                if (r < WB) {
                    double acc = 0.0;
#pragma unroll 5
                    for (int k = 0; k < KQ; ++k) acc += term(r, k0 + k);
                    red[wave * WB + r] = acc;
                }
            }
            __syncthreads();
        };
        quarters([&](int r, int k) { return A[r * LDA + k] * vz[k]; });   // z = G b
        if (tid < WB) {
            const double z = ((red[tid] + red[WB + tid]) + red[2 * WB + tid]) + red[3 * WB + tid];
            vz[WB + tid] = z;
            bz[static_cast<int64_t>(i) * WB + tid] = z;
        }
        __syncthreads();
        quarters([&](int r, int k) { return Ep[k * WB + r] * vz[WB + k]; });   // E_p^T z
        if (tid < WB)
            SPb[static_cast<int64_t>(i) * WB + tid] = ((red[tid] + red[WB + tid]) + red[2 * WB + tid]) + red[3 * WB + tid];
        __syncthreads();
        if (hn) {
            quarters([&](int r, int k) { return Ei[r * WB + k] * vz[WB + k]; });   // E_i z
            if (tid < WB)
                SNb[static_cast<int64_t>(i) * WB + tid] =
                    ((red[tid] + red[WB + tid]) + red[2 * WB + tid]) + red[3 * WB + tid];
        }
    }
}

// Block 0 after the last level sl: D_0 -= Sp_sl, b_0 -= SPb_sl (its earlier
// levels came through the combine workgroups) while staging, the same
// Gauss-Jordan inversion, then x_0 = G b_0 (one workgroup).
template <int T>
__global__ __launch_bounds__(kThreads) void top_kernel(const double* __restrict__ D, const double* __restrict__ SP,
                                                      const double* __restrict__ bz, const double* __restrict__ SPb,
                                                      double* __restrict__ x, int32_t sl, int32_t mc,
                                                      int32_t* __restrict__ status) {
    using L = Lds<T>;
    constexpr int WB = L::WB, LDA = L::LDA, LDC = L::LDC, PER = T * T, KQ = WB / 4;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;
    double* C = A + WB * LDA;
    double* vz = C + WB * LDC;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t B2 = static_cast<int64_t>(WB) * WB;
    {
        double g[PER], a1[PER];
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            g[qq] = D[tid + kThreads * qq];
            a1[qq] = sl > 0 ? SP[sl * B2 + tid + kThreads * qq] : 0.0;
        }
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            const int e = tid + kThreads * qq;
            A[(e / WB) * LDA + e % WB] = sl > 0 ? g[qq] - a1[qq] : g[qq];
        }
    }
    if (mc > 1) {
        // bordered solve: X_0 = G R_0 for the WB x mc right-hand side (R in LDS
        // behind vz, row stride mc + 1); each thread sums whole dot products
        double* R = vz + 2 * WB;
        const int64_t RB = static_cast<int64_t>(WB) * mc;
        {   // all loads first (WB * mc / kThreads <= 12 per thread), then the stores
            constexpr int kMaxPer = 16 * 6 * 32 / kThreads;
            const int per = WB * mc / kThreads;
            double bv[kMaxPer], sv[kMaxPer];
#pragma unroll
            for (int q = 0; q < kMaxPer; ++q) {
                const int e = tid + kThreads * q;
                bv[q] = q < per ? bz[e] : 0.0;
                sv[q] = q < per && sl > 0 ? SPb[sl * RB + e] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < kMaxPer; ++q) {
                const int e = tid + kThreads * q;
                if (q < per) R[(e / mc) * (mc + 1) + e % mc] = sl > 0 ? bv[q] - sv[q] : bv[q];
            }
        }
        __syncthreads();
        const bool bad = gj_invert<T>(A, C);
        if (bad && tid == 0) *status = 1;
        for (int e = tid; e < WB * mc; e += kThreads) {
            const int r = e / mc, c = e % mc;
            double acc = 0.0;
#pragma unroll 8
            for (int k = 0; k < WB; ++k) acc = fma(A[r * LDA + k], R[k * (mc + 1) + c], acc);
            x[e] = acc;
        }
        return;
    }
    if (tid < WB) vz[tid] = sl > 0 ? bz[tid] - SPb[static_cast<int64_t>(sl) * WB + tid] : bz[tid];
    __syncthreads();
    const bool bad = gj_invert<T>(A, C);
    if (bad && tid == 0) *status = 1;
    double* red = C;   // [4][WB]: the quarters of x = G b
    const int k0 = wave * KQ;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int r = lane + 64 * h;
        if (r < WB) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < KQ; ++k) acc += A[r * LDA + k0 + k] * vz[k0 + k];
            red[wave * WB + r] = acc;
        }
    }
    __syncthreads();
    if (tid < WB) x[tid] = ((red[tid] + red[WB + tid]) + red[2 * WB + tid]) + red[3 * WB + tid];
}

// Block 0 of a Schur-accumulating bordered solve (gn_bcr.hpp BcrSchur), one
// workgroup: D_0 and its reduced RHS block R_0 = [b_0 | y_0] (the last level's
// Sp folded in), X_0 = G_0 R_0, then the border: S = C - sum_k P_k[B, B] -
// R_0[:, B]^T X_0[:, B] and s = r_b - (the same with column 0), the slots in
// slot order (deterministic), S padded to 32 x 32 with the identity and
// inverted by gj_invert<2>, x_b = S^-1 s; and x_0 = X_0[:, 0] - X_0[:, B] x_b.
template <int T>
__global__ __launch_bounds__(kThreads) void top_schur_kernel(const double* __restrict__ D,
                                                            const double* __restrict__ SP,
                                                            const double* __restrict__ bz,
                                                            const double* __restrict__ SPb, double* __restrict__ x,
                                                            int32_t sl, int32_t mc, BcrSchur sc,
                                                            int32_t* __restrict__ status, int32_t* ready, int32_t nb) {
    using L = Lds<T>;
    constexpr int WB = L::WB, LDA = L::LDA, LDC = 17, PER = T * T;
    constexpr int WC = WB > 32 ? WB : 32;   // C scratch rows (the 32 x 32 border inverse too)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* A = lds;                  // [WB][LDA]: D_0, then G_0
    double* C = A + WB * LDA;         // [WC][17]
    double* R = C + WC * LDC;         // [WB][mc + 1]: R_0
    double* X0 = R + WB * (mc + 1);   // [WB][mc + 1]: X_0 = G_0 R_0
    double* Sm = X0 + WB * (mc + 1);  // [32][33]: S, then S^-1
    double* sv = Sm + 32 * 33;        // [32]: s
    double* xbs = sv + 32;            // [32]: x_b
    double* P0 = xbs + 32;            // [32][33]: R_0^T X_0 (mc <= 32)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lk = lane >> 4;
    constexpr int K4 = WB / 4;
    const int64_t B2 = static_cast<int64_t>(WB) * WB, RB = static_cast<int64_t>(WB) * mc;
    {
        double g[PER], a1[PER];
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            g[qq] = D[tid + kThreads * qq];
            a1[qq] = sl > 0 ? SP[sl * B2 + tid + kThreads * qq] : 0.0;
        }
#pragma unroll
        for (int qq = 0; qq < PER; ++qq) {
            const int e = tid + kThreads * qq;
            A[(e / WB) * LDA + e % WB] = sl > 0 ? g[qq] - a1[qq] : g[qq];
        }
    }
    for (int e = tid; e < WB * mc; e += kThreads) {
        const double v = bz[e];
        R[(e / mc) * (mc + 1) + e % mc] = sl > 0 ? v - SPb[sl * RB + e] : v;
    }
    __syncthreads();
    if (gj_invert<T>(A, C) && tid == 0) *status = 1;   // ends with a barrier
    const int nct = mc / 16;
    // X_0 = G_0 R_0 as MFMA tiles (wave w: tiles w, w + 4, ...), then
    // P_0 = R_0^T X_0 (nct x nct tiles)
    for (int t = wave; t < T * nct; t += 4) {
        const int ti = t / nct, tc = t - ti * nct;
        double af[K4], bf[K4];
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) {
            af[k4] = A[(16 * ti + lr) * LDA + 4 * k4 + lk];
            bf[k4] = R[(4 * k4 + lk) * (mc + 1) + 16 * tc + lr];
        }
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) acc = mma(af[k4], bf[k4], acc);
#pragma unroll
        for (int g = 0; g < 4; ++g) X0[(16 * ti + lk + 4 * g) * (mc + 1) + 16 * tc + lr] = acc[g];
    }
    __syncthreads();
    for (int t = wave; t < nct * nct; t += 4) {
        const int ti = t / nct, tc = t - ti * nct;
        double af[K4], bf[K4];
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) {
            af[k4] = R[(4 * k4 + lk) * (mc + 1) + 16 * ti + lr];
            bf[k4] = X0[(4 * k4 + lk) * (mc + 1) + 16 * tc + lr];
        }
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) acc = mma(af[k4], bf[k4], acc);
#pragma unroll
        for (int g = 0; g < 4; ++g) P0[(16 * ti + lk + 4 * g) * 33 + 16 * tc + lr] = acc[g];
    }
    __syncthreads();
    // [S | s] entries e = k * (nbd + 1) + l (l = nbd: s), at most 4 per thread
    const int nbd = sc.nbd, ncol = nbd + 1;
    for (int e = tid; e < 32 * 32; e += kThreads) {   // identity padding
        const int r = e >> 5, c = e & 31;
        if (r >= nbd || c >= nbd) Sm[r * 33 + c] = r == c ? 1.0 : 0.0;
    }
    if (tid < 32 && tid >= nbd) sv[tid] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = tid + kThreads * q;
        if (e < nbd * ncol) {
            const int k = e / ncol, l = e % ncol;
            const int pc = l < nbd ? 1 + l : 0;   // P column: B_l, or the rhs
            const double cv = l < nbd ? (l <= k ? sc.BR[static_cast<int64_t>(k) * sc.nvt + sc.nv_band + l]
                                                : sc.BR[static_cast<int64_t>(l) * sc.nvt + sc.nv_band + k])
                                      : sc.rhs[sc.nv_band + k];
            double acc = 0.0;
            int t = 0;
            for (; t + 4 <= sc.n_slots; t += 4) {   // four slots' loads in flight, summed in slot order
                double pv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) pv[u] = sc.P[(static_cast<int64_t>(t + u) * mc + 1 + k) * mc + pc];
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += pv[u];
            }
            for (; t < sc.n_slots; ++t) acc += sc.P[(static_cast<int64_t>(t) * mc + 1 + k) * mc + pc];
            acc += P0[(1 + k) * 33 + pc];
            if (l < nbd) Sm[k * 33 + l] = cv - acc;
            else sv[k] = cv - acc;
        }
    }
    __syncthreads();
    if (gj_invert<2>(Sm, C) && tid == 0) *status = 1;   // ends with a barrier
    if (tid < nbd) {
        double v = 0.0;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) v = fma(Sm[tid * 33 + k], sv[k], v);
        xbs[tid] = v;
        sc.xb[tid] = v;
    }
    __syncthreads();
    if (tid < WB) {
        double a = 0.0;
        for (int k = 0; k < nbd; ++k) a = fma(X0[tid * (mc + 1) + 1 + k], xbs[k], a);
        x[tid] = X0[tid * (mc + 1)] - a;
    }
}

// Back-substitution of a Schur-accumulating bordered solve (one column):
// x_i = (z_i[:, 0] - z_i[:, B] x_b) - X_i x_p - Y_i x_n, z_i from bzo (row
// stride mc).  Thread (tr, tc) sums its share of the row's terms (columns
// tc + 16 w of X / Y, z columns tc + 16 m) and the DPP row sum adds them.
template <int T>
__global__ __launch_bounds__(kThreads) void back_schur_kernel(const double* __restrict__ Xs,
                                                             const double* __restrict__ Ys,
                                                             const double* __restrict__ bzo, double* __restrict__ x,
                                                             const double* __restrict__ xb, int32_t nbd, int32_t nb,
                                                             int32_t s, int32_t mc);

// A double moved between lanes of a 16-lane row by DPP (both halves).
template <int CTRL>
__device__ __forceinline__ double dpp_row(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b & 0xffffffff), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Back-substitution of the odd blocks of level s: x_i = z_i - X_i x_p - Y_i x_n
// (16 x 16 threads: thread (tr, tc) sums columns tc + 16 w of rows tr + 16 u from
// 128 B row segments; DPP row sums).
template <int T>
__global__ __launch_bounds__(kThreads) void back_kernel(const double* __restrict__ Xs, const double* __restrict__ Ys,
                                                       const double* __restrict__ bz, double* __restrict__ x,
                                                       int32_t nb, int32_t s) {
    constexpr int WB = 16 * T;
    const int tid = threadIdx.x;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const bool hn = n < nb;
    const int64_t B2 = static_cast<int64_t>(WB) * WB;
    const int tr = tid >> 4, tc = tid & 15;
    const double* X = Xs + i * B2;
    const double* Y = Ys + i * B2;
    // every X / Y / x_p / x_n / z load in flight before the first FMA (no LDS
    // staging, no barrier: the level is a chain of load latencies)
    double xv[T][T], yv[T][T], zv[T], vp[T], vn[T];
#pragma unroll
    for (int w = 0; w < T; ++w) {
        vp[w] = x[static_cast<int64_t>(p) * WB + tc + 16 * w];
        vn[w] = hn ? x[static_cast<int64_t>(n) * WB + tc + 16 * w] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
#pragma unroll
        for (int w = 0; w < T; ++w) {
            xv[u][w] = X[(tr + 16 * u) * WB + tc + 16 * w];
            yv[u][w] = hn ? Y[(tr + 16 * u) * WB + tc + 16 * w] : 0.0;
        }
        zv[u] = tc == 0 ? bz[static_cast<int64_t>(i) * WB + tr + 16 * u] : 0.0;
    }
    double v[T];
#pragma unroll
    for (int u = 0; u < T; ++u) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int w = 0; w < T; ++w) {
            a0 = fma(xv[u][w], vp[w], a0);
            a1 = fma(yv[u][w], vn[w], a1);
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
        for (int u = 0; u < T; ++u) {
            const int r = tr + 16 * u;
            x[static_cast<int64_t>(i) * WB + r] = zv[u] - v[u];
        }
    }
}

template <int T>
__global__ __launch_bounds__(kThreads) void back_schur_kernel(const double* __restrict__ Xs,
                                                             const double* __restrict__ Ys,
                                                             const double* __restrict__ bzo, double* __restrict__ x,
                                                             const double* __restrict__ xb, int32_t nbd, int32_t nb,
                                                             int32_t s, int32_t mc) {
    constexpr int WB = 16 * T;
    const int tid = threadIdx.x;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const bool hn = n < nb;
    const int64_t B2 = static_cast<int64_t>(WB) * WB, RB = static_cast<int64_t>(WB) * mc;
    const int tr = tid >> 4, tc = tid & 15;
    const double* X = Xs + i * B2;
    const double* Y = Ys + i * B2;
    const int nzc = mc / 16;   // z columns per thread: tc + 16 m (mc <= 32)
    double xv[T][T], yv[T][T], vp[T], vn[T], zv[T][2], cf[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {   // coefficient of z column c: 1 (the rhs), -x_b[c - 1], 0 past the border
        const int c = tc + 16 * m;
        cf[m] = m < nzc ? (c == 0 ? 1.0 : (c <= nbd ? -xb[c - 1] : 0.0)) : 0.0;
    }
#pragma unroll
    for (int w = 0; w < T; ++w) {
        vp[w] = x[static_cast<int64_t>(p) * WB + tc + 16 * w];
        vn[w] = hn ? x[static_cast<int64_t>(n) * WB + tc + 16 * w] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
#pragma unroll
        for (int w = 0; w < T; ++w) {
            xv[u][w] = X[(tr + 16 * u) * WB + tc + 16 * w];
            yv[u][w] = hn ? Y[(tr + 16 * u) * WB + tc + 16 * w] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < 2; ++m)
            zv[u][m] = m < nzc ? bzo[i * RB + static_cast<int64_t>(tr + 16 * u) * mc + tc + 16 * m] : 0.0;
    }
    double v[T];
#pragma unroll
    for (int u = 0; u < T; ++u) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int w = 0; w < T; ++w) {
            a0 = fma(xv[u][w], vp[w], a0);
            a1 = fma(yv[u][w], vn[w], a1);
        }
        v[u] = (a0 + a1) - fma(cf[1], zv[u][1], cf[0] * zv[u][0]);   // -(this thread's share of x)
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
        v[u] += dpp_row<0xB1>(v[u]);
        v[u] += dpp_row<0x4E>(v[u]);
        v[u] += dpp_row<0x124>(v[u]);
        v[u] += dpp_row<0x128>(v[u]);
    }
    if (tc == 0) {
#pragma unroll
        for (int u = 0; u < T; ++u) x[static_cast<int64_t>(i) * WB + tr + 16 * u] = -v[u];
    }
}

// Every back-substitution level of a Schur-accumulating bordered solve in ONE
// launch, on ONE XCD (a level is ~1 us of load latency; as its own launch it
// takes 4.8 us: profiles/r05_gn_kernel_stats.csv).  Only the workgroups with
// blockIdx % 8 == 0 work — round-robin dispatch puts them all on the same XCD
// (as the ICP gangs rely on), whose L2 is the one coherence point they need —
// workgroup 8 w taking the w-th odd block in coarsest-level-first order.  A
// block's x is published as data-tagged granules (tag 1 in the high word,
// 32-bit halves of the doubles in the low; one relaxed
// agent-scope store each, no fence: the data IS the flag, as in the ICP gang
// exchange; the granules are zeroed by each iteration's linearisation
// launch, so the tag is a constant) and its consumers poll them; block 0 (the
// top launch's) is read plainly.  Producers have lower indices than their consumers and dispatch is
// in index order, so the lowest unfinished block can always run.  A wait
// longer than `wait` s_memrealtime ticks sets *status |= 2 (a wrong result
// the caller reports, never a hang).
template <int T>
__global__ __launch_bounds__(kThreads) void back_schur_xcd_kernel(const double* __restrict__ Xs,
                                                                 const double* __restrict__ Ys,
                                                                 const double* __restrict__ bzo, double* x,
                                                                 const double* __restrict__ xb, int32_t nbd,
                                                                 int32_t nb, int32_t mc, uint64_t* xg, uint32_t wait,
                                                                 int32_t* __restrict__ status) {
    constexpr int WB = 16 * T;
    __shared__ uint32_t xh[2][2 * WB];   // the neighbours' x as 32-bit halves (lo, hi)
    const int tid = threadIdx.x;
    if (blockIdx.x & 7) return;   // (uniform) not on the working XCD

    int w = static_cast<int>(blockIdx.x >> 3);
    int s = 1;
    while (2 * s < nb) s *= 2;   // the top level
    for (;;) {
        const int n_odd = (nb - s + 2 * s - 1) / (2 * s);
        if (w < n_odd || s == 1) break;
        w -= n_odd;
        s /= 2;
    }
    const int i = s + 2 * s * w;
    if (i >= nb) return;   // (uniform) past the last odd block
    const int p = i - s, n = i + s;
    const bool hn = n < nb;
    constexpr uint32_t ep = 1;   // the tag (granules zeroed by the linearisation launch)
    const int64_t B2 = static_cast<int64_t>(WB) * WB, RB = static_cast<int64_t>(WB) * mc;
    const int tr = tid >> 4, tc = tid & 15;
    const double* X = Xs + i * B2;
    const double* Y = Ys + i * B2;
    const int nzc = mc / 16;
    // this block's own operands (earlier launches) in flight while the neighbours are polled
    double xv[T][T], yv[T][T], vp[T], vn[T], zv[T][2], cf[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int c = tc + 16 * m;
        cf[m] = m < nzc ? (c == 0 ? 1.0 : (c <= nbd ? -xb[c - 1] : 0.0)) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
#pragma unroll
        for (int ww = 0; ww < T; ++ww) {
            xv[u][ww] = X[(tr + 16 * u) * WB + tc + 16 * ww];
            yv[u][ww] = hn ? Y[(tr + 16 * u) * WB + tc + 16 * ww] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < 2; ++m)
            zv[u][m] = m < nzc ? bzo[i * RB + static_cast<int64_t>(tr + 16 * u) * mc + tc + 16 * m] : 0.0;
    }
    // the neighbours' x: granules (2 WB per block) polled until their tags are
    // this iteration's; block 0 plain
    for (int e = tid; e < 4 * WB; e += kThreads) {
        const int side = e / (2 * WB), g = e - side * 2 * WB;
        const int j = side ? n : p;
        if (side && !hn) continue;
        if (j == 0) {
            const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(x[g >> 1]));
            xh[side][g] = static_cast<uint32_t>((g & 1) ? bits >> 32 : bits);
            continue;
        }
        const uint64_t* src = xg + static_cast<int64_t>(j) * 2 * WB + g;
        uint64_t v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (static_cast<uint32_t>(v >> 32) != ep) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            do {
                __builtin_amdgcn_s_sleep(1);
                v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_s_memrealtime() - t0 > wait) {
                    atomicOr(status, 2);
                    break;
                }
            } while (static_cast<uint32_t>(v >> 32) != ep);
        }
        xh[side][g] = static_cast<uint32_t>(v);
    }
    __syncthreads();
    const double* xp_s = reinterpret_cast<const double*>(xh[0]);
    const double* xn_s = reinterpret_cast<const double*>(xh[1]);
#pragma unroll
    for (int ww = 0; ww < T; ++ww) {
        vp[ww] = xp_s[tc + 16 * ww];
        vn[ww] = hn ? xn_s[tc + 16 * ww] : 0.0;
    }
    double v[T];
#pragma unroll
    for (int u = 0; u < T; ++u) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int ww = 0; ww < T; ++ww) {
            a0 = fma(xv[u][ww], vp[ww], a0);
            a1 = fma(yv[u][ww], vn[ww], a1);
        }
        v[u] = (a0 + a1) - fma(cf[1], zv[u][1], cf[0] * zv[u][0]);
    }
#pragma unroll
    for (int u = 0; u < T; ++u) {
        v[u] += dpp_row<0xB1>(v[u]);
        v[u] += dpp_row<0x4E>(v[u]);
        v[u] += dpp_row<0x124>(v[u]);
        v[u] += dpp_row<0x128>(v[u]);
    }
    // lanes tc = 0 / 1 of each row publish the lo / hi granule of its rows
    // (every lane of the row holds the row sum); tc = 0 also writes x
    if (tc < 2) {
        const uint64_t tag = static_cast<uint64_t>(ep) << 32;
        uint64_t* dst = xg + static_cast<int64_t>(i) * 2 * WB;
#pragma unroll
        for (int u = 0; u < T; ++u) {
            const int r = tr + 16 * u;
            const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(-v[u]));
            if (tc == 0) x[static_cast<int64_t>(i) * WB + r] = -v[u];
            __hip_atomic_store(dst + 2 * r + tc, tag | (tc ? bits >> 32 : bits & 0xffffffffull), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Bordered solves: x_i = z_i - X_i x_p - Y_i x_n for WB x mc blocks (row
// stride mc, mc a multiple of 16) as MFMA tiles, wave w taking output tiles w,
// w + 4, ... (fixed k order: deterministic).  The level is a chain of load
// latencies, not of MFMAs: every operand of a tile (X / Y fragments, the x_p /
// x_n B fragments straight from global memory, z) is loaded at once, with no
// LDS staging or barrier.
template <int T>
__global__ __launch_bounds__(kThreads) void back_multi_kernel(const double* __restrict__ Xs,
                                                             const double* __restrict__ Ys,
                                                             const double* __restrict__ bz, double* __restrict__ x,
                                                             int32_t nb, int32_t s, int32_t mc) {
    constexpr int WB = 16 * T, K4 = WB / 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lk = lane >> 4;
    const int i = s + 2 * s * blockIdx.x;
    const int p = i - s, n = i + s;
    const bool hn = n < nb;
    const int64_t B2 = static_cast<int64_t>(WB) * WB, RB = static_cast<int64_t>(WB) * mc;
    const double* X = Xs + i * B2;
    const double* Y = Ys + i * B2;
    const double* xp = x + p * RB;
    const double* xn = x + n * RB;
    const int nct = mc / 16;
    for (int t = wave; t < T * nct; t += 4) {
        const int ti = t / nct, tc = t - ti * nct;
        double ax[K4], ay[K4], bp[K4], bn[K4], zv[4];
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) {
            ax[k4] = X[(16 * ti + lr) * WB + 4 * k4 + lk];
            ay[k4] = hn ? Y[(16 * ti + lr) * WB + 4 * k4 + lk] : 0.0;
            bp[k4] = xp[(4 * k4 + lk) * mc + 16 * tc + lr];
            bn[k4] = hn ? xn[(4 * k4 + lk) * mc + 16 * tc + lr] : 0.0;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) zv[g] = bz[i * RB + (16 * ti + lk + 4 * g) * mc + 16 * tc + lr];
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k4 = 0; k4 < K4; ++k4) {
            acc = mma(ax[k4], bp[k4], acc);
            acc = mma(ay[k4], bn[k4], acc);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t o = i * RB + (16 * ti + lk + 4 * g) * mc + 16 * tc + lr;
            x[o] = zv[g] - acc[g];
        }
    }
}

// Border of a bordered solve: S = C - B^T Z_B and
// s = r_b - B^T Z_r over the band rows coupled to the border (nbr_rows: B is
// zero elsewhere), staged in chunks with every load in flight and summed in a
// fixed order; S padded to 32 x 32 with the identity, inverted by the same
// blocked Gauss-Jordan as the BCR blocks (gj_invert<2>), x_b = S^-1 s.
constexpr int kBorderMax = 31;
constexpr int kBorderChunk = 64;
__global__ __launch_bounds__(kThreads) void border_solve_kernel(const double* __restrict__ Z,
                                                               const double* __restrict__ BR,
                                                               const double* __restrict__ rhs,
                                                               const int32_t* __restrict__ nbr_rows, int32_t n_nbr,
                                                               int32_t nv_band, int32_t nbd, int32_t nvt, int32_t mc,
                                                               double* __restrict__ xb, int32_t* __restrict__ status) {
    constexpr int LDA = 33, LDC = 17;
    __shared__ double A[32 * LDA];
    __shared__ double C[32 * LDC];
    __shared__ double sv[32];
    __shared__ double Bs[kBorderChunk][33];   // B^T columns of the chunk's coupled rows
    __shared__ double Zs[kBorderChunk][33];   // their Z rows (column 0: Z_r, 1 + k: Z_B)
    const int tid = threadIdx.x;
    const int ncol = nbd + 1;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};   // entries e = tid + 256 q of [S | s]
    double cv[4] = {0.0, 0.0, 0.0, 0.0};    // their C / r_b values, loaded before the chunks
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = tid + kThreads * q;
        if (e < nbd * ncol) {
            const int k = e / ncol, l = e % ncol;
            cv[q] = l < nbd ? (l <= k ? BR[static_cast<int64_t>(k) * nvt + nv_band + l]
                                      : BR[static_cast<int64_t>(l) * nvt + nv_band + k])
                            : rhs[nv_band + k];
        }
    }
    for (int t0 = 0; t0 < n_nbr; t0 += kBorderChunk) {
        const int nt = min(kBorderChunk, n_nbr - t0);
        __syncthreads();
        {   // every row index, then every B / Z value in flight, then the LDS stores
            constexpr int kPer = kBorderChunk * 32 / kThreads;
            int rv[kPer];
            double bv[kPer], zv[kPer];
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                const int e = tid + kThreads * q;
                rv[q] = e < nt * 32 ? nbr_rows[t0 + (e >> 5)] : 0;
            }
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                const int e = tid + kThreads * q, k = e & 31;
                const bool in = e < nt * 32;
                bv[q] = in && k < nbd ? BR[static_cast<int64_t>(k) * nvt + rv[q]] : 0.0;
                zv[q] = in && k < ncol ? Z[static_cast<int64_t>(rv[q]) * mc + (k < nbd ? 1 + k : 0)] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                const int e = tid + kThreads * q;
                if (e < nt * 32) {
                    Bs[e >> 5][e & 31] = bv[q];
                    Zs[e >> 5][e & 31] = zv[q];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + kThreads * q;
            if (e < nbd * ncol) {
                const int k = e / ncol, l = e % ncol;
                double a = acc[q];
                for (int t = 0; t < nt; ++t) a = fma(Bs[t][k], Zs[t][l], a);
                acc[q] = a;
            }
        }
    }
    for (int e = tid; e < 32 * 32; e += kThreads) {   // identity padding
        const int r = e >> 5, c = e & 31;
        if (r >= nbd || c >= nbd) A[r * LDA + c] = r == c ? 1.0 : 0.0;
    }
    if (tid < 32 && tid >= nbd) sv[tid] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = tid + kThreads * q;
        if (e < nbd * ncol) {
            const int k = e / ncol, l = e % ncol;
            if (l < nbd) A[k * LDA + l] = cv[q] - acc[q];
            else sv[k] = cv[q] - acc[q];
        }
    }
    __syncthreads();
    const bool bad = gj_invert<2>(A, C);   // ends with a barrier
    if (bad && tid == 0) *status = 1;
    if (tid < nbd) {
        double v = 0.0;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) v = fma(A[tid * LDA + k], sv[k], v);
        xb[tid] = v;
    }
}

}  // namespace bcrgj

constexpr int kBcrGjSlots = 2 * 256;   // odd-kernel workgroups resident at once (2 per CU)
// odd blocks from which a level inverts them once (inv_kernel; 0 = never, the
// default: measured in round 6 at C4, splitting level 1 (234 blocks) or levels
// 1-2 costs 2-4 %: 5,340-5,347 it/s unsplit against 5,240-5,271 / 5,094-5,211,
// bit-identical chi2; profiles/r06_gn_ab_split.txt)
constexpr int kGjSplitMin = 0;

BcrGjBufs bcr_gj_bufs(double* work, int32_t nv, int32_t Wb, int32_t mc) {
    const int64_t nb = (nv + Wb - 1) / Wb;
    const int64_t B2 = static_cast<int64_t>(Wb) * Wb;
    const int64_t RB = static_cast<int64_t>(Wb) * mc;
    BcrGjBufs b;
    b.D = work;
    b.E0 = b.D + nb * B2;
    b.E1 = b.E0 + nb * B2;
    b.Xs = b.E1 + nb * B2;
    b.Ys = b.Xs + nb * B2;
    b.SP = b.Ys + nb * B2;
    b.SN = b.SP + nb * B2;
    b.bz = b.SN + nb * B2;
    b.SPb = b.bz + nb * RB;
    b.SNb = b.SPb + nb * RB;
    b.x = b.SNb + nb * RB;
    b.bzo = b.x + nb * RB;
    b.ready = reinterpret_cast<int32_t*>(b.bzo + nb * RB);
    b.xg = reinterpret_cast<uint64_t*>(b.bzo + nb * RB + (nb + 1) / 2 + 1);
    return b;
}

int64_t bcr_gj_work_size(int32_t nv, int32_t Wb, int32_t mc) {
    const int64_t nb = (nv + Wb - 1) / Wb;
    // + the epoch word (ready) and the back-substitution's tagged granules
    return 7 * nb * Wb * Wb + 5 * nb * Wb * static_cast<int64_t>(mc) + (nb + 1) / 2 + 1 + 2 * nb * Wb;
}

// The levels of the explicit-inverse reduction, after bcr_load_kernel filled
// D, E0 and bz, and the block-0 solve (x_0 in b.x).
int bcr_gj_levels(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, int32_t* status, hipStream_t st,
                  const BcrSchur* sc) {
    const int nb = (nv + Wb - 1) / Wb;
    const int mct = mc > 1 ? mc / 16 : 0;   // RHS column tiles (bordered solves)
    if (sc && (mc > 32 || mc < 16)) return fail(SLAM_EINVAL, "gn: Schur border with %d RHS columns", mc);
    using OddFn = void (*)(double*, const double*, double*, double*, double*, double*, double*, double*,
                           double*, double*, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t*, double*,
                           const int32_t*, double*, int32_t);
    using InvFn = void (*)(double*, const double*, const double*, int32_t, int32_t, int32_t*);
    static const InvFn invs[6] = {bcrgj::inv_kernel<1>, bcrgj::inv_kernel<2>, bcrgj::inv_kernel<3>,
                                  bcrgj::inv_kernel<4>, bcrgj::inv_kernel<5>, bcrgj::inv_kernel<6>};
    // levels with at least this many odd blocks invert them once (inv_kernel),
    // before the products (SLAMHIP_GN_SPLIT_MIN=n selects it for A/B; 0 = never)
    static const int split_min = [] {
        const char* e = getenv("SLAMHIP_GN_SPLIT_MIN");
        return e ? atoi(e) : kGjSplitMin;
    }();
    static const OddFn odds[6] = {bcrgj::odd_kernel<1>, bcrgj::odd_kernel<2>, bcrgj::odd_kernel<3>,
                                  bcrgj::odd_kernel<4>, bcrgj::odd_kernel<5>, bcrgj::odd_kernel<6>};
    static const size_t lds1[6] = {bcrgj::Lds<1>::bytes, bcrgj::Lds<2>::bytes, bcrgj::Lds<3>::bytes,
                                   bcrgj::Lds<4>::bytes, bcrgj::Lds<5>::bytes, bcrgj::Lds<6>::bytes};
    static const size_t ldsm[6] = {bcrgj::Lds<1>::bytes_multi, bcrgj::Lds<2>::bytes_multi,
                                   bcrgj::Lds<3>::bytes_multi, bcrgj::Lds<4>::bytes_multi,
                                   bcrgj::Lds<5>::bytes_multi, bcrgj::Lds<6>::bytes_multi};
    static const size_t ldss[6] = {bcrgj::Lds<1>::bytes_schur, bcrgj::Lds<2>::bytes_schur,
                                   bcrgj::Lds<3>::bytes_schur, bcrgj::Lds<4>::bytes_schur,
                                   bcrgj::Lds<5>::bytes_schur, bcrgj::Lds<6>::bytes_schur};
    const size_t* lds = sc ? ldss : mct > 0 ? ldsm : lds1;
    static bool attrs = false;
    if (!attrs) {   // not a stream operation: the launch sequence stays graph-capturable
        for (int t = 0; t < 6; ++t) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(odds[t]), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(ldss[t]));
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(invs[t]), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(lds1[t]));
        }
        attrs = true;
    }
    const int T = Wb / 16;
    int lv = 0, last = 1;
    for (int s = 1; s < nb; s *= 2, ++lv) {
        const int n_odd = (nb - s + 2 * s - 1) / (2 * s);   // i = s, 3s, ... < nb
        const int n_even = (nb + 2 * s - 1) / (2 * s);      // j = 0, 2s, ... < nb
        double* Ec = (lv & 1) ? b.E1 : b.E0;
        double* En = (lv & 1) ? b.E0 : b.E1;
        // column tiles per workgroup (cpw), by a cost model of the measured phases
        // (inversion ~42k cycles, X / Y product ~6k, Sp + E' ~11k per column
        // tile) over the rounds of kBcrGjSlots resident workgroups.  (A third
        // workgroup set for E' beside Sp measured slower: 2,530 -> 2,395 it/s.)
        // (preinv: the inversion runs once per block before, a workgroup only stages G_i)
        const int preinv = split_min > 0 && n_odd >= split_min ? 1 : 0;
        int cpw = T;
        double best = 1e30;
        for (int c = 1; c <= T; ++c) {
            const int wgs = n_odd * (2 * ((T + c - 1) / c) + max(mct, 1));
            const int rounds = (wgs + kBcrGjSlots - 1) / kBcrGjSlots;
            const double est = rounds * ((preinv ? 4.0 : 42.0) + c * 17.0);
            if (est < best) {
                best = est;
                cpw = c;
            }
        }
        const int ng = (T + cpw - 1) / cpw;
        // + the combine workgroups of the blocks that stay even (j = 0, 2s, ...)
        const int n_comb = s > 1 ? n_even : 0;
        if (preinv)
            hipLaunchKernelGGL(invs[T - 1], dim3(n_odd), dim3(bcrgj::kThreads), lds1[T - 1], st, b.D, b.SP, b.SN, nb, s,
                               status);
        hipLaunchKernelGGL(odds[T - 1], dim3(n_odd + n_comb, max(2 * ng + max(mct, 1), bcrgj::kCombineSplit)),
                           dim3(bcrgj::kThreads), lds[T - 1], st, b.D, Ec, En, b.Xs, b.Ys, b.SP, b.SN, b.bz, b.SPb,
                           b.SNb, nb, s, cpw, n_odd, mc, status, sc ? b.bzo : nullptr, sc ? sc->pslot : nullptr,
                           sc ? sc->P : nullptr, preinv);
        last = s;
    }
    // block 0 (always even): the last level's Sp, then x_0
    using TopFn = void (*)(const double*, const double*, const double*, const double*, double*, int32_t, int32_t,
                           int32_t*);
    static const TopFn tops[6] = {bcrgj::top_kernel<1>, bcrgj::top_kernel<2>, bcrgj::top_kernel<3>,
                                  bcrgj::top_kernel<4>, bcrgj::top_kernel<5>, bcrgj::top_kernel<6>};
    static bool attrs_t = false;
    if (!attrs_t) {
        for (int t = 0; t < 6; ++t)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tops[t]), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(lds1[t] + sizeof(double) * 96 * 65));
        attrs_t = true;
    }
    if (sc) {   // block 0 + the border's Schur complement and x_b
        using TopSFn = void (*)(const double*, const double*, const double*, const double*, double*, int32_t, int32_t,
                                BcrSchur, int32_t*, int32_t*, int32_t);
        static const TopSFn topss[6] = {bcrgj::top_schur_kernel<1>, bcrgj::top_schur_kernel<2>,
                                        bcrgj::top_schur_kernel<3>, bcrgj::top_schur_kernel<4>,
                                        bcrgj::top_schur_kernel<5>, bcrgj::top_schur_kernel<6>};
        auto top_s_lds = [](int wb) {
            const int wc = wb > 32 ? wb : 32;
            return sizeof(double) * (static_cast<size_t>(wb) * (wb + 1) + static_cast<size_t>(wc) * 17 +
                                     2 * static_cast<size_t>(wb) * 33 + 2 * 32 * 33 + 64);
        };
        static bool attrs_s = false;
        if (!attrs_s) {
            for (int t = 0; t < 6; ++t)
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(topss[t]),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(top_s_lds(16 * (t + 1))));
            attrs_s = true;
        }
        hipLaunchKernelGGL(topss[T - 1], dim3(1), dim3(bcrgj::kThreads), top_s_lds(Wb), st, b.D, b.SP, b.bz, b.SPb,
                           b.x, nb > 1 ? last : 0, mc, *sc, status, b.ready, nb);
        return check_launch("gn bcr (explicit inverse, Schur border) kernels");
    }
    const size_t lds_top = lds1[T - 1] + (mct > 0 ? sizeof(double) * Wb * (mc + 1) : 0);
    hipLaunchKernelGGL(tops[T - 1], dim3(1), dim3(bcrgj::kThreads), lds_top, st, b.D, b.SP, b.bz, b.SPb, b.x,
                       nb > 1 ? last : 0, mc, status);
    return check_launch("gn bcr (explicit inverse) kernels");
}

// Back-substitution, level by level in reverse, after the top kernel wrote x_0.
int bcr_border_solve(const double* Z, const double* BR, const double* rhs, const int32_t* nbr_rows, int32_t n_nbr,
                     int32_t nv_band, int32_t nbd, int32_t nvt, int32_t mc, double* xb, int32_t* status,
                     hipStream_t st) {
    if (nbd < 1 || nbd > bcrgj::kBorderMax) return fail(SLAM_EINVAL, "gn: border of %d scalars", nbd);
    hipLaunchKernelGGL(bcrgj::border_solve_kernel, dim3(1), dim3(bcrgj::kThreads), 0, st, Z, BR, rhs, nbr_rows, n_nbr,
                       nv_band, nbd, nvt, mc, xb, status);
    return check_launch("gn border solve");
}

static int g_fused = [] {   // default on; SLAMHIP_GN_FUSED_BACK=0 turns it off
    const char* e = getenv("SLAMHIP_GN_FUSED_BACK");
    return e && e[0] == '0' ? 0 : 1;
}();
static uint32_t g_fused_wait = 20000000;   // 0.2 s of s_memrealtime ticks per wait
void bcr_gj_set_fused(int on) { g_fused = on ? 1 : 0; }
int bcr_gj_get_fused() { return g_fused; }
void bcr_gj_set_fused_wait(uint32_t ticks) { g_fused_wait = ticks; }

int bcr_gj_back(const BcrGjBufs& b, int32_t nv, int32_t Wb, int32_t mc, hipStream_t st, const BcrSchur* sc) {
    const int nb = (nv + Wb - 1) / Wb;
    // the XCD-local tagged hand-offs (every level in one launch; default since
    // round 5: 5,418-5,453 it/s against 5,385-5,388 with a launch per level,
    // profiles/r05_gn_ab_fused2.txt; the pose update fused into it as well was
    // slower, 5,244-5,306: each workgroup's scattered pose read-modify-write
    // holds its slot longer and delays the finer levels' dispatch); they rest
    // on the round-robin workgroup -> XCD dispatch: a violated
    // assumption times out (status 2; slamhip.gn re-runs the step with
    // bcr_gj_set_fused(0)), never a hang or a silent wrong answer.  The first
    // form (flags with agent-scope release / acquire across XCDs) was slower
    // than the launches (2,926-2,949 it/s, profiles/r05_gn_ab_schur.txt)
    if (sc && g_fused && nb > 1) {   // every level in one launch on one XCD (tagged granules)
        using BackXFn = void (*)(const double*, const double*, const double*, double*, const double*, int32_t, int32_t,
                                 int32_t, uint64_t*, uint32_t, int32_t*);
        static const BackXFn backxs[6] = {bcrgj::back_schur_xcd_kernel<1>, bcrgj::back_schur_xcd_kernel<2>,
                                          bcrgj::back_schur_xcd_kernel<3>, bcrgj::back_schur_xcd_kernel<4>,
                                          bcrgj::back_schur_xcd_kernel<5>, bcrgj::back_schur_xcd_kernel<6>};
        hipLaunchKernelGGL(backxs[Wb / 16 - 1], dim3(8 * (nb - 1)), dim3(bcrgj::kThreads), 0, st, b.Xs, b.Ys, b.bzo,
                           b.x, sc->xb, sc->nbd, nb, mc, b.xg, g_fused_wait, sc->status);
        return check_launch("gn bcr (explicit inverse, Schur border) XCD-local back-substitution");
    }
    if (sc) {   // one column: z_i[:, 0] - z_i[:, B] x_b
        using BackSFn = void (*)(const double*, const double*, const double*, double*, const double*, int32_t, int32_t,
                                 int32_t, int32_t);
        static const BackSFn backss[6] = {bcrgj::back_schur_kernel<1>, bcrgj::back_schur_kernel<2>,
                                          bcrgj::back_schur_kernel<3>, bcrgj::back_schur_kernel<4>,
                                          bcrgj::back_schur_kernel<5>, bcrgj::back_schur_kernel<6>};
        int s = 1;
        while (s < nb) s *= 2;
        for (s /= 2; s >= 1; s /= 2) {
            const int n_odd = (nb - s + 2 * s - 1) / (2 * s);
            hipLaunchKernelGGL(backss[Wb / 16 - 1], dim3(n_odd), dim3(bcrgj::kThreads), 0, st, b.Xs, b.Ys, b.bzo, b.x,
                               sc->xb, sc->nbd, nb, s, mc);
        }
        return check_launch("gn bcr (explicit inverse, Schur border) back-substitution");
    }
    using BackFn = void (*)(const double*, const double*, const double*, double*, int32_t, int32_t);
    static const BackFn backs[6] = {bcrgj::back_kernel<1>, bcrgj::back_kernel<2>, bcrgj::back_kernel<3>,
                                    bcrgj::back_kernel<4>, bcrgj::back_kernel<5>, bcrgj::back_kernel<6>};
    using BackMFn = void (*)(const double*, const double*, const double*, double*, int32_t, int32_t, int32_t);
    static const BackMFn backms[6] = {bcrgj::back_multi_kernel<1>, bcrgj::back_multi_kernel<2>,
                                      bcrgj::back_multi_kernel<3>, bcrgj::back_multi_kernel<4>,
                                      bcrgj::back_multi_kernel<5>, bcrgj::back_multi_kernel<6>};
    int s = 1;
    while (s < nb) s *= 2;
    for (s /= 2; s >= 1; s /= 2) {
        const int n_odd = (nb - s + 2 * s - 1) / (2 * s);
        if (mc > 1)
            hipLaunchKernelGGL(backms[Wb / 16 - 1], dim3(n_odd), dim3(bcrgj::kThreads), 0, st, b.Xs, b.Ys, b.bz, b.x,
                               nb, s, mc);
        else
            hipLaunchKernelGGL(backs[Wb / 16 - 1], dim3(n_odd), dim3(bcrgj::kThreads), 0, st, b.Xs, b.Ys, b.bz, b.x,
                               nb, s);
    }
    return check_launch("gn bcr (explicit inverse) back-substitution");
}

}  // namespace slamhip
