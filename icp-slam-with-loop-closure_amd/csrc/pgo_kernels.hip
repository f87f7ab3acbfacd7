// pgo_kernels.hip — SE(2) pose-graph relaxation kernels for gfx950 (MI355X).
//
// Rebuilds src/pose_graph_optimization.py (cohnt/ICP-SLAM-with-Loop-Closure):
//
//   pose_graph_optimization_step_sgd  (:7-49)
//     pass 1 (:13-24)  sgd_weights_kernel: M[i] = sum over loop edges e with
//                      a_e < i <= b_e of diag(W_e), accumulated in edge order
//                      (one thread per node, so every M[i] is the reference's
//                      sequential sum), W_e = inv(R sigma R^T); gamma = the
//                      first minimum-norm diag(W_e) (sgd_gamma_kernel).
//     pass 2 (:27-49)  sgd_prefix_kernel: prefix sums C of 1/M (pose-independent
//                      within a step); sgd_relax_kernel: ONE persistent workgroup
//                      walks the loop edges in networkx order (each edge reads
//                      poses the previous edges moved — a true sequential
//                      dependency), ramps (a, b] by C differences and moves the
//                      tail i > b by beta through lazy per-block offsets.
//   recompute_pose_graph_orientation (:51-57)  orient_kernel.
//
// Rounding: the per-edge residual, d = 2 inv(R^T sigma R) r and the clamp are
// evaluated like the reference; the ramp uses prefix-sum differences and the
// tail shifts are summed per block instead of the reference's left-to-right
// running sums, so poses agree to rounding (tests: 1e-9 on positions after 20
// steps of the reference's lap graph).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace slamhip {

struct M3 {
    double a[3][3];
};

// A @ B with the OpenBLAS dgemm FMA chain (see se2_mul).
__device__ __forceinline__ M3 m3_mul(const M3& x, const M3& y) {
    M3 z;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            z.a[i][j] = fma(x.a[i][2], y.a[2][j], fma(x.a[i][1], y.a[1][j], x.a[i][0] * y.a[0][j]));
    return z;
}

__device__ __forceinline__ M3 m3_transpose(const M3& x) {
    M3 z;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) z.a[i][j] = x.a[j][i];
    return z;
}

// Inverse by LU with partial pivoting (dgesv on the identity), enough for the
// well-conditioned R sigma R^T blocks here.
__device__ __forceinline__ M3 m3_inv(const M3& m) {
    double A[3][3], X[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            A[i][j] = m.a[i][j];
            X[i][j] = (i == j) ? 1.0 : 0.0;
        }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int p = k;
        for (int i = k + 1; i < 3; ++i)
            if (fabs(A[i][k]) > fabs(A[p][k])) p = i;
        if (p != k) {
            for (int j = 0; j < 3; ++j) {
                double t = A[k][j]; A[k][j] = A[p][j]; A[p][j] = t;
                t = X[k][j]; X[k][j] = X[p][j]; X[p][j] = t;
            }
        }
        for (int i = k + 1; i < 3; ++i) {
            const double l = A[i][k] / A[k][k];
            for (int j = k; j < 3; ++j) A[i][j] -= l * A[k][j];
            for (int j = 0; j < 3; ++j) X[i][j] -= l * X[k][j];
        }
    }
    M3 r;
    for (int j = 0; j < 3; ++j)
        for (int i = 2; i >= 0; --i) {
            double s = X[i][j];
            for (int k = i + 1; k < 3; ++k) s -= A[i][k] * r.a[k][j];
            r.a[i][j] = s / A[i][i];
        }
    return r;
}

// Closed-form 3x3 inverse (adjugate times one reciprocal of the determinant):
// the relaxation's dependent chain keeps one fp64 division instead of the
// nine of the pivoted LU (agrees with it to rounding; tests at 1e-9).
__device__ __forceinline__ M3 m3_inv_adj(const M3& m) {
    const double(&a)[3][3] = m.a;
    const double c00 = fma(a[1][1], a[2][2], -a[1][2] * a[2][1]);
    const double c01 = fma(a[1][2], a[2][0], -a[1][0] * a[2][2]);
    const double c02 = fma(a[1][0], a[2][1], -a[1][1] * a[2][0]);
    const double id = 1.0 / fma(a[0][0], c00, fma(a[0][1], c01, a[0][2] * c02));
    M3 r;
    r.a[0][0] = c00 * id;
    r.a[1][0] = c01 * id;
    r.a[2][0] = c02 * id;
    r.a[0][1] = fma(a[0][2], a[2][1], -a[0][1] * a[2][2]) * id;
    r.a[1][1] = fma(a[0][0], a[2][2], -a[0][2] * a[2][0]) * id;
    r.a[2][1] = fma(a[0][1], a[2][0], -a[0][0] * a[2][1]) * id;
    r.a[0][2] = fma(a[0][1], a[1][2], -a[0][2] * a[1][1]) * id;
    r.a[1][2] = fma(a[0][2], a[1][0], -a[0][0] * a[1][2]) * id;
    r.a[2][2] = fma(a[0][0], a[1][1], -a[0][1] * a[1][0]) * id;
    return r;
}

// construct_R (src/pose_graph_optimization.py:76-85)
__device__ __forceinline__ M3 rot_z(double theta) {
    double s, c;
    sincos(theta, &s, &c);
    M3 r;
    r.a[0][0] = c;   r.a[0][1] = -s;  r.a[0][2] = 0.0;
    r.a[1][0] = s;   r.a[1][1] = c;   r.a[1][2] = 0.0;
    r.a[2][0] = 0.0; r.a[2][1] = 0.0; r.a[2][2] = 1.0;
    return r;
}

__device__ __forceinline__ M3 diag3(double v) {
    M3 r;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) r.a[i][j] = (i == j) ? v : 0.0;
    return r;
}

__device__ __forceinline__ bool is_loop_edge(int a, int b) { return a - b != 1 && b - a != 1; }

// x mod 2 pi into [0, 2 pi) (Python's float %) without fmod's remainder loop:
// one floor, one fma and a one-step correction (agrees with the exact
// remainder to ~1e-16 |x|; tests at 1e-9).
__device__ __forceinline__ double py_mod_2pi(double x) {
    const double m = 2.0 * M_PI;
    double r = fma(-floor(x * (1.0 / m)), m, x);
    r = r < 0.0 ? r + m : r;
    return r >= m ? r - m : r;
}

// diag(inv(R sigma R^T)) of edge e (pass 1), 3 doubles per edge.
__global__ void sgd_dw_kernel(const double* __restrict__ poses, const int32_t* __restrict__ ea,
                              const int32_t* __restrict__ eb, int32_t E, double sigma,
                              double* __restrict__ dw) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const M3 R = rot_z(poses[3 * ea[e] + 2]);
    const M3 W = m3_inv(m3_mul(m3_mul(R, diag3(sigma)), m3_transpose(R)));
    dw[3 * e + 0] = W.a[0][0];
    dw[3 * e + 1] = W.a[1][1];
    dw[3 * e + 2] = W.a[2][2];
}

// gamma: first edge (networkx order) whose diag(W) has the smallest squared
// norm, among edges that touch at least one node (a < b).  One wave.
__global__ void sgd_gamma_kernel(const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
                                 int32_t E, const double* __restrict__ dw, double* __restrict__ gamma) {
    double bestv = INFINITY;
    int bestj = -1;
    for (int e = threadIdx.x; e < E; e += 64) {
        const int a = ea[e], b = eb[e];
        if (!is_loop_edge(a, b) || a >= b) continue;
        const double* w = dw + 3 * e;
        const double n2 = fma(w[2], w[2], fma(w[1], w[1], w[0] * w[0]));
        if (n2 < bestv) { bestv = n2; bestj = e; }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(bestv, off, 64);
        const int oj = __shfl_xor(bestj, off, 64);
        if (ov < bestv || (ov == bestv && oj >= 0 && (bestj < 0 || oj < bestj))) { bestv = ov; bestj = oj; }
    }
    if (threadIdx.x == 0) {
        for (int j = 0; j < 3; ++j) gamma[j] = bestj >= 0 ? dw[3 * bestj + j] : INFINITY;
    }
}

// M[i][j] in edge order; also 1/M for the relaxation pass.  One thread / node.
// Only loop edges with a < b cover any node (a < i <= b), i.e. exactly the
// compacted active list (sgd_compact_kernel, networkx order kept), so each
// node sums over K edges instead of all E, in the same order.
__global__ void sgd_weights_kernel(int32_t N, const int32_t* __restrict__ A, const int32_t* __restrict__ B,
                                   const int32_t* __restrict__ IDX, const int32_t* __restrict__ Kp,
                                   const double* __restrict__ dw, double* __restrict__ invM) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int K = *Kp;
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    for (int k = 0; k < K; ++k) {
        if (A[k] < i && i <= B[k]) {
            const double* w = dw + 3 * static_cast<int64_t>(IDX[k]);
            m0 = m0 + w[0];
            m1 = m1 + w[1];
            m2 = m2 + w[2];
        }
    }
    invM[3 * i + 0] = 1.0 / m0;
    invM[3 * i + 1] = 1.0 / m1;
    invM[3 * i + 2] = 1.0 / m2;
}

constexpr int kRelaxBlock = 512;
#ifndef SLAM_RELAX_THREADS
#define SLAM_RELAX_THREADS 256
#endif
constexpr int kRelaxThreads = SLAM_RELAX_THREADS;   // the relaxation workgroup: one wave per SIMD (512: 14.9 ms/step at C4, 256: 13.1, 128: 13.0)

// Inclusive prefix sums of 1/M per column: C[0] = 0, C[i+1] = C[i] + invM[i].
// One workgroup, chunked block scan (fixed order).  The relaxation then reads
// the ramp sum over (a, i] as C[i+1] - C[a+1] instead of scanning per edge.
__global__ __launch_bounds__(kRelaxBlock) void sgd_prefix_kernel(const double* __restrict__ invM, int32_t N,
                                                                 double* __restrict__ C) {
    constexpr int WAVES = kRelaxBlock / 64;
    __shared__ double red[WAVES][3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int chunk = (N + kRelaxBlock - 1) / kRelaxBlock;
    const int lo = tid * chunk, hi = min(lo + chunk, N);
    // 1/M is +inf for nodes no loop edge covers (M = 0); they lie in no ramp
    // range (a, b], so they contribute 0 to the prefix.
    auto w = [&](int i, int j) { const double v = invM[3 * i + j]; return isfinite(v) ? v : 0.0; };
    double loc[3] = {0.0, 0.0, 0.0};
    for (int i = lo; i < hi; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) loc[j] += w(i, j);
    double inc[3] = {loc[0], loc[1], loc[2]};
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double o = __shfl_up(inc[j], off, 64);
            if (lane >= off) inc[j] = o + inc[j];
        }
    if (lane == 63)
#pragma unroll
        for (int j = 0; j < 3; ++j) red[wave][j] = inc[j];
    __syncthreads();
    double run[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double w0 = 0.0;
        for (int q = 0; q < wave; ++q) w0 += red[q][j];
        run[j] = w0 + (inc[j] - loc[j]);
    }
    if (tid == 0)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[j] = 0.0;
    for (int i = lo; i < hi; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            run[j] += w(i, j);
            C[3 * (i + 1) + j] = run[j];
        }
}

// Active loop edges (|a - b| != 1 and a < b: the edges pass 2 applies) in
// networkx order, compacted into (A, B, TF) so the relaxation walks only them
// with one level of dependent loads.  One workgroup, ordered ballot compaction.
__global__ __launch_bounds__(1024) void sgd_compact_kernel(const int32_t* __restrict__ ea,
                                                           const int32_t* __restrict__ eb,
                                                           const double* __restrict__ tf, int32_t E,
                                                           int32_t* __restrict__ A, int32_t* __restrict__ B,
                                                           double* __restrict__ TF, int32_t* __restrict__ IDX,
                                                           int32_t* __restrict__ K) {
    __shared__ int wcount[16];
    __shared__ int base;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int e0 = 0; e0 < E; e0 += 1024) {
        const int e = e0 + tid;
        int a = 0, b = 0;
        bool act = false;
        if (e < E) {
            a = ea[e];
            b = eb[e];
            act = is_loop_edge(a, b) && a < b;
        }
        const uint64_t m = __ballot(act);
        const int pos_w = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                           __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
        if (lane == 0) wcount[wave] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wave; ++w) off += wcount[w];
        if (act) {
            const int k = off + pos_w;
            A[k] = a;
            B[k] = b;
            IDX[k] = e;
#pragma unroll
            for (int q = 0; q < 9; ++q) TF[9 * static_cast<int64_t>(k) + q] = tf[9 * static_cast<int64_t>(e) + q];
        }
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int w = 0; w < 16; ++w) t += wcount[w];
            base += t;
        }
        __syncthreads();
    }
    if (tid == 0) *K = base;
}

// Pass 2: one workgroup, sequential over the active loop edges.  Poses live in
// LDS when they fit (N <= kLdsPoses), otherwise in global memory (one CU:
// workgroup-scope barriers order them).  An edge (a, b) moves node i by
//   beta (C[i+1] - C[a+1]) / tw   for a < i <= b   (the ramp, C = prefix of 1/M)
//   beta                          for i > b        (the tail).
// Nodes are grouped in blocks of 2^sh; only the remainder of a's block and
// b's block are updated explicitly (<= 2^(sh+1) nodes, one per thread).  Whole
// blocks inside (a, b) take the ramp lazily as coefficients of C
// (cA[q] += beta/tw, off[q] -= beta C[a+1]/tw) and whole blocks after b the tail
// (off[q] += beta), so that a node's pose is
//   P[i] = stored[i] + off[q] + cA[q] C[i+1],   q = i >> sh,
// and an edge costs O(2^sh + N / 2^sh) parallel work and ONE barrier.
constexpr int kLdsPoses = 6144;
constexpr int kMaxOffBlocks = 2048;

template <bool IN_LDS>
__global__ __launch_bounds__(kRelaxThreads) void sgd_relax_kernel(
    double* __restrict__ g_poses, int32_t N, const int32_t* __restrict__ A, const int32_t* __restrict__ B,
    const double* __restrict__ TF, const int32_t* __restrict__ Kp, const double* __restrict__ C,
    const double* __restrict__ gamma, double lr, double sigma, int32_t sh) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nblk = ((N - 1) >> sh) + 1;
    double* off = reinterpret_cast<double*>(smem);                // [nblk][3] lazy offsets
    double* cA = off + 3 * nblk;                                  // [nblk][3] lazy ramp coefficients
    double* P = IN_LDS ? cA + 3 * nblk : g_poses;
    __shared__ uint32_t rd_count;   // waves done reading P[a], P[b] (all edges so far)
    const int tid = threadIdx.x;
    const int K = *Kp;
    const int bs = 1 << sh;
    if (tid == 0) rd_count = 0;

    for (int i = tid; i < 3 * nblk; i += kRelaxThreads) {
        off[i] = 0.0;
        cA[i] = 0.0;
    }
    if (IN_LDS) {
        for (int i = tid; i < 3 * N; i += kRelaxThreads) P[i] = g_poses[i];
    }
    __syncthreads();

    double alpha[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        alpha[j] = 1.0 / gamma[j];
        alpha[j] *= lr;
    }
    const M3 S = diag3(sigma);

    // explicit node of thread tid for edge (a, b): the remainder of a's block,
    // then b's block (when different); -1 when the thread has none
    auto explicit_node = [&](int a, int b) {
        const int ba = a >> sh, bb = b >> sh;
        const int n1 = min(N, (ba + 1) << sh) - (a + 1);
        const int n2 = bb > ba ? min(N, (bb + 1) << sh) - (bb << sh) : 0;
        return tid < n1 ? a + 1 + tid : (tid < n1 + n2 ? (bb << sh) + (tid - n1) : -1);
    };
    // Edge k's pose-independent operands are loaded during edge k-1.
    struct Pre {
        int a, b, ni;
        double z[9], ca[3], cb[3], ci[3], irtw[3];
    };
    auto fetch = [&](int k, Pre& q) {
        q.a = A[k];
        q.b = B[k];
#pragma unroll
        for (int t = 0; t < 9; ++t) q.z[t] = TF[9 * static_cast<int64_t>(k) + t];
        q.ni = explicit_node(q.a, q.b);
        const int i0 = q.ni >= 0 ? q.ni : q.a;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            q.ca[j] = C[3 * (q.a + 1) + j];
            q.cb[j] = C[3 * (q.b + 1) + j];
            q.ci[j] = C[3 * (i0 + 1) + j];
            q.irtw[j] = 1.0 / (q.cb[j] - q.ca[j]);   // pose-independent: off the dependent chain
        }
    };
    Pre cur, nxt;
    if (K > 0) fetch(0, cur);
    for (int k = 0; k < K; ++k) {
        if (k + 1 < K) fetch(k + 1, nxt);
        const int a = cur.a, b = cur.b;

        // ---- residual (src/pose_graph_optimization.py:29-34), uniform -----------
        const int ba = a >> sh, bb = b >> sh;
        double pa[3], pb[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            pa[j] = P[3 * a + j] + off[3 * ba + j] + cA[3 * ba + j] * cur.ca[j];
            pb[j] = P[3 * b + j] + off[3 * bb + j] + cA[3 * bb + j] * cur.cb[j];
        }
        const M3 R = rot_z(pa[2]);                // construct_R(pg, a)
        M3 Pa = R;                                // utils.pose_to_mat(poses[a])
        Pa.a[0][2] = pa[0];
        Pa.a[1][2] = pa[1];
        M3 Z;
#pragma unroll
        for (int t = 0; t < 9; ++t) Z.a[t / 3][t % 3] = cur.z[t];
        const M3 Pb = m3_mul(Pa, Z);
        double r[3];
        r[0] = Pb.a[0][2] - pb[0];
        r[1] = Pb.a[1][2] - pb[1];
        r[2] = py_mod_2pi(atan2(Pb.a[1][0], Pb.a[0][0]) - pb[2]);
        const M3 Wi = m3_inv_adj(m3_mul(m3_mul(m3_transpose(R), S), R));
        double beta[3];
        const int L = b - a;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const M3& w = Wi;
            const double dj = fma(2.0 * w.a[j][2], r[2], fma(2.0 * w.a[j][1], r[1], (2.0 * w.a[j][0]) * r[0]));
            double bj = (static_cast<double>(L) * dj) * alpha[j];
            if (fabs(bj) > fabs(r[j])) bj = r[j];
            beta[j] = bj;
        }
        // Every thread read P[a] and P[b] above, and node b is one of this
        // edge's explicit nodes: its owner may not write it before every wave
        // has read it.  Each wave counts itself in after its residual chain
        // (which consumed the reads); only the owner of b waits for the count
        // (normally already complete), the other threads go on.  Release (every
        // lane's reads of P ordered before the count) / acquire (the owner's
        // write of P[b] ordered after it), workgroup scope; with P in LDS the
        // fence covers LDS only (it does not wait for the next edge's
        // prefetched global operands)
        if constexpr (IN_LDS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if ((tid & 63) == 0) __hip_atomic_fetch_add(&rd_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t rd_target = static_cast<uint32_t>(kRelaxThreads / 64) * static_cast<uint32_t>(k + 1);
        // ---- explicit nodes (a's block remainder, b's block) ----------------------
        {
            int i = cur.ni;
            int t = tid;
            double cij[3] = {cur.ci[0], cur.ci[1], cur.ci[2]};
            while (i >= 0) {
                if (i == b) {
                    while (__hip_atomic_load(&rd_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < rd_target)
                        __builtin_amdgcn_s_sleep(1);
                    if constexpr (IN_LDS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
                if (i <= b) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) P[3 * i + j] += beta[j] * ((cij[j] - cur.ca[j]) * cur.irtw[j]);
                } else {
#pragma unroll
                    for (int j = 0; j < 3; ++j) P[3 * i + j] += beta[j];
                }
                t += kRelaxThreads;   // more than one explicit node per thread only when 2^(sh+1) > block
                if (t >= 2 * bs) break;
                const int n1 = min(N, (ba + 1) << sh) - (a + 1);
                const int n2 = bb > ba ? min(N, (bb + 1) << sh) - (bb << sh) : 0;
                i = t < n1 ? a + 1 + t : (t < n1 + n2 ? (bb << sh) + (t - n1) : -1);
                if (i >= 0)
#pragma unroll
                    for (int j = 0; j < 3; ++j) cij[j] = C[3 * (i + 1) + j];
            }
        }
        // ---- whole blocks: ramp (ba, bb) as C coefficients, tail (bb, nblk) --------
        for (int q = ba + 1 + tid; q < nblk; q += kRelaxThreads) {
            if (q < bb) {
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const double g = beta[j] * cur.irtw[j];
                    cA[3 * q + j] += g;
                    off[3 * q + j] -= g * cur.ca[j];
                }
            } else if (q > bb) {
#pragma unroll
                for (int j = 0; j < 3; ++j) off[3 * q + j] += beta[j];
            }
        }
        __syncthreads();
        cur = nxt;
    }
    // fold the lazy terms back
    for (int i = tid; i < N; i += kRelaxThreads) {
        const int q = i >> sh;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double v = P[3 * i + j] + off[3 * q + j] + cA[3 * q + j] * C[3 * (i + 1) + j];
            if (IN_LDS) g_poses[3 * i + j] = v; else P[3 * i + j] = v;
        }
    }
}

// First loop of recompute_pose_graph_orientation: theta_i from the unit
// direction to the next pose, i = 1 .. N-2.  Reads columns 0-1, writes 2.
__global__ void orient_kernel(double* __restrict__ poses, int32_t N) {
    const int i = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N - 1) return;
    double vx = poses[3 * (i + 1)] - poses[3 * i];
    double vy = poses[3 * (i + 1) + 1] - poses[3 * i + 1];
    const double n = sqrt(fma(vy, vy, vx * vx));
    if (n > 0.0) {
        vx = vx / n;
        vy = vy / n;
        poses[3 * i + 2] = atan2(vy, vx);
    }
}

// Second half of recompute_pose_graph_orientation (:68-74) with icp_recompute:
// the reverse-order loop theta_i = theta_{i-1} + atan2(T_i[1,0], T_i[0,0])
// reads theta_{i-1} BEFORE its own update, so every node is independent.
// tf holds the N-1 rotation-only ICP results of pairs (i, i-1), i = 1..N-1.
__global__ void copy_theta_kernel(const double* __restrict__ poses, int32_t N, double* __restrict__ th) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) th[i] = poses[3 * i + 2];
}

__global__ void apply_theta_kernel(double* __restrict__ poses, int32_t N, const double* __restrict__ th,
                                   const double* __restrict__ tf) {
    const int i = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double* t = tf + 9 * static_cast<int64_t>(i - 1);
    poses[3 * i + 2] = th[i - 1] + atan2(t[3], t[0]);
}

}  // namespace slamhip

using namespace slamhip;

extern "C" {

int64_t slam_pgo_sgd_work_size(int32_t N, int32_t E) {
    // doubles: invM (3N) | dw (3E) | gamma (4) | C (3N+3) | TF (9E) | then int32: A, B, IDX (E each) | K
    return 3 * static_cast<int64_t>(N) + 3 * static_cast<int64_t>(E) + 4 + 3 * (static_cast<int64_t>(N) + 1) +
           9 * static_cast<int64_t>(E) + (3 * static_cast<int64_t>(E) + 2) / 2;
}

int slam_pgo_sgd_step_f64(double* poses, int32_t N, const int32_t* ea, const int32_t* eb,
                          const double* tf, int32_t E, double learning_rate,
                          double loop_closure_uncertainty, double* work, void* stream) {
    if (N < 0 || E < 0) return fail(SLAM_EINVAL, "sgd: N=%d E=%d", N, E);
    if (N == 0 || E == 0) return ok();
    if (!poses || !ea || !eb || !tf || !work) return fail(SLAM_EINVAL, "sgd: null array argument");
    hipStream_t s = as_stream(stream);
    double* invM = work;
    double* dw = work + 3 * static_cast<int64_t>(N);
    double* gamma = dw + 3 * static_cast<int64_t>(E);
    double* C = gamma + 4;
    double* TF = C + 3 * (static_cast<int64_t>(N) + 1);
    int32_t* A = reinterpret_cast<int32_t*>(TF + 9 * static_cast<int64_t>(E));
    int32_t* Bv = A + E;
    int32_t* IDX = Bv + E;
    int32_t* Kp = IDX + E;
    hipLaunchKernelGGL(sgd_dw_kernel, dim3((E + 255) / 256), dim3(256), 0, s, poses, ea, eb, E,
                       loop_closure_uncertainty, dw);
    hipLaunchKernelGGL(sgd_gamma_kernel, dim3(1), dim3(64), 0, s, ea, eb, E, dw, gamma);
    hipLaunchKernelGGL(sgd_compact_kernel, dim3(1), dim3(1024), 0, s, ea, eb, tf, E, A, Bv, TF, IDX, Kp);
    hipLaunchKernelGGL(sgd_weights_kernel, dim3((N + 127) / 128), dim3(128), 0, s, N, A, Bv, IDX, Kp, dw,
                       invM);
    hipLaunchKernelGGL(sgd_prefix_kernel, dim3(1), dim3(kRelaxBlock), 0, s, invM, N, C);
    // lazy-offset block size 2^sh: >= 64 nodes, at most kMaxOffBlocks blocks
    int sh = 6;
    while ((((N - 1) >> sh) + 1) > kMaxOffBlocks) ++sh;
    const size_t offb = 2 * 3 * static_cast<size_t>(((N - 1) >> sh) + 1) * sizeof(double);   // off + cA
    if (N <= kLdsPoses) {
        const size_t lds = offb + 3 * static_cast<size_t>(N) * sizeof(double);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(sgd_relax_kernel<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        hipLaunchKernelGGL(sgd_relax_kernel<true>, dim3(1), dim3(kRelaxThreads), lds, s, poses, N, A, Bv, TF,
                           Kp, C, gamma, learning_rate, loop_closure_uncertainty, sh);
    } else {
        // off + cA reach 2 x 3 x 2048 doubles (96 KiB): above the 64 KiB default
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(sgd_relax_kernel<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(offb));
        hipLaunchKernelGGL(sgd_relax_kernel<false>, dim3(1), dim3(kRelaxThreads), offb, s, poses, N, A, Bv,
                           TF, Kp, C, gamma, learning_rate, loop_closure_uncertainty, sh);
    }
    return check_launch("pgo sgd kernels");
}

// Second half of recompute_pose_graph_orientation (:68-74) with icp_recompute:
// the reverse-order loop theta_i = theta_{i-1} + atan2(T_i[1,0], T_i[0,0])
// reads theta_{i-1} BEFORE its own update, so every node is independent once
// the old thetas are snapshotted (work: N doubles).
int slam_pgo_orient_from_tf_f64(double* poses, int32_t N, const double* tf, double* work, void* stream) {
    if (N < 2) return ok();
    if (!poses || !tf || !work) return fail(SLAM_EINVAL, "orient_from_tf: null array");
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(copy_theta_kernel, dim3((N + 255) / 256), dim3(256), 0, s, poses, N, work);
    hipLaunchKernelGGL(apply_theta_kernel, dim3((N - 1 + 255) / 256), dim3(256), 0, s, poses, N, work, tf);
    return check_launch("pgo orient_from_tf kernels");
}

int slam_pgo_orient_f64(double* poses, int32_t N, void* stream) {
    if (N < 3) return ok();
    if (!poses) return fail(SLAM_EINVAL, "orient: null poses");
    hipLaunchKernelGGL(orient_kernel, dim3((N - 2 + 255) / 256), dim3(256), 0, as_stream(stream), poses, N);
    return check_launch("pgo orient kernel");
}

}  // extern "C"
