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
//                      within a step), sgd_irtw_kernel: 1 / (C[b+1] - C[a+1]) per
//                      edge; sgd_relax_kernel: ONE persistent wave (poses in
//                      LDS; a 256-thread workgroup when they are not) walks the
//                      loop edges in networkx order (each edge reads poses the
//                      previous edges moved — a true sequential dependency),
//                      ramps (a, b] by C differences and moves the tail i > b by
//                      beta through lazy per-block offsets.
//   recompute_pose_graph_orientation (:51-57)  orient_kernel.
//
// Rounding: the per-edge residual and the clamp are evaluated like the
// reference, d = 2 inv(R^T sigma R) r as (2 / sigma) r (exact for a rotation R;
// the reference's LAPACK inverse differs in the last bits); the ramp uses prefix-sum differences and the
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
// The relaxation workgroup: poses in LDS -> ONE wave (LDS operations of a wave
// complete in order: no barriers, no read-count protocol, and every LDS read of
// an edge's updates in flight at once); poses in global memory -> 256 threads
// with the workgroup protocol (512: 14.9 ms/step at C4, 256: 13.1, 128: 13.0
// before the one-wave path).
template <bool IN_LDS>
constexpr int relax_threads() {
    return IN_LDS ? 64 : 256;
}
constexpr int kRelaxSlots = 2;   // explicit nodes per thread with prefetched C values

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

// 1 / (C[b+1] - C[a+1]) per active edge (the ramp's reciprocal total weight;
// pose-independent within a step), off the relaxation's sequential chain.
__global__ void sgd_irtw_kernel(const int32_t* __restrict__ A, const int32_t* __restrict__ B,
                                const int32_t* __restrict__ Kp, const double* __restrict__ C, int32_t E,
                                double* __restrict__ RT) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E || k >= *Kp) return;
    const int a = A[k], b = B[k];
#pragma unroll
    for (int j = 0; j < 3; ++j) RT[3 * k + j] = 1.0 / (C[3 * (b + 1) + j] - C[3 * (a + 1) + j]);
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

// Diagnostics build (-DSLAM_SGD_STAMPS): thread 0's s_memtime cycles per phase
// of the relaxation loop summed over edges (tools/sgd_stamps.py).
#ifdef SLAM_SGD_STAMPS
__device__ unsigned long long g_sgd_stamps[8];
#define SGD_STAMP(q)                                                    \
    do {                                                                \
        if (threadIdx.x == 0) {                                         \
            const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
            acc_[q] += t1_ - t0_;                                       \
            t0_ = t1_;                                                  \
        }                                                               \
    } while (0)
#else
#define SGD_STAMP(q) \
    do {             \
    } while (0)
#endif

// Vector (vmcnt-counted) loads of uniform addresses: buffer loads through a
// descriptor of the array (the compiler turns plain uniform loads of
// read-only memory into scalar loads, which count on lgkmcnt).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t vrsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ int vld_i(__amdgpu_buffer_rsrc_t r, int i) {
    return static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(r, i * 4, 0, 0));
}
__device__ __forceinline__ double vld_d(__amdgpu_buffer_rsrc_t r, int i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, i * 8, 0, 0);
    return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(v[1]) << 32) | v[0]));
}

template <bool IN_LDS, int BR>
__global__ __launch_bounds__(relax_threads<IN_LDS>()) void sgd_relax_kernel(
    double* __restrict__ g_poses, int32_t N, const int32_t* A, const int32_t* B, const double* TF,
    const double* RT, const int32_t* __restrict__ Kp, const double* C, const double* __restrict__ gamma, double lr,
    double sigma, int32_t sh) {
    // The prefetch of A, B, TF and C goes through vld (vector loads counted by
    // vmcnt): as scalar loads (uniform addresses) they shared lgkmcnt with the
    // LDS traffic, so every LDS wait of an edge also waited for the next
    // edges' prefetch from memory.
    constexpr int kRelaxThreads = relax_threads<IN_LDS>();
    constexpr bool kOneWave = kRelaxThreads == 64;
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
    const double w2 = 2.0 / sigma;

    // explicit node t (a thread slot) of edge (a, b): the remainder of a's
    // block, then b's block (when different); -1 past them
    auto node_of = [&](int a, int b, int t) {
        const int ba = a >> sh, bb = b >> sh;
        const int n1 = min(N, (ba + 1) << sh) - (a + 1);
        const int n2 = bb > ba ? min(N, (bb + 1) << sh) - (bb << sh) : 0;
        return t < n1 ? a + 1 + t : (t < n1 + n2 ? (bb << sh) + (t - n1) : -1);
    };
    // Operands in three stages so that no load sits on the per-edge chain:
    // (a, b) of edge k + 2 are loaded during edge k; edge k + 1's transform and
    // C values (which need its a and b) are issued during edge k; edge k uses
    // what arrived meanwhile.
    const auto rA = vrsrc(A), rB = vrsrc(B), rTF = vrsrc(TF), rRT = vrsrc(RT), rC = vrsrc(C);
    struct Ops {
        int a, b, ni[kRelaxSlots];
        double z[9], ca[3], cb[3], irtw[3], ci[kRelaxSlots][3];
    };
    auto issue = [&](int k, int a, int b, Ops& q) {
        q.a = a;
        q.b = b;
#pragma unroll
        for (int t = 0; t < 9; ++t) q.z[t] = vld_d(rTF, 9 * k + t);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            q.ca[j] = vld_d(rC, 3 * (a + 1) + j);
            q.cb[j] = vld_d(rC, 3 * (b + 1) + j);
            q.irtw[j] = vld_d(rRT, 3 * k + j);
        }
#pragma unroll
        for (int u = 0; u < kRelaxSlots; ++u) {
            q.ni[u] = node_of(a, b, tid + u * kRelaxThreads);
            const int i0 = q.ni[u] >= 0 ? q.ni[u] : a;
#pragma unroll
            for (int j = 0; j < 3; ++j) q.ci[u][j] = vld_d(rC, 3 * (i0 + 1) + j);
        }
    };
    Ops cur, nxt;
    int an = 0, bn = 0;   // edge k + 1's (a, b)
    long long th_bits = 0;   // heading bits of the cached sin/cos (valid once th_set)
    bool th_set = false;
    double sn_c = 0.0, cs_c = 1.0;
    if (K > 0) {
        issue(0, A[0], B[0], cur);
        an = A[min(1, K - 1)];
        bn = B[min(1, K - 1)];
    }
#ifdef SLAM_SGD_STAMPS
    unsigned long long t0_ = __builtin_amdgcn_s_memtime();
    unsigned long long acc_[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (int k = 0; k < K; ++k) {
        // unconditional loads (indices clamped at the last edge): the compiler
        // then knows how many loads are younger than each operand and waits
        // only for that one, not for everything just issued (vmcnt(0))
        const int k2 = min(k + 2, K - 1);
        const int a2 = vld_i(rA, k2), b2 = vld_i(rB, k2);   // made uniform at the end of the edge
        issue(min(k + 1, K - 1), an, bn, nxt);
        const int a = cur.a, b = cur.b;
        const double(&irtw)[3] = cur.irtw;   // 1 / (C[b+1] - C[a+1]): sgd_irtw_kernel
        SGD_STAMP(0);

        const int ba = a >> sh, bb = b >> sh;
        // one wave: the reads of this edge's updates go out with the residual's
        // (nothing writes them before the updates below), so their latency hides
        // under the residual chain: a's block remainder and b's block (<=
        // kRelaxSlots nodes per lane; 2^(sh+1) = 128 = kRelaxSlots x 64 for
        // LDS-resident graphs), whole blocks (ba, nblk) in BR rounds
        double pv[kRelaxSlots][3], ov[BR][3], cv[BR][3];
        if constexpr (kOneWave) {
#pragma unroll
            for (int u = 0; u < kRelaxSlots; ++u) {
                const int i = cur.ni[u] >= 0 ? cur.ni[u] : a;
#pragma unroll
                for (int j = 0; j < 3; ++j) pv[u][j] = P[3 * i + j];
            }
#pragma unroll
            for (int r = 0; r < BR; ++r) {
                const int q = ba + 1 + tid + r * kRelaxThreads;
                const int qc = q < nblk ? q : ba;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    ov[r][j] = off[3 * qc + j];
                    cv[r][j] = cA[3 * qc + j];
                }
            }
        }

        // ---- residual (src/pose_graph_optimization.py:29-34), uniform -----------
        double pa[3], pb[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            pa[j] = P[3 * a + j] + off[3 * ba + j] + cA[3 * ba + j] * cur.ca[j];
            pb[j] = P[3 * b + j] + off[3 * bb + j] + cA[3 * bb + j] * cur.cb[j];
        }
        // construct_R(pg, a): sin/cos cached across edges of the same heading
        // bits (consecutive edges leaving one node: nothing moves node a between
        // them), so the cached values are the ones sincos would return
        if (!th_set || __double_as_longlong(pa[2]) != th_bits) {
            sincos(pa[2], &sn_c, &cs_c);
            th_bits = __double_as_longlong(pa[2]);
            th_set = true;
        }
        M3 R;
        R.a[0][0] = cs_c;  R.a[0][1] = -sn_c; R.a[0][2] = 0.0;
        R.a[1][0] = sn_c;  R.a[1][1] = cs_c;  R.a[1][2] = 0.0;
        R.a[2][0] = 0.0;   R.a[2][1] = 0.0;   R.a[2][2] = 1.0;
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
        // d = 2 inv(R^T sigma I R) r = (2 / sigma) r: R is a rotation, so the
        // inverse is I / sigma exactly; the reference's LAPACK inverse of the
        // rounded product differs from it in the last bits only (and beta is
        // clamped to r whenever 2 (b - a) lr > 1, e.g. always at lr = 1)
        double beta[3];
        const int L = b - a;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double dj = w2 * r[j];
            double bj = (static_cast<double>(L) * dj) * alpha[j];
            if (fabs(bj) > fabs(r[j])) bj = r[j];
            beta[j] = bj;
        }
        SGD_STAMP(1);
        // Several waves: every thread read P[a] and P[b] above, and node b is
        // one of this edge's explicit nodes, so its owner may not write it
        // before every wave has read it.  Each wave counts itself in after its
        // residual chain (which consumed the reads); only the owner of b waits
        // for the count (normally already complete).  Release (every lane's
        // reads of P before the count) / acquire (the owner's write of P[b]
        // after it), workgroup scope; with P in LDS the fence covers LDS only.
        // One wave: LDS operations of a wave complete in order, nothing to do.
        if constexpr (!kOneWave) {
            if constexpr (IN_LDS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if ((tid & 63) == 0) __hip_atomic_fetch_add(&rd_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const uint32_t rd_target = static_cast<uint32_t>(kRelaxThreads / 64) * static_cast<uint32_t>(k + 1);
        SGD_STAMP(2);
        if constexpr (kOneWave) {
            // ---- one wave: the writes of the values read above ----------------------
            SGD_STAMP(3);
#pragma unroll
            for (int u = 0; u < kRelaxSlots; ++u) {
                const int i = cur.ni[u];
                if (i >= 0) {
#pragma unroll
                    for (int j = 0; j < 3; ++j)
                        P[3 * i + j] = pv[u][j] + (i <= b ? beta[j] * ((cur.ci[u][j] - cur.ca[j]) * irtw[j]) : beta[j]);
                }
            }
#pragma unroll
            for (int r = 0; r < BR; ++r) {
                const int q = ba + 1 + tid + r * kRelaxThreads;
                if (q < bb) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const double g = beta[j] * irtw[j];
                        cA[3 * q + j] = cv[r][j] + g;
                        off[3 * q + j] = ov[r][j] - g * cur.ca[j];
                    }
                } else if (q > bb && q < nblk) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) off[3 * q + j] = ov[r][j] + beta[j];
                }
            }
        } else {
            // ---- explicit nodes (a's block remainder, b's block) ----------------------
            auto move = [&](int i, const double (&ci)[3]) {
                if constexpr (!kOneWave) {
                    if (i == b) {
                        while (__hip_atomic_load(&rd_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < rd_target)
                            __builtin_amdgcn_s_sleep(1);
                        if constexpr (IN_LDS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    }
                }
                if (i <= b) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) P[3 * i + j] += beta[j] * ((ci[j] - cur.ca[j]) * irtw[j]);
                } else {
#pragma unroll
                    for (int j = 0; j < 3; ++j) P[3 * i + j] += beta[j];
                }
            };
#pragma unroll
            for (int u = 0; u < kRelaxSlots; ++u)
                if (cur.ni[u] >= 0) move(cur.ni[u], cur.ci[u]);
            // more explicit nodes than prefetched slots only when 2^(sh+1) > kRelaxSlots * threads
            for (int t = tid + kRelaxSlots * kRelaxThreads; t < 2 * bs; t += kRelaxThreads) {
                const int i = node_of(a, b, t);
                if (i < 0) break;
                const double ci[3] = {C[3 * (i + 1)], C[3 * (i + 1) + 1], C[3 * (i + 1) + 2]};
                move(i, ci);
            }
            SGD_STAMP(3);
            // ---- whole blocks: ramp (ba, bb) as C coefficients, tail (bb, nblk) --------
            for (int q = ba + 1 + tid; q < nblk; q += kRelaxThreads) {
                if (q < bb) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const double g = beta[j] * irtw[j];
                        cA[3 * q + j] += g;
                        off[3 * q + j] -= g * cur.ca[j];
                    }
                } else if (q > bb) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) off[3 * q + j] += beta[j];
                }
            }
        }
        SGD_STAMP(4);
        if constexpr (!kOneWave) __syncthreads();
        SGD_STAMP(5);
        cur = nxt;
        an = __builtin_amdgcn_readfirstlane(a2);
        bn = __builtin_amdgcn_readfirstlane(b2);
    }
#ifdef SLAM_SGD_STAMPS
    if (threadIdx.x == 0)
        for (int q = 0; q < 6; ++q) g_sgd_stamps[q] += acc_[q];
#endif
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

// Diagnostics: copy (and clear) the relaxation's phase cycles; SLAM_EINVAL
// unless built with -DSLAM_SGD_STAMPS.
int slam_pgo_sgd_stamps(unsigned long long* out8) {
#ifdef SLAM_SGD_STAMPS
    if (!out8) return fail(SLAM_EINVAL, "sgd stamps: null");
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_sgd_stamps), 8 * sizeof(unsigned long long));
    unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sgd_stamps), z, sizeof(z));
    return ok();
#else
    (void)out8;
    return fail(SLAM_EINVAL, "sgd stamps: built without SLAM_SGD_STAMPS");
#endif
}

int64_t slam_pgo_sgd_work_size(int32_t N, int32_t E) {
    // doubles: invM (3N) | dw (3E) | gamma (4) | C (3N+3) | TF (9E) | RT (3E) | then int32: A, B, IDX (E each) | K
    return 3 * static_cast<int64_t>(N) + 3 * static_cast<int64_t>(E) + 4 + 3 * (static_cast<int64_t>(N) + 1) +
           12 * static_cast<int64_t>(E) + (3 * static_cast<int64_t>(E) + 2) / 2;
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
    double* RT = TF + 9 * static_cast<int64_t>(E);
    int32_t* A = reinterpret_cast<int32_t*>(RT + 3 * static_cast<int64_t>(E));
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
    hipLaunchKernelGGL(sgd_irtw_kernel, dim3((E + 255) / 256), dim3(256), 0, s, A, Bv, Kp, C, E, RT);
    // lazy-offset block size 2^sh: >= 64 nodes, at most kMaxOffBlocks blocks
    int sh = 6;
    while ((((N - 1) >> sh) + 1) > kMaxOffBlocks) ++sh;
    const size_t offb = 2 * 3 * static_cast<size_t>(((N - 1) >> sh) + 1) * sizeof(double);   // off + cA
    if (N <= kLdsPoses) {
        // one wave; whole-block updates in BR rounds of 64 (nblk <= 96 here)
        const size_t lds = offb + 3 * static_cast<size_t>(N) * sizeof(double);
        const int nblk = ((N - 1) >> sh) + 1;
        auto kern = nblk <= 64 ? sgd_relax_kernel<true, 1> : sgd_relax_kernel<true, 2>;
        static_assert(((kLdsPoses - 1) >> 6) + 1 <= 2 * 64, "BR = 2 covers every LDS-resident graph");
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds));
        hipLaunchKernelGGL(kern, dim3(1), dim3(relax_threads<true>()), lds, s, poses, N, A, Bv, TF, RT, Kp, C,
                           gamma, learning_rate, loop_closure_uncertainty, sh);
    } else {
        // off + cA reach 2 x 3 x 2048 doubles (96 KiB): above the 64 KiB default
        auto kern = sgd_relax_kernel<false, 1>;
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(offb));
        hipLaunchKernelGGL(kern, dim3(1), dim3(relax_threads<false>()), offb, s, poses, N, A, Bv, TF, RT, Kp, C,
                           gamma, learning_rate, loop_closure_uncertainty, sh);
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
