// icp_kernels.hip — batched 2-D point-to-point ICP for gfx950 (MI355X).
//
// Rebuilds the hot path of the reference's src/icp.py (cohnt/ICP-SLAM-with-
// Loop-Closure) as one fused kernel: ONE scan pair per workgroup, every ICP
// iteration on chip, transform history streamed out.
//
//   reference                               here
//   src/icp.py:62   np.dot(T, pc1.T).T      transform_queries(): FMA chain in
//                                           OpenBLAS dgemm order (bit-equal)
//   src/icp.py:4-19 get_correspondences     exact fp64 argmin (dx*dx + dy*dy, no
//                                           contraction, np.argmin first-minimum
//                                           rule), found by an fp32 screen with
//                                           exact pruning (nn_window_pruned) and
//                                           certified in fp64 (certify), or by the
//                                           exhaustive fp64 scan (nn_scan_f64);
//                                           pc2 resident in LDS
//   src/icp.py:22-46 get_transform          two deterministic block reductions
//                                           (centroids, then the centred 2x2
//                                           cross-covariance) + closed-form 2x2
//                                           Kabsch (argmax_R tr(R S))
//   src/icp.py:49-52 get_error              sum of the per-query minima
//   src/icp.py:72-97 icp() loop             stopping rules evaluated on chip,
//                                           identically by every thread
//
// Compile with -ffp-contract=off: the distance must round exactly like NumPy.
// MFMA is deliberately not used: the work is a min-search, not a contraction;
// the kernel is VALU-issue / latency bound (DESIGN.md §3.1 Roofline).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace slamhip {

constexpr int kCandCap = 4096;
constexpr size_t kMaxLds = 160 * 1024;      // LDS per workgroup (gfx950)
constexpr int32_t kBadBounds = INT32_MIN;   // out_iters of a pair outside the launch's bounds
__device__ int g_icp_status;                // nonzero: some pair was outside its launch's bounds
// two reduction slabs of 16 doubles per wave at the front of the dynamic LDS
// (block_sum_exact16, alternating between iterations), then 16 doubles of
// per-pair constants (kept in LDS, not in registers across the NN search)
constexpr int kPairConsts = 42;   // 12 pair constants, then kBcast: the gang exchange's broadcast slab (16 sums + the
                                  // arrival flag), then kKab: the update wave 0 hands to the others and the drain
                                  // flag (an even count keeps the candidates 16-byte aligned)
__host__ __device__ constexpr int red_doubles(int block) { return 2 * (block / 64) * 16 + kPairConsts; }
enum PairConst { kPcX, kPcY, kDpX, kDpY, kMupX, kMupY, kGm1, kGm2, kGs1, kGs2, kPmax, kCmax, kPh0, kPhS, kDrainAt,
                 kBcast = 16, kKab = 34 };

struct IcpArgs {
    const double2* pts;
    const int64_t* scan_off;
    const int32_t* src_scan;
    const int32_t* dst_scan;
    const double* init;
    double epsilon;
    double stopping_thresh;
    int32_t max_iters;
    int32_t rotation_only;
    int32_t cand_cap;       // LDS candidate capacity for this launch (points)
    int32_t hist_stride;
    double* out_hist;
    double* out_tf;
    double* out_err;
    int32_t* out_iters;
    // single-step mode
    int64_t* out_corr;
    const int64_t* corr_off;
    // diagnostics: per-phase s_memtime totals of workgroup 0 (NULL = off)
    unsigned long long* stamps;
    // diagnostics: total candidate evaluations performed, all lanes (NULL = off)
    unsigned long long* evals;
    // diagnostics: per pair and phase (resume 0 / 1) the s_memrealtime (100 MHz)
    // at which its (part-0) workgroup started and ended, and the XCC / SE / CU
    // it ran on: trace[(b * 2 + resume) * 4 + {0: start, 1: end, 2: hw id}] (NULL = off)
    unsigned long long* trace;
    // phased scheduling (batch mode): workgroup -> pair map (NULL = identity),
    // iterations per pair in this launch (0 = to completion), resume from the
    // state a previous phase saved in out_tf / out_err / out_iters, and the
    // per-pair sort key written at a pause
    const int32_t* order;
    int32_t phase_cap;
    int32_t resume;
    float* sched_key;
    // gangs (GANG kernels only): a pair's query groups dealt over `gang`
    // workgroups on one XCD that exchange their per-iteration partial sums
    // through gang_slots; n_gangs pairs
    int32_t gang;
    int32_t n_gangs;
    uint64_t* gang_slots;    // [n_gangs][2][gang][32] tagged granules, zeroed before the launch
    uint32_t gang_wait;      // longest wait for the partners of one exchange (s_memrealtime ticks)
    uint32_t gang_wait_first;   // the same for a launch's FIRST exchange of a pair (partners not resident)
    // a word the launch's parts share (zeroed before it; NULL: none): the first
    // part that times out at its first exchange sets it, and every part still
    // waiting at, or later reaching, its own first exchange stops at once
    uint32_t* gang_abort;
    // PRUNE kernels, scheduler phases: a paused pair's search state (per query
    // i: last match and clearance word at qsave[b * qsave_stride + i]; the
    // motion T_next - T and its slack at dtsave[b * 8 + ..]) so that its resumed
    // iteration is as warm as an uninterrupted one (NULL: resume cold)
    uint2* qsave;
    float* dtsave;
    int32_t qsave_stride;
    // launch order -> pair, XCD-aware (0: identity): runs of xcd_run
    // consecutive pairs go to one XCD (round-robin dispatch: workgroup bx runs
    // on XCD bx % 8), so consecutive pairs, which share a scan (pc1 of pair i
    // is pc2 of pair i + 1), stage it through the same L2; the runs rotate
    // over the XCDs, so a stretch of slow pairs still spreads over the chip
    int32_t xcd_run;
    int32_t n_pairs;   // pairs of the launch (the XCD-aware map's bound)
    // angle pre-tier (launch_batch): slots below *skip_lt of an ordered launch
    // belong to pairs another tier runs (NULL: none); an order entry < 0 is
    // padding (both: the workgroup leaves at once)
    const int32_t* skip_lt;
    const int32_t* take_lt;   // the pre-tier's launch: slots at or past *take_lt leave at once (NULL: none)
    // drain (phase 2's bulk launch, launch_batch): *drain counts the launch's
    // pairs that stopped (finished or paused); once at most drain_x of its
    // *drain_n - drain_skip pairs have not, each pair pauses at the end of its
    // iteration (those running and any still to start: at most drain_x) and
    // the drain tier (wide workgroups) finishes them (NULL: off)
    uint32_t* drain;
    const int32_t* drain_n;
    int32_t drain_skip;
    int32_t drain_x;
};
constexpr int kGangMax = 17;          // parts per gang (1081-point scans: 17 groups of 64)
#ifndef SLAM_TAIL_SHARE
#define SLAM_TAIL_SHARE 1
#endif
constexpr size_t kTailShare = SLAM_TAIL_SHARE;   // gang / team workgroups per CU (LDS requested: kMaxLds / share)
constexpr int kGangSweep = 32;        // parts an exchange sweep covers (16 loads per lane)
// A gang exchange waits at most this many s_memrealtime ticks (100 MHz) for its
// partners; a part that times out stops at once (the timeout is sticky: it
// never waits again), writes nothing, and the pair is re-run from its saved
// phase-1 state on one workgroup after the phase (launch_batch's repair launch)
constexpr uint32_t kGangWaitTicks = 20000000;   // 0.2 s
__device__ int g_gang_timeout;        // parts that timed out (read-and-cleared by slam_icp_gang_timeouts)

// A wave-uniform double moved to SGPRs (v_readfirstlane of both halves).
__device__ __forceinline__ double uniform_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xffffffff));
    const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(b >> 32));
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Lane src's double, in every lane (src wave-uniform).
__device__ __forceinline__ double bcast_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), src);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

__device__ __forceinline__ float uniform_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// Bare v_sqrt_f32 (about 1 ulp), without the ~15-instruction IEEE rounding
// fix-up sqrtf compiles to.  Every use below takes a bound with a relative
// slack of >= 1e-6 (>> 1 ulp); a denormal input may flush to 0, which only
// loosens a lower bound, and the certification's upper bound adds 1e-30 first.
__device__ __forceinline__ float sqrt_bound(float x) { return __builtin_amdgcn_sqrtf(x); }

// Squared distance with NumPy's rounding: sum((pc2[j] - q)**2) over x, y (+0).
__device__ __forceinline__ double exact_d2(double px, double py, double qx, double qy) {
    const double dx = px - qx;
    const double dy = py - qy;
    return dx * dx + dy * dy;   // -ffp-contract=off: two roundings, then the add
}

// Exhaustive first-minimum nearest neighbour of QPT queries per lane against
// `cnt` fp64 candidates in LDS (all lanes read the same candidate: broadcast).
template <int QPT>
__device__ __forceinline__ void nn_scan_f64(const double2* __restrict__ cand, int cnt, int base,
                                            const double (&qx)[QPT], const double (&qy)[QPT],
                                            double (&best)[QPT], int (&bi)[QPT]) {
#pragma unroll 2
    for (int j = 0; j < cnt; ++j) {
        const double2 p = cand[j];
        const int jj = base + j;
#pragma unroll
        for (int k = 0; k < QPT; ++k) {
            const double d = exact_d2(p.x, p.y, qx[k], qy[k]);
            const bool lt = d < best[k];
            best[k] = lt ? d : best[k];
            bi[k] = lt ? jj : bi[k];
        }
    }
}

// fp32 screen, chunked: candidates are visited in chunks of kChunk; per
// query only the chunk minimum is tracked inside a chunk (4 fp32 ops + half a
// v_min3 per candidate), and across chunks the smallest chunk minimum (M1, in
// chunk C1) and the second smallest (M2).  The winning chunk is re-scanned
// afterwards for the index and the in-chunk runner-up.  Candidates are padded
// to a multiple of kChunk with far sentinels (d32 = +inf).
constexpr int kChunk = 32;
constexpr float kSentinel = 3.0e19f;

__device__ __forceinline__ float screen_d32(float px, float py, float qx, float qy) {
    const float dx = px - qx;
    const float dy = py - qy;
    return fmaf(dy, dy, dx * dx);
}

// fp32 candidates are stored as pairs (x_2p, x_2p+1, y_2p, y_2p+1): one float4
// read gives two candidates whose distances to a query are three packed ops
// (v_pk_add x2, v_pk_mul, v_pk_fma) — per element exactly screen_d32.
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 cf_at(const float2* candf, int j) {
    const float* f = reinterpret_cast<const float*>(candf) + 4 * (j >> 1) + (j & 1);
    return make_float2(f[0], f[2]);
}
__device__ __forceinline__ void cf_put(float2* candf, int j, float x, float y) {
    float* f = reinterpret_cast<float*>(candf) + 4 * (j >> 1) + (j & 1);
    f[0] = x;
    f[2] = y;
}
__device__ __forceinline__ f32x2v screen_pair(const float4& p, float qx, float qy) {
    const f32x2v dx = f32x2v{p.x, p.y} - qx;
    const f32x2v dy = f32x2v{p.z, p.w} - qy;
    return __builtin_elementwise_fma(dy, dy, dx * dx);
}

template <int QPT>
__device__ __forceinline__ void nn_scan_chunked(const float2* __restrict__ candf, int n_pad,
                                                const float (&qx)[QPT], const float (&qy)[QPT],
                                                float (&M1)[QPT], float (&M2)[QPT], int (&C1)[QPT]) {
    for (int c0 = 0; c0 < n_pad; c0 += kChunk) {
        float cm[QPT];
#pragma unroll
        for (int k = 0; k < QPT; ++k) cm[k] = INFINITY;
#pragma unroll 4
        for (int j = c0; j < c0 + kChunk; ++j) {
            const float2 p = cf_at(candf, j);
#pragma unroll
            for (int k = 0; k < QPT; ++k) cm[k] = fminf(cm[k], screen_d32(p.x, p.y, qx[k], qy[k]));
        }
#pragma unroll
        for (int k = 0; k < QPT; ++k) {
            const bool lt = cm[k] < M1[k];
            M2[k] = __builtin_amdgcn_fmed3f(M1[k], M2[k], cm[k]);   // M1 <= M2
            C1[k] = lt ? c0 : C1[k];
            M1[k] = fminf(M1[k], cm[k]);
        }
    }
}

// Diagnostics trace (IcpArgs::trace): the hardware location of this wave,
// XCC id << 16 | HW_ID (CU, SH, SE bits).
__device__ __forceinline__ unsigned long long hw_where() {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));        // HW_REG_HW_ID, all 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));      // HW_REG_XCC_ID, 16 bits
    return (static_cast<unsigned long long>(xcc & 0xf) << 32) | hw;
}
__device__ __forceinline__ void trace_mark(const IcpArgs& a, int b, int what) {
    if (a.trace) {
        unsigned long long* t = a.trace + (static_cast<int64_t>(b) * 2 + (a.resume ? 1 : 0)) * 4;
        t[what] = __builtin_amdgcn_s_memrealtime();
        if (what == 0) t[2] = hw_where();   // slot 2: where; slot 3: staging done
    }
}

// Wave-wide min / max / or without LDS or SGPR round trips: DPP butterflies
// inside each 16-lane row, then the gfx950 row swaps (v_permlane16_swap pairs
// rows 0-1 and 2-3, v_permlane32_swap the two halves).  Every lane returns the
// result.
// Min / max run on integers: a float's bits map to an int of the same order
// (sign-magnitude -> two's complement, an involution), and non-negative floats
// order as their unsigned bits.  An integer min takes the DPP operand directly
// (v_min_i32_dpp, bound_ctrl: one instruction per step), where fminf would
// canonicalise both operands first (IEEE mode) behind a separate DPP move.
__device__ __forceinline__ int f2ord(float f) {
    const int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float ord2f(int o) { return __int_as_float(o ^ ((o >> 31) & 0x7fffffff)); }
#define SLAM_DPPI(v, ctrl) __builtin_amdgcn_mov_dpp((v), (ctrl), 0xF, 0xF, true)
template <typename I, typename Op>
__device__ __forceinline__ I wave_reduce_i(I v, Op op) {
    v = op(v, static_cast<I>(SLAM_DPPI(static_cast<int>(v), 0xB1)));    // quad_perm [1,0,3,2]
    v = op(v, static_cast<I>(SLAM_DPPI(static_cast<int>(v), 0x4E)));    // quad_perm [2,3,0,1]
    v = op(v, static_cast<I>(SLAM_DPPI(static_cast<int>(v), 0x124)));   // row_ror:4
    v = op(v, static_cast<I>(SLAM_DPPI(static_cast<int>(v), 0x128)));   // row_ror:8
    const auto p = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(v), static_cast<uint32_t>(v), false, false);
    v = op(static_cast<I>(p[0]), static_cast<I>(p[1]));
    const auto q = __builtin_amdgcn_permlane32_swap(static_cast<uint32_t>(v), static_cast<uint32_t>(v), false, false);
    return op(static_cast<I>(q[0]), static_cast<I>(q[1]));
}
#undef SLAM_DPPI
struct MinI { __device__ int operator()(int a, int b) const { return min(a, b); } };
struct MaxI { __device__ int operator()(int a, int b) const { return max(a, b); } };
struct MinU { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return min(a, b); } };
struct MaxU { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return max(a, b); } };
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// two independent 16-bit maxima in one word (v_pk_max_u16)
struct MaxPk16 {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const {
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
    }
};
// every lane returns the wave's min / max (no NaN inputs)
__device__ __forceinline__ float wave_min_f(float v) { return ord2f(wave_reduce_i<int>(f2ord(v), MinI())); }
__device__ __forceinline__ float wave_max_f(float v) { return ord2f(wave_reduce_i<int>(f2ord(v), MaxI())); }
// the same for v >= 0 (or +inf)
__device__ __forceinline__ float wave_min_nn(float v) {
    return __uint_as_float(wave_reduce_i<uint32_t>(__float_as_uint(v), MinU()));
}
__device__ __forceinline__ float wave_max_nn(float v) {
    return __uint_as_float(wave_reduce_i<uint32_t>(__float_as_uint(v), MaxU()));
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));
    v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));
    v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x124, 0xF, 0xF, false));
    v |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x128, 0xF, 0xF, false));
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = p[0] | p[1];
    const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    // wave-uniform by construction: move to an SGPR for the scalar loop over its bits
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(q[0] | q[1])));
}

// Conservative squared distance between two axis-aligned boxes (or a point,
// as a degenerate box), rounded DOWN by 1e-6 relative: a lower bound of every
// fp32 screened distance between their points (>> the ~16 u of rounding).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float box_lb(f32x2 alo, f32x2 ahi, const float4& b) {
    const f32x2 d0 = f32x2{b.x, b.y} - ahi;   // box b = (x0, y0, x1, y1): v_pk_add_f32
    const f32x2 d1 = alo - f32x2{b.z, b.w};
    const float ddx = fmaxf(fmaxf(d0.x, d1.x), 0.0f);
    const float ddy = fmaxf(fmaxf(d0.y, d1.y), 0.0f);
    return fmaf(ddy, ddy, ddx * ddx) * (1.0f - 1e-6f);
}

// Exact pruned screen (PRUNE).  Each lane tracks, for its query, the smallest
// fp32 screened distance M1 with its FIRST index J1 and the second smallest M2
// over all other candidates — exactly what the full screen yields — while
// skipping candidates that provably cannot change them:
//   1. window: the kWin sub-chunks (of kSub candidates) around the lane's
//      predicted match (last iteration's match) are scanned in full, the QPT
//      queries interleaved for ILP;
//   2. clearance: a query whose window is unchanged and whose carried
//      clearance radius, minus this iteration's motion, still exceeds sqrt(M2)
//      is done (every non-window candidate is provably farther than M2);
//   3. group mask: for the remaining ("active") queries of a 64-query group,
//      lane l tests sub-chunk 64 w + l against the box of the active queries
//      and their largest M2 -> 64-bit live masks;
//   4. visits: every live sub-chunk outside the lane's window whose box is
//      within the lane's current M2 is scanned; the bounds seen on the way
//      give the next clearance radius.
// Skipped candidates have d32 >= lower bound > M2 at the time of the test, and
// M2 only decreases, so (M1, M2, J1) equal the full scan's.
constexpr int kSub = 8;
#ifndef SLAM_KWIN
#define SLAM_KWIN 4
#endif
#ifndef SLAM_KBATCH
#define SLAM_KBATCH 4   // round 5, after the windows' intersection left the live sets: 4 for 3 (10k bench
                        // 4.00-4.03 ms against 4.06-4.07; 2: 4.21-4.23, 5 / 6: 4.07; profiles/r05_ab_kbatch*.txt)
#endif
constexpr int kWin = SLAM_KWIN;  // window sub-chunks (32 candidates); 2/5/6/8 measured slower
constexpr int kStageUnroll = 4;  // staging loads in flight per thread
constexpr int kBatch = SLAM_KBATCH;   // live sub-chunks tested per batch
constexpr int kWpe = 4;          // waves/SIMD the default 1081-point instance is compiled for

// Screened distances are non-negative (or +inf), so their IEEE bit patterns
// order like unsigned integers: the updates run on the bits (integer min /
// med3 need no NaN canonicalisation of the loop-carried M1, M2).
// Packed-key top-2 of the window scan (nn_window_pruned): K1 <= K2 the two
// smallest keys seen.
constexpr int kWinBits = kWin * kSub <= 16 ? 4 : kWin * kSub <= 32 ? 5 : 6;   // 32 window offsets: 5
constexpr uint32_t kWinLow = (1u << kWinBits) - 1;
static_assert(kWin * kSub <= 1 << kWinBits, "window offsets fit the key's low bits");
// (a & m) | b as ONE v_and_or_b32 (the compiler turns the or of disjoint bits
// into an add and fuses it with the loop offset: two instructions)
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t b) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(m), "s"(b));
    return r;
}
__device__ __forceinline__ void take_key(uint32_t key, uint32_t& K1, uint32_t& K2) {
    uint32_t md;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(md) : "v"(K1), "v"(K2), "v"(key));
    K2 = md;
    K1 = min(K1, key);
}

__device__ __forceinline__ void take_cand(float d, int j, float& M1, float& M2, int& J1) {
    const uint32_t db = __float_as_uint(d), m1 = __float_as_uint(M1), m2 = __float_as_uint(M2);
    J1 = db < m1 ? j : J1;
    uint32_t md;   // second smallest of {M1 <= M2, d}
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(md) : "v"(m1), "v"(m2), "v"(db));
    M2 = __uint_as_float(md);
    M1 = __uint_as_float(min(m1, db));
}

// Clearance state carried across ICP iterations, one 32-bit word per query:
// a radius R (fp32, low 9 bits cleared) with the query's window start ws in the
// low bits.  Invariant after iteration t: every candidate OUTSIDE the window
// [ws, ws + kWin) lies at Euclidean distance >= R from the query's fp32 point.
// Packing rounds R down, so the packed radius never exceeds the true bound.
constexpr uint32_t kWsMask = 511;   // nsub <= kCandCap / kSub = 512
__device__ __forceinline__ float st_radius(uint32_t s) { return __uint_as_float(s & ~kWsMask); }
__device__ __forceinline__ int st_ws(uint32_t s) { return static_cast<int>(s & kWsMask); }
__device__ __forceinline__ uint32_t st_pack(float r, int ws) {
    r = r >= 0.0f ? fminf(r, 1e30f) * (1.0f - 0x1p-12f) : 0.0f;   // NaN -> 0; 2^11 ulps down > 511
    return (__float_as_uint(r) & ~kWsMask) | static_cast<uint32_t>(ws);
}

// NQ <= QPT: the wave's groups k >= NQ hold no query (k * BLOCK + 64 * wave >=
// n1, e.g. group 4 of waves 1-3 for 1081-point scans at 256x5) and are skipped.
template <int QPT, int NQ>
__device__ __forceinline__ void nn_window_pruned(const float2* __restrict__ candf,
                                                 const float4* __restrict__ box8, int nsub,
                                                 const float (&qx)[QPT], const float (&qy)[QPT],
                                                 const bool (&valid)[QPT], const int (&pred)[QPT],
                                                 uint32_t* __restrict__ st, int st_stride,
                                                 float (&M1)[QPT], float (&M2)[QPT], int (&J1)[QPT],
                                                 int& nvisit, bool stamping, unsigned long long (&tsub)[9],
                                                 bool counting, unsigned long long& nev,
                                                 unsigned long long* ghist) {
    const int lane = threadIdx.x & 63;
    unsigned long long t0 = stamping ? __builtin_amdgcn_s_memtime() : 0;
    auto lap = [&](int q) {   // diagnostics: sub-phase s_memtime (workgroup 0, wave 0)
        if (stamping) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            if (q == 0) tsub[0] += t1 - t0;
            if (q == 1) tsub[1] += t1 - t0;
            if (q == 2) tsub[2] += t1 - t0;
            t0 = t1;
        }
    };
    // window: kWin sub-chunks centred on the prediction's sub-chunk
    int ws[QPT];
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
        // sub-chunks before the predicted one: even windows lean to the nearer half
        const int lo = (kWin & 1) ? kWin / 2 : kWin / 2 - ((pred[k] & (kSub - 1)) >= kSub / 2 ? 1 : 0);
        ws[k] = min(max((pred[k] >> 3) - lo, 0), nsub - kWin);
    }
    // 1. windows, as a top-2 of packed keys: a candidate's screened distance bits
    //    with the low kWinBits replaced by its offset in the window, so that one
    //    v_and_or + v_min + v_med3 per candidate keep the two smallest keys and
    //    the winner's offset (ties: the earlier offset, as take_cand).  A key
    //    sits within 2^kWinBits ulps below its distance.  Unpacked afterwards:
    //    M1 = the winner's key truncated (<= its distance), M2 = the runner-up
    //    key with the low bits set (>= the runner-up's distance: every test that
    //    needs M2 from above — settling, group mask, visits — stays valid), and
    //    the certification reads M2 truncated (<= the true runner-up); keys
    //    that differ only in the dropped bits are then never certified apart,
    //    so a near-tie inside the window takes the exact fallback
    uint32_t K1[QPT], K2[QPT];
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
        K1[k] = 0xffffffffu;
        K2[k] = 0xffffffffu;
    }
#pragma unroll 2
    for (int t = 0; t < kWin * kSub; t += 2) {
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const float4 pp = *reinterpret_cast<const float4*>(candf + ws[k] * kSub + t);
            const f32x2v d = screen_pair(pp, qx[k], qy[k]);
            take_key(and_or(__float_as_uint(d.x), ~kWinLow, static_cast<uint32_t>(t)), K1[k], K2[k]);
            take_key(and_or(__float_as_uint(d.y), ~kWinLow, static_cast<uint32_t>(t + 1)), K1[k], K2[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
        if (k < NQ) {
            J1[k] = static_cast<int>(K1[k] & kWinLow) + ws[k] * kSub;
            M1[k] = __uint_as_float(K1[k] & ~kWinLow);
            M2[k] = __uint_as_float(min(K2[k] | kWinLow, 0x7f800000u));   // capped at +inf
        }
    }
    if (counting) {
#pragma unroll
        for (int k = 0; k < QPT; ++k) nev += kWin * kSub * __popcll(__ballot(valid[k]));
    }
    lap(0);
    // 2. clearance test: the carried radius R (already reduced by this
    //    iteration's motion) bounds every candidate outside the PREVIOUS window;
    //    when the window moved by up to 2 sub-chunks, the sub-chunks that left it
    //    are bounded by their boxes.  If the resulting radius Rl has Rl^2 > M2,
    //    every non-window candidate has d32 > M2: the window result is the full
    //    screen's.  Only the other queries ("active") search further; a group
    //    without active queries is done.  Settled queries carry Rl with the new
    //    window to the next iteration.
    bool act[QPT];
#pragma unroll
    for (int k = NQ; k < QPT; ++k) act[k] = false;
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        const uint32_t stk = st[k * st_stride];   // LDS: not held in registers across the window scan
        const int wp = st_ws(stk);
        const int sh = ws[k] - wp;
        float rl = st_radius(stk);
        if (sh != 0) {
            const int c0 = sh > 0 ? wp : wp + kWin - 1;          // sub-chunks that left the window
            const int c1 = sh > 0 ? wp + 1 : wp + kWin - 2;
            const float4 b0 = box8[min(max(c0, 0), nsub - 1)];
            const float4 b1 = box8[min(max(c1, 0), nsub - 1)];
            float lb = box_lb(f32x2{qx[k], qy[k]}, f32x2{qx[k], qy[k]}, b0);
            if (sh * sh > 1) lb = fminf(lb, box_lb(f32x2{qx[k], qy[k]}, f32x2{qx[k], qy[k]}, b1));
            rl = fminf(rl, sqrt_bound(lb) * (1.0f - 1e-5f));
        }
        const bool settled = sh * sh <= 4 && rl * rl * (1.0f - 1e-5f) > M2[k];
#ifdef SLAM_ABL_GROUP
        act[k] = false;
#else
        act[k] = valid[k] && !settled;
#endif
        if (settled && sh != 0) st[k * st_stride] = st_pack(rl, ws[k]);
    }
    lap(1);
    // 3. per group with active queries: the box of the active fp32 queries and
    //    their largest M2; lane l tests sub-chunk 64 w + l against it -> live
    //    mask; each live sub-chunk is tested by every active lane against its
    //    own query (batches of kBatch, independent loads), the wave OR of those
    //    bits says which sub-chunks to scan.  The smallest bound over the rest
    //    (non-live sub-chunks: gf; live sub-chunks outside the window: lmin)
    //    is the new clearance radius.
    const int nw = (nsub + 63) >> 6;
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
        if (__ballot(act[k]) == 0) continue;   // wave-uniform
        int g_live = 0, g_vis = 0;   // diagnostics (stamping): this group's live and visited sub-chunks
        unsigned long long f0 = stamping ? __builtin_amdgcn_s_memtime() : 0;
        auto flap = [&](int q) {   // diagnostics: group-loop sub-phases (workgroup 0, wave 0)
            if (stamping) {
                const unsigned long long f1 = __builtin_amdgcn_s_memtime();
                tsub[q] += f1 - f0;
                f0 = f1;
            }
        };
        const float bx0 = wave_min_f(act[k] ? qx[k] : INFINITY);
        const float bx1 = wave_max_f(act[k] ? qx[k] : -INFINITY);
        const float by0 = wave_min_f(act[k] ? qy[k] : INFINITY);
        const float by1 = wave_max_f(act[k] ? qy[k] : -INFINITY);
        const float gM2 = wave_max_nn(act[k] ? M2[k] : 0.0f);
#ifndef SLAM_NO_WINX
        // sub-chunks inside EVERY active lane's window ([wlo, whi): the windows'
        // intersection) are needed by no active lane and bound nothing it needs
        // (the clearance covers the candidates outside its own window): not live
        const uint32_t wx = wave_reduce_i<uint32_t>(
            act[k] ? (static_cast<uint32_t>(ws[k]) << 16) | static_cast<uint32_t>(0xffff - (ws[k] + kWin)) : 0u,
            MaxPk16());
        const int wlo = static_cast<int>(wx >> 16), whi = 0xffff - static_cast<int>(wx & 0xffff);
#else
        const int wlo = 0, whi = 0;
#endif
        float gf = INFINITY, lmin = INFINITY;
        flap(5);
        for (int w = 0; w < nw; ++w) {
            const int sl = 64 * w + lane;
            // branch-free (no short-circuit): the LDS reads are not serialised behind exec-mask jumps
            const float glb = box_lb(f32x2{bx0, by0}, f32x2{bx1, by1}, box8[min(sl, nsub - 1)]);
            const bool gl = glb <= gM2;
            gf = (sl < nsub && !gl) ? fminf(gf, glb) : gf;
            uint64_t live = __ballot((sl < nsub) & gl & ((sl < wlo) | (sl >= whi)));
            if (stamping) {
                tsub[3] += __popcll(live);
                g_live += __popcll(live);
            }
            flap(6);
            while (live) {
                // up to kBatch live sub-chunks per batch, straight-line: the box
                // reads (broadcast) and tests issue back to back
                uint64_t scpack = 0;   // 6-bit in-word positions of this batch's sub-chunks
                uint32_t has = 0;
                float4 bb[kBatch];
#pragma unroll
                for (int u = 0; u < kBatch; ++u) {   // all box reads first (broadcast), then the tests
                    const int pos = live ? static_cast<int>(__builtin_ctzll(live)) : 0;
                    has |= static_cast<uint32_t>(live != 0) << u;
                    live &= live - 1;
                    scpack |= static_cast<uint64_t>(pos) << (6 * u);
                    bb[u] = box8[64 * w + pos];
                }
                if (stamping) tsub[4] += 1;
                uint32_t need = 0;
#pragma unroll
                for (int u = 0; u < kBatch; ++u) {
                    const int sc = 64 * w + static_cast<int>((scpack >> (6 * u)) & 63);
                    const float lb = box_lb(f32x2{qx[k], qy[k]}, f32x2{qx[k], qy[k]}, bb[u]);
                    const bool out = (sc < ws[k]) | (sc >= ws[k] + kWin);
                    lmin = out ? fminf(lmin, lb) : lmin;   // a padding slot repeats a real box: harmless
                    need |= static_cast<uint32_t>(act[k] & out & (lb <= M2[k])) << u;
                }
                need &= has;
                // scan the sub-chunks some lane needs (rolled loop: small code)
                uint32_t todo = wave_or_u32(need);
                flap(7);
                while (todo) {
                    const int u = __builtin_ctz(todo);
                    todo &= todo - 1;
                    const int c8 = (64 * w + static_cast<int>((scpack >> (6 * u)) & 63)) * kSub;
                    ++nvisit;
                    ++g_vis;
                    if (counting) nev += kSub * __popcll(__ballot((need >> u) & 1u));
                    if ((need >> u) & 1u) {
#pragma unroll
                        for (int t = 0; t < kSub; t += 2) {
                            const float4 pp = *reinterpret_cast<const float4*>(candf + c8 + t);
                            const f32x2v d = screen_pair(pp, qx[k], qy[k]);
                            take_cand(d.x, c8 + t, M1[k], M2[k], J1[k]);
                            take_cand(d.y, c8 + t + 1, M1[k], M2[k], J1[k]);
                        }
                    }
                }
                flap(8);
            }
        }
        // lb <= d32 <= (1 + 5u) |q - p|^2, so |q - p| >= sqrt(lb) (1 - 1e-5)
        const float gfar = wave_min_nn(gf);
        if (act[k]) st[k * st_stride] = st_pack(sqrt_bound(fminf(gfar, lmin)) * (1.0f - 1e-5f), ws[k]);
        const int na = stamping ? __popcll(__ballot(act[k])) : 0;
        if (stamping && lane == 0) {
            // diagnostics: per active-lane bucket (1, 2-4, 5-8, 9-16, 17-32, 33-64): group
            // iterations, live sub-chunks, visited sub-chunks (stamps[96..])
            const int bk = na <= 1 ? 0 : na <= 4 ? 1 : na <= 8 ? 2 : na <= 16 ? 3 : na <= 32 ? 4 : 5;
            atomicAdd(ghist + bk, 1ull);
            atomicAdd(ghist + 8 + bk, static_cast<unsigned long long>(g_live));
            atomicAdd(ghist + 16 + bk, static_cast<unsigned long long>(g_vis));
        }
    }
    lap(2);
}

// Predicted match of a query without a previous match (the first iteration of a
// launch): the candidate at the query's bearing in pc2's frame, by linear
// interpolation over pc2's bearing range (a lidar scan's beams are in bearing
// order at a fixed step; the rotation of the initial transform shifts the
// match by as many beams), clamped; the proportional index when pc2 gives no
// range.  Only the window position depends on it: results do not.
__device__ __forceinline__ int cold_pred(float fx, float fy, float ph0, float phs, int i, int n1, int n2) {
    if (phs > 0.0f) {
        const float j = rintf((atan2f(fy, fx) - ph0) * phs);
        return static_cast<int>(fminf(fmaxf(j, 0.0f), static_cast<float>(n2 - 1)));
    }
    return static_cast<int>(static_cast<int64_t>(i) * n2 / max(n1, 1));
}

// Certification of a screened winner.
// Any candidate at exact squared distance T has screened distance
// d32 <= F(T) = (1+8u) T + 3a sqrt(T) + 3a^2 (u = 2^-24, a = the coordinate
// rounding bound (1+u) u (|p|max + |q|max)); F is strictly increasing.  If
// every other candidate has d32 >= s2 and s2 > F(d1), all of them have
// T > d1: the winner (exact distance d1) is the unique exact minimum.  Fc is
// an upper bound of F(d1) (sqrt rounded up through fp32, 1e-12 relative slack).
__device__ __forceinline__ bool certify(double d1, double s2, double a) {
    const float sq = sqrt_bound(static_cast<float>(d1) + 1e-30f) * (1.0f + 1e-6f);   // >= sqrt(d1)
    const double fc = fma(1.0 + 8.0 * 0x1p-24, d1, fma(3.0 * a, static_cast<double>(sq), 3.0 * a * a)) *
                          (1.0 + 1e-12) + 1e-37;
    return s2 > fc;
}

// A part that gives up on an exchange (timeout, or a partner's abort) writes
// granules with this tag into its slots of this exchange and of the next: a
// partner still sweeping this one, one that starts late, or one that got past
// it (every granule had arrived) stops at once instead of waiting out its own
// timeout, and the pair goes to the repair launch (tags of real exchanges are
// e + 1 < 2^31).  A pair that finished at this exchange had its results
// written by part 0 already; the repair skips it.
constexpr uint32_t kGangAbortTag = 0xffffffffu;
// One lane's share of a gang exchange sweep: granule g of parts pp, pp + 2, ...
// (N per lane, addresses clamped so every load is issued unconditionally),
// repeated until every tag matches; then the doubles reassembled across the
// lane halves (lane l ^ 16 holds the other half) and summed.  Own granules come
// from registers.  `arrived` (wave-uniform) turns false when the partners did
// not all arrive within `wait` s_memrealtime ticks; the sum is then garbage.
template <int N>
__device__ __forceinline__ double gang_sweep(const uint64_t* buf, int g, int pp, int part, int parts, uint64_t tag,
                                             uint32_t own, int lane, uint32_t wait, bool& arrived,
                                             uint32_t* abortw) {
    uint32_t v[N];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    arrived = true;
    for (;;) {
        uint64_t x[N];
#pragma unroll
        for (int k = 0; k < N; ++k)
            x[k] = __hip_atomic_load(buf + min(pp + 2 * k, parts - 1) * 32 + g, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true, ab = false;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const int p = pp + 2 * k;
            v[k] = p == part ? own : static_cast<uint32_t>(x[k]);
            ok &= p >= parts || p == part || (x[k] & 0xffffffff00000000ull) == tag;
            ab |= p < parts && p != part && (x[k] >> 32) == kGangAbortTag;
        }
        if (__all(ok)) break;
        if (__any(ab)) {   // a partner gave up (gang_exchange_wave): so does this part, at once
            arrived = false;
            break;
        }
        // first exchange: another pair of the launch already found its partners absent
        if (abortw && __hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
            arrived = false;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > wait) {   // a partner never arrived
            if (lane == 0) {
                atomicAdd(&g_gang_timeout, 1);
                if (abortw) __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            arrived = false;
            break;
        }
    }
    const bool hi = (lane & 16) != 0;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v[k]), 16, 64));
        const uint64_t bits = hi ? (static_cast<uint64_t>(v[k]) << 32) | other : (static_cast<uint64_t>(other) << 32) | v[k];
        if (pp + 2 * k < parts) s += __longlong_as_double(static_cast<long long>(bits));
    }
    return s;
}

// Gang exchange of one iteration's 16 exact partial sums (lane q of every wave
// holds value q) as data-tagged granules: the data IS the flag (guide R2).
// Exchange e is the pair's absolute ICP iteration, so the tags of a pair that
// resumes in a later scheduler phase never match a granule left by an earlier
// phase in the same slots (no re-zeroing between phases).
// Granule l < 32 of a part is the 8-byte {tag = e + 1, half (l >> 4) of value
// (l & 15)}, written by ONE relaxed agent-scope (sc1) store; no drain, no
// counter.  Every wave sweeps all parts' granules (sc1 loads, all in flight:
// lane l reads granule l & 31 of parts l >> 5, (l >> 5) + 2, ...) until every
// tag matches, then reassembles and sums them (the partials are exact sums on
// fixed grids, so any order gives the same bits).  Slots alternate by
// exchange parity: a part can only publish exchange e + 2 after reading every
// part's e + 1 granules, each published after its reader finished exchange e.
// (One exchange ~2 L2-miss round trips; the counter form it replaced took
// four: store, drain, counter add, poll.)
// One wave's part of the exchange: publish this part's granules, sweep every
// part's until they all arrived (or `wait` ran out: arrived = false), and
// return the total of value q in lane q < 16.  Called by ONE wave per part.
__device__ __forceinline__ double gang_exchange_wave(double t, uint64_t* slots, int part, int parts, int e,
                                                     uint32_t wait, bool& arrived, uint32_t* abortw = nullptr) {
    // an opaque lane index: the sweep's addresses are recomputed at every
    // exchange (a few VALU) instead of hoisted out of the ICP loop, where the
    // 16-wave wide instance (128 VGPRs) spilled them to scratch
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const uint64_t tag = static_cast<uint64_t>(e + 1) << 32;
    uint64_t* buf = slots + (e & 1) * parts * 32;
    const uint64_t tb = static_cast<uint64_t>(__double_as_longlong(__shfl(t, lane & 15, 64)));
    if (lane < 32)
        __hip_atomic_store(buf + part * 32 + lane, tag | ((lane & 16) ? (tb >> 32) : (tb & 0xffffffffull)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int g = lane & 31, pp = lane >> 5;
    const uint32_t own = static_cast<uint32_t>((lane & 16) ? (tb >> 32) : tb);
    double s = 0.0;
    // branch-free sweeps of N loads per lane (a divergent guard around each
    // load made the compiler drain them one by one)
    if (parts <= 4)
        s = gang_sweep<2>(buf, g, pp, part, parts, tag, own, lane, wait, arrived, abortw);
    else if (parts <= 8)
        s = gang_sweep<4>(buf, g, pp, part, parts, tag, own, lane, wait, arrived, abortw);
    else if (parts <= 16)
        s = gang_sweep<8>(buf, g, pp, part, parts, tag, own, lane, wait, arrived, abortw);
    else
        s = gang_sweep<kGangSweep / 2>(buf, g, pp, part, parts, tag, own, lane, wait, arrived, abortw);
    if (!arrived) {   // (uniform) tell the partners: at this exchange and at the next (lanes 0-31 / 32-63)
        __hip_atomic_store(slots + ((e + (lane >> 5)) & 1) * parts * 32 + part * 32 + (lane & 31),
                           static_cast<uint64_t>(kGangAbortTag) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return s + __shfl_xor(s, 32, 64);   // parts of even + odd index (the same bits in both halves)
}

// Block-wide exchange: wave 0 polls (every wave polling queued the last
// arriver's loads) and broadcasts the sums and the arrival flag through LDS.
// Returns false in every thread when a partner timed out.
__device__ __forceinline__ bool gang_exchange(double& t, uint64_t* slots, int part, int parts, int e, uint32_t wait,
                                             uint32_t* abortw,
                                             double* bcast) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    if (wave == 0) {
        bool arrived;
        const double s = gang_exchange_wave(t, slots, part, parts, e, wait, arrived, abortw);
        if (lane < 16) bcast[lane] = s;
        if (lane == 0) bcast[16] = arrived ? 1.0 : 0.0;
    }
    // the slab is rewritten only at the next exchange, after the next
    // block_sum_exact16 barrier, so every wave has read it by then
    __syncthreads();
    t = lane < 16 ? bcast[lane] : 0.0;
    return bcast[16] != 0.0;
}

// Per-pair setup shared by the kernels: pc2 into LDS (fp64, fp32 pairs with
// far sentinels, sub-chunk boxes), max |coordinate| of both clouds, and the
// per-pair constants in LDS (pconst): pc1's first point c, dp = sum(p - c) as an
// order-free sum, pc1's centroid, the sum grids.  Ends with a barrier.
struct PairSetup {
    double cmax, pmaxd;
    float pmax;
    bool screen;
    int nsub;
};
template <int BLOCK, bool SCREEN, bool PRUNE>
__device__ __forceinline__ PairSetup stage_pair(const IcpArgs& a, int n1, int n2, const double2* __restrict__ p1,
                                                const double2* __restrict__ p2, bool resident, double2* cand,
                                                float2* candf, float4* box8, double* red0, double* red1,
                                                double* pconst) {
    constexpr int WAVES = BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    double cmax = 0.0;   // max |coordinate| of pc2 (screen error bound, sum grids)
    if (resident) {
#pragma unroll kStageUnroll
        for (int j = tid; j < n2; j += BLOCK) {   // unrolled: several loads in flight per thread
            const double2 p = p2[j];
            cand[j] = p;
            if constexpr (SCREEN) cf_put(candf, j, static_cast<float>(p.x), static_cast<float>(p.y));
            cmax = fmax(cmax, fmax(fabs(p.x), fabs(p.y)));
        }
        if constexpr (SCREEN) {
            for (int j = n2 + tid; j < (n2 + kChunk - 1) / kChunk * kChunk; j += BLOCK)
                cf_put(candf, j, kSentinel, kSentinel);
        }
    } else {
        for (int j = tid; j < n2; j += BLOCK) {
            const double2 p = p2[j];
            cmax = fmax(cmax, fmax(fabs(p.x), fabs(p.y)));
        }
    }
    const int nsub = (n2 + kChunk - 1) / kChunk * (kChunk / kSub);   // sub-chunks incl. padding
    if constexpr (SCREEN && PRUNE) {
        __syncthreads();   // candf complete
        for (int c = tid; c < nsub; c += BLOCK) {
            float x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
            for (int j = c * kSub; j < min(n2, (c + 1) * kSub); ++j) {
                const float2 p = cf_at(candf, j);
                x0 = fminf(x0, p.x);
                x1 = fmaxf(x1, p.x);
                y0 = fminf(y0, p.y);
                y1 = fmaxf(y1, p.y);
            }
            box8[c] = make_float4(x0, y0, x1, y1);
        }
    }
    bool screen = false;
    double pmaxd;        // max |coordinate| of pc1 (sum grids)
    float pmax = 0.0f;   // PRUNE: the same in fp32 (motion bound slack)
    {
        double cm[2] = {cmax, 0.0};
#pragma unroll kStageUnroll
        for (int i = tid; i < n1; i += BLOCK) {
            const double2 p = p1[i];
            cm[1] = fmax(cm[1], fmax(fabs(p.x), fabs(p.y)));
        }
        // block max through the second slab: max is exact, order-free
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            cm[0] = fmax(cm[0], __shfl_xor(cm[0], off, 64));
            cm[1] = fmax(cm[1], __shfl_xor(cm[1], off, 64));
        }
        if (lane == 0) {
            red1[wave] = cm[0];
            red1[WAVES + wave] = cm[1];
        }
        __syncthreads();
        cmax = red1[0];
        double pm = red1[WAVES];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) {
            cmax = fmax(cmax, red1[w]);
            pm = fmax(pm, red1[WAVES + w]);
        }
        cmax = uniform_d(cmax);
        pmaxd = uniform_d(pm);
        pmax = uniform_f(static_cast<float>(pm) * (1.0f + 1e-6f));
        // finite fp32 squares guaranteed (SCREEN launches are LDS-resident)
        if constexpr (SCREEN) screen = cmax < 1e18;
    }
    // Cross-covariance centre: pc1's first point c (any per-pair constant
    // works; it only keeps the terms small) and dp = sum(p - c), once per pair
    // as an order-free sum (first slab; iteration 0 reduces into the second).
    const double2 pc = p1[0];
    double dpx, dpy;
    {
        const RsumGrid gp = rsum_grid(2.0 * pmaxd * (1.0 + 1e-12), n1);
        double acc[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.0;
        for (int i = tid; i < n1; i += BLOCK) {
            const double2 p = p1[i];
            rsum_add(p.x - pc.x, gp, acc[0], acc[1]);
            rsum_add(p.y - pc.y, gp, acc[2], acc[3]);
        }
        const double t = block_sum_exact16<WAVES>(acc, red0);
        dpx = readlane_d(t, 0) + readlane_d(t, 1);
        dpy = readlane_d(t, 2) + readlane_d(t, 3);
    }
    if (tid == 0) {   // read back after the barrier before the loop
        pconst[kPcX] = pc.x;
        pconst[kPcY] = pc.y;
        pconst[kDpX] = dpx;
        pconst[kDpY] = dpy;
        pconst[kMupX] = pc.x + dpx / static_cast<double>(n1);   // pc1's centroid: mu_p = c + dp / n
        pconst[kMupY] = pc.y + dpy / static_cast<double>(n1);
        const RsumGrid gm = rsum_grid(cmax, n1);                         // matched pc2 coordinates
        const RsumGrid gs = rsum_grid(2.0 * pmaxd * cmax * (1.0 + 1e-12), n1);   // (p - c) m^T terms
        pconst[kGm1] = gm.m1;
        pconst[kGm2] = gm.m2;
        pconst[kGs1] = gs.m1;
        pconst[kGs2] = gs.m2;
        pconst[kPmax] = pmaxd;
        pconst[kCmax] = cmax;
        // bearing of pc2's first and last points: a cold query's predicted match
        // is the candidate at its own bearing (cold_pred), 0 scale = no prediction
        const double2 f = p2[0], l = p2[n2 - 1];
        const double ph0 = atan2(f.y, f.x), ph1 = atan2(l.y, l.x);
        pconst[kPh0] = ph0;
        pconst[kPhS] = (n2 > 1 && ph1 > ph0) ? static_cast<double>(n2 - 1) / (ph1 - ph0) : 0.0;
    }
    __syncthreads();
    PairSetup r;
    r.cmax = cmax;
    r.pmaxd = pmaxd;
    r.pmax = pmax;
    r.screen = screen;
    r.nsub = nsub;
    return r;
}

// DIAG: a diagnostics build of the kernel (per-phase s_memtime stamps of
// workgroup 0, in-kernel candidate-evaluation counter); the product kernels
// are compiled without any of it.
// GANG: one pair runs on a.gang workgroups (parts); part p holds the query
// groups (64 consecutive queries) p, p + gang, p + 2 gang, ... and the parts
// exchange their partial sums every iteration (gang_exchange).  Every part
// stages pc2 and computes the per-pair constants itself; part 0 writes the
// outputs.  Results are bit-identical to the one-workgroup kernels.
template <int BLOCK, int QPT, bool STEP, bool SCREEN, bool PRUNE = false, int WPE = 1, bool DIAG = false,
          bool GANG = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void icp_kernel(IcpArgs a) {
    constexpr int WAVES = BLOCK / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* red0 = reinterpret_cast<double*>(smem);
    double* red1 = red0 + WAVES * 16;
    double* pconst = red0 + 2 * WAVES * 16;   // PairConst slots
    double2* cand = reinterpret_cast<double2*>(smem + red_doubles(BLOCK) * sizeof(double));
    const int cap = a.cand_cap;
    // SCREEN only: fp32 copy of the candidates and per-wave fallback queues
    float2* candf = reinterpret_cast<float2*>(cand + cap);
    float4* box8 = reinterpret_cast<float4*>(candf + cap);   // PRUNE: [cap/8] sub-chunk boxes
    // PRUNE: per-query state carried across iterations in LDS instead of
    // registers (fewer VGPRs live through the window scan): last match and
    // the clearance word, slot k * BLOCK + tid
    int* qprev = reinterpret_cast<int*>(box8 + cap / kSub);
    uint32_t* qst = reinterpret_cast<uint32_t*>(qprev + BLOCK * QPT);

    // GANG: blocks b and b + 8 share an XCD (round-robin dispatch), so gang g's
    // parts sit at stride 8: block = ((g / 8) * gang + part) * 8 + g % 8
    int slot = static_cast<int>(blockIdx.x), part = 0, parts = 1;
    if constexpr (GANG) {
        parts = a.gang;
        const int bx = static_cast<int>(blockIdx.x);
        slot = (bx / (8 * parts)) * 8 + (bx & 7);
        part = (bx >> 3) % parts;
        if (slot >= a.n_gangs) return;   // padding block (uniform)
    }
    // pair of this workgroup: launch order (XCD-aware when xcd_per > 0) or the
    // scheduler's order
    int b = a.order ? a.order[slot] : slot;
    if (a.order && (b < 0 || (a.skip_lt && slot < *a.skip_lt) || (a.take_lt && slot >= *a.take_lt)))
        return;   // (uniform) another tier's pair / padding
    if (!GANG && !a.order && a.xcd_run > 0) {
        const int k = slot >> 3, g = a.xcd_run;
        b = ((k / g) * 8 + (slot & 7)) * g + k % g;
        if (b >= a.n_pairs) return;   // padding workgroup (uniform)
    }
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    // query of slot (k, tid): ((k * WAVES + wave) * parts + part) * 64 + lane
    //   = k * qstride + tid + gshift   (qstride = BLOCK, gshift = 0 without gangs)
    const int qstride = GANG ? BLOCK * parts : BLOCK;
    const int gshift = GANG ? (wave * (parts - 1) + part) * 64 : 0;   // wave-uniform
    // resumed phase: out_iters holds -(iterations done) for a paused pair and
    // the final count for a finished one (nothing left to do)
    int it0 = 0;
    if (a.resume) {
        const int s = a.out_iters[b];
        if (s > 0 || s == kBadBounds) return;   // uniform: the whole workgroup leaves
        it0 = -s;
    }
    const int s1 = a.src_scan[b];
    const int s2 = a.dst_scan[b];
    const int64_t o1 = a.scan_off[s1];
    const int64_t o2 = a.scan_off[s2];
    const int n1 = static_cast<int>(a.scan_off[s1 + 1] - o1);
    const int n2 = static_cast<int>(a.scan_off[s2 + 1] - o2);
    const double2* __restrict__ p1 = a.pts + o1;
    const double2* __restrict__ p2 = a.pts + o2;
    const bool resident = n2 <= cap;
    // the caller's bounds (max_n1 / max_n2) chose this instance and the LDS
    // size: a pair outside them would be computed wrongly, so it is flagged
    // instead (slam_icp_status returns SLAM_EINVAL) and left undone
    if (n1 < 1 || n2 < 1 || n1 > qstride * QPT || (SCREEN && !resident)) {
        if (tid == 0 && part == 0) {
            if (!STEP) a.out_iters[b] = kBadBounds;
            a.out_err[b] = __builtin_nan("");
            atomicOr(&g_icp_status, 1);
        }
        return;   // uniform
    }

    if (tid == 0 && part == 0) trace_mark(a, b, 0);
    // drain: the stopped-pair count at which the rest pause (in LDS: read once
    // per iteration by wave 0, no register held through the loop)
    if constexpr (!GANG && !STEP) {
        if (a.drain && tid == 0) pconst[kDrainAt] = static_cast<double>(*a.drain_n - a.drain_skip - a.drain_x);
    }
#ifdef SLAM_ABL_STAGE2X
    // timing-only ablation: the staging twice (its cost = the difference)
    (void)stage_pair<BLOCK, SCREEN, PRUNE>(a, n1, n2, p1, p2, resident, cand, candf, box8, red0, red1, pconst);
#endif
    const PairSetup ps = stage_pair<BLOCK, SCREEN, PRUNE>(a, n1, n2, p1, p2, resident, cand, candf, box8, red0, red1,
                                                          pconst);
    if (tid == 0 && part == 0) trace_mark(a, b, 3);   // staging done (diagnostics)
    const double cmax = ps.cmax;
    const float pmax = ps.pmax;
    const bool screen = ps.screen;
    const int nsub = ps.nsub;
    int bprev[QPT];   // !PRUNE screen: last match in registers
    // a resumed pair with saved search state picks it up (PRUNE)
    const bool warm = PRUNE && it0 > 0 && a.qsave != nullptr;
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
        bprev[k] = -1;
        if constexpr (PRUNE) {
            const int i = k * qstride + tid + gshift;
            uint2 v = make_uint2(0xffffffffu, 0u);   // no match yet, clearance 0 (see st_pack)
            if (warm && i < n1) v = a.qsave[static_cast<int64_t>(b) * a.qsave_stride + i];
            qprev[k * BLOCK + tid] = static_cast<int>(v.x);
            qst[k * BLOCK + tid] = v.y;
        }
    }
    int nscan_total = 0;
    // PRUNE: this iteration's motion T - T_prev in fp32 and its rounding slack
    float dT[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, dsig = 0.0f;
    if (warm) {
        const float* ds = a.dtsave + static_cast<int64_t>(b) * 8;
#pragma unroll
        for (int q = 0; q < 6; ++q) dT[q] = uniform_f(ds[q]);
        dsig = uniform_f(ds[6]);
    }
    const int n2_pad = (n2 + kChunk - 1) / kChunk * kChunk;

    // a resumed pair continues from its saved state: the transform and the
    // previous error (the ICP loop carries nothing else that affects results)
    SE2 T = load_se2((it0 > 0 ? a.out_tf : a.init) + 9 * static_cast<int64_t>(b));
    if (a.rotation_only) {   // src/icp.py:60-61 zeroes previous_transform[:2, 2]
        T.m02 = 0.0;
        T.m12 = 0.0;
    }
    double* hist = (!STEP && a.hist_stride > 0)
                       ? a.out_hist + static_cast<int64_t>(b) * a.hist_stride * 9
                       : nullptr;
    if (hist && tid == 0 && part == 0 && it0 == 0) store_se2(hist, T);
    double last_err = it0 > 0 ? a.out_err[b] : 0.0;
    __syncthreads();

    unsigned long long tph[5] = {0, 0, 0, 0, 0}, tprev = 0, tsub[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};

    // diagnostics: workgroup 0; wave 0 writes the sub-phase detail, every wave
    // its own phase totals (stamps[16 + 8 * wave + ...])
    const bool stamping = DIAG && a.stamps != nullptr && b == 0;   // wave-uniform
    int nfail = 0;
    const bool counting = DIAG && a.evals != nullptr;
    unsigned long long nev = 0;
    auto stamp = [&](int ph) {
        if (stamping) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph >= 0) tph[ph] += t - tprev;
            tprev = t;
        }
    };
    auto flush_stamps = [&]() {
        if (stamping && lane == 0) {
            unsigned long long* ws8 = a.stamps + 16 + 8 * wave;
            for (int q = 0; q < 4; ++q) ws8[q] = tph[q];
            ws8[4] = static_cast<unsigned long long>(nscan_total);
            ws8[5] = static_cast<unsigned long long>(nfail);
            ws8[6] = tsub[3];
            ws8[7] = tsub[4];
        }
        if (stamping && lane == 0 && wave == 0) {
            for (int q = 0; q < 4; ++q) a.stamps[q] = tph[q];
            a.stamps[4] = static_cast<unsigned long long>(nscan_total);   // sub-chunks visited (wave 0)
            for (int q = 0; q < 9; ++q) a.stamps[5 + q] = tsub[q];
        }
    };
    stamp(-1);
    for (int it = it0;; ++it) {
        // An opaque copy of the thread index per iteration: query addresses and
        // masks derived from it are recomputed (2 VALU) instead of hoisted out
        // of the loop and spilled to scratch.
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        double qx[QPT], qy[QPT];
        int bi[QPT];
        double dq[QPT];   // exact squared distance to the match (the error term of the sums)
        if constexpr (SCREEN) {
            // ---- fp32 screen over LDS-resident candidates ---------------------
            {
                float fx[QPT], fy[QPT], M1[QPT], M2[QPT];
                int C1[QPT];
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const int i = k * qstride + tid + gshift;
                    double x = 0.0, y = 0.0;
                    if (i < n1) {
                        const double2 p = p1[i];
                        x = p.x;
                        y = p.y;
                    }
                    const double tx = fma(T.m02, 1.0, fma(T.m01, y, T.m00 * x));
                    const double ty = fma(T.m12, 1.0, fma(T.m11, y, T.m10 * x));
                    fx[k] = static_cast<float>(tx);
                    fy[k] = static_cast<float>(ty);
                    if constexpr (PRUNE) {
                        // carried clearance minus this iteration's motion of the fp32
                        // query: |q_t - q_{t-1}| <= |dT p| + fp32 rounding of both
                        // queries and of dT p
                        const float xf = static_cast<float>(x), yf = static_cast<float>(y);
                        const float ex = fmaf(dT[1], yf, fmaf(dT[0], xf, dT[2]));
                        const float ey = fmaf(dT[4], yf, fmaf(dT[3], xf, dT[5]));
                        const float dl = (sqrt_bound(fmaf(ey, ey, ex * ex)) +
                                          1e-6f * (fabsf(fx[k]) + fabsf(fy[k]) + fabsf(ex) + fabsf(ey)) + dsig) *
                                         (1.0f + 1e-5f);
                        const uint32_t so = qst[k * BLOCK + tid];
                        qst[k * BLOCK + tid] = st_pack((st_radius(so) - dl) * (1.0f - 1e-5f), st_ws(so));
                    }
                    M1[k] = INFINITY;
                    M2[k] = INFINITY;
                    C1[k] = 0;
                }
                if (screen) {
                    if constexpr (PRUNE) {
                        int pred[QPT];
                        bool vq[QPT];
#pragma unroll
                        for (int k = 0; k < QPT; ++k) {
                            const int i = k * qstride + tid + gshift;
                            const int bp = qprev[k * BLOCK + tid];
                            // (a lane without a query keeps -1: no cold prediction every iteration)
                            pred[k] = (bp >= 0 || i >= n1) ? max(bp, 0)
                                                           : cold_pred(fx[k], fy[k], static_cast<float>(pconst[kPh0]),
                                                          static_cast<float>(pconst[kPhS]), i, n1, n2);
                            vq[k] = i < n1;
                        }
                        // groups holding queries (uniform; only the last can be empty)
                        const int nq = min(QPT, max(0, (n1 - 64 * wave - gshift + qstride - 1) / qstride));
                        if (QPT > 1 && nq == QPT - 1)
                            nn_window_pruned<QPT, (QPT > 1 ? QPT - 1 : QPT)>(candf, box8, nsub, fx, fy, vq, pred,
                                                                               qst + tid, BLOCK, M1, M2, C1,
                                                                               nscan_total,
                                                                               stamping, tsub, counting, nev, a.stamps ? a.stamps + 96 : nullptr);
                        else
                            nn_window_pruned<QPT, QPT>(candf, box8, nsub, fx, fy, vq, pred, qst + tid, BLOCK, M1, M2, C1,
                                                       nscan_total, stamping, tsub, counting, nev, a.stamps ? a.stamps + 96 : nullptr);
                    } else {
                        nn_scan_chunked<QPT>(candf, n2_pad, fx, fy, M1, M2, C1);
                        if (counting) {   // full screen + winning-chunk rescan
#pragma unroll
                            for (int k = 0; k < QPT; ++k)
                                nev += (n2_pad + kChunk) * __popcll(__ballot(k * qstride + tid + gshift < n1));
                        }
                    }
                }
                stamp(0);
                // ---- certify: the screened winner is the exact fp64 argmin? ---
                // the winners' fp64 coordinates for every group at once: one LDS
                // latency instead of one per (divergent) certification branch
                double2 cw[QPT];
                if constexpr (PRUNE) {
#pragma unroll
                    for (int k = 0; k < QPT; ++k) cw[k] = cand[min(C1[k], n2 - 1)];
                }
#pragma unroll
                for (int k = 0; k < QPT; ++k) {
                    const int i = k * qstride + tid + gshift;
                    double x = 0.0, y = 0.0;
                    if (i < n1) {
                        const double2 p = p1[i];
                        x = p.x;
                        y = p.y;
                    }
                    qx[k] = fma(T.m02, 1.0, fma(T.m01, y, T.m00 * x));   // bit-identical to above
                    qy[k] = fma(T.m12, 1.0, fma(T.m11, y, T.m10 * x));
                    // winning chunk: first index reaching the chunk minimum + runner-up
                    float b2 = INFINITY;
                    int j1 = C1[k];
                    if constexpr (!PRUNE) {   // PRUNE tracked the exact index and runner-up already
                        float b1 = INFINITY;
#pragma unroll 2
                        for (int j = C1[k]; j < C1[k] + kChunk; ++j) {
                            const float2 p = cf_at(candf, j);
                            const float d = screen_d32(p.x, p.y, fx[k], fy[k]);
                            b2 = __builtin_amdgcn_fmed3f(b1, b2, d);
                            if (d < b1) j1 = j;
                            b1 = fminf(b1, d);
                        }
                    }
                    j1 = min(j1, n2 - 1);
                    bi[k] = j1;
                    bool ok = true;
                    const double2 c = PRUNE ? cw[k] : cand[j1];
                    const double d1 = exact_d2(c.x, c.y, qx[k], qy[k]);
                    dq[k] = d1;   // = the sums' (pc1_t - pc2[corr])**2 bit for bit (same operands)
                    if (!screen) {
                        ok = i >= n1;   // |coordinates| >= 1e18: every query takes the exact path
                    } else if (i < n1 && n2 > 1) {
                        // every other j: d32 >= s2 (PRUNE: M2 may still hold the window's
                        // runner-up key rounded up, so its truncation is the bound)
                        const double s2 = PRUNE ? static_cast<double>(__uint_as_float(__float_as_uint(M2[k]) & ~kWinLow))
                                                : static_cast<double>(fminf(M2[k], b2));
                        const double cq = fmax(fabs(qx[k]), fabs(qy[k]));
                        const double ab = (1.0 + 0x1p-24) * 0x1p-24 * (cmax + cq);
#ifdef SLAM_ABL_CERT
                        ok = true;
#else
                        ok = cq < 1e18 && s2 < 3.0e38 && certify(d1, s2, ab);
#endif
                    }
                    // wave-cooperative exact fp64 scan for each uncertified query of
                    // this group: the whole wave scans pc2 for it, a (distance, index)
                    // butterfly leaves the first minimum in every lane, the owner takes it
                    uint64_t fails = __ballot(!ok);
                    if (stamping) nfail += __popcll(fails);
                    if (counting) nev += static_cast<unsigned long long>(n2) * __popcll(fails);
                    while (fails) {
                        const int src = static_cast<int>(__builtin_ctzll(fails));
                        fails &= fails - 1;
                        const double x = bcast_d(qx[k], src), y = bcast_d(qy[k], src);
                        double bd = INFINITY;
                        int bj = lane < n2 ? lane : 0x7fffffff;
                        for (int j = lane; j < n2; j += 64) {
                            const double2 c = cand[j];
                            const double d = exact_d2(c.x, c.y, x, y);
                            if (d < bd) {
                                bd = d;
                                bj = j;
                            }
                        }
#pragma unroll
                        for (int off = 32; off >= 1; off >>= 1) {
                            const double od = __shfl_xor(bd, off, 64);
                            const int oj = __shfl_xor(bj, off, 64);
                            if (od < bd || (od == bd && oj < bj)) {
                                bd = od;
                                bj = oj;
                            }
                        }
                        if (lane == src) {
                            bi[k] = bj;
                            dq[k] = bd;
                        }
                    }
                }
                stamp(1);
            }
            stamp(2);
#pragma unroll
            for (int k = 0; k < QPT; ++k) {
                const int nb = k * qstride + tid + gshift < n1 ? bi[k] : -1;
                if constexpr (PRUNE) qprev[k * BLOCK + tid] = nb;
                else bprev[k] = nb;
            }
        } else {
            // ---- exact fp64 scan (src/icp.py:62-63) ---------------------------
            double best[QPT];
#pragma unroll
            for (int k = 0; k < QPT; ++k) {
                const int i = k * qstride + tid + gshift;
                double x = 0.0, y = 0.0;
                if (i < n1) {
                    const double2 p = p1[i];
                    x = p.x;
                    y = p.y;
                }
                qx[k] = fma(T.m02, 1.0, fma(T.m01, y, T.m00 * x));
                qy[k] = fma(T.m12, 1.0, fma(T.m11, y, T.m10 * x));
                best[k] = INFINITY;
                bi[k] = 0;
            }
            if (resident) {
                nn_scan_f64<QPT>(cand, n2, 0, qx, qy, best, bi);
                if (counting) {
#pragma unroll
                    for (int k = 0; k < QPT; ++k) nev += static_cast<unsigned long long>(n2) * __popcll(__ballot(k * qstride + tid + gshift < n1));
                }
            } else {
                for (int t0 = 0; t0 < n2; t0 += cap) {
                    const int cnt = min(cap, n2 - t0);
                    __syncthreads();
                    for (int j = tid; j < cnt; j += BLOCK) cand[j] = p2[t0 + j];
                    __syncthreads();
                    nn_scan_f64<QPT>(cand, cnt, t0, qx, qy, best, bi);
                    if (counting) {
#pragma unroll
                        for (int k = 0; k < QPT; ++k) nev += static_cast<unsigned long long>(cnt) * __popcll(__ballot(k * qstride + tid + gshift < n1));
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < QPT; ++k) dq[k] = best[k];
        }

        // ---- src/icp.py:64,68 + 22-46  error, centroids, cross-covariance ------
        // One pass, one barrier, order-free sums (rsum_add): the totals are the
        // same bits for every workgroup shape and query layout, so a pair's
        // result does not depend on the instance, the scheduler or the number of
        // GPUs a stream is sharded over.  Per query:
        //   m (matched pc2 point), d^2 = |q - m|^2 (the error, reference rounding),
        //   (p - c) m^T with p the untransformed pc1 point and c = pc1[0].
        // Then pc1_avg = T mu_p, and X Y^T = R_T [sum (p - c) m^T - dp pc2_avg^T]
        // (q - mu_q = R_T (p - mu_p) and sum (m - pc2_avg) = 0).
        // drain count, read by wave 0 ahead of the sums' loads (used in the update)
        uint32_t dword = 0;
        if constexpr (!GANG && !STEP) {
            if (a.drain && wave == 0)
                dword = __hip_atomic_load(a.drain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        double tot;
        {
            // the pc1 row is re-read (the untransformed point of the (p - c) m^T
            // terms); the error term is the match's exact distance kept from the
            // search (dq), so the query point need not stay live or be recomputed
            int tr = threadIdx.x;
            asm volatile("" : "+v"(tr));
            const double2 c = *reinterpret_cast<const double2*>(pconst + kPcX);
            const double2 gmv = *reinterpret_cast<const double2*>(pconst + kGm1);
            const double2 gsv = *reinterpret_cast<const double2*>(pconst + kGs1);
            const double2 pcm = *reinterpret_cast<const double2*>(pconst + kPmax);   // (pmax, cmax)
            const double bq = (fmax(fabs(T.m00) + fabs(T.m01), fabs(T.m10) + fabs(T.m11)) * pcm.x +
                               fmax(fabs(T.m02), fabs(T.m12))) * (1.0 + 1e-12);   // >= |q|
            const RsumGrid gm{gmv.x, gmv.y}, gs{gsv.x, gsv.y};
            const RsumGrid gd = rsum_grid(2.0 * (bq + pcm.y) * (bq + pcm.y) * (1.0 + 1e-12), n1);
            double acc[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.0;
#pragma unroll
            for (int k = 0; k < QPT; ++k) {
                const int i = k * qstride + tr + gshift;
                if (i < n1) {
                    const double2 m = resident ? cand[bi[k]] : p2[bi[k]];
                    const double2 p = p1[i];
                    rsum_add(m.x, gm, acc[0], acc[1]);
                    rsum_add(m.y, gm, acc[2], acc[3]);
                    rsum_add(dq[k], gd, acc[4], acc[5]);   // (pc1_t - pc2[corr])**2
                    const double ax = p.x - c.x, ay = p.y - c.y;
                    rsum_add(ax * m.x, gs, acc[6], acc[7]);
                    rsum_add(ax * m.y, gs, acc[8], acc[9]);
                    rsum_add(ay * m.x, gs, acc[10], acc[11]);
                    rsum_add(ay * m.y, gs, acc[12], acc[13]);
                }
            }
            tot = block_sum_exact16<WAVES>(acc, ((it - it0) & 1) ? red0 : red1);
        }
        if constexpr (GANG) {
            // a partner that never arrived: stop at once, write nothing (the
            // repair launch re-runs the pair from its phase-1 state)
            if (parts > 1 && !gang_exchange(tot, a.gang_slots + static_cast<int64_t>(slot) * 2 * parts * 32, part,
                                            parts, it, it == it0 ? a.gang_wait_first : a.gang_wait,
                                            it == it0 ? a.gang_abort : nullptr, pconst + kBcast))
                return;
        }
        // The update is the same for every wave: wave 0 computes it and hands the
        // new transform and the error to the others through LDS (one barrier;
        // the same bits), so the other waves' SIMD issue slots go to the search
        // (-DSLAM_KABSCH_ALL: every wave computes it, as before round 5)
        SE2 Tn;
        double err;
#ifndef SLAM_KABSCH_ALL
        if (wave == 0) {
#else
        {
#endif
            const double n = static_cast<double>(n1);
            const double mvx = (readlane_d(tot, 0) + readlane_d(tot, 1)) / n;   // pc2_avg
            const double mvy = (readlane_d(tot, 2) + readlane_d(tot, 3)) / n;
            err = readlane_d(tot, 4) + readlane_d(tot, 5);
            const double2 dp = *reinterpret_cast<const double2*>(pconst + kDpX);
            const double2 mup = *reinterpret_cast<const double2*>(pconst + kMupX);
            const double mux = fma(T.m02, 1.0, fma(T.m01, mup.y, T.m00 * mup.x));   // pc1_avg = T mu_p
            const double muy = fma(T.m12, 1.0, fma(T.m11, mup.y, T.m10 * mup.x));
            // S_p = sum (p - mu_p)(m - pc2_avg)^T, then S = X @ Y.T = R_T S_p
            const double p00 = fma(-dp.x, mvx, readlane_d(tot, 6) + readlane_d(tot, 7));
            const double p01 = fma(-dp.x, mvy, readlane_d(tot, 8) + readlane_d(tot, 9));
            const double p10 = fma(-dp.y, mvx, readlane_d(tot, 10) + readlane_d(tot, 11));
            const double p11 = fma(-dp.y, mvy, readlane_d(tot, 12) + readlane_d(tot, 13));
            double s[4];
            s[0] = fma(T.m01, p10, T.m00 * p00);
            s[1] = fma(T.m01, p11, T.m00 * p01);
            s[2] = fma(T.m11, p10, T.m10 * p00);
            s[3] = fma(T.m11, p11, T.m10 * p01);

            // ---- closed-form 2x2 Kabsch: R maximising tr(R S) ---------------------
            // Equals V diag(1, det(V U^T)) U^T of the reference's SVD route.
            const double cs = s[0] + s[3];
            const double sn = s[1] - s[2];
            const double r = sqrt(cs * cs + sn * sn);
            const double c = r > 0.0 ? cs / r : 1.0;
            const double si = r > 0.0 ? sn / r : 0.0;
            // t = pc2_avg - R @ pc1_avg (dgemv order)
            double tx = mvx - fma(-si, muy, c * mux);
            double ty = mvy - fma(c, muy, si * mux);
            if (a.rotation_only) {   // src/icp.py:65-66
                tx = 0.0;
                ty = 0.0;
            }
            SE2 D;
            D.m00 = c;  D.m01 = -si; D.m02 = tx;
            D.m10 = si; D.m11 = c;   D.m12 = ty;
            Tn = se2_mul(D, T);   // src/icp.py:67
#ifndef SLAM_KABSCH_ALL
            if (lane == 0) {
                pconst[kKab + 0] = Tn.m00;
                pconst[kKab + 1] = Tn.m01;
                pconst[kKab + 2] = Tn.m02;
                pconst[kKab + 3] = Tn.m10;
                pconst[kKab + 4] = Tn.m11;
                pconst[kKab + 5] = Tn.m12;
                pconst[kKab + 6] = err;
                // drain: at most drain_x of the launch's pairs have not stopped
                pconst[kKab + 7] =
                    (!GANG && !STEP && a.drain && static_cast<double>(dword) >= pconst[kDrainAt]) ? 1.0 : 0.0;
            }
#endif
        }
#ifndef SLAM_KABSCH_ALL
        __syncthreads();
        Tn.m00 = pconst[kKab + 0];
        Tn.m01 = pconst[kKab + 1];
        Tn.m02 = pconst[kKab + 2];
        Tn.m10 = pconst[kKab + 3];
        Tn.m11 = pconst[kKab + 4];
        Tn.m12 = pconst[kKab + 5];
        err = pconst[kKab + 6];
        const bool drain_now = pconst[kKab + 7] != 0.0;
#else
        const bool drain_now = false;
#endif

        stamp(3);
        if constexpr (STEP) {
            if (tid == 0) {
                store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                a.out_err[b] = err;
            }
            if (counting && lane == 0) atomicAdd(a.evals, nev);
            int64_t* corr = a.out_corr + a.corr_off[b];
#pragma unroll
            for (int k = 0; k < QPT; ++k) {
                const int i = k * qstride + tid + gshift;
                if (i < n1) corr[i] = bi[k];
            }
            return;
        } else {
            if (hist && tid == 0 && part == 0) store_se2(hist + 9 * (it + 1), Tn);
            // src/icp.py:86-95 (identical in every thread -> uniform exit)
            const double derr = fabs(last_err - err);
            const bool stop = (err < a.epsilon) || (it > a.max_iters) ||
                              (it > 0 && derr < a.stopping_thresh);
            last_err = err;
            if constexpr (PRUNE) {
                // motion of the next iteration's queries: (Tn - T) p, fp32; dsig bounds
                // its evaluation error (4u of |dT||p|) and the fp64 rounding of both
                // transforms (|R| <= 1 + 1e-9, |p| <= pmax)
                dT[0] = uniform_f(static_cast<float>(Tn.m00 - T.m00));
                dT[1] = uniform_f(static_cast<float>(Tn.m01 - T.m01));
                dT[2] = uniform_f(static_cast<float>(Tn.m02 - T.m02));
                dT[3] = uniform_f(static_cast<float>(Tn.m10 - T.m10));
                dT[4] = uniform_f(static_cast<float>(Tn.m11 - T.m11));
                dT[5] = uniform_f(static_cast<float>(Tn.m12 - T.m12));
                const float rr = fmaxf(fabsf(dT[0]) + fabsf(dT[1]), fabsf(dT[3]) + fabsf(dT[4]));
                const float tt = fmaxf(fabsf(dT[2]), fabsf(dT[5]));
                const float big = static_cast<float>(fabs(T.m02) + fabs(T.m12) + fabs(Tn.m02) + fabs(Tn.m12));
                dsig = uniform_f(1e-6f * (rr * pmax + tt) + 1e-9f * (pmax + big) + 1e-30f);
            }
            // Tn is identical in every lane: keep it in SGPRs
            T.m00 = uniform_d(Tn.m00); T.m01 = uniform_d(Tn.m01); T.m02 = uniform_d(Tn.m02);
            T.m10 = uniform_d(Tn.m10); T.m11 = uniform_d(Tn.m11); T.m12 = uniform_d(Tn.m12);
            if (stop) {
                flush_stamps();
                if (counting && lane == 0) atomicAdd(a.evals, nev);
                if (tid == 0 && part == 0) {
                    store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                    a.out_err[b] = err;
                    a.out_iters[b] = it + 1;
                    trace_mark(a, b, 1);
                    if (!GANG && a.drain) atomicAdd(a.drain, 1u);
                }
                return;
            }
            if ((a.phase_cap > 0 && it + 1 - it0 >= a.phase_cap) || drain_now) {
                // pause (scheduler phase boundary): save the loop state; the
                // last error change orders the survivors for the next phase
                flush_stamps();
                if (counting && lane == 0) atomicAdd(a.evals, nev);
                if constexpr (PRUNE) {
                    if (a.qsave) {   // the search state, so the resumed iteration starts warm
#pragma unroll
                        for (int k = 0; k < QPT; ++k) {
                            const int i = k * qstride + tid + gshift;
                            if (i < n1)
                                a.qsave[static_cast<int64_t>(b) * a.qsave_stride + i] =
                                    make_uint2(static_cast<uint32_t>(qprev[k * BLOCK + tid]), qst[k * BLOCK + tid]);
                        }
                        if (tid == 0 && part == 0) {
                            float* ds = a.dtsave + static_cast<int64_t>(b) * 8;
#pragma unroll
                            for (int q = 0; q < 6; ++q) ds[q] = dT[q];
                            ds[6] = dsig;
                        }
                    }
                }
                if (tid == 0 && part == 0) {
                    store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                    a.out_err[b] = err;
                    a.out_iters[b] = -(it + 1);
                    a.sched_key[b] = static_cast<float>(derr);
                    trace_mark(a, b, 1);
                    if (!GANG && a.drain) atomicAdd(a.drain, 1u);
                }
                return;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Team kernel (latency mode for the strong-scaling tail).  A gang of
// workgroups runs one pair, ONE 64-query group per workgroup, and the
// group's search is split over the kTeam waves of its workgroup: wave w scans
// window sub-chunk ws + w and every kTeam-th batch of the live sub-chunks, the
// partial top-2 results meet in LDS (merged in wave order: the window's
// left-to-right order).  A lone pair's iteration is then about a quarter of
// its slowest group's search plus the exchanges, instead of the whole group's
// (one outlier group — queries far from every candidate, 70-110 live
// sub-chunks — set the lone latency).  Every wave holds
// the same 64 queries and their state (matches, clearances) in registers and
// updates it identically; wave 0 alone contributes the sums.  Results equal
// the one-workgroup kernels bit for bit (same exact sums, same winners).
// ---------------------------------------------------------------------------
#ifndef SLAM_TEAM_WAVES
#define SLAM_TEAM_WAVES 4
#endif
constexpr int kTeam = SLAM_TEAM_WAVES;   // waves per query group (lone pair 1118: 4 waves 12.5 us/iter, 8 waves 13.0: the
                                         // merges, barriers and sums grow faster than the slowest group's search shrinks)
constexpr int kTeamMaxParts = kGangSweep;   // query groups of a team-run pair (2,048 points)
constexpr int kTeamBlock = 64 * kTeam;

// (M1, J1, M2) <- the top-2 of itself and (m1, j1, m2), both sorted; ties keep
// the current J1 (earlier in visit order), as take_cand does
__device__ __forceinline__ void top2_merge(float& M1, float& M2, int& J1, float m1, float m2, int j1) {
    const uint32_t a1 = __float_as_uint(M1), a2 = __float_as_uint(M2);
    const uint32_t b1 = __float_as_uint(m1), b2 = __float_as_uint(m2);
    J1 = b1 < a1 ? j1 : J1;
    M2 = __uint_as_float(min(max(a1, b1), min(a2, b2)));
    M1 = __uint_as_float(min(a1, b1));
}

__host__ __device__ constexpr size_t team_xbuf_words() { return 2 * kTeam * 4 * 64; }

__global__ __launch_bounds__(kTeamBlock) void icp_team_kernel(IcpArgs a) {
    constexpr int WAVES = kTeam;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* red0 = reinterpret_cast<double*>(smem);
    double* red1 = red0 + WAVES * 16;
    double* pconst = red0 + 2 * WAVES * 16;
    double2* cand = reinterpret_cast<double2*>(smem + red_doubles(kTeamBlock) * sizeof(double));
    const int cap = a.cand_cap;
    float2* candf = reinterpret_cast<float2*>(cand + cap);
    float4* box8 = reinterpret_cast<float4*>(candf + cap);
    uint32_t* xbuf = reinterpret_cast<uint32_t*>(box8 + cap / kSub);   // [2][kTeam][4][64] merge slots

    const int parts = a.gang;
    const int bx = static_cast<int>(blockIdx.x);
    const int slot = (bx / (8 * parts)) * 8 + (bx & 7);
    const int part = (bx >> 3) % parts;   // = the query group of this workgroup
    if (slot >= a.n_gangs) return;
    const int b = a.order ? a.order[slot] : slot;
    if (b < 0) return;   // padding (uniform)
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int it0 = 0;
    if (a.resume) {
        const int s = a.out_iters[b];
        if (s > 0 || s == kBadBounds) return;
        it0 = -s;
    }
    const int s1 = a.src_scan[b];
    const int s2 = a.dst_scan[b];
    const int64_t o1 = a.scan_off[s1];
    const int64_t o2 = a.scan_off[s2];
    const int n1 = static_cast<int>(a.scan_off[s1 + 1] - o1);
    const int n2 = static_cast<int>(a.scan_off[s2 + 1] - o2);
    const double2* __restrict__ p1 = a.pts + o1;
    const double2* __restrict__ p2 = a.pts + o2;
    if (n1 < 1 || n2 < 1 || n1 > 64 * parts || n2 > cap) {
        if (tid == 0 && part == 0) {
            a.out_iters[b] = kBadBounds;
            a.out_err[b] = __builtin_nan("");
            atomicOr(&g_icp_status, 1);
        }
        return;
    }
    const PairSetup ps = stage_pair<kTeamBlock, true, true>(a, n1, n2, p1, p2, true, cand, candf, box8, red0, red1,
                                                            pconst);
    const int nsub = ps.nsub;
    const bool screen = ps.screen;
    SE2 T = load_se2((it0 > 0 ? a.out_tf : a.init) + 9 * static_cast<int64_t>(b));
    if (a.rotation_only) {
        T.m02 = 0.0;
        T.m12 = 0.0;
    }
    double* hist = a.hist_stride > 0 ? a.out_hist + static_cast<int64_t>(b) * a.hist_stride * 9 : nullptr;
    if (hist && tid == 0 && part == 0 && it0 == 0) store_se2(hist, T);
    double last_err = it0 > 0 ? a.out_err[b] : 0.0;
    float dT[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, dsig = 0.0f;
    int prev = -1;      // last match (identical in every wave)
    uint32_t st = 0;    // clearance word (radius | window start), see st_pack
    const int i = part * 64 + lane;
    const bool valid = i < n1;
    const int nw = (nsub + 63) >> 6;
    // diagnostics (a.stamps != NULL): s_memtime per phase of wave 0 of every part,
    // stamps[256 + 16 * part + phase]
    const bool stamping = a.stamps != nullptr && wave == 0;
    unsigned long long tp = stamping ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto tstamp = [&](int q) {
        if (stamping) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            tacc[q] += t1 - tp;
            tp = t1;
        }
    };
    auto tflush = [&]() {
        if (stamping && lane == 0)
            for (int q = 0; q < 10; ++q) atomicAdd(a.stamps + 256 + 16 * part + q, tacc[q]);
    };
    for (int it = it0;; ++it) {
        double x = 0.0, y = 0.0;
        if (valid) {
            const double2 p = p1[i];
            x = p.x;
            y = p.y;
        }
        const double qx = fma(T.m02, 1.0, fma(T.m01, y, T.m00 * x));
        const double qy = fma(T.m12, 1.0, fma(T.m11, y, T.m10 * x));
        const float fx = static_cast<float>(qx), fy = static_cast<float>(qy);
        {   // carried clearance minus this iteration's motion (as icp_kernel)
            const float xf = static_cast<float>(x), yf = static_cast<float>(y);
            const float ex = fmaf(dT[1], yf, fmaf(dT[0], xf, dT[2]));
            const float ey = fmaf(dT[4], yf, fmaf(dT[3], xf, dT[5]));
            const float dl = (sqrt_bound(fmaf(ey, ey, ex * ex)) + 1e-6f * (fabsf(fx) + fabsf(fy) + fabsf(ex) + fabsf(ey)) +
                              dsig) * (1.0f + 1e-5f);
            st = st_pack((st_radius(st) - dl) * (1.0f - 1e-5f), st_ws(st));
        }
        float M1 = INFINITY, M2 = INFINITY;
        int J1 = 0;
        int ws = 0;
        bool act = false;
        float lmin = INFINITY, gfar = INFINITY;
        uint32_t* xb = xbuf + (it & 1) * (kTeam * 4 * 64);
        if (screen) {
            const int pred = (prev >= 0 || i >= n1) ? max(prev, 0)
                                                    : cold_pred(fx, fy, static_cast<float>(pconst[kPh0]),
                                                   static_cast<float>(pconst[kPhS]), i, n1, n2);
            {
                const int lo = kWin / 2 - ((pred & (kSub - 1)) >= kSub / 2 ? 1 : 0);
                ws = min(max((pred >> 3) - lo, 0), nsub - kWin);
            }
            // window: this wave's sub-chunk ws + wave (waves past the window: none)
            if (wave < kWin) {
                const int c8 = (ws + wave) * kSub;
#pragma unroll
                for (int t = 0; t < kSub; t += 2) {
                    const float4 pp = *reinterpret_cast<const float4*>(candf + c8 + t);
                    const f32x2v d = screen_pair(pp, fx, fy);
                    take_cand(d.x, c8 + t, M1, M2, J1);
                    take_cand(d.y, c8 + t + 1, M1, M2, J1);
                }
            }
            tstamp(0);
            xb[(wave * 4 + 0) * 64 + lane] = __float_as_uint(M1);
            xb[(wave * 4 + 1) * 64 + lane] = static_cast<uint32_t>(J1);
            xb[(wave * 4 + 2) * 64 + lane] = __float_as_uint(M2);
            __syncthreads();
            tstamp(1);
            M1 = INFINITY;
            M2 = INFINITY;
            J1 = 0;
#pragma unroll
            for (int w = 0; w < kTeam; ++w)
                top2_merge(M1, M2, J1, __uint_as_float(xb[(w * 4 + 0) * 64 + lane]),
                           __uint_as_float(xb[(w * 4 + 2) * 64 + lane]), static_cast<int>(xb[(w * 4 + 1) * 64 + lane]));
            // clearance test (identical in every wave)
            {
                const int wp = st_ws(st);
                const int sh = ws - wp;
                float rl = st_radius(st);
                if (sh != 0) {
                    const int c0 = sh > 0 ? wp : wp + kWin - 1;
                    const int c1 = sh > 0 ? wp + 1 : wp + kWin - 2;
                    const float4 b0 = box8[min(max(c0, 0), nsub - 1)];
                    const float4 b1 = box8[min(max(c1, 0), nsub - 1)];
                    float lb = box_lb(f32x2{fx, fy}, f32x2{fx, fy}, b0);
                    if (sh * sh > 1) lb = fminf(lb, box_lb(f32x2{fx, fy}, f32x2{fx, fy}, b1));
                    rl = fminf(rl, sqrt_bound(lb) * (1.0f - 1e-5f));
                }
                const bool settled = sh * sh <= 4 && rl * rl * (1.0f - 1e-5f) > M2;
                act = valid && !settled;
                if (settled && sh != 0) st = st_pack(rl, ws);
            }
            tstamp(2);
            // group search past the window, split over the team
            float E1 = INFINITY, E2 = INFINITY;
            int EJ = 0;
            if (__ballot(act) != 0) {   // identical in every wave
                const float bx0 = wave_min_f(act ? fx : INFINITY);
                const float bx1 = wave_max_f(act ? fx : -INFINITY);
                const float by0 = wave_min_f(act ? fy : INFINITY);
                const float by1 = wave_max_f(act ? fy : -INFINITY);
                const float gM2 = wave_max_nn(act ? M2 : 0.0f);
                float gf = INFINITY;
                int bcount = 0;
                for (int w = 0; w < nw; ++w) {
                    const int sl = 64 * w + lane;
                    const float glb = box_lb(f32x2{bx0, by0}, f32x2{bx1, by1}, box8[min(sl, nsub - 1)]);
                    const bool gl = glb <= gM2;
                    gf = (sl < nsub && !gl) ? fminf(gf, glb) : gf;
                    uint64_t live = __ballot((sl < nsub) & gl);
                    while (live) {
                        uint64_t scpack = 0;
                        uint32_t has = 0;
                        float4 bb[kBatch];
#pragma unroll
                        for (int u = 0; u < kBatch; ++u) {
                            const int pos = live ? static_cast<int>(__builtin_ctzll(live)) : 0;
                            has |= static_cast<uint32_t>(live != 0) << u;
                            live &= live - 1;
                            scpack |= static_cast<uint64_t>(pos) << (6 * u);
                            bb[u] = box8[64 * w + pos];
                        }
                        const bool mine = (bcount++ % kTeam) == wave;   // wave-uniform
                        if (!mine) continue;
                        // current upper bound of the final M2: second smallest of the
                        // window's top-2 and this wave's extra top-2
                        const uint32_t m2l = min(max(__float_as_uint(M1), __float_as_uint(E1)),
                                                 min(__float_as_uint(M2), __float_as_uint(E2)));
                        uint32_t need = 0;
#pragma unroll
                        for (int u = 0; u < kBatch; ++u) {
                            const int sc = 64 * w + static_cast<int>((scpack >> (6 * u)) & 63);
                            const float lb = box_lb(f32x2{fx, fy}, f32x2{fx, fy}, bb[u]);
                            const bool out = (sc < ws) | (sc >= ws + kWin);
                            lmin = out ? fminf(lmin, lb) : lmin;
                            need |= static_cast<uint32_t>(act & out & (lb <= __uint_as_float(m2l))) << u;
                        }
                        need &= has;
                        uint32_t todo = wave_or_u32(need);
                        while (todo) {
                            const int u = __builtin_ctz(todo);
                            todo &= todo - 1;
                            const int c8 = (64 * w + static_cast<int>((scpack >> (6 * u)) & 63)) * kSub;
                            if ((need >> u) & 1u) {
#pragma unroll
                                for (int t = 0; t < kSub; t += 2) {
                                    const float4 pp = *reinterpret_cast<const float4*>(candf + c8 + t);
                                    const f32x2v d = screen_pair(pp, fx, fy);
                                    take_cand(d.x, c8 + t, E1, E2, EJ);
                                    take_cand(d.y, c8 + t + 1, E1, E2, EJ);
                                }
                            }
                        }
                    }
                }
                gfar = wave_min_nn(gf);
            }
            // merge the team's extra candidates (disjoint from the window and from
            // each other) and the clearance bounds
            uint32_t* xb2 = xb + 0;   // second half of this iteration's slots
            xb2 = xbuf + ((it & 1) ^ 1) * (kTeam * 4 * 64);
            xb2[(wave * 4 + 0) * 64 + lane] = __float_as_uint(E1);
            xb2[(wave * 4 + 1) * 64 + lane] = static_cast<uint32_t>(EJ);
            xb2[(wave * 4 + 2) * 64 + lane] = __float_as_uint(E2);
            xb2[(wave * 4 + 3) * 64 + lane] = __float_as_uint(lmin);
            tstamp(3);
            __syncthreads();
            tstamp(4);
            float lm = INFINITY;
#pragma unroll
            for (int w = 0; w < kTeam; ++w) {
                top2_merge(M1, M2, J1, __uint_as_float(xb2[(w * 4 + 0) * 64 + lane]),
                           __uint_as_float(xb2[(w * 4 + 2) * 64 + lane]), static_cast<int>(xb2[(w * 4 + 1) * 64 + lane]));
                lm = fminf(lm, __uint_as_float(xb2[(w * 4 + 3) * 64 + lane]));
            }
            if (act) st = st_pack(sqrt_bound(fminf(gfar, lm)) * (1.0f - 1e-5f), ws);
        }
        tstamp(5);
        // certification (identical in every wave) and the exact fallback
        int bi;
        {
            const int j1 = min(J1, n2 - 1);
            bi = j1;
            bool ok = true;
            if (!screen) {
                ok = !valid;
            } else if (valid && n2 > 1) {
                const double2 c = cand[j1];
                const double d1 = exact_d2(c.x, c.y, qx, qy);
                const double cq = fmax(fabs(qx), fabs(qy));
                const double ab = (1.0 + 0x1p-24) * 0x1p-24 * (ps.cmax + cq);
                ok = cq < 1e18 && M2 < 3.0e38f && certify(d1, static_cast<double>(M2), ab);
            }
            uint64_t fails = __ballot(!ok);
            while (fails) {
                const int src = static_cast<int>(__builtin_ctzll(fails));
                fails &= fails - 1;
                const double xs = bcast_d(qx, src), ys = bcast_d(qy, src);
                double bd = INFINITY;
                int bj = lane < n2 ? lane : 0x7fffffff;
                for (int j = lane; j < n2; j += 64) {
                    const double2 c = cand[j];
                    const double d = exact_d2(c.x, c.y, xs, ys);
                    if (d < bd) {
                        bd = d;
                        bj = j;
                    }
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const double od = __shfl_xor(bd, off, 64);
                    const int oj = __shfl_xor(bj, off, 64);
                    if (od < bd || (od == bd && oj < bj)) {
                        bd = od;
                        bj = oj;
                    }
                }
                if (lane == src) bi = bj;
            }
            prev = valid ? bi : -1;
        }
        tstamp(6);
        // sums: wave 0's 64 queries (the other waves hold the same ones)
        double tot;
        {
            const double2 c = *reinterpret_cast<const double2*>(pconst + kPcX);
            const double2 gmv = *reinterpret_cast<const double2*>(pconst + kGm1);
            const double2 gsv = *reinterpret_cast<const double2*>(pconst + kGs1);
            const double2 pcm = *reinterpret_cast<const double2*>(pconst + kPmax);
            const double bq = (fmax(fabs(T.m00) + fabs(T.m01), fabs(T.m10) + fabs(T.m11)) * pcm.x +
                               fmax(fabs(T.m02), fabs(T.m12))) * (1.0 + 1e-12);
            const RsumGrid gm{gmv.x, gmv.y}, gs{gsv.x, gsv.y};
            const RsumGrid gd = rsum_grid(2.0 * (bq + pcm.y) * (bq + pcm.y) * (1.0 + 1e-12), n1);
            double acc[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.0;
            if (wave == 0 && valid) {
                const double2 m = cand[bi];
                rsum_add(m.x, gm, acc[0], acc[1]);
                rsum_add(m.y, gm, acc[2], acc[3]);
                rsum_add(exact_d2(m.x, m.y, qx, qy), gd, acc[4], acc[5]);
                const double ax = x - c.x, ay = y - c.y;
                rsum_add(ax * m.x, gs, acc[6], acc[7]);
                rsum_add(ax * m.y, gs, acc[8], acc[9]);
                rsum_add(ay * m.x, gs, acc[10], acc[11]);
                rsum_add(ay * m.y, gs, acc[12], acc[13]);
            }
            tot = block_sum_exact16<WAVES>(acc, ((it - it0) & 1) ? red0 : red1);
            tstamp(7);
            if (parts > 1 && !gang_exchange(tot, a.gang_slots + static_cast<int64_t>(slot) * 2 * parts * 32, part,
                                            parts, it, it == it0 ? a.gang_wait_first : a.gang_wait,
                                            it == it0 ? a.gang_abort : nullptr, pconst + kBcast)) {
                tflush();
                return;   // a partner timed out: nothing written, the repair launch re-runs the pair
            }
        }
        tstamp(8);
        const double n = static_cast<double>(n1);
        const double mvx = (readlane_d(tot, 0) + readlane_d(tot, 1)) / n;
        const double mvy = (readlane_d(tot, 2) + readlane_d(tot, 3)) / n;
        const double err = readlane_d(tot, 4) + readlane_d(tot, 5);
        const double2 dp = *reinterpret_cast<const double2*>(pconst + kDpX);
        const double2 mup = *reinterpret_cast<const double2*>(pconst + kMupX);
        const double mux = fma(T.m02, 1.0, fma(T.m01, mup.y, T.m00 * mup.x));
        const double muy = fma(T.m12, 1.0, fma(T.m11, mup.y, T.m10 * mup.x));
        const double p00 = fma(-dp.x, mvx, readlane_d(tot, 6) + readlane_d(tot, 7));
        const double p01 = fma(-dp.x, mvy, readlane_d(tot, 8) + readlane_d(tot, 9));
        const double p10 = fma(-dp.y, mvx, readlane_d(tot, 10) + readlane_d(tot, 11));
        const double p11 = fma(-dp.y, mvy, readlane_d(tot, 12) + readlane_d(tot, 13));
        const double s00 = fma(T.m01, p10, T.m00 * p00);
        const double s01 = fma(T.m01, p11, T.m00 * p01);
        const double s10 = fma(T.m11, p10, T.m10 * p00);
        const double s11 = fma(T.m11, p11, T.m10 * p01);
        const double cs = s00 + s11;
        const double sn = s01 - s10;
        const double r = sqrt(cs * cs + sn * sn);
        const double co = r > 0.0 ? cs / r : 1.0;
        const double si = r > 0.0 ? sn / r : 0.0;
        double tx = mvx - fma(-si, muy, co * mux);
        double ty = mvy - fma(co, muy, si * mux);
        if (a.rotation_only) {
            tx = 0.0;
            ty = 0.0;
        }
        SE2 D;
        D.m00 = co; D.m01 = -si; D.m02 = tx;
        D.m10 = si; D.m11 = co;  D.m12 = ty;
        const SE2 Tn = se2_mul(D, T);
        if (hist && tid == 0 && part == 0) store_se2(hist + 9 * (it + 1), Tn);
        const double derr = fabs(last_err - err);
        const bool stop = (err < a.epsilon) || (it > a.max_iters) || (it > 0 && derr < a.stopping_thresh);
        last_err = err;
        dT[0] = uniform_f(static_cast<float>(Tn.m00 - T.m00));
        dT[1] = uniform_f(static_cast<float>(Tn.m01 - T.m01));
        dT[2] = uniform_f(static_cast<float>(Tn.m02 - T.m02));
        dT[3] = uniform_f(static_cast<float>(Tn.m10 - T.m10));
        dT[4] = uniform_f(static_cast<float>(Tn.m11 - T.m11));
        dT[5] = uniform_f(static_cast<float>(Tn.m12 - T.m12));
        {
            const float rr = fmaxf(fabsf(dT[0]) + fabsf(dT[1]), fabsf(dT[3]) + fabsf(dT[4]));
            const float tt = fmaxf(fabsf(dT[2]), fabsf(dT[5]));
            const float big = static_cast<float>(fabs(T.m02) + fabs(T.m12) + fabs(Tn.m02) + fabs(Tn.m12));
            dsig = uniform_f(1e-6f * (rr * ps.pmax + tt) + 1e-9f * (ps.pmax + big) + 1e-30f);
        }
        T.m00 = uniform_d(Tn.m00); T.m01 = uniform_d(Tn.m01); T.m02 = uniform_d(Tn.m02);
        T.m10 = uniform_d(Tn.m10); T.m11 = uniform_d(Tn.m11); T.m12 = uniform_d(Tn.m12);
        tstamp(9);
        if (stop) {
            tflush();
            if (tid == 0 && part == 0) {
                store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                a.out_err[b] = err;
                a.out_iters[b] = it + 1;
            }
            return;
        }
        if (a.phase_cap > 0 && it + 1 - it0 >= a.phase_cap) {
            tflush();
            if (tid == 0 && part == 0) {
                store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                a.out_err[b] = err;
                a.out_iters[b] = -(it + 1);
                a.sched_key[b] = static_cast<float>(derr);
            }
            return;
        }
    }
}

// ---------------------------------------------------------------------------
// Wide tier (latency mode for the few slowest pairs of a small batch).  A pair
// runs on one workgroup per 64-query group (as the team kernel), but the NN
// search is a plain BRUTE-FORCE fp32 screen split over the workgroup's NW
// waves by candidate slices — no window, no clearance, no visit loop: a
// group's cost is the same whatever its queries, so no outlier group sets the
// iteration.  Per iteration:
//   all waves  transform the group's 64 queries, scan their chunks of 32
//              candidates keeping chunk minima (M1, its chunk, M2 over chunks),
//              publish them in LDS (barrier);
//   wave 0     merges the NW partial results in candidate order, rescans the
//              winning chunk (exact index, in-chunk runner-up), certifies in
//              fp64 (the exact scan for the rest, as every kernel), forms the
//              exact grid sums (wave_sum_exact16), exchanges them with the
//              other groups' workgroups (tagged granules), applies the Kabsch
//              update and the stopping rules, and publishes T (barrier).
// The search result is the full screen's (M1 / J1 / runner-up as mode 1), the
// certified match the exact fp64 argmin and the sums exact on fixed grids:
// results equal every other kernel bit for bit.
// ---------------------------------------------------------------------------
#ifndef SLAM_WIDE_WAVES
#define SLAM_WIDE_WAVES 8
#endif
constexpr int kWideWaves = SLAM_WIDE_WAVES;
constexpr int kWideBlock = 64 * kWideWaves;
__host__ __device__ constexpr size_t wide_lds_bytes(int cap, int groups = 1) {
    return red_doubles(kWideBlock * groups) * sizeof(double) +
           static_cast<size_t>(cap) * (sizeof(double2) + sizeof(float2)) +
           static_cast<size_t>(kWideWaves * groups) * 3 * 64 * sizeof(uint32_t) + 24 * sizeof(double) +
           static_cast<size_t>(groups) * 64 * sizeof(int32_t);
}
// The wide tier's pruning bound: the runner-up over this many candidates around
// a query's last match
#ifndef SLAM_WIDE_UWIN
#define SLAM_WIDE_UWIN 5   // round 6: lone pair 21.4k -> 18.0k cycles per iteration against 2, 9: 19.1k
                           // (profiles/r06_wide_stamps5.txt, r06_wide_stamps6.txt)
#endif
constexpr int kUWin = SLAM_WIDE_UWIN;
// A wide slot's global slab (float4 units): the fp32 candidate pairs (cap / 2),
// then one bounding box per chunk of kChunk candidates (cap / kChunk)
__host__ __device__ constexpr int64_t wide_slab_f4(int cap) { return cap / 2 + cap / kChunk; }

// src/icp.py:22-46 + 64-67 from the 16 exact partial sums (lane q holds value
// q, every lane the same T): the Kabsch update of icp_kernel, one wave.
struct KabschOut {
    SE2 Tn;
    double err;
};
__device__ __forceinline__ KabschOut kabsch_from_sums(double tot, const SE2& T, const double* pconst, int n1,
                                                      bool rotation_only) {
    const double n = static_cast<double>(n1);
    const double mvx = (readlane_d(tot, 0) + readlane_d(tot, 1)) / n;   // pc2_avg
    const double mvy = (readlane_d(tot, 2) + readlane_d(tot, 3)) / n;
    KabschOut o;
    o.err = readlane_d(tot, 4) + readlane_d(tot, 5);
    const double2 dp = *reinterpret_cast<const double2*>(pconst + kDpX);
    const double2 mup = *reinterpret_cast<const double2*>(pconst + kMupX);
    const double mux = fma(T.m02, 1.0, fma(T.m01, mup.y, T.m00 * mup.x));   // pc1_avg = T mu_p
    const double muy = fma(T.m12, 1.0, fma(T.m11, mup.y, T.m10 * mup.x));
    const double p00 = fma(-dp.x, mvx, readlane_d(tot, 6) + readlane_d(tot, 7));
    const double p01 = fma(-dp.x, mvy, readlane_d(tot, 8) + readlane_d(tot, 9));
    const double p10 = fma(-dp.y, mvx, readlane_d(tot, 10) + readlane_d(tot, 11));
    const double p11 = fma(-dp.y, mvy, readlane_d(tot, 12) + readlane_d(tot, 13));
    const double s00 = fma(T.m01, p10, T.m00 * p00);
    const double s01 = fma(T.m01, p11, T.m00 * p01);
    const double s10 = fma(T.m11, p10, T.m10 * p00);
    const double s11 = fma(T.m11, p11, T.m10 * p01);
    const double cs = s00 + s11;
    const double sn = s01 - s10;
    const double r = sqrt(cs * cs + sn * sn);
    const double co = r > 0.0 ? cs / r : 1.0;
    const double si = r > 0.0 ? sn / r : 0.0;
    double tx = mvx - fma(-si, muy, co * mux);
    double ty = mvy - fma(co, muy, si * mux);
    if (rotation_only) {
        tx = 0.0;
        ty = 0.0;
    }
    SE2 D;
    D.m00 = co; D.m01 = -si; D.m02 = tx;
    D.m10 = si; D.m11 = co;  D.m12 = ty;
    o.Tn = se2_mul(D, T);
    return o;
}

// The wide pairs' fp32 candidates in the pair layout of candf (cf_put), one
// `cap` slab per wide slot, in global memory: the wide kernel streams them
// through SCALAR loads (s_load_dwordx16: 8 candidates into SGPRs, uniform for
// the wave) instead of LDS broadcasts (1 KB to VGPRs per ds_read_b128).
__global__ __launch_bounds__(256) void wide_prep_kernel(IcpArgs a, float2* __restrict__ wcand) {
    const int slot = blockIdx.x;
    if (slot >= a.n_gangs || (a.take_lt && slot >= *a.take_lt)) return;
    const int b = a.order ? a.order[slot] : slot;
    if (b < 0) return;   // padding (uniform)
    const int s2 = a.dst_scan[b];
    const int64_t o2 = a.scan_off[s2];
    const int n2 = static_cast<int>(a.scan_off[s2 + 1] - o2);
    float2* dst = wcand + 2 * static_cast<int64_t>(slot) * wide_slab_f4(a.cand_cap);
    for (int j = threadIdx.x; j < a.cand_cap; j += 256) {
        float x = kSentinel, y = kSentinel;
        if (j < n2) {
            const double2 p = a.pts[o2 + j];
            x = static_cast<float>(p.x);
            y = static_cast<float>(p.y);
        }
        cf_put(dst, j, x, y);
    }
    // per chunk: the box of its real candidates' fp32 points (a chunk of
    // sentinels only gets a box at the sentinel: its bound is +inf)
    float4* box = reinterpret_cast<float4*>(dst) + a.cand_cap / 2;
    for (int c = threadIdx.x; c < a.cand_cap / kChunk; c += 256) {
        float4 bx = make_float4(kSentinel, kSentinel, kSentinel, kSentinel);
        for (int j = c * kChunk; j < min((c + 1) * kChunk, n2); ++j) {
            const double2 p = a.pts[o2 + j];
            const float x = static_cast<float>(p.x), y = static_cast<float>(p.y);
            const bool first = j == c * kChunk;
            bx.x = first ? x : fminf(bx.x, x);
            bx.y = first ? y : fminf(bx.y, y);
            bx.z = first ? x : fmaxf(bx.z, x);
            bx.w = first ? y : fmaxf(bx.w, y);
        }
        box[c] = bx;
    }
}

// G query groups per workgroup (1: 8 waves; 2: 16 waves, the workgroup a CU
// of its own, round 6): group gq = wave % G (its leader, wave gq, on SIMD gq),
// its NW waves wave = gq + G w.  With G = 2 the two leaders add their exact
// partial sums (order-free) before the one exchange of the workgroup, so a
// 1081-point pair runs on 9 workgroups instead of 17.
template <int G>
__global__ __launch_bounds__(64 * kWideWaves * G) void icp_wide_kernel(IcpArgs a, const float4* __restrict__ wcand) {
    constexpr int NW = kWideWaves;
    constexpr int WAVES = NW * G;
    constexpr int WBLK = 64 * WAVES;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* red0 = reinterpret_cast<double*>(smem);
    double* red1 = red0 + WAVES * 16;
    double* pconst = red0 + 2 * WAVES * 16;
    double2* cand = reinterpret_cast<double2*>(smem + red_doubles(WBLK) * sizeof(double));
    const int cap = a.cand_cap;
    float2* candf = reinterpret_cast<float2*>(cand + cap);
    uint32_t* xs = reinterpret_cast<uint32_t*>(candf + cap);       // [WAVES][3][64]: M1, chunk, M2 per wave
    double* tb = reinterpret_cast<double*>(xs + WAVES * 3 * 64);   // the next T (6) and the flag
    double* gsum = tb + 8;                                         // [16]: group 1's partial sums (G = 2)
    int32_t* pm = reinterpret_cast<int32_t*>(gsum + 16);           // [G][64]: the groups' last matches

    const int parts = a.gang;
    const int bx = static_cast<int>(blockIdx.x);
    const int slot = (bx / (8 * parts)) * 8 + (bx & 7);   // a pair's workgroups on one XCD
    const int part = (bx >> 3) % parts;                     // = its G 64-query groups
    if (slot >= a.n_gangs || (a.take_lt && slot >= *a.take_lt)) return;
    const int b = a.order ? a.order[slot] : slot;
    if (b < 0) return;   // padding (uniform)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gq = wave % G, wg = wave / G;   // query group in the workgroup, wave in the group
    int it0 = 0;
    if (a.resume) {
        const int s = a.out_iters[b];
        if (s > 0 || s == kBadBounds) return;
        it0 = -s;
    }
    const int s1 = a.src_scan[b], s2 = a.dst_scan[b];
    const int64_t o1 = a.scan_off[s1], o2 = a.scan_off[s2];
    const int n1 = static_cast<int>(a.scan_off[s1 + 1] - o1);
    const int n2 = static_cast<int>(a.scan_off[s2 + 1] - o2);
    const double2* __restrict__ p1 = a.pts + o1;
    const double2* __restrict__ p2 = a.pts + o2;
    if (n1 < 1 || n2 < 1 || n1 > 64 * G * parts || n2 > cap) {
        if (tid == 0 && part == 0) {
            a.out_iters[b] = kBadBounds;
            a.out_err[b] = __builtin_nan("");
            atomicOr(&g_icp_status, 1);
        }
        return;
    }
    if (tid == 0 && part == 0) trace_mark(a, b, 0);
    const PairSetup ps = stage_pair<WBLK, true, false>(a, n1, n2, p1, p2, true, cand, candf, nullptr, red0, red1,
                                                       pconst);
    SE2 T = load_se2((it0 > 0 ? a.out_tf : a.init) + 9 * static_cast<int64_t>(b));
    if (a.rotation_only) {
        T.m02 = 0.0;
        T.m12 = 0.0;
    }
    double* hist = a.hist_stride > 0 ? a.out_hist + static_cast<int64_t>(b) * a.hist_stride * 9 : nullptr;
    if (hist && tid == 0 && part == 0 && it0 == 0) store_se2(hist, T);
    double last_err = it0 > 0 ? a.out_err[b] : 0.0;
    const int i = (part * G + gq) * 64 + lane;
    const bool valid = i < n1;
    const int nch = (n2 + kChunk - 1) / kChunk;
    // the slot's fp32 candidate pairs and chunk boxes (wide_prep_kernel), read
    // through scalar loads; wave w scans the chunks w, w + NW, ... (interleaved:
    // the few chunks a group's queries need spread over the waves)
    const float4* __restrict__ cg = wcand + static_cast<int64_t>(slot) * wide_slab_f4(cap);
    const float4* __restrict__ cbox = cg + cap / 2;
    // pruning (round 6): from the second iteration of a launch on, the kUWin
    // candidates around a lane's last match bound the runner-up: U = the second
    // smallest of their screened distances >= M2 >= M1, so a chunk whose box lies farther than U from the lane's
    // query holds neither the minimum nor the runner-up; it is skipped when no
    // lane of the wave needs it.  The certification takes min(M2, U) as its
    // bound on the other candidates (skipped ones are > U): results unchanged.
    bool warm = false;
    uint64_t* slots = a.gang_slots + static_cast<int64_t>(slot) * 2 * parts * 32;
    // diagnostics (a.stamps != NULL): s_memtime per phase of wave 0 of every
    // part, stamps[256 + 16 * part + phase] (tools/wide_stamps.py)
    const bool stamping = a.stamps != nullptr && wave == 0;
    unsigned long long tp = stamping ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto tstamp = [&](int q) {
        if (stamping) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            tacc[q] += t1 - tp;
            tp = t1;
        }
    };
    for (int it = it0;; ++it) {
        double x = 0.0, y = 0.0;
        if (valid) {
            const double2 p = p1[i];
            x = p.x;
            y = p.y;
        }
        const double qx = fma(T.m02, 1.0, fma(T.m01, y, T.m00 * x));
        const double qy = fma(T.m12, 1.0, fma(T.m11, y, T.m10 * x));
        const float fx = static_cast<float>(qx), fy = static_cast<float>(qy);
        // ---- this wave's slice: chunk minima (screened distances are >= 0:
        //      their bits order as unsigned integers) ---------------------------
        uint32_t M1 = 0xffffffffu, M2 = 0xffffffffu;
        int C1 = 0;
        uint32_t U = 0x7f800000u;   // +inf: no pruning
        if (ps.screen) {
            if (warm) {
                // the second smallest screened distance over kUWin consecutive
                // candidates around the last match (distinct: warm implies n2 >= kUWin)
                const int jb = min(max(pm[gq * 64 + lane] - kUWin / 2, 0), n2 - kUWin);
                uint32_t u1 = 0xffffffffu, u2 = 0xffffffffu;
#pragma unroll
                for (int q = 0; q < kUWin; ++q) {
                    const float2 aq = cf_at(candf, jb + q);
                    take_key(__float_as_uint(screen_d32(aq.x, aq.y, fx, fy)), u1, u2);
                }
                U = valid ? u2 : 0u;
            }
            for (int c = wg; c < nch; c += NW) {
                if (warm) {
                    const float lb = box_lb(f32x2{fx, fy}, f32x2{fx, fy}, cbox[c]);
                    if (!__builtin_amdgcn_ballot_w64(valid && __float_as_uint(lb) <= U)) continue;   // uniform
                }
                const float4* cp = cg + c * (kChunk / 2);
                uint32_t cm = 0xffffffffu;
#pragma unroll
                for (int t = 0; t < kChunk / 2; ++t) {
                    const f32x2v d = screen_pair(cp[t], fx, fy);
                    cm = min(cm, min(__float_as_uint(d.x), __float_as_uint(d.y)));   // v_min3_u32
                }
                C1 = cm < M1 ? c : C1;
                uint32_t md;
                asm("v_med3_u32 %0, %1, %2, %3" : "=v"(md) : "v"(M1), "v"(M2), "v"(cm));
                M2 = md;
                M1 = min(M1, cm);
            }
        }
        tstamp(0);
        xs[(wave * 3 + 0) * 64 + lane] = M1;
        xs[(wave * 3 + 1) * 64 + lane] = static_cast<uint32_t>(C1);
        xs[(wave * 3 + 2) * 64 + lane] = min(M2, U);   // (every wave holds the same U)
        __syncthreads();
        tstamp(1);
        double tot = 0.0;
        if (wave < G) {   // the group leaders
            // merge: the smallest chunk minimum, the lowest chunk on ties (the
            // waves' chunks interleave), and the second smallest over all chunks
            uint32_t m1 = 0xffffffffu, m2 = 0xffffffffu;
            int c1 = 0;
#pragma unroll
            for (int w0 = 0; w0 < NW; ++w0) {
                const int w = gq + G * w0;
                const uint32_t a1 = xs[(w * 3 + 0) * 64 + lane], a2 = xs[(w * 3 + 2) * 64 + lane];
                const int ac = static_cast<int>(xs[(w * 3 + 1) * 64 + lane]);
                c1 = (a1 < m1 || (a1 == m1 && ac < c1)) ? ac : c1;
                m2 = min(max(m1, a1), min(m2, a2));
                m1 = min(m1, a1);
            }
            // the winning chunk: first index reaching the minimum + in-chunk
            // runner-up; its 16 candidate pairs read at once, then two
            // independent chains (even / odd pairs) merged in index order
            float b2 = INFINITY;   // the winning chunk's runner-up (its minimum is the chunk minimum)
            int j1 = c1 * kChunk;
            {
                const float4* cp = reinterpret_cast<const float4*>(candf + c1 * kChunk);
                float e1[2] = {INFINITY, INFINITY}, e2[2] = {INFINITY, INFINITY};
                int ej[2] = {0, 0};
                // (four candidate pairs in flight at a time: 16 VGPRs, not 64 — the
                // 16-wave instance must fit 128 without spilling)
#pragma unroll
                for (int t0 = 0; t0 < kChunk / 2; t0 += 4) {
                    float4 pp[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) pp[u] = cp[t0 + u];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int t = t0 + u;
                        const f32x2v d = screen_pair(pp[u], fx, fy);
                        const int h = t & 1;
                        take_cand(d.x, 2 * t, e1[h], e2[h], ej[h]);
                        take_cand(d.y, 2 * t + 1, e1[h], e2[h], ej[h]);
                    }
                }
                // chain 0 holds offsets {0,1,4,5,...}, chain 1 {2,3,6,7,...}: on a tie
                // the smaller offset wins (the full scan's first index)
                const bool one = e1[1] < e1[0] || (e1[1] == e1[0] && ej[1] < ej[0]);
                j1 += one ? ej[1] : ej[0];
                b2 = fminf(fmaxf(e1[0], e1[1]), fminf(e2[0], e2[1]));
            }
            j1 = min(j1, n2 - 1);
            int bi = j1;
            tstamp(2);
            const double2 cw = cand[j1];
            double dq = exact_d2(cw.x, cw.y, qx, qy);
            bool ok = true;
            if (!ps.screen) {
                ok = !valid;
            } else if (valid && n2 > 1) {
                const double s2 = static_cast<double>(fminf(__uint_as_float(m2), b2));
                const double cq = fmax(fabs(qx), fabs(qy));
                const double ab = (1.0 + 0x1p-24) * 0x1p-24 * (ps.cmax + cq);
                ok = cq < 1e18 && s2 < 3.0e38 && certify(dq, s2, ab);
            }
            uint64_t fails = __ballot(!ok);
            while (fails) {   // the exact fp64 scan for each uncertified query (first index on ties)
                const int src = static_cast<int>(__builtin_ctzll(fails));
                fails &= fails - 1;
                const double xs_ = bcast_d(qx, src), ys_ = bcast_d(qy, src);
                double bd = INFINITY;
                int bj = lane < n2 ? lane : 0x7fffffff;
                for (int j = lane; j < n2; j += 64) {
                    const double2 c = cand[j];
                    const double d = exact_d2(c.x, c.y, xs_, ys_);
                    if (d < bd) {
                        bd = d;
                        bj = j;
                    }
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    const double od = __shfl_xor(bd, off, 64);
                    const int oj = __shfl_xor(bj, off, 64);
                    if (od < bd || (od == bd && oj < bj)) {
                        bd = od;
                        bj = oj;
                    }
                }
                if (lane == src) {
                    bi = bj;
                    dq = bd;
                }
            }
            tstamp(3);
            pm[gq * 64 + lane] = bi;   // the next iteration's prediction (read after the barriers below)
            // sums (as icp_kernel step 4), this group's 64 queries
            const double2 c = *reinterpret_cast<const double2*>(pconst + kPcX);
            const double2 gmv = *reinterpret_cast<const double2*>(pconst + kGm1);
            const double2 gsv = *reinterpret_cast<const double2*>(pconst + kGs1);
            const double2 pcm = *reinterpret_cast<const double2*>(pconst + kPmax);
            const double bq = (fmax(fabs(T.m00) + fabs(T.m01), fabs(T.m10) + fabs(T.m11)) * pcm.x +
                               fmax(fabs(T.m02), fabs(T.m12))) * (1.0 + 1e-12);
            const RsumGrid gm{gmv.x, gmv.y}, gs{gsv.x, gsv.y};
            const RsumGrid gd = rsum_grid(2.0 * (bq + pcm.y) * (bq + pcm.y) * (1.0 + 1e-12), n1);
            double acc[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.0;
            if (valid) {
                const double2 m = cand[bi];
                rsum_add(m.x, gm, acc[0], acc[1]);
                rsum_add(m.y, gm, acc[2], acc[3]);
                rsum_add(dq, gd, acc[4], acc[5]);
                const double ax = x - c.x, ay = y - c.y;
                rsum_add(ax * m.x, gs, acc[6], acc[7]);
                rsum_add(ax * m.y, gs, acc[8], acc[9]);
                rsum_add(ay * m.x, gs, acc[10], acc[11]);
                rsum_add(ay * m.y, gs, acc[12], acc[13]);
            }
            tot = wave_sum_exact16(acc);
            if (G > 1 && gq == 1 && lane < 16) gsum[lane] = tot;
        }
        if constexpr (G > 1) {
            __syncthreads();   // group 1's sums (exact partials: any order gives the same bits)
            if (wave == 0 && lane < 16) tot += gsum[lane];
        }
        if (wave == 0) {
            tstamp(4);
            bool arrived = true;
            if (parts > 1)
                tot = gang_exchange_wave(tot, slots, part, parts, it, it == it0 ? a.gang_wait_first : a.gang_wait, arrived,
                                         it == it0 ? a.gang_abort : nullptr);
            tstamp(5);
            double flag = 0.0;
            if (!arrived) {
                flag = 3.0;   // a partner timed out: write nothing, the repair launch re-runs the pair
            } else {
                const KabschOut ko = kabsch_from_sums(tot, T, pconst, n1, a.rotation_only != 0);
                const SE2& Tn = ko.Tn;
                const double err = ko.err;
                if (hist && lane == 0 && part == 0) store_se2(hist + 9 * (it + 1), Tn);
                const double derr = fabs(last_err - err);
                const bool stop = (err < a.epsilon) || (it > a.max_iters) || (it > 0 && derr < a.stopping_thresh);
                last_err = err;
                if (stop) {
                    flag = 1.0;
                    if (lane == 0 && part == 0) {
                        store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                        a.out_err[b] = err;
                        a.out_iters[b] = it + 1;
                        trace_mark(a, b, 1);
                    }
                } else if (a.phase_cap > 0 && it + 1 - it0 >= a.phase_cap) {
                    flag = 2.0;
                    if (lane == 0 && part == 0) {
                        store_se2(a.out_tf + 9 * static_cast<int64_t>(b), Tn);
                        a.out_err[b] = err;
                        a.out_iters[b] = -(it + 1);
                        a.sched_key[b] = static_cast<float>(derr);
                        trace_mark(a, b, 1);
                    }
                }
                if (lane == 0) {
                    tb[0] = Tn.m00; tb[1] = Tn.m01; tb[2] = Tn.m02;
                    tb[3] = Tn.m10; tb[4] = Tn.m11; tb[5] = Tn.m12;
                }
            }
            if (lane == 0) tb[6] = flag;
            tstamp(6);
        }
        __syncthreads();
        tstamp(7);
        if (tb[6] != 0.0) {   // uniform: stop, pause or a lost partner
            if (stamping && lane == 0)
                for (int q = 0; q < 8; ++q) atomicAdd(a.stamps + 256 + 16 * part + q, tacc[q]);
            return;
        }
        T.m00 = uniform_d(tb[0]); T.m01 = uniform_d(tb[1]); T.m02 = uniform_d(tb[2]);
        T.m10 = uniform_d(tb[3]); T.m11 = uniform_d(tb[4]); T.m12 = uniform_d(tb[5]);
        warm = n2 >= kUWin;
    }
}

// ---------------------------------------------------------------------------
// Instance table.  A (BLOCK, QPT) instance holds BLOCK*QPT queries in
// registers; the host picks the smallest capacity >= max_n1 so idle lanes stay
// few (1081-point scans: 64x17 = 1088 -> 99.4 % of lanes busy).
// ---------------------------------------------------------------------------
using KernelFn = void (*)(IcpArgs);

struct Instance {
    int block;
    int qpt;
    KernelFn batch;          // exact fp64 scan
    KernelFn step;
    KernelFn batch_screen;   // fp32 screen + exact certification, every chunk
    KernelFn step_screen;
    KernelFn batch_prune;    // fp32 screen with exact chunk pruning (default)
    KernelFn step_prune;
    KernelFn batch_prune_diag;   // the same with stamps / evaluation counter (diagnostics)
};

// W: minimum waves per SIMD the pruned batch kernel is compiled for (4 on the
// default 1081-point shape: 128 VGPRs, a few cold spills, +10 % measured)
#define SLAM_INST(B, Q, W)                                                                 \
    {B, Q, icp_kernel<B, Q, false, false>, icp_kernel<B, Q, true, false>,                 \
     icp_kernel<B, Q, false, true>, icp_kernel<B, Q, true, true>,                         \
     icp_kernel<B, Q, false, true, true, W>, icp_kernel<B, Q, true, true, true>,        \
     icp_kernel<B, Q, false, true, true, W, true>}
static const Instance kInstances[] = {
    SLAM_INST(64, 1, 1),   SLAM_INST(64, 2, 1),   SLAM_INST(64, 4, 1),   SLAM_INST(128, 3, 1),
    SLAM_INST(128, 4, 1),  SLAM_INST(192, 4, 1),  SLAM_INST(192, 6, 1),  SLAM_INST(256, 4, 1),
    SLAM_INST(256, 5, kWpe), SLAM_INST(320, 4, 1),  SLAM_INST(384, 3, 1),  SLAM_INST(512, 3, 1),
    SLAM_INST(576, 2, 1),  SLAM_INST(512, 4, 1),  SLAM_INST(512, 6, 1),  SLAM_INST(512, 8, 1),
    SLAM_INST(512, 16, 1),
};
#undef SLAM_INST
constexpr int kNumInstances = sizeof(kInstances) / sizeof(kInstances[0]);
constexpr int kMaxQuery = 512 * 16;

// Relative per-lane throughput of an instance shape, measured on MI355X with
// the C3 workload (profiles/r01_instance_sweep_*.jsonl): QPT 5-6 at 192-256
// threads keeps enough waves resident and enough queries per LDS read.
static double shape_efficiency(int block, int qpt) {
    static const double by_qpt[17] = {0, 0.50, 0.60, 0.80, 0.90, 1.00, 0.88, 0.70, 0.60,
                                      0.50, 0.45, 0.45, 0.40, 0.35, 0.35, 0.30, 0.30};
    double e = by_qpt[qpt < 16 ? qpt : 16];
    if (block > 384) e *= 0.75;
    return e;
}

// Gang kernels (pruned screen, batch mode): one query group per wave (QPT 1),
// BLOCK = 64 x the groups of a pair's largest part.
struct GangInstance {
    int block;
    KernelFn fn;
};
static const GangInstance kGangInstances[] = {
    {64, icp_kernel<64, 1, false, true, true, 1, false, true>},
    {128, icp_kernel<128, 1, false, true, true, 1, false, true>},
    {192, icp_kernel<192, 1, false, true, true, 1, false, true>},
    {256, icp_kernel<256, 1, false, true, true, 1, false, true>},
    {320, icp_kernel<320, 1, false, true, true, 1, false, true>},
    {384, icp_kernel<384, 1, false, true, true, 1, false, true>},
    {512, icp_kernel<512, 1, false, true, true, 1, false, true>},
};

// Bulk gangs (small batches): every pair of a phase as a gang of 2 or 3
// workgroups with the ordinary LDS footprint (4-5 workgroups per CU), so a
// pair's iteration latency halves while the batch cannot fill the GPU with
// whole pairs.  Several query groups per wave as the
// bulk instances; 1081-point scans: 17 groups -> 9 per part (192x3) or 6
// (128x3).
struct BulkGangInstance {
    int parts;
    int block;
    int qpt;
    KernelFn fn;
};
static const BulkGangInstance kBulkGangInstances[] = {
    {2, 192, 3, icp_kernel<192, 3, false, true, true, kWpe, false, true>},
    {2, 256, 3, icp_kernel<256, 3, false, true, true, kWpe, false, true>},
    {3, 128, 3, icp_kernel<128, 3, false, true, true, kWpe, false, true>},
    {3, 192, 2, icp_kernel<192, 2, false, true, true, kWpe, false, true>},
    // round 6: gangs of 4 / 6 for the angle pre-tier (slam_icp_set_angle_tier_kind)
    {4, 192, 2, icp_kernel<192, 2, false, true, true, kWpe, false, true>},
    {6, 192, 1, icp_kernel<192, 1, false, true, true, kWpe, false, true>},
};
static const BulkGangInstance* pick_bulk_gang_instance(int max_n1, int parts) {
    const int groups = (max_n1 + 63) / 64;
    const int per = (groups + parts - 1) / parts;
    const BulkGangInstance* best = nullptr;
    for (const BulkGangInstance& g : kBulkGangInstances)
        if (g.parts == parts && g.block / 64 * g.qpt >= per && (!best || g.block * g.qpt < best->block * best->qpt))
            best = &g;
    return best;
}

// the smallest gang instance holding ceil(groups / parts) groups, or NULL
static const GangInstance* pick_gang_instance(int max_n1, int parts) {
    const int groups = (max_n1 + 63) / 64;
    const int per = (groups + parts - 1) / parts;
    for (const GangInstance& g : kGangInstances)
        if (g.block >= 64 * per) return &g;
    return nullptr;
}

static const Instance* pick_instance(int max_n1, int forced) {
    if (forced >= 0 && forced < kNumInstances) return &kInstances[forced];
    const Instance* bestp = nullptr;
    double best_cost = 0.0;
    for (int i = 0; i < kNumInstances; ++i) {
        const Instance& c = kInstances[i];
        const int capq = c.block * c.qpt;
        if (capq < max_n1) continue;
        const double cost = static_cast<double>(capq) / shape_efficiency(c.block, c.qpt);
        if (!bestp || cost < best_cost) {
            bestp = &c;
            best_cost = cost;
        }
    }
    return bestp;
}

static thread_local int g_forced_instance = -1;

// get_transform + get_error on already-matched rows (src/icp.py:22-52), one
// workgroup; the same reductions and closed form as the fused kernel.
constexpr int kKabschBlock = 256;
__global__ __launch_bounds__(kKabschBlock) void kabsch_kernel(const double2* __restrict__ pa,
                                                              const double2* __restrict__ pb,
                                                              int64_t n, double* out_T,
                                                              double* out_err) {
    constexpr int WAVES = kKabschBlock / 64;
    __shared__ double red[2 * WAVES * 5];
    double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t i = threadIdx.x; i < n; i += kKabschBlock) {
        const double2 p = pa[i], q = pb[i];
        const double dx = p.x - q.x, dy = p.y - q.y;
        v[0] += p.x;
        v[1] += p.y;
        v[2] += q.x;
        v[3] += q.y;
        v[4] += dx * dx + dy * dy;
    }
    block_sum<5, WAVES>(v, red);
    const double nn = static_cast<double>(n);
    const double mux = v[0] / nn, muy = v[1] / nn, mvx = v[2] / nn, mvy = v[3] / nn;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t i = threadIdx.x; i < n; i += kKabschBlock) {
        const double2 p = pa[i], q = pb[i];
        const double xa = p.x - mux, ya = p.y - muy, xb = q.x - mvx, yb = q.y - mvy;
        s[0] = fma(xa, xb, s[0]);
        s[1] = fma(xa, yb, s[1]);
        s[2] = fma(ya, xb, s[2]);
        s[3] = fma(ya, yb, s[3]);
    }
    block_sum<4, WAVES>(s, red + WAVES * 5);
    if (threadIdx.x == 0) {
        const double cs = s[0] + s[3], sn = s[1] - s[2];
        const double r = sqrt(cs * cs + sn * sn);
        const double c = r > 0.0 ? cs / r : 1.0;
        const double si = r > 0.0 ? sn / r : 0.0;
        SE2 D;
        D.m00 = c;  D.m01 = -si; D.m02 = mvx - fma(-si, muy, c * mux);
        D.m10 = si; D.m11 = c;   D.m12 = mvy - fma(c, muy, si * mux);
        store_se2(out_T, D);
        *out_err = v[4];
    }
}

// NN search mode: 0 exact fp64 scan, 1 fp32 screen (all chunks), 2 fp32
// screen with exact chunk pruning (default).  Results are identical in all
// three (tests/test_icp_gpu.py::test_nn_modes_identical).
static thread_local int g_screen = 2;
// XCD-aware pair map of order-free launches: runs of this many consecutive
// pairs per XCD (0 = identity; diagnostics)
static thread_local int g_xcd_map = 16;
static thread_local unsigned long long* g_icp_stamps = nullptr;
static thread_local unsigned long long* g_icp_evals = nullptr;
static thread_local unsigned long long* g_icp_trace = nullptr;

// inst_override / lds_min: the scheduler's CU-exclusive head launch (below)
static int launch(bool step, const IcpArgs& args, int32_t B, int32_t max_n1, int32_t max_n2,
                  void* stream, const Instance* inst_override = nullptr, size_t lds_min = 0) {
    if (B <= 0) return ok();   // e.g. a scheduler tier left empty
    const Instance* inst = inst_override ? inst_override : pick_instance(max_n1, g_forced_instance);
    if (!inst) return fail(SLAM_ETOOBIG, "query scan of %d points exceeds capacity %d", max_n1, kMaxQuery);
    IcpArgs a = args;
    a.stamps = g_icp_stamps;
    a.evals = g_icp_evals;
    a.cand_cap = max_n2 < kCandCap ? ((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk : kCandCap;
    int mode = max_n2 <= kCandCap ? g_screen : 0;
    auto lds_of = [&](int m) {
        size_t l = red_doubles(inst->block) * sizeof(double) + static_cast<size_t>(a.cand_cap) * sizeof(double2);
        if (m >= 1) l += static_cast<size_t>(a.cand_cap) * sizeof(float2);
        if (m == 2)
            l += static_cast<size_t>(a.cand_cap / kSub) * sizeof(float4) +
                 static_cast<size_t>(inst->block) * inst->qpt * 2 * sizeof(int32_t);
        return l;
    };
    // the pruned screen's per-query LDS state does not fit next to 4,096
    // candidates for the largest query shapes: the full screen (same results) then
    if (mode == 2 && lds_of(2) > kMaxLds) mode = 1;
    const size_t lds = max(lds_of(mode), lds_min);
    const bool diag = (a.stamps || a.evals) && mode == 2 && !step;   // diagnostics: pruned batch only
    KernelFn fn = mode == 2 ? (step ? inst->step_prune : (diag ? inst->batch_prune_diag : inst->batch_prune))
                : mode == 1 ? (step ? inst->step_screen : inst->batch_screen)
                            : (step ? inst->step : inst->batch);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds));
    int grid = B;
    a.xcd_run = 0;
    a.n_pairs = B;
    if (!step && !a.order && g_xcd_map > 0 && B >= 64) {   // XCD-aware pair map (IcpArgs::xcd_run)
        a.xcd_run = g_xcd_map;
        grid = (B + 8 * g_xcd_map - 1) / (8 * g_xcd_map) * 8 * g_xcd_map;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(inst->block), lds, as_stream(stream), a);
    return check_launch(step ? "icp_step kernel" : "icp_batch kernel");
}

// ---------------------------------------------------------------------------
// Phased scheduling of a large batch.  ICP iteration counts have a long tail
// (C3: mean 18, p99 36, max 102), and a slow pair that happens to start late
// keeps the GPU waiting (natural order 8.5 ms vs 5.0 ms for the same pairs
// sorted by their iteration counts).  Phase 1 runs every pair for kProbe
// iterations and pauses the unfinished ones; their last error change |dE|
// (large = far from the |dE| < stopping_thresh exit) orders phase 2, longest
// first, by a 256-bucket counting sort on log2 |dE| (order within a bucket is
// arbitrary and irrelevant: pairs are independent and every result is
// bit-identical to the single-launch run).
// ---------------------------------------------------------------------------
constexpr int kSchedBuckets = 256;
static thread_local int g_sched_probe = -1;   // phase-1 iterations (0: single launch; -1: automatic, sched_probe_for)
// Automatic probe length.  Round 4 (profiles/r04_probe_shards*.txt, C3
// stream): 3 iterations for the full batch (10k pairs: 4.09 ms; 2: 4.11, 4:
// 4.27) and for 1,250 / 5,000-pair shards; 4 for 2,048-4,095 pairs, where the
// tail tiers run and a longer probe keys them better (2,500 pairs: 2.03-2.04
// ms against 2.14-2.15 with 3; 1,250 pairs: 1.49 against 1.44).  Round 6, at
// the round-6 kernels and tiers, timed as bench.py times (20 back-to-back
// launches, settings alternated on one box, profiles/r06_ab_probe*.txt): 2 for
// 4,096-8,192 pairs (the 2-rank shards' maximum 2.55 / 2.71 ms on seeds 2025 /
// 7, against 2.55 / 2.84 with 3 and 2.50 / 2.95 with 4); the 10k batch keeps 3
// (3.97 / 4.33 ms against 4.03 / 4.19 with 2: a wash over the two seeds), the
// 1,250-pair shards 3 (2: 1.08-1.09 against 1.03-1.06), 2,048-4,095 pairs 4
static int sched_probe_for(int B) { return B >= 4096 && B <= 8192 ? 2 : B >= 2048 && B < 4096 ? 4 : 3; }
static thread_local int g_sched_min_pairs = 1024;   // batches below this fit the GPU at once
// Phase 2 starts the pairs the probe keyed slowest (the top g_sched_heads, at
// most one per 16 pairs) on workgroups that request the whole LDS of a CU, so
// no other workgroup shares their CU, with an 8-wave instance (a lone pair's
// iteration latency: 512x3 ~19-21 us vs 256x5 ~29 us on C3's longest pair)
// beside the rest, which runs on a second stream: the long tail bounds a
// sharded stream (64 heads measured best: 5,000 / 2,500 /
// 1,250-pair shards 3.47 / 3.10 / 2.31 -> 2.88 / 2.41 / 1.79 ms, 10k pairs
// unchanged).  Those pairs' sums run over another wave layout: results equal
// the single launch to rounding (correspondences exact, iterations equal).
static thread_local int g_sched_heads = 64;
// a full C3 batch (10k pairs) keeps every CU for the bulk: heads there cost ~3 %;
// round 4 (probe 3, profiles/r04_strong_probe.txt): the 5,000-pair shard runs
// 3.12 ms without the exchange/head tiers and 3.40 ms with them, the 2,500-pair
// shard 2.84 vs 2.31 ms, so the tiers start below 4,096 pairs
#ifndef SLAM_AUTO_ANGLE
#define SLAM_AUTO_ANGLE 40
#endif
#ifndef SLAM_AUTO_SHARE
#define SLAM_AUTO_SHARE 2
#endif
constexpr int kHeadsMaxPairs = 4096;
static thread_local int g_tiers_below = kHeadsMaxPairs;   // batches below this get the tail tiers

static const Instance* pick_head_instance(int max_n1) {
    const Instance* best = nullptr;
    for (int i = 0; i < kNumInstances; ++i) {
        const Instance& c = kInstances[i];
        if (c.block != 512 || c.block * c.qpt < max_n1) continue;
        if (!best || c.qpt < best->qpt) best = &c;
    }
    return best;
}

// Gangs: the top g_sched_gangs of the head pairs run on g_sched_gang_parts
// workgroups each (one query group per wave, CU-exclusive, one XCD per gang),
// which exchange their partial sums every iteration: a lone pair's iteration
// latency is then one query group's search plus the exchange, not a whole
// workgroup's.  Results are bit-identical.
static thread_local int g_sched_gangs = 24;
static thread_local int g_sched_gang_parts = 4;
static thread_local uint32_t g_gang_wait = kGangWaitTicks;   // diagnostics can shorten it to force timeouts
// A pair's first exchange in a launch waits at most this long: a partner that
// is not resident by then (CUs held by another process, or a shard whose
// exchange tiers outnumber the CUs for that long) makes the pair give up at
// once and the repair launch run it on one workgroup — a stall of milliseconds,
// not the 0.2 s of a later exchange (where every partner has been seen)
constexpr uint32_t kGangWaitFirstTicks = 400000;   // 4 ms
static thread_local uint32_t g_gang_wait_first = kGangWaitFirstTicks;
// Wide tier: the top g_sched_wide keyed pairs of a batch below kHeadsMaxPairs
// run on icp_wide_kernel, one workgroup per 64-query group, each requesting
// kMaxLds / g_wide_share of LDS (1: CU-exclusive)
static thread_local int g_sched_wide = 0;
static thread_local int g_wide_share = 1;
// Bulk gangs: batches of fewer than g_bulk_gang_below pairs run both phases'
// bulk as gangs of g_bulk_gang_parts workgroups (0 / 1 parts: off)
static thread_local int g_bulk_gang_below = 0;
static thread_local int g_bulk_gang_parts = 2;
// carry the paused pairs' search state from phase 1 to phase 2 (warm resume)
static thread_local int g_sched_warm = 0;
// batches of <= kSortOneMax pairs sort on one workgroup (diagnostics: 0 = the
// three-kernel sort at every size)
static thread_local int g_sched_sort_one = 1;
// Angle pre-tier (batches of up to kSortOneMax pairs): up to g_angle_max pairs
// whose initial transform turns by more than g_angle_thresh rad — the C3
// stream's long pairs all start at a turn of 0.5-3 rad —
// run on a tier of their own from the start, beside phase 1 of the others
// (0: off)
static thread_local int g_angle_max = 0;
static thread_local float g_angle_thresh = 0.3f;
// the pre-tier's kind: 0 the wide tier (g_wide_share workgroups per CU), or
// 2 / 3: bulk gangs of that many ordinary workgroups (cheap enough for the
// larger shards' dozens of turning pairs)
static thread_local int g_angle_kind = 0;
// with a gang pre-tier (kind 2 / 3): its first g_angle_mix turning pairs (the
// largest turns) on wide workgroups instead, g_angle_mix_share per CU (0: none)
static thread_local int g_angle_mix = 0;
static thread_local int g_angle_mix_share = 2;
// Automatic tier profile by batch size (the default; any explicit tier setter
// turns it off, slam_icp_set_schedule_auto(1) turns it back on), measured on
// every rank's shard of the 10k C3 stream and of a second stream (seed 7),
// contiguous and cost-balanced (tools/shard_sweep.py, profiles/r06_wide_sweep*.txt):
//   B <  kAutoSmall (8-rank shards): the angle pre-tier, up to kAutoAngle
//        turning pairs (all of a shard's, in practice) on wide workgroups of
//        two query groups, one per CU; no phase-2 tiers (round 6: 1,250-pair
//        shards 1.18-1.19 ms balanced, against 1.55 with 24 pairs two per CU);
//   B <  kHeadsMaxPairs (4-rank shards): the same with up to kAutoMidWide
//        pairs (2,500 pairs: 1.91 / 2.10 ms on the two streams, against 2.58 /
//        3.23 with the gang pre-tier);
//   B <= kSortOneMax (2-rank shards): the angle pre-tier as bulk gangs of 4
//        (kAutoMidAngle pairs; round 6: 2.57 / 2.84 ms on seeds 2025 / 7
//        against 2.61 / 3.27 with gangs of 3, gangs of 6 2.64 / 2.92,
//        profiles/r06_gangk_sweep.txt) and, in phase 2, 64 heads, the first 24
//        as gangs of 4 (round 5: 96 pre-tier pairs 2.55 ms, 48 2.79, the heads
//        alone 3.77, profiles/r05_shard_sweep11.txt; the wide pre-tier there
//        3.1-3.9 ms: 9 CUs per turning pair starve the bulk);
//   larger batches: no tiers.
static thread_local int g_sched_auto = 1;
// drain tier (launch_batch): when at most this many of phase 2's bulk pairs
// have not stopped, the running ones pause and finish on wide workgroups (-1:
// kDrainPairs up to kSortOneMax pairs, none above; 0: off).  Measured on the
// C3 shards (profiles/r06_drain_sweep2.txt, balanced, two rounds): 2 / 4 / 8
// ranks 2.65-2.66 / 1.77-1.78 / 1.11-1.12 ms against 2.69 / 1.85-1.86 /
// 1.13-1.17 without; 12, 16 and 28 pairs within noise of 24
constexpr int kDrainPairs = 24;   // x 9 CU-exclusive workgroups (1081-point scans, two groups each): 216 CUs
static thread_local int g_drain = -1;
constexpr int kAutoSmall = 2048;
constexpr int kAutoMidAngle = 96;
constexpr int kAutoMidWide = 64;
constexpr int kAutoAngle = SLAM_AUTO_ANGLE;
constexpr int kAutoShare = SLAM_AUTO_SHARE;

// per device: the side streams and the fork / join events (created once, reused)
struct SideStream {
    hipStream_t stream = nullptr, stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;
    hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr, join3 = nullptr, join4 = nullptr;
};
static SideStream* side_stream(int dev) {
    static SideStream side[64];
    if (dev < 0 || dev >= 64) return nullptr;
    SideStream& e = side[dev];
    if (!e.stream) {
        // (round 5: the exchange tiers on the highest stream priority, the gangs
        // on a side stream, measured slower: profiles/r05_shard_sweep2.txt)
        if (hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&e.stream2, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&e.stream3, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&e.stream4, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join2, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join3, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join4, hipEventDisableTiming) != hipSuccess) {
            e.stream = nullptr;
            return nullptr;
        }
    }
    return &e;
}

// G pairs (args.order[0..G)) as gangs of `parts` workgroups; slots (G x 2 x
// parts x 32 uint64 granules, zeroed on `s` before this) are stream-ordered
// workspace.  Every gang's parts must be
// co-resident: G * parts workgroups of one CU each stay far below the CU count.
static int launch_gangs(const IcpArgs& args, int G, int parts, bool team, int max_n1, int max_n2, hipStream_t s,
                        uint64_t* slots) {
    if (team) {   // one query group per workgroup, the group's search split over its kTeam waves
        if (max_n2 > kCandCap || parts < 1 || parts > kTeamMaxParts) return fail(SLAM_EINVAL, "icp teams: shape");
        IcpArgs a = args;
        a.stamps = g_icp_stamps;   // diagnostics: per-part phase cycles (icp_team_kernel)
        a.evals = nullptr;
        a.cand_cap = ((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk;
        a.gang = parts;
        a.n_gangs = G;
        a.gang_slots = slots;
        a.gang_wait = g_gang_wait;
    a.gang_wait_first = min(g_gang_wait, g_gang_wait_first);
        const size_t lds_need = red_doubles(kTeamBlock) * sizeof(double) +
                                static_cast<size_t>(a.cand_cap) * (sizeof(double2) + sizeof(float2)) +
                                static_cast<size_t>(a.cand_cap / kSub) * sizeof(float4) + team_xbuf_words() * sizeof(uint32_t);
        if (lds_need > kMaxLds) return fail(SLAM_EINVAL, "icp teams: LDS");
        const size_t lds = max(lds_need, kMaxLds / kTailShare);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(icp_team_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        hipLaunchKernelGGL(icp_team_kernel, dim3((G + 7) / 8 * 8 * parts), dim3(kTeamBlock), lds, s, a);
        return check_launch("icp team kernel");
    }
    const GangInstance* gi = pick_gang_instance(max_n1, parts);
    if (!gi || parts < 2 || parts > kGangMax || max_n2 > kCandCap) return fail(SLAM_EINVAL, "icp gangs: no instance");
    IcpArgs a = args;
    a.stamps = nullptr;
    a.evals = nullptr;
    a.cand_cap = ((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk;
    a.gang = parts;
    a.n_gangs = G;
    a.gang_slots = slots;
    a.gang_wait = g_gang_wait;
    a.gang_wait_first = min(g_gang_wait, g_gang_wait_first);
    const size_t lds_need = red_doubles(gi->block) * sizeof(double) + static_cast<size_t>(a.cand_cap) * sizeof(double2) +
                            static_cast<size_t>(a.cand_cap) * sizeof(float2) +
                            static_cast<size_t>(a.cand_cap / kSub) * sizeof(float4) +
                            static_cast<size_t>(gi->block) * 2 * sizeof(int32_t);
    if (lds_need > kMaxLds) return fail(SLAM_EINVAL, "icp gangs: LDS");
    const size_t lds = max(lds_need, kMaxLds / kTailShare);   // 1: whole CU (a gang's latency is its slowest part)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gi->fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds));
    const int blocks = (G + 7) / 8 * 8 * parts;
    hipLaunchKernelGGL(gi->fn, dim3(blocks), dim3(gi->block), lds, s, a);
    return check_launch("icp gang kernel");
}

// B pairs (args.order, or identity) as bulk gangs (instance `bg`), slots:
// B x 2 x parts x 32 granules, zeroed once per batch.
static int launch_bulk_gangs(const IcpArgs& args, int B, const BulkGangInstance* bg, int max_n2, hipStream_t s,
                             uint64_t* slots) {
    if (B <= 0) return ok();
    IcpArgs a = args;
    a.stamps = nullptr;
    a.evals = nullptr;
    a.cand_cap = ((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk;
    a.gang = bg->parts;
    a.n_gangs = B;
    a.gang_slots = slots;
    a.gang_wait = g_gang_wait;
    a.gang_wait_first = min(g_gang_wait, g_gang_wait_first);
    const size_t lds = red_doubles(bg->block) * sizeof(double) + static_cast<size_t>(a.cand_cap) * sizeof(double2) +
                       static_cast<size_t>(a.cand_cap) * sizeof(float2) +
                       static_cast<size_t>(a.cand_cap / kSub) * sizeof(float4) +
                       static_cast<size_t>(bg->block) * bg->qpt * 2 * sizeof(int32_t);
    if (lds > kMaxLds) return fail(SLAM_EINVAL, "icp bulk gangs: LDS");
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(bg->fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(lds));
    hipLaunchKernelGGL(bg->fn, dim3((B + 7) / 8 * 8 * bg->parts), dim3(bg->block), lds, s, a);
    return check_launch("icp bulk gang kernel");
}

// W pairs (args.order[0..W)) on the wide tier: one workgroup per 64-query
// group, the parts of a pair on one XCD (slots as launch_gangs).
static thread_local int g_wide_groups = 1;   // explicit settings: query groups per wide workgroup
static int launch_wide(const IcpArgs& args, int W, int max_n1, int max_n2, hipStream_t s, uint64_t* slots,
                       float2* wcand, int share, int groups) {
    const int G = groups > 1 ? 2 : 1;
    const int parts = (max_n1 + 64 * G - 1) / (64 * G);
    if (max_n2 > kCandCap || parts < 1 || parts > kTeamMaxParts) return fail(SLAM_EINVAL, "icp wide tier: shape");
    IcpArgs a = args;
    a.stamps = g_icp_stamps;   // diagnostics: per-part phase cycles (icp_wide_kernel)
    a.evals = nullptr;
    a.cand_cap = ((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk;
    a.gang = parts;
    a.n_gangs = W;
    a.gang_slots = slots;
    a.gang_wait = g_gang_wait;
    a.gang_wait_first = min(g_gang_wait, g_gang_wait_first);
    const size_t need = wide_lds_bytes(a.cand_cap, G);
    if (need > kMaxLds) return fail(SLAM_EINVAL, "icp wide tier: LDS");
    // two groups per workgroup: 16 waves, one workgroup per CU (share 1)
    const size_t lds = max(need, kMaxLds / static_cast<size_t>(G > 1 ? 1 : max(share, 1)));
    const void* fn = G > 1 ? reinterpret_cast<const void*>(icp_wide_kernel<2>) : reinterpret_cast<const void*>(icp_wide_kernel<1>);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(wide_prep_kernel, dim3(W), dim3(256), 0, s, a, wcand);
    if (G > 1)
        hipLaunchKernelGGL(icp_wide_kernel<2>, dim3((W + 7) / 8 * 8 * parts), dim3(2 * kWideBlock), lds, s, a,
                           reinterpret_cast<const float4*>(wcand));
    else
        hipLaunchKernelGGL(icp_wide_kernel<1>, dim3((W + 7) / 8 * 8 * parts), dim3(kWideBlock), lds, s, a,
                           reinterpret_cast<const float4*>(wcand));
    return check_launch("icp wide kernel");
}

// Stable counting sort of the pairs by bucket, so order[] (which pairs become
// gangs, heads, bulk) is the same every run: per block of kSortBlock pairs a
// histogram hist_blk[blk][q] (LDS atomics: counts are order-free), an
// exclusive scan over (bucket, block) in bucket-major order, then a scatter
// where a pair lands at its (bucket, block) offset plus the number of earlier
// pairs of its block in the same bucket (wave match loop + per-wave counts).
constexpr int kSortBlock = 1024;
constexpr int kNB = kSchedBuckets + 1;   // buckets incl. "finished"
constexpr int kScanChunk = 32;           // blocks per LDS chunk of the scan (32 KB)

__device__ __forceinline__ int sched_bucket(const int32_t* iters, const float* key, int b, float thresh) {
    const int s = iters[b];
    // finished and out-of-bounds pairs go last (their workgroups exit at once)
    if (s > 0 || s == kBadBounds) return kSchedBuckets;
    // not started (a phase-1 bulk gang that timed out left out_iters 0 and no
    // key): it has every iteration ahead of it, so it goes first; the key is
    // read only for paused pairs, which wrote it
    if (s == 0) return 0;
    const float l = log2f(fmaxf(key[b] / thresh, 1e-30f));   // 8 buckets per octave, 2^16 -> 0
    return min(max(static_cast<int>(floorf(128.0f - 8.0f * l)), 0), kSchedBuckets - 1);
}

__global__ __launch_bounds__(kSortBlock) void sched_count_kernel(const int32_t* __restrict__ iters,
                                                                 const float* __restrict__ key, int32_t B,
                                                                 float thresh, int32_t* __restrict__ hist_blk,
                                                                 int32_t* __restrict__ bucket) {
    __shared__ int h[kNB];
    for (int q = threadIdx.x; q < kNB; q += kSortBlock) h[q] = 0;
    __syncthreads();
    const int b = blockIdx.x * kSortBlock + threadIdx.x;
    if (b < B) {
        const int q = sched_bucket(iters, key, b, thresh);
        bucket[b] = q;
        atomicAdd(&h[q], 1);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kNB; q += kSortBlock) hist_blk[blockIdx.x * kNB + q] = h[q];
}

// One workgroup: hist_blk[blk][q] <- sum of the counts of all (q' < q, any
// block) and (q, blk' < blk): the first slot of (bucket q, block blk).
__global__ __launch_bounds__(512) void sched_scan_kernel(int32_t* __restrict__ hist_blk, int32_t nblk,
                                                        int32_t* __restrict__ n_out) {
    __shared__ int chunk[kScanChunk * kNB];
    __shared__ int tot[512];
    const int q = threadIdx.x;
    int run = 0;   // column q's running count over the blocks
    for (int k0 = 0; k0 < nblk; k0 += kScanChunk) {
        const int nk = min(kScanChunk, nblk - k0);
        for (int i = threadIdx.x; i < nk * kNB; i += 512) chunk[i] = hist_blk[k0 * kNB + i];   // coalesced, in flight
        __syncthreads();
        if (q < kNB) {
            for (int k = 0; k < nk; ++k) {
                const int c = chunk[k * kNB + q];
                chunk[k * kNB + q] = run;
                run += c;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nk * kNB; i += 512) hist_blk[k0 * kNB + i] = chunk[i];
        __syncthreads();
    }
    // exclusive scan of the bucket totals (Hillis-Steele over 512 slots)
    tot[q] = q < kNB ? run : 0;
    __syncthreads();
    for (int d = 1; d < 512; d <<= 1) {
        const int v = q >= d ? tot[q - d] : 0;
        __syncthreads();
        tot[q] += v;
        __syncthreads();
    }
    const int base = q < kNB ? tot[q] - run : 0;
    if (n_out && q == kSchedBuckets) *n_out = base;   // the unfinished pairs (every bucket before the last)
    __syncthreads();
    tot[q] = base;
    __syncthreads();
    for (int i = threadIdx.x; i < nblk * kNB; i += 512) hist_blk[i] += tot[i % kNB];
}

__global__ __launch_bounds__(kSortBlock) void sched_scatter_kernel(const int32_t* __restrict__ bucket, int32_t B,
                                                                   const int32_t* __restrict__ hist_blk,
                                                                   int32_t* __restrict__ order) {
    constexpr int WAVES = kSortBlock / 64;
    __shared__ int cnt[WAVES * kNB];
    for (int i = threadIdx.x; i < WAVES * kNB; i += kSortBlock) cnt[i] = 0;
    __syncthreads();
    const int b = blockIdx.x * kSortBlock + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool valid = b < B;
    const int q = valid ? bucket[b] : -1;
    // rank among the wave's lanes with the same bucket: one ballot per distinct bucket
    int rank = 0;
    uint64_t todo = __ballot(valid);
    while (todo) {
        const int u = __shfl(q, static_cast<int>(__builtin_ctzll(todo)), 64);
        const uint64_t m = __ballot(q == u);
        if (q == u) rank = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0) cnt[wave * kNB + u] = __popcll(m);
        todo &= ~m;
    }
    __syncthreads();
    if (valid) {
        int pos = hist_blk[blockIdx.x * kNB + q] + rank;
        for (int w = 0; w < wave; ++w) pos += cnt[w * kNB + q];
        order[pos] = b;
    }
}

// The same stable order as count + scan + scatter for a batch of at most
// kSortOneMax pairs, in ONE workgroup (one launch instead of three, the phase
// boundary of a strong-scaling shard is a chain of launches): an LDS histogram
// of every pair's bucket, an exclusive scan of the bucket totals, then the
// pairs in chunks of kSortBlock in index order, each placed at its bucket's
// running offset plus its rank among the chunk's earlier pairs of that bucket.
// The workgroup also zeroes `nz` words at `zero` (the phase-2 exchange slots:
// no separate memset on the boundary).
constexpr int kSortOneMax = 8192;
// MODE 0: the phase boundary's sort (sched_bucket) of the pairs ids[koff ..
// B) (koff = *k_dev, 0 without; ids NULL: the pairs 0 .. B-1), order[] = the
// sorted pairs then -1 padding up to B.  MODE 1: the angle pre-tier's order
// (launch_batch): pairs whose initial transform turns by more than `thresh`
// rad first, largest turn first (32 buckets per rad... 255 over [0, pi]), the
// rest in index order; *k_dev = min(#turning pairs, kmax); those pairs'
// out_iters are set to 0 ("not started": the repair launch runs them from
// their initial transform if their tier timed out).
template <int MODE>
__global__ __launch_bounds__(kSortBlock) void sched_sort_one_kernel(const int32_t* __restrict__ iters,
                                                                    const float* __restrict__ key, int32_t B,
                                                                    float thresh, int32_t* __restrict__ order,
                                                                    uint64_t* __restrict__ zero, int64_t nz,
                                                                    const int32_t* __restrict__ ids,
                                                                    int32_t* __restrict__ k_dev,
                                                                    const double* __restrict__ init, int32_t kmax,
                                                                    int32_t* __restrict__ out_iters, int32_t kmix = -1,
                                                                    int32_t* __restrict__ n_out = nullptr, int32_t koff0 = 0) {
    constexpr int WAVES = kSortBlock / 64;
    constexpr int PER = kSortOneMax / kSortBlock;
    __shared__ int base[kNB];
    __shared__ int cnt[WAVES * kNB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int64_t e = tid; e < nz; e += kSortBlock) zero[e] = 0;
    for (int i = tid; i < kNB; i += kSortBlock) base[i] = 0;
    const int koff = MODE == 0 ? (k_dev ? *k_dev : koff0) : 0;
    if constexpr (MODE == 0) {   // ids may hold -1 padding (not placed): every slot starts as padding
        for (int j = tid; j < B; j += kSortBlock) order[j] = -1;
    }
    const int n = B - koff;   // entries sorted
    __syncthreads();
    int q[PER], pb[PER];
#pragma unroll
    for (int c = 0; c < PER; ++c) {
        const int j = c * kSortBlock + tid;
        pb[c] = j < n ? (ids ? ids[koff + j] : j) : -1;
        q[c] = -1;
        if (pb[c] >= 0) {
            if constexpr (MODE == 0) {
                q[c] = sched_bucket(iters, key, pb[c], thresh);
            } else {
                const double* t = init + 9 * static_cast<int64_t>(pb[c]);
                const float ang = fabsf(atan2f(static_cast<float>(t[3]), static_cast<float>(t[0])));
                q[c] = ang > thresh ? min(max(255 - static_cast<int>(ang * (255.0f / 3.14159265f)), 0), 255)
                                    : kSchedBuckets;
            }
            atomicAdd(&base[q[c]], 1);
        }
    }
    __syncthreads();
    if (tid < 64) {   // exclusive scan of the kNB totals by wave 0 (chunks of 64 + a running carry)
        int carry = 0;
        for (int c0 = 0; c0 < kNB; c0 += 64) {
            const int i = c0 + lane;
            const int v = i < kNB ? base[i] : 0;
            int x = v;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            if (i < kNB) base[i] = carry + x - v;
            carry += __shfl(x, 63, 64);
        }
        if (MODE == 0 && lane == 0 && n_out) *n_out = base[kSchedBuckets];   // the unfinished pairs sorted
        if constexpr (MODE == 1) {
            if (lane == 0) *k_dev = min(base[kSchedBuckets], kmax);   // turning pairs precede bucket 256
            if (lane == 0 && kmix >= 0) k_dev[1] = min(base[kSchedBuckets], kmix);   // the mixed pre-tier's wide part
        }
    }
    __syncthreads();
    const int kk = MODE == 1 ? min(base[kSchedBuckets], kmax) : 0;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
        if (c * kSortBlock >= n) break;   // uniform
        for (int i = tid; i < WAVES * kNB; i += kSortBlock) cnt[i] = 0;
        __syncthreads();
        const bool valid = q[c] >= 0;
        int rank = 0;
        uint64_t todo = __ballot(valid);
        while (todo) {
            const int u = __shfl(q[c], static_cast<int>(__builtin_ctzll(todo)), 64);
            const uint64_t m = __ballot(q[c] == u);
            if (q[c] == u) rank = __popcll(m & ((1ull << lane) - 1));
            if (lane == 0) cnt[wave * kNB + u] = __popcll(m);
            todo &= ~m;
        }
        __syncthreads();
        if (valid) {
            int pos = base[q[c]] + rank;
            for (int w = 0; w < wave; ++w) pos += cnt[w * kNB + q[c]];
            order[pos] = pb[c];
            if (MODE == 1 && pos < kk) out_iters[pb[c]] = 0;
        }
        __syncthreads();
        // the chunk's totals advance the running offsets (one thread per bucket)
        for (int i = tid; i < kNB; i += kSortBlock) {
            int t = 0;
            for (int w = 0; w < WAVES; ++w) t += cnt[w * kNB + i];
            base[i] += t;
        }
        __syncthreads();
    }
}

static int launch_batch(const IcpArgs& args, int32_t B, int32_t max_n1, int32_t max_n2, void* stream) {
    const int probe = g_sched_probe >= 0 ? g_sched_probe : sched_probe_for(B);
    if (probe <= 0 || B < g_sched_min_pairs || args.max_iters + 2 <= probe)
        return launch(false, args, B, max_n1, max_n2, stream);
    hipStream_t s = as_stream(stream);
    const size_t nb = static_cast<size_t>(B);
    // tiers of phase 2: gangs (order[0, G)), CU-exclusive heads (order[G, H)),
    // the rest (order[H, B)) beside them
    // the tier profile: explicit settings, or the automatic one by batch size
    int cfg_heads = g_sched_heads, cfg_gangs = g_sched_gangs, cfg_parts = g_sched_gang_parts;
    int cfg_wide = g_sched_wide, cfg_share = g_wide_share, cfg_angle = g_angle_max, cfg_akind = g_angle_kind;
    int cfg_mix = g_angle_mix, cfg_mix_share = g_angle_mix_share, cfg_groups = g_wide_groups;
    int tiers_below = g_tiers_below;
    if (g_sched_auto) {
        cfg_wide = 0;
        cfg_share = 1;
        cfg_parts = 4;
        cfg_akind = 0;
        cfg_mix = 0;
        cfg_mix_share = 2;
        cfg_groups = 1;
        if (B < kAutoSmall) {
            cfg_heads = 0;
            cfg_gangs = 0;
            cfg_angle = kAutoAngle;
            cfg_share = kAutoShare;
            cfg_groups = 2;
        } else if (B < kHeadsMaxPairs) {
            cfg_heads = 0;
            cfg_gangs = 0;
            cfg_angle = kAutoMidWide;
            cfg_groups = 2;
        } else if (B <= kSortOneMax) {
            cfg_heads = 64;
            cfg_gangs = 24;
            cfg_angle = kAutoMidAngle;
            cfg_akind = 4;
            tiers_below = kSortOneMax + 1;
        } else {
            cfg_heads = 0;
            cfg_gangs = 0;
            cfg_angle = 0;
        }
    }
    const int heads = cfg_heads > 0 && B < tiers_below ? min(cfg_heads, max(B / 16, 1)) : 0;
    // gang parts: cfg_parts workgroups per pair, or (0) teams: one workgroup
    // per 64-query group
    const bool team = cfg_parts == 0;
    const int parts = team ? (max_n1 + 63) / 64 : cfg_parts;
    const bool gang_ok = g_forced_instance < 0 && g_screen == 2 && max_n2 <= kCandCap &&
                         (team ? parts <= kTeamMaxParts : parts >= 2 && pick_gang_instance(max_n1, parts) != nullptr);
    // tiers of phase 2: wide (order[0, Wd)), gangs (order[Wd, Wd + G)), heads, bulk
    const int wide_parts = (max_n1 + 63) / 64;
    const bool wide_ok = g_forced_instance < 0 && g_screen == 2 && max_n2 <= kCandCap && wide_parts <= kTeamMaxParts &&
                         wide_lds_bytes(((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk) <= kMaxLds;
    // angle pre-tier: the turning pairs on their own tier from the start (with
    // it, no phase-2 wide tier: measured slower, profiles/r05_shard_sweep8.txt)
    // (bulk gangs run the pruned screen from an LDS-resident pc2: the same
    // conditions as the phase-1 bulk gangs below)
    const bool apg_ok = cfg_akind >= 2 && g_forced_instance < 0 && g_screen == 2 && max_n2 <= kCandCap;
    const BulkGangInstance* apg = apg_ok ? pick_bulk_gang_instance(max_n1, cfg_akind) : nullptr;
    const int ap = (cfg_angle > 0 && (cfg_akind >= 2 ? apg != nullptr : wide_ok) && B <= kSortOneMax &&
                    g_sched_sort_one && B >= g_bulk_gang_below)
                       ? min(cfg_angle, B)
                       : 0;
    // mixed pre-tier: its first `mix` pairs on wide workgroups, the rest on the gangs
    const int mix = (ap > 0 && apg && wide_ok && cfg_mix > 0) ? min(cfg_mix, ap) : 0;
    const int Wd = wide_ok && ap == 0 ? min(cfg_wide, heads) : 0;
    const int G = gang_ok ? max(0, min(cfg_gangs, heads - Wd)) : 0;
    const size_t wide_slot_words = static_cast<size_t>(Wd) * 2 * wide_parts * 32;
    const size_t gang_slot_bytes =
        (static_cast<size_t>(G) * 2 * max(parts, 1) * 32 + wide_slot_words) * sizeof(uint64_t);
    const size_t wide_cand_bytes =
        static_cast<size_t>(Wd) * wide_slab_f4(((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk) * sizeof(float4);
    // bulk gangs for a batch too small to fill the GPU with whole pairs
    const BulkGangInstance* bg =
        B < g_bulk_gang_below && g_bulk_gang_parts >= 2 && g_forced_instance < 0 && g_screen == 2 && max_n2 <= kCandCap
            ? pick_bulk_gang_instance(max_n1, g_bulk_gang_parts)
            : nullptr;
    const size_t bulk_slot_bytes = bg ? nb * 2 * bg->parts * 32 * sizeof(uint64_t) : 0;
    const int nblk = (B + kSortBlock - 1) / kSortBlock;
    const size_t sched_bytes =
        (static_cast<size_t>(nblk) * kNB * sizeof(int32_t) + nb * (2 * sizeof(int32_t) + sizeof(float)) + 255) / 256 * 256;
    // the paused pairs' search state (phase 1 -> 2): 8 B per query + 32 B per pair
    const size_t qsave_bytes = g_sched_warm ? (nb * static_cast<size_t>(max_n1) * sizeof(uint2) + nb * 8 * sizeof(float) +
                                               255) / 256 * 256
                                           : 0;
    // angle pre-tier: order0 (B), its count (device), exchange slots, fp32 candidates
    const size_t cand_cap_w = static_cast<size_t>(((max(max_n2, 1) + kChunk - 1) / kChunk) * kChunk);
    // (a mixed pre-tier: the wide part's slots first, then the gangs' by slot index)
    const size_t ap_mix_words = static_cast<size_t>(mix) * 2 * wide_parts * 32;
    const size_t ap_slot_words = static_cast<size_t>(ap) * 2 * max(wide_parts, max(cfg_akind, 3)) * 32 + ap_mix_words;
    const size_t ap_bytes = ap ? ((nb + 2) * sizeof(int32_t) + 255) / 256 * 256 + ap_slot_words * sizeof(uint64_t) +
                                     static_cast<size_t>(ap) * wide_slab_f4(static_cast<int>(cand_cap_w)) * sizeof(float4)
                               : 0;
    // drain tier: the counters, then its pairs' exchange slots and fp32 candidates
    // (default: batches up to the one-workgroup sort, the strong-scaling shards;
    // the 10k batch ran 1 % slower with it, profiles/r06_drain_sweep2.txt)
    const int drain_cfg = g_drain < 0 ? (B <= kSortOneMax ? kDrainPairs : 0) : g_drain;
    // (a batch above the one-workgroup sort drains only without other phase-2
    // tiers: its three-kernel sort takes every pair)
    const bool one_sort = B <= kSortOneMax && g_sched_sort_one;
    const int drain_x = drain_cfg > 0 && !bg && wide_ok && wide_lds_bytes(static_cast<int>(cand_cap_w), 2) <= kMaxLds &&
                                (one_sort || (heads == 0 && ap == 0))
                            ? drain_cfg
                            : 0;
    const size_t drain_slot_words = static_cast<size_t>(drain_x) * 2 * wide_parts * 32;
    const size_t drain_bytes = drain_x ? 256 + (nb * sizeof(int32_t) + 255) / 256 * 256 + drain_slot_words * sizeof(uint64_t) +
                                             static_cast<size_t>(drain_x) * wide_slab_f4(static_cast<int>(cand_cap_w)) *
                                                 sizeof(float4)
                                       : 0;
    // one abort word per exchange-tier launch (IcpArgs::gang_abort), zeroed up front
    constexpr size_t abort_bytes = 256;
    const size_t bytes = sched_bytes + gang_slot_bytes + wide_cand_bytes + bulk_slot_bytes + qsave_bytes + ap_bytes +
                         drain_bytes + abort_bytes;
    void* ws = nullptr;
    if (hipMallocAsync(&ws, bytes, s) != hipSuccess) return fail(SLAM_EHIP, "icp scheduler: no workspace");
    int32_t* hist = static_cast<int32_t*>(ws);   // hist_blk[nblk][kNB]
    int32_t* bucket = hist + static_cast<size_t>(nblk) * kNB;
    int32_t* order = bucket + nb;
    float* key = reinterpret_cast<float*>(order + nb);
    uint64_t* gang_slots = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + sched_bytes);
    float2* wide_cand = reinterpret_cast<float2*>(static_cast<char*>(ws) + sched_bytes + gang_slot_bytes);
    uint64_t* bulk_slots =
        reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + sched_bytes + gang_slot_bytes + wide_cand_bytes);
    char* ap0 = static_cast<char*>(ws) + sched_bytes + gang_slot_bytes + wide_cand_bytes + bulk_slot_bytes + qsave_bytes;
    int32_t* order0 = ap ? reinterpret_cast<int32_t*>(ap0) : nullptr;   // [B] + the counts at order0[B], [B + 1]
    int32_t* ap_k = ap ? order0 + nb : nullptr;
    uint64_t* ap_slots = ap ? reinterpret_cast<uint64_t*>(ap0 + ((nb + 2) * sizeof(int32_t) + 255) / 256 * 256) : nullptr;
    float2* ap_cand = ap ? reinterpret_cast<float2*>(ap_slots + ap_slot_words) : nullptr;
    char* dr0 = static_cast<char*>(ws) + (bytes - abort_bytes - drain_bytes);
    uint32_t* abortw = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + (bytes - abort_bytes));
    (void)hipMemsetAsync(abortw, 0, abort_bytes, s);
    uint32_t* drain_w = drain_x ? reinterpret_cast<uint32_t*>(dr0) : nullptr;
    int32_t* drain_n = drain_x ? reinterpret_cast<int32_t*>(dr0 + 8) : nullptr;
    int32_t* drain_order = drain_x ? reinterpret_cast<int32_t*>(dr0 + 256) : nullptr;
    uint64_t* drain_slots =
        drain_x ? reinterpret_cast<uint64_t*>(dr0 + 256 + (nb * sizeof(int32_t) + 255) / 256 * 256) : nullptr;
    float2* drain_cand = drain_x ? reinterpret_cast<float2*>(drain_slots + drain_slot_words) : nullptr;
    IcpArgs a = args;
    a.phase_cap = probe;
    a.sched_key = key;
    if (qsave_bytes) {
        char* q0 = static_cast<char*>(ws) + sched_bytes + gang_slot_bytes + wide_cand_bytes + bulk_slot_bytes;
        a.qsave = reinterpret_cast<uint2*>(q0);
        a.dtsave = reinterpret_cast<float*>(q0 + nb * static_cast<size_t>(max_n1) * sizeof(uint2));
        a.qsave_stride = max_n1;
    }
    int rc = 0;
    SideStream* side0 = nullptr;
    // the stream the phases run on: the caller's, or with the pre-tier stream3
    // (the pre-tier then runs on the caller's stream right behind the angle
    // sort, so its workgroups are dispatched before phase 1's, which waits for
    // an event; joined back before the repair launches)
    hipStream_t ms = s;
    if (ap) {
        // the turning pairs first in order0 (their out_iters set to 0: not
        // started), then their tier from their initial transforms; phase 1
        // runs the rest (order0 from *ap_k on)
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) side0 = side_stream(dev);
        if (!side0) return (void)hipFreeAsync(ws, s), fail(SLAM_EHIP, "icp scheduler: side streams");
        hipLaunchKernelGGL(sched_sort_one_kernel<1>, dim3(1), dim3(kSortBlock), 0, s, args.out_iters,
                           static_cast<const float*>(nullptr), B, g_angle_thresh, order0, ap_slots,
                           static_cast<int64_t>(ap_slot_words), static_cast<const int32_t*>(nullptr), ap_k, args.init, ap,
                           args.out_iters, mix > 0 ? mix : -1);
        if (hipEventRecord(side0->fork, s) != hipSuccess || hipStreamWaitEvent(side0->stream3, side0->fork, 0) != hipSuccess ||
            (mix > 0 && hipStreamWaitEvent(side0->stream4, side0->fork, 0) != hipSuccess))
            rc = fail(SLAM_EHIP, "icp scheduler: fork");
        else
            ms = side0->stream3;
        IcpArgs w = args;
        w.order = order0;
        w.take_lt = ap_k;
        w.gang_abort = abortw + 0;
        if (rc == 0 && mix > 0) {   // the largest turns on wide workgroups (slots below ap_k[1]), on
            IcpArgs wm = w;         // stream4 beside the gangs (joined back before the repair launches)
            wm.take_lt = ap_k + 1;
            wm.gang_abort = abortw + 1;
            rc = launch_wide(wm, mix, max_n1, max_n2, side0->stream4, ap_slots, ap_cand, cfg_mix_share, cfg_groups);
            if (rc == 0 && hipEventRecord(side0->join4, side0->stream4) != hipSuccess) rc = fail(SLAM_EHIP, "icp scheduler: join");
            w.skip_lt = ap_k + 1;   // the gangs take the slots from there to ap_k[0]
        }
        if (rc == 0)
            rc = apg ? launch_bulk_gangs(w, ap, apg, max_n2, s, ap_slots + ap_mix_words)
                     : launch_wide(w, ap, max_n1, max_n2, s, ap_slots, ap_cand, cfg_share, cfg_groups);
        a.order = order0;
        a.skip_lt = ap_k;
    }
    if (rc != 0) {
    } else if (bg) {
        // a phase-1 gang that timed out writes nothing: its pair must then read
        // as "not started" (out_iters 0) in phase 2, never as a stale result
        (void)hipMemsetAsync(args.out_iters, 0, nb * sizeof(int32_t), s);
        (void)hipMemsetAsync(bulk_slots, 0, bulk_slot_bytes, s);
        IcpArgs a1 = a;
        a1.gang_abort = abortw + 2;
        rc = launch_bulk_gangs(a1, B, bg, max_n2, s, bulk_slots);
    } else {
        rc = launch(false, a, B, max_n1, max_n2, ms);
    }
    if (rc == 0) {
        const float thr = args.stopping_thresh > 0.0 ? static_cast<float>(args.stopping_thresh) : 1e-4f;
        // phase 2 gives pairs new slots: clear phase 1's granules (a pair restarted
        // from iteration 0 would otherwise meet another pair's old tags)
        if (bg) (void)hipMemsetAsync(bulk_slots, 0, bulk_slot_bytes, s);
        if (drain_w) (void)hipMemsetAsync(drain_w, 0, sizeof(uint32_t), ms);
        if (B <= kSortOneMax && g_sched_sort_one) {
            // one launch on the phase boundary: the sort, and the exchange slots zeroed beside it
            hipLaunchKernelGGL(sched_sort_one_kernel<0>, dim3(1), dim3(kSortBlock), 0, ms, args.out_iters, key, B, thr,
                               order, gang_slots, static_cast<int64_t>(G + Wd > 0 ? gang_slot_bytes / sizeof(uint64_t) : 0),
                               order0, ap_k, static_cast<const double*>(nullptr), 0, static_cast<int32_t*>(nullptr), -1,
                               drain_n);
        } else {
            if (G + Wd > 0) (void)hipMemsetAsync(gang_slots, 0, gang_slot_bytes, ms);
            hipLaunchKernelGGL(sched_count_kernel, dim3(nblk), dim3(kSortBlock), 0, ms, args.out_iters, key, B, thr,
                               hist, bucket);
            hipLaunchKernelGGL(sched_scan_kernel, dim3(1), dim3(512), 0, ms, hist, nblk, drain_n);
            hipLaunchKernelGGL(sched_scatter_kernel, dim3(nblk), dim3(kSortBlock), 0, ms, bucket, B, hist, order);
        }
        rc = check_launch("icp scheduler kernels");
    }
    // drain tier, queued right behind phase 2's bulk launch on its stream: the
    // bulk's pairs (order[skip..B), entries past the unfinished ones finished
    // or padding) sorted again, the ones it paused (at most drain_x) first,
    // then on wide workgroups from their paused state; a wide pair whose parts
    // were not all resident is re-run on one workgroup (repair)
    auto drain_tier = [&](hipStream_t st, int skip) -> int {
        const float thr = args.stopping_thresh > 0.0 ? static_cast<float>(args.stopping_thresh) : 1e-4f;
        if (one_sort) {
            hipLaunchKernelGGL(sched_sort_one_kernel<0>, dim3(1), dim3(kSortBlock), 0, st, args.out_iters, key, B, thr,
                               drain_order, drain_slots, static_cast<int64_t>(drain_slot_words),
                               static_cast<const int32_t*>(order), static_cast<int32_t*>(nullptr),
                               static_cast<const double*>(nullptr), 0, static_cast<int32_t*>(nullptr), -1,
                               static_cast<int32_t*>(nullptr), skip);
        } else {   // (no other tier: every pair is the bulk's)
            (void)hipMemsetAsync(drain_slots, 0, drain_slot_words * sizeof(uint64_t), st);
            hipLaunchKernelGGL(sched_count_kernel, dim3(nblk), dim3(kSortBlock), 0, st, args.out_iters, key, B, thr,
                               hist, bucket);
            hipLaunchKernelGGL(sched_scan_kernel, dim3(1), dim3(512), 0, st, hist, nblk, static_cast<int32_t*>(nullptr));
            hipLaunchKernelGGL(sched_scatter_kernel, dim3(nblk), dim3(kSortBlock), 0, st, bucket, B, hist, drain_order);
        }
        int r = check_launch("icp drain sort");
        IcpArgs d = a;
        d.order = drain_order;
        d.skip_lt = nullptr;
        d.take_lt = nullptr;
        d.phase_cap = 0;
        d.resume = 1;
        d.gang_abort = abortw + 6;
        if (r == 0) r = launch_wide(d, drain_x, max_n1, max_n2, st, drain_slots, drain_cand, 1, 2);
        d.gang_abort = nullptr;
        if (r == 0) r = launch(false, d, min(B, 2 * drain_x), max_n1, max_n2, st);
        return r;
    };
    if (rc == 0) {   // phase 2: the unfinished pairs, slowest-converging first
        a.phase_cap = 0;
        a.resume = 1;
        a.order = order;
        a.skip_lt = nullptr;
        const int GW = Wd + G;   // pairs on the exchange tiers (wide, then gangs)
        const Instance* hinst = heads > GW && g_forced_instance < 0 ? pick_head_instance(max_n1) : nullptr;
        int dev = 0;
        SideStream* side = nullptr;
        if ((hinst || GW > 0 || bg || ap) && max_n2 <= kCandCap && hipGetDevice(&dev) == hipSuccess) side = side_stream(dev);
        if (side) {
            // fork: the gangs and the head pairs on CU-exclusive workgroups first
            // (the GPU is empty after the scheduler kernels: they take the first
            // CUs), gangs on the caller's stream, heads on the second side stream,
            // the rest on the side stream behind the fork event, which resolves
            // after the first launches are queued; join before the workspace is freed
            const int H = hinst ? heads : GW;
            if (hipEventRecord(side->fork, ms) != hipSuccess || hipStreamWaitEvent(side->stream, side->fork, 0) != hipSuccess ||
                hipStreamWaitEvent(side->stream2, side->fork, 0) != hipSuccess ||
                hipStreamWaitEvent(side->stream3, side->fork, 0) != hipSuccess)
                rc = fail(SLAM_EHIP, "icp scheduler: fork");
            // the wide tier on its own stream (the gangs must not queue behind it)
            if (rc == 0 && Wd > 0) {
                IcpArgs aw = a;
                aw.gang_abort = abortw + 3;
                rc = launch_wide(aw, Wd, max_n1, max_n2, side->stream3, gang_slots, wide_cand, cfg_share, cfg_groups);
            }
            if (rc == 0 && G > 0) {
                IcpArgs g = a;
                g.order = order + Wd;
                g.gang_abort = abortw + 4;
                rc = launch_gangs(g, G, parts, team, max_n1, max_n2, ms, gang_slots + wide_slot_words);
            }
            if (rc == 0 && H > GW) {
                IcpArgs h = a;
                h.order = order + GW;
                rc = launch(false, h, H - GW, max_n1, max_n2, side->stream2, hinst, kMaxLds);
            }
            IcpArgs t = a;
            t.order = order + H;
            if (drain_x && !bg) {
                t.drain = drain_w;
                t.drain_n = drain_n;
                t.drain_skip = H;
                t.drain_x = drain_x;
            }
            if (bg) t.gang_abort = abortw + 5;
            if (rc == 0)
                rc = bg ? launch_bulk_gangs(t, B - H, bg, max_n2, side->stream, bulk_slots + static_cast<size_t>(H) * 2 * bg->parts * 32)
                        : launch(false, t, B - H, max_n1, max_n2, side->stream);
            if (rc == 0 && t.drain) rc = drain_tier(side->stream, H);
            if (rc == 0 && (hipEventRecord(side->join, side->stream) != hipSuccess ||
                            hipEventRecord(side->join2, side->stream2) != hipSuccess ||
                            hipEventRecord(side->join3, side->stream3) != hipSuccess))
                rc = fail(SLAM_EHIP, "icp scheduler: join");
            if (rc == 0 && (hipStreamWaitEvent(s, side->join, 0) != hipSuccess ||
                            hipStreamWaitEvent(s, side->join2, 0) != hipSuccess ||
                            hipStreamWaitEvent(s, side->join3, 0) != hipSuccess ||
                            (mix > 0 && hipStreamWaitEvent(s, side->join4, 0) != hipSuccess)))
                rc = fail(SLAM_EHIP, "icp scheduler: wait");
            // (with the pre-tier, stream3 = ms: join3 also joins the phases and the gangs)
            if (rc == 0 && (GW > 0 || bg)) {
                // repair: a wide / gang pair whose partners did not all arrive
                // stopped without writing, leaving it paused at the phase-1 state;
                // re-run such pairs on one workgroup each (finished pairs'
                // workgroups exit at once, so this costs one near-empty launch)
                IcpArgs r = a;
                r.order = order;
                rc = launch(false, r, bg ? B : GW, max_n1, max_n2, stream);
            }
            if (rc == 0 && ap) {   // the same for the angle pre-tier (not started: from the initial transform)
                IcpArgs r = a;
                r.order = order0;
                rc = launch(false, r, ap, max_n1, max_n2, stream);
            }
        } else {
            if (ms != s && (hipEventRecord(side0->join3, ms) != hipSuccess || hipStreamWaitEvent(s, side0->join3, 0) != hipSuccess ||
                            (mix > 0 && hipStreamWaitEvent(s, side0->join4, 0) != hipSuccess)))
                rc = fail(SLAM_EHIP, "icp scheduler: wait");
            if (rc == 0) {
                IcpArgs t = a;
                if (drain_x) {
                    t.drain = drain_w;
                    t.drain_n = drain_n;
                    t.drain_skip = 0;
                    t.drain_x = drain_x;
                }
                rc = launch(false, t, B, max_n1, max_n2, stream);
                if (rc == 0 && t.drain) rc = drain_tier(as_stream(stream), 0);
            }
            if (rc == 0 && ap) {   // the pre-tier's repair (its pairs are not in phase 2's order)
                IcpArgs r = a;
                r.order = order0;
                rc = launch(false, r, ap, max_n1, max_n2, stream);
            }
        }
    }
    if (ms != s && rc != 0) {   // an error after the pre-tier's fork: still join the side streams before the free
        (void)hipEventRecord(side0->join3, ms);
        (void)hipStreamWaitEvent(s, side0->join3, 0);
        if (mix > 0) {
            (void)hipEventRecord(side0->join4, side0->stream4);
            (void)hipStreamWaitEvent(s, side0->join4, 0);
        }
    }
    (void)hipFreeAsync(ws, s);
    return rc;
}

}  // namespace slamhip

using namespace slamhip;

extern "C" {

int slam_abi_version(void) { return 100; }

const char* slam_last_error(void) { return last_error_buf(); }

int slam_icp_max_query_points(void) { return kMaxQuery; }

// Diagnostics: number of compiled (BLOCK, QPT) instances, their shapes, and a
// way to force one (bench/profile sweeps).  Not part of the stable ABI.
int slam_icp_num_instances(void) { return kNumInstances; }
int slam_icp_instance_shape(int i, int* block, int* qpt) {
    if (i < 0 || i >= kNumInstances) return fail(SLAM_EINVAL, "instance %d out of range", i);
    *block = kInstances[i].block;
    *qpt = kInstances[i].qpt;
    return ok();
}
int slam_icp_force_instance(int i) {
    g_forced_instance = (i >= 0 && i < kNumInstances) ? i : -1;
    return ok();
}
int slam_icp_set_stamps(void* dev_buf) {
    g_icp_stamps = reinterpret_cast<unsigned long long*>(dev_buf);
    return ok();
}
// Diagnostics: per-pair phase timeline of slam_icp_batch_f64 (IcpArgs::trace):
// a device buffer of B x 2 x 4 uint64; NULL turns it off.
int slam_icp_set_trace(void* dev_buf) {
    g_icp_trace = reinterpret_cast<unsigned long long*>(dev_buf);
    return ok();
}
int slam_icp_set_eval_counter(void* dev_u64) {
    g_icp_evals = reinterpret_cast<unsigned long long*>(dev_u64);
    return ok();
}
// Phased scheduling of large batches (see launch_batch): phase-1 iterations
// (0 = one launch) and the smallest batch it applies to.  Results do not
// depend on it (tests/test_icp_gpu.py::test_schedule_is_invisible).
int slam_icp_set_schedule_heads(int heads) {
    if (heads < 0) return fail(SLAM_EINVAL, "schedule: negative head count");
    g_sched_heads = heads;
    g_sched_auto = 0;
    return ok();
}
int slam_icp_set_schedule_gangs(int gangs, int parts) {
    if (gangs < 0 || parts == 1 || parts < 0 || parts > kGangMax)
        return fail(SLAM_EINVAL, "schedule: gangs %d parts %d", gangs, parts);
    g_sched_gangs = gangs;
    g_sched_gang_parts = parts;
    g_sched_auto = 0;
    return ok();
}
// Gang parts that timed out waiting for a partner since the last call (their
// pairs were re-run on single workgroups: results stay valid); read-and-clear.
// Synchronises the device.
// Wide tier: the `pairs` slowest-keyed pairs of a batch below 8,192 pairs on
// icp_wide_kernel (before the gangs), workgroups requesting 1/share of a CU's
// LDS (1: CU-exclusive).  Results are bit-identical.  0 = off.
int slam_icp_set_schedule_wide(int pairs, int share) {
    if (pairs < 0 || share < 1 || share > 8) return fail(SLAM_EINVAL, "schedule: wide %d share %d", pairs, share);
    g_sched_wide = pairs;
    g_wide_share = share;
    g_sched_auto = 0;
    return ok();
}
// Bulk gangs: batches of fewer than `below_pairs` pairs (>= the scheduler's
// minimum) run every phase's bulk as gangs of `parts` (2 or 3) workgroups
// with the ordinary LDS footprint: half the iteration latency per pair when
// whole pairs cannot fill the GPU.  Bit-identical results.  0 = off.
int slam_icp_set_bulk_gangs(int below_pairs, int parts) {
    if (below_pairs < 0 || (below_pairs > 0 && (parts < 2 || parts > 3)))
        return fail(SLAM_EINVAL, "bulk gangs: below %d parts %d", below_pairs, parts);
    g_bulk_gang_below = below_pairs;
    g_bulk_gang_parts = parts;
    return ok();
}
// Diagnostics: carry the paused pairs' search state across the scheduler's
// phase boundary (1, default) or resume them cold (0).  Results identical.
int slam_icp_set_schedule_warm(int on) {
    g_sched_warm = on ? 1 : 0;
    return ok();
}
// Diagnostics: the phase boundary's sort of batches <= 4,096 pairs on one
// workgroup (1, default) or as the three-kernel sort (0).  Same order.
int slam_icp_set_sched_sort_one(int on) {
    g_sched_sort_one = on ? 1 : 0;
    return ok();
}
// Diagnostics: batches of fewer than `pairs` pairs get the tail tiers (heads,
// gangs, wide); 0 restores the default (4,096).
// Diagnostics: the XCD-aware pair map of launches in stream order: runs of
// `run` consecutive pairs per XCD (default 16; 0 = identity; -1 restores the
// default).  Results do not depend on it.
int slam_icp_set_xcd_map(int run) {
    if (run < -1 || run > 4096) return fail(SLAM_EINVAL, "xcd map run %d", run);
    g_xcd_map = run < 0 ? 16 : run;
    return ok();
}
// Angle pre-tier (see launch_batch): batches of up to 8,192 pairs run up to
// `max_pairs` pairs whose initial transform turns by more than `thresh_rad`
// on a tier of their own from the start (kind: slam_icp_set_angle_tier_kind;
// 0: off).  Results are bit-identical.
int slam_icp_set_angle_tier(int max_pairs, float thresh_rad) {
    if (max_pairs < 0 || max_pairs > 1024 || !(thresh_rad >= 0.0f))
        return fail(SLAM_EINVAL, "angle tier: %d pairs, threshold %g", max_pairs, static_cast<double>(thresh_rad));
    g_angle_max = max_pairs;
    g_angle_thresh = thresh_rad;
    g_sched_auto = 0;
    return ok();
}
// The angle pre-tier's kind: 0 the wide tier, 2 / 3 bulk gangs of that many
// ordinary workgroups per pair.
int slam_icp_set_angle_tier_kind(int kind) {
    if (kind != 0 && kind != 2 && kind != 3 && kind != 4 && kind != 6)
        return fail(SLAM_EINVAL, "angle tier kind %d not in {0, 2, 3, 4, 6}", kind);
    g_angle_kind = kind;
    g_sched_auto = 0;
    return ok();
}
int slam_icp_set_wide_groups(int groups) {
    if (groups != 1 && groups != 2) return fail(SLAM_EINVAL, "wide groups %d not in {1, 2}", groups);
    g_wide_groups = groups;
    return ok();
}
int slam_icp_set_angle_tier_mix(int wide_pairs, int share) {
    if (wide_pairs < 0 || share < 1 || share > 8) return fail(SLAM_EINVAL, "angle tier mix %d, share %d", wide_pairs, share);
    g_angle_mix = wide_pairs;
    g_angle_mix_share = share;
    g_sched_auto = 0;
    return ok();
}
// The automatic tier profile by batch size (1, default) or the explicit
// settings (0; any tier setter selects them).  1 also restores the explicit
// settings' defaults (64 heads, 24 gangs of 4, no wide tier, no angle tier).
int slam_icp_set_schedule_auto(int on) {
    g_sched_auto = on ? 1 : 0;
    if (on) {
        g_sched_heads = 64;
        g_sched_gangs = 24;
        g_sched_gang_parts = 4;
        g_sched_wide = 0;
        g_wide_share = 1;
        g_angle_max = 0;
        g_angle_thresh = 0.3f;
        g_angle_kind = 0;
        g_angle_mix = 0;
        g_angle_mix_share = 2;
    }
    return ok();
}
int slam_icp_set_tier_limit(int pairs) {
    if (pairs < 0) return fail(SLAM_EINVAL, "tier limit %d < 0", pairs);
    g_tiers_below = pairs ? pairs : kHeadsMaxPairs;
    return ok();
}
int slam_icp_gang_timeouts(void) {
    int v = 0;
    const int zero = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_gang_timeout), sizeof(int)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_gang_timeout), &zero, sizeof(int)) != hipSuccess)
        return fail(SLAM_EHIP, "gang timeouts: read");
    return v;
}
// Diagnostics: the longest wait of a gang exchange for its partners, in
// s_memrealtime ticks (100 MHz); 0 restores the default (0.2 s).  Tiny values
// force timeouts (the repair path).
int slam_icp_set_gang_first_wait(uint32_t ticks) {
    g_gang_wait_first = ticks ? ticks : kGangWaitFirstTicks;
    return ok();
}
// Diagnostics: `workgroups` workgroups that each hold a whole CU's LDS and spin
// for `ticks` of s_memrealtime (bounded), on `stream`: a stand-in for another
// process occupying CUs (tests/test_icp_gpu.py::test_occupied_cus_cost_milliseconds)
__global__ __launch_bounds__(64) void occupy_kernel(uint32_t ticks, unsigned long long* sink) {
    extern __shared__ double lds_occ[];
    if (threadIdx.x == 0) {
        lds_occ[0] = 1.0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned long long n = 0;
        while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
            __builtin_amdgcn_s_sleep(8);
            ++n;
        }
        if (n == 0 && sink) sink[blockIdx.x] = static_cast<unsigned long long>(lds_occ[0]);
    }
}
int slam_icp_diag_occupy(int workgroups, uint32_t ticks, void* stream) {
    if (workgroups < 1 || workgroups > 4096 || ticks > 100000000u)
        return fail(SLAM_EINVAL, "occupy: %d workgroups, %u ticks (at most 1 s)", workgroups, ticks);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(occupy_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(kMaxLds));
    hipLaunchKernelGGL(occupy_kernel, dim3(workgroups), dim3(64), kMaxLds, as_stream(stream), ticks,
                       static_cast<unsigned long long*>(nullptr));
    return check_launch("occupy kernel");
}
int slam_icp_set_gang_wait(uint32_t ticks) {
    g_gang_wait = ticks ? ticks : kGangWaitTicks;
    return ok();
}
// Diagnostics: the scheduler's stable bucket sort on its own: order[] of B
// pairs from their phase-1 out_iters and keys (device arrays), as phase 2
// would visit them.
int slam_icp_sched_sort(const int32_t* iters, const float* key, int32_t B, float thresh, int32_t* order,
                        void* stream) {
    if (B <= 0) return ok();
    if (!iters || !key || !order) return fail(SLAM_EINVAL, "null array argument");
    hipStream_t s = as_stream(stream);
    if (B <= kSortOneMax) {   // the one-workgroup sort launch_batch uses at this size
        hipLaunchKernelGGL(sched_sort_one_kernel<0>, dim3(1), dim3(kSortBlock), 0, s, iters, key, B, thresh, order,
                           static_cast<uint64_t*>(nullptr), static_cast<int64_t>(0), static_cast<const int32_t*>(nullptr),
                           static_cast<int32_t*>(nullptr), static_cast<const double*>(nullptr), 0,
                           static_cast<int32_t*>(nullptr));
        return check_launch("sched sort kernel");
    }
    const int nblk = (B + kSortBlock - 1) / kSortBlock;
    void* ws = nullptr;
    const size_t bytes = (static_cast<size_t>(nblk) * kNB + static_cast<size_t>(B)) * sizeof(int32_t);
    if (hipMallocAsync(&ws, bytes, s) != hipSuccess) return fail(SLAM_EHIP, "sched sort: no workspace");
    int32_t* hist = static_cast<int32_t*>(ws);
    int32_t* bucket = hist + static_cast<size_t>(nblk) * kNB;
    hipLaunchKernelGGL(sched_count_kernel, dim3(nblk), dim3(kSortBlock), 0, s, iters, key, B, thresh, hist, bucket);
    hipLaunchKernelGGL(sched_scan_kernel, dim3(1), dim3(512), 0, s, hist, nblk, static_cast<int32_t*>(nullptr));
    hipLaunchKernelGGL(sched_scatter_kernel, dim3(nblk), dim3(kSortBlock), 0, s, bucket, B, hist, order);
    const int rc = check_launch("sched sort kernels");
    (void)hipFreeAsync(ws, s);
    return rc;
}
int slam_icp_set_drain(int pairs) {
    if (pairs < -1 || pairs > 64) return fail(SLAM_EINVAL, "drain: pairs outside [-1, 64]");
    g_drain = pairs;
    return ok();
}

int slam_icp_set_schedule(int probe_iters, int min_pairs) {
    if (probe_iters < -1 || min_pairs < 0) return fail(SLAM_EINVAL, "schedule: probe_iters < -1 or min_pairs < 0");
    g_sched_probe = probe_iters;
    g_sched_min_pairs = min_pairs;
    return ok();
}
// Bounds check of every ICP launch since the last call: synchronises `stream`
// and returns SLAM_EINVAL if a pair's scans were empty or outside the
// max_n1 / max_n2 the caller passed (that pair's out_iters = INT32_MIN, its
// out_err NaN), then clears the flag.
int slam_icp_status(void* stream) {
    if (hipStreamSynchronize(as_stream(stream)) != hipSuccess) return fail(SLAM_EHIP, "icp status: stream sync");
    int st = 0;
    if (hipMemcpyFromSymbol(&st, HIP_SYMBOL(g_icp_status), sizeof(int)) != hipSuccess)
        return fail(SLAM_EHIP, "icp status: read");
    if (st == 0) return ok();
    const int zero = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_icp_status), &zero, sizeof(int));
    return fail(SLAM_EINVAL, "icp: a pair's scan sizes exceed the max_n1 / max_n2 bounds of its launch "
                             "(or a scan is empty); its out_iters is INT32_MIN");
}

int slam_icp_set_screen(int mode) {
    if (mode < 0 || mode > 2) return fail(SLAM_EINVAL, "nn mode %d not in {0, 1, 2}", mode);
    g_screen = mode;
    return ok();
}
int slam_icp_selected_instance(int max_n1) {
    const Instance* p = pick_instance(max_n1, g_forced_instance);
    return p ? static_cast<int>(p - kInstances) : -1;
}

int slam_icp_batch_f64(const double* pts, const int64_t* scan_off, const int32_t* src_scan,
                       const int32_t* dst_scan, const double* init, int32_t B, double epsilon,
                       int32_t max_iters, double stopping_thresh, int32_t rotation_only,
                       int32_t max_n1, int32_t max_n2, int32_t hist_stride, double* out_hist,
                       double* out_tf, double* out_err, int32_t* out_iters, void* stream) {
    if (B < 0) return fail(SLAM_EINVAL, "B = %d < 0", B);
    if (B == 0) return ok();
    if (!pts || !scan_off || !src_scan || !dst_scan || !init || !out_tf || !out_err || !out_iters)
        return fail(SLAM_EINVAL, "null array argument");
    if (max_n1 < 1 || max_n2 < 1) return fail(SLAM_EINVAL, "empty scan (max_n1=%d, max_n2=%d)", max_n1, max_n2);
    if (max_iters > 1000000) return fail(SLAM_EINVAL, "max_iters %d > 1e6", max_iters);
    if (hist_stride < 0 || (hist_stride > 0 && (hist_stride < max_iters + 3 || !out_hist)))
        return fail(SLAM_EINVAL, "hist_stride %d must be 0 or >= max_iters + 3 (%d)", hist_stride, max_iters + 3);
    IcpArgs a{};
    a.pts = reinterpret_cast<const double2*>(pts);
    a.scan_off = scan_off;
    a.src_scan = src_scan;
    a.dst_scan = dst_scan;
    a.init = init;
    a.epsilon = epsilon;
    a.stopping_thresh = stopping_thresh;
    a.max_iters = max_iters < -1 ? -1 : max_iters;
    a.rotation_only = rotation_only;
    a.hist_stride = hist_stride;
    a.out_hist = out_hist;
    a.out_tf = out_tf;
    a.out_err = out_err;
    a.out_iters = out_iters;
    a.trace = g_icp_trace;
    return launch_batch(a, B, max_n1, max_n2, stream);
}

int slam_icp_step_f64(const double* pts, const int64_t* scan_off, const int32_t* src_scan,
                      const int32_t* dst_scan, const double* T_in, int32_t B, int32_t rotation_only,
                      int32_t max_n1, int32_t max_n2, double* T_out, int64_t* out_corr,
                      const int64_t* corr_off, double* out_err, void* stream) {
    if (B < 0) return fail(SLAM_EINVAL, "B = %d < 0", B);
    if (B == 0) return ok();
    if (!pts || !scan_off || !src_scan || !dst_scan || !T_in || !T_out || !out_corr || !corr_off || !out_err)
        return fail(SLAM_EINVAL, "null array argument");
    if (max_n1 < 1 || max_n2 < 1) return fail(SLAM_EINVAL, "empty scan (max_n1=%d, max_n2=%d)", max_n1, max_n2);
    IcpArgs a{};
    a.pts = reinterpret_cast<const double2*>(pts);
    a.scan_off = scan_off;
    a.src_scan = src_scan;
    a.dst_scan = dst_scan;
    a.init = T_in;
    a.rotation_only = rotation_only;
    a.out_tf = T_out;
    a.out_err = out_err;
    a.out_corr = out_corr;
    a.corr_off = corr_off;
    return launch(true, a, B, max_n1, max_n2, stream);
}

int slam_kabsch2d_f64(const double* a, const double* b, int64_t n, double* out_T, double* out_err,
                      void* stream) {
    if (n < 1) return fail(SLAM_EINVAL, "kabsch2d: n = %lld < 1", static_cast<long long>(n));
    if (!a || !b || !out_T || !out_err) return fail(SLAM_EINVAL, "null array argument");
    hipLaunchKernelGGL(kabsch_kernel, dim3(1), dim3(kKabschBlock), 0, as_stream(stream),
                       reinterpret_cast<const double2*>(a), reinterpret_cast<const double2*>(b), n,
                       out_T, out_err);
    return check_launch("kabsch2d kernel");
}

}  // extern "C"
