/*
 * slamhip.h — C-ABI of the MI355X-native ICP + SE(2) pose-graph hot path.
 *
 * Drop-in boundary for cohnt/ICP-SLAM-with-Loop-Closure (reference at
 * /root/reference).  The reference is pure Python/NumPy, so its "FFI" for this
 * path is the Python call surface of src/icp.py and
 * src/pose_graph_optimization.py; the build's drop-in modules
 * (the .py modules in icp-slam-with-loop-closure_amd/src) bind these entry points with
 * ctypes.  Each entry point names the reference
 * function(s) it replaces.
 *
 * Conventions (all entry points):
 *   - every array argument is a DEVICE pointer (hipMalloc / torch-ROCm
 *     storage) owned by the caller; scalars are host values;
 *   - points are packed (x, y) float64 pairs ("double2"); the homogeneous
 *     coordinate of the reference's (n, 3) arrays is implicit and must be 1
 *     (np.c_[points, ones] as scripts/main.py:242-243 builds them);
 *   - 3x3 SE(2) matrices are 9 float64, row-major, last row [0, 0, 1];
 *   - launches are asynchronous and ordered on `stream` (a hipStream_t; NULL
 *     = the legacy default stream) and copy nothing to the host; nothing is
 *     allocated persistently.  One exception to "allocates nothing": a
 *     slam_icp_batch_f64 call of >= 1024 pairs takes a transient
 *     stream-ordered workspace (hipMallocAsync / hipFreeAsync, 12 B per pair),
 *     which stream capture records as graph memory nodes;
 *   - return 0 on success, a negative SLAM_E* code on failure; the message is
 *     available from slam_last_error() (thread-local);
 *   - the tuning and diagnostics switches (slam_icp_set_*, slam_gn_set_*)
 *     are per host thread (thread-local, like slam_last_error): a thread's
 *     settings never change another thread's launches;
 *   - one host thread per device at a time: the batch scheduler's side
 *     streams and fork / join events are one set per device.
 */
#ifndef SLAMHIP_H
#define SLAMHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLAM_OK 0
#define SLAM_EINVAL (-1)   /* bad shape / argument */
#define SLAM_EHIP (-2)     /* HIP runtime error (launch, device) */
#define SLAM_ETOOBIG (-3)  /* a scan larger than the compiled query capacity */

/* Library identity: ABI version (major*100 + minor). */
int slam_abi_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* slam_last_error(void);
/* Largest query scan (pc1) one workgroup can hold (points). */
int slam_icp_max_query_points(void);

/*
 * Batched ICP, one scan pair per workgroup, all iterations on chip.
 * Replaces src/icp.py:72-97 `icp(pc1, pc2, init_transform, epsilon,
 * max_iters, stopping_thresh, rotation_only)` for B independent pairs, i.e.
 * the joblib fan-out of scripts/main.py:240-247,
 * src/pose_graph_optimization.py:59-68 and src/loop_closure_detection.py:134-142.
 *
 *   pts       all scans, packed double2, scan s = pts[scan_off[s] .. scan_off[s+1])
 *   scan_off  int64[n_scans + 1]
 *   src_scan  int32[B]  pc1 (moving/query cloud) of pair b
 *   dst_scan  int32[B]  pc2 (reference cloud) of pair b
 *   init      float64[B][9] initial transforms
 *   max_n1/max_n2  host upper bounds of the pc1 / pc2 sizes in this batch
 *                  (select the kernel instance and LDS size).  The kernel
 *                  checks every pair against them: a pair with an empty scan
 *                  or n1 > max_n1's instance capacity or n2 > max_n2's LDS
 *                  capacity is not computed (out_iters = INT32_MIN, out_err =
 *                  NaN) and raises the flag slam_icp_status() reports
 *   hist_stride    0, or >= max_iters + 3: out_hist[b] holds the full
 *                  transform list [init, T1, ..., T_k] the reference returns
 *   out_hist  float64[B][hist_stride][9] (NULL if hist_stride == 0)
 *   out_tf    float64[B][9]  final transform (transforms[-1])
 *   out_err   float64[B]     returned error (of the penultimate transform)
 *   out_iters int32[B]       number of ICP iterations k (len(transforms) - 1)
 * Stopping rules are the reference's: err < epsilon; iteration > max_iters;
 * |last_err - err| < stopping_thresh from the second iteration on.
 * Batches of >= 1024 pairs run in two phases (slam_icp_set_schedule) with a
 * transient stream-ordered workspace of 12 B/pair (hipMallocAsync/FreeAsync).
 */
int slam_icp_batch_f64(const double* pts, const int64_t* scan_off,
                       const int32_t* src_scan, const int32_t* dst_scan,
                       const double* init, int32_t B,
                       double epsilon, int32_t max_iters, double stopping_thresh,
                       int32_t rotation_only, int32_t max_n1, int32_t max_n2,
                       int32_t hist_stride, double* out_hist, double* out_tf,
                       double* out_err, int32_t* out_iters, void* stream);

/*
 * Synchronises `stream` and reports the device-side bounds check of every
 * slam_icp_batch_f64 / slam_icp_step_f64 launch since the previous call:
 * SLAM_OK, or SLAM_EINVAL when some pair was outside its launch's max_n1 /
 * max_n2 (see above); the flag is then cleared.
 */
int slam_icp_status(void* stream);

/*
 * One ICP iteration per pair.  Replaces src/icp.py:55-69 `icp_iteration(pc1,
 * pc2, previous_transform, rotation_only)`; with T_in = identity it is
 * src/icp.py:10-19 `get_correspondences(pc1, pc2)` (an identity transform
 * reproduces the query coordinates exactly).
 *   T_in      float64[B][9]
 *   T_out     float64[B][9]   transform @ previous_transform
 *   out_corr  int64[...]      correspondences of pair b written at
 *                             out_corr[corr_off[b] + i], i < n1(b)
 *   corr_off  int64[B]
 *   out_err   float64[B]      get_error of the pre-update cloud
 */
int slam_icp_step_f64(const double* pts, const int64_t* scan_off,
                      const int32_t* src_scan, const int32_t* dst_scan,
                      const double* T_in, int32_t B, int32_t rotation_only,
                      int32_t max_n1, int32_t max_n2, double* T_out,
                      int64_t* out_corr, const int64_t* corr_off,
                      double* out_err, void* stream);

/*
 * Rigid 2-D fit of matched rows a[i] -> b[i] (n rows each, double2).
 * Replaces src/icp.py:22-46 `get_transform(pc1, pc2)` (out_T) and
 * src/icp.py:49-52 `get_error(pc1, pc2)` (out_err, the SUM of squares).
 */
int slam_kabsch2d_f64(const double* a, const double* b, int64_t n,
                      double* out_T, double* out_err, void* stream);

/*
 * One stochastic-gradient relaxation step, in place on poses (N x 3).
 * Replaces src/pose_graph_optimization.py:7-49
 * `pose_graph_optimization_step_sgd(pose_graph, learning_rate,
 * loop_closure_uncertainty)`.  Edges (ea[e] -> eb[e], tf[e] 3x3) must be in
 * the pose graph's networkx iteration order; |a-b| == 1 edges are skipped as
 * in the reference.  `work`: float64[slam_pgo_sgd_work_size(N, E)] scratch.
 */
int slam_pgo_sgd_step_f64(double* poses, int32_t N, const int32_t* ea,
                          const int32_t* eb, const double* tf, int32_t E,
                          double learning_rate, double loop_closure_uncertainty,
                          double* work, void* stream);

/* float64 elements of the `work` scratch slam_pgo_sgd_step_f64 needs. */
int64_t slam_pgo_sgd_work_size(int32_t N, int32_t E);

/*
 * Heading recompute from positions, in place.  Replaces the first loop of
 * src/pose_graph_optimization.py:51-57 `recompute_pose_graph_orientation`.
 */
int slam_pgo_orient_f64(double* poses, int32_t N, void* stream);

/*
 * Second half of recompute_pose_graph_orientation with icp_recompute
 * (src/pose_graph_optimization.py:68-74): theta_i = theta_{i-1} +
 * atan2(tf_i[1,0], tf_i[0,0]) for i = 1..N-1, theta_{i-1} taken BEFORE its
 * own update (the reference's reverse-order loop).  tf: float64[N-1][9]
 * rotation-only ICP results of pairs (i, i-1); work: float64[N].
 */
int slam_pgo_orient_from_tf_f64(double* poses, int32_t N, const double* tf,
                                double* work, void* stream);

/*
 * One Gauss-Newton iteration of the SE(2) pose graph (north-star solve; the
 * reference has only the SGD relaxation).  Problem: the graph as
 * src/pose_graph.py:61-73 exports it to g2o — edge e: ea[e] -> eb[e] with
 * relative measurement tf[e] and isotropic information w[e]; node columns
 * node_col[n] (-1 = fixed) in a bandwidth-reducing order; H lower band of
 * half-width W scalars; slot_* list the edge contributions of every H block
 * (see slamhip/gn.py GnPlan).  Poses are updated in place; chi2 before the
 * step -> *out_chi2 (device); *status != 0 if H was not positive definite.
 */
int64_t slam_gn_work_size(int32_t N, int32_t E, int32_t W);
int slam_gn_max_lds_band(void);
int slam_gn_iteration_f64(double* poses, int32_t N, const int32_t* ea,
                          const int32_t* eb, const double* tf, const double* w,
                          int32_t E, const int32_t* node_col,
                          const int32_t* slot_rc, const int32_t* slot_ptr,
                          const int32_t* slot_items, int32_t n_slots,
                          int32_t nv, int32_t W, double* work,
                          double* out_chi2, int32_t* status, void* stream);

/*
 * The same iteration for a band + border plan (slamhip/gn.py GnPlan with a
 * border, e.g. C4's lap graph cut at one place): scalars [0, nv_band) form
 * the band of half-width W, the last nv - nv_band <= 31 scalars a border
 * coupled to band rows nbr_rows[0..n_nbr) only.  Solved as H = [A B; B^T C]:
 * Z = A^-1 [r_a | B] by block cyclic reduction with several right-hand
 * sides, S = C - B^T Z_B, x_b = S^-1 (r_b - B^T Z_r), x_a = Z_r - Z_B x_b.
 * work: slam_gn_work_size_bordered(N, E, W, nv - nv_band) doubles.
 */
int64_t slam_gn_work_size_bordered(int32_t N, int32_t E, int32_t W,
                                   int32_t n_border);
int slam_gn_iteration_bordered_f64(double* poses, int32_t N, const int32_t* ea,
                                   const int32_t* eb, const double* tf,
                                   const double* w, int32_t E,
                                   const int32_t* node_col,
                                   const int32_t* slot_rc,
                                   const int32_t* slot_ptr,
                                   const int32_t* slot_items, int32_t n_slots,
                                   int32_t nv, int32_t W, int32_t nv_band,
                                   const int32_t* nbr_rows, int32_t n_nbr,
                                   double* work, double* out_chi2,
                                   int32_t* status, void* stream);
/* The same bordered iteration with the border's Schur complement accumulated
 * DURING the band's elimination: every eliminated
 * block i with pslot[i] = k >= 0 (the blocks whose reduced rows couple to the
 * border; slamhip.gn.GnPlan lists them symbolically) adds Y_i^T D_i^-1 Y_i to
 * slot k of pwork (n_pslot x mc x mc doubles, mc = 16 ceil((nbd + 1) / 16)),
 * the top block forms S and x_b = S^-1 s, and the back-substitution runs on
 * one column.  Same result as slam_gn_iteration_bordered_f64 to rounding;
 * needs the explicit-inverse cyclic reduction (SLAM_EINVAL otherwise).
 * The back-substitution runs as ONE XCD-local launch by default
 * (slam_gn_set_fused_back): a fused wait that timed out sets *status |= 2,
 * the step is then invalid and is re-run with slam_gn_set_fused_back(0)
 * (slamhip.gn does this).
 * work: slam_gn_work_size_bordered(N, E, W, nv - nv_band) doubles. */
int slam_gn_iteration_schur_f64(double* poses, int32_t N, const int32_t* ea,
                                const int32_t* eb, const double* tf,
                                const double* w, int32_t E,
                                const int32_t* node_col,
                                const int32_t* slot_rc,
                                const int32_t* slot_ptr,
                                const int32_t* slot_items, int32_t n_slots,
                                int32_t nv, int32_t W, int32_t nv_band,
                                const int32_t* pslot, int32_t n_pslot,
                                double* pwork, double* work,
                                double* out_chi2, int32_t* status,
                                void* stream);
/* The Schur path's back-substitution: one XCD-local launch (1, default) or
 * one launch per level (0). */
int slam_gn_set_fused_back(int on);
int slam_gn_get_fused_back(void);
/* 1 when slam_gn_iteration_schur_f64 can run in this process (the
 * explicit-inverse cyclic reduction is the solver: not with
 * slam_gn_set_solver(1) or the SLAMHIP_BCR_CHOL / SLAMHIP_BCR_LEGACY A/B
 * switches), 0 otherwise: a bordered plan then takes
 * slam_gn_iteration_bordered_f64. */
int slam_gn_schur_supported(void);
/* Diagnostics: the fused back-substitution's longest wait in s_memrealtime
 * ticks (0: the default 0.2 s); a tiny wait forces the timeout path. */
int slam_gn_set_fused_wait(uint32_t ticks);

/* ---- occupancy grid (src/produce_occupancy_grid.py) ------------------------
 * pts: packed (x, y) scan points, scan_off (S+1), pose4 (S x 4: cos theta,
 * sin theta, x, y of each scan's pose; cos/sin as np.cos/np.sin give them).
 * slam_grid_global_points_f64 replaces construct_global_points (:75-87):
 * gpts (P x 2) and bounds = (min x, max x, min y, max y) of all of them.
 * slam_grid_update_i8 replaces update_occupancy_grid / the beam loop of
 * produce_occupancy_grid (:54-73, bresenham_update :89-121): the int8 grid
 * (H x W, row = y) is updated in place with the reference's per-beam rule.
 * work: slam_grid_work_size(S, H, W) BYTES. */
int64_t slam_grid_work_size(int32_t S, int32_t H, int32_t W);
int slam_grid_global_points_f64(const double* pts, const int64_t* scan_off, int32_t S, const double* pose4,
                                double* gpts, double* bounds, void* work, void* stream);
int slam_grid_update_i8(const double* gpts, const int64_t* scan_off, int32_t S, const double* pose4, int64_t P,
                        double min_x, double min_y, double cell_width, int32_t H, int32_t W, int32_t k_hit,
                        int32_t k_miss, int8_t* grid, void* work, void* stream);

/* Diagnostics (kernel-shape sweeps; not needed by callers). */
int slam_icp_num_instances(void);
int slam_icp_instance_shape(int i, int* block, int* qpt);
int slam_icp_force_instance(int i);
int slam_icp_selected_instance(int max_n1);
/* NN search mode: 0 exact fp64 scan, 1 fp32 screen (all chunks), 2 fp32
 * screen with exact pruning (per-lane windows + sub-chunk boxes, default);
 * identical results. */
int slam_icp_set_screen(int mode);
/* Phased scheduling of slam_icp_batch_f64 for batches of >= min_pairs pairs:
 * every pair runs probe_iters iterations, then the unfinished ones resume in
 * order of their last error change (slowest-converging first), so the long
 * tail of iteration counts does not start late.  probe_iters = 0: one launch;
 * -1 (default): automatic — 3, or 4 for batches of 2,048-4,095 pairs and 2
 * for 4,096-8,192.
 * Defaults (-1, 1024).  Results are identical either way. */
int slam_icp_set_schedule(int probe_iters, int min_pairs);
/* Phase 2 of the scheduler starts the (at most) `heads` pairs the probe keyed
 * slowest (one per 16 pairs at most) first, on CU-exclusive 512-thread
 * workgroups; the rest runs beside them on a library-owned second stream,
 * joined back before the call's work ends: the strong-scaling tail.  Batches
 * below 4,096 pairs only (larger shards keep every CU for the bulk).  Sums
 * are order-free (exact on fixed grids), so results are bit-identical to the
 * single launch.  0 = off; default 64. */
int slam_icp_set_schedule_heads(int heads);
/* The first `gangs` of those head pairs run as gangs of `parts` workgroups
 * (2..17) each: a pair's 64-query groups are dealt over the parts, which sit on
 * one XCD, hold one CU each, and exchange their exact partial sums every
 * iteration through a stream-ordered workspace (data-tagged 8-byte granules,
 * agent-scope write-through stores, bounded polling).  parts = 0: teams, one
 * workgroup per 64-query group (pairs up to 2,048 points), the group's search
 * split over the workgroup's four waves (latency mode).  Results are
 * bit-identical to the one-workgroup kernels.  gangs = 0: off; defaults
 * (24, 4).  SLAM_EINVAL for gangs < 0, parts 1, < 0 or > 17. */
int slam_icp_set_schedule_gangs(int gangs, int parts);
/* Wide tier: the `pairs` slowest-keyed pairs (taken before the gangs) run on
 * one workgroup per 64-query group (pairs up to 2,048 points) whose NW waves
 * split a brute-force fp32 screen by candidate slices (no pruning, so no
 * outlier group sets the iteration time); the groups exchange their exact
 * partial sums every iteration like the gangs.  Workgroups request 1/share of
 * a CU's LDS (1: CU-exclusive).  Bit-identical results; 0 = off. */
int slam_icp_set_schedule_wide(int pairs, int share);
/* Bulk gangs: batches of fewer than `below_pairs` pairs run the bulk of both
 * scheduler phases as gangs of `parts` (2 or 3) workgroups with the ordinary
 * LDS footprint — half (a third) of a pair's iteration latency when whole
 * pairs cannot fill the GPU (strong-scaling shards).  Bit-identical results.
 * below_pairs = 0: off. */
int slam_icp_set_bulk_gangs(int below_pairs, int parts);
/* Diagnostics: the scheduler can save a paused pair's search state (last match
 * and clearance per query, 8 B, and the pending motion bound) so its phase-2
 * iteration starts warm (1; a transient workspace of 8 B per query — measured
 * no faster on C3, round 4); 0 (default) resumes cold.  Results are identical. */
int slam_icp_set_schedule_warm(int on);
/* Gang parts that waited longer than the gang wait for a partner since the
 * last call (read-and-clear; synchronises the device): 4 ms at a pair's first
 * exchange of a launch (a partner that is not resident by then, e.g. CUs held
 * by another process), 0.2 s later on.  Such a part stops at once without
 * writing and marks its next exchange so that partners already past this one
 * stop there too; a first-exchange timeout also stops every other pair of the
 * same launch at its first exchange (one wait per launch, not per pair);
 * after phase 2 the scheduler re-runs every exchange-tier pair
 * that did not finish on one workgroup from its saved state, so the results
 * stay valid (and bit-identical): this count is a warning, not an error.
 * Scheduler order is a stable sort (deterministic). */
int slam_icp_gang_timeouts(void);
/* Diagnostics: the gang wait in s_memrealtime ticks (100 MHz); 0 = default.
 * Tiny values force timeouts, exercising the repair path (the first
 * exchange's wait is the smaller of this and slam_icp_set_gang_first_wait's). */
int slam_icp_set_gang_wait(uint32_t ticks);
/* Diagnostics: the first exchange's wait in ticks; 0 = default (4 ms). */
int slam_icp_set_gang_first_wait(uint32_t ticks);
/* Diagnostics: `workgroups` workgroups that each hold a whole CU's LDS and
 * spin for `ticks` (<= 1 s) on `stream` — a stand-in for another process
 * occupying CUs while a batch runs. */
int slam_icp_diag_occupy(int workgroups, uint32_t ticks, void* stream);
/* Diagnostics: phase 2's visiting order of B pairs from their phase-1
 * out_iters (> 0: finished) and keys (last |dE|), by the scheduler's stable
 * bucket sort (device arrays; order[] receives B pair indices). */
int slam_icp_sched_sort(const int32_t* iters, const float* key, int32_t B, float thresh, int32_t* order,
                        void* stream);
/* Diagnostics: batches of <= 8,192 pairs sort at the phase boundary on one
 * workgroup (1, default; slam_icp_sched_sort uses it at those sizes too) or
 * with the three-kernel sort (0).  The order is the same. */
int slam_icp_set_sched_sort_one(int on);
/* Diagnostics: batches of fewer than `pairs` pairs get the scheduler's tail
 * tiers (heads, gangs, wide); 0 restores the default (4,096). */
int slam_icp_set_tier_limit(int pairs);
/* Diagnostics: the angle pre-tier — batches of up to 8,192 pairs run up to
 * `max_pairs` pairs whose initial transform turns by more than `thresh_rad`
 * on a tier of their own from the start (slam_icp_set_angle_tier_kind),
 * beside the two-phase schedule of the others (0: off).  Results are
 * bit-identical. */
int slam_icp_set_angle_tier(int max_pairs, float thresh_rad);
/* Diagnostics: the angle pre-tier's kind, 0 the wide tier, 2 / 3 / 4 / 6 bulk
 * gangs of that many ordinary workgroups per pair. */
int slam_icp_set_angle_tier_kind(int kind);
/* Diagnostics: with a gang pre-tier (kind 2 / 3), its first wide_pairs
 * turning pairs (the largest turns) run on wide workgroups, `share` per CU,
 * the rest on the gangs (0: none).  Bit-identical. */
int slam_icp_set_angle_tier_mix(int wide_pairs, int share);
/* Diagnostics: query groups per wide-tier workgroup: 1 (8 waves, `share`
 * workgroups per CU) or 2 (16 waves, one workgroup per CU; a 1081-point pair
 * on 9 workgroups).  Bit-identical. */
int slam_icp_set_wide_groups(int groups);
/* The scheduler's automatic tier profile by batch size (1, default; DESIGN.md
 * section 6): below 2,048 pairs up to 40 turning pre-tier pairs, below 4,096
 * up to 64, on wide workgroups of two query groups (one per CU); 4,096 - 8,192
 * pairs up to 96 pre-tier pairs on gangs of 4 plus 64 phase-2 heads, the
 * first 24 as gangs of 4; larger batches no tiers.  0: the explicit settings;
 * any of the tier setters above selects them, 1 restores their defaults too. */
int slam_icp_set_schedule_auto(int on);
/* The drain tier of phased batches: once every pair of phase 2's bulk launch
 * has started and at most `pairs` still run, each of them pauses at the end of
 * its iteration and they finish on wide workgroups (two query groups, one per
 * CU), from their paused state, bit-identical.  -1: the default (24 for
 * batches up to 8,192 pairs, off above), 0: off, at most 64 (more than
 * 256 / parts pairs cannot all be resident: their exchanges time out and the
 * repair launch finishes them). */
int slam_icp_set_drain(int pairs);
/* Diagnostics: the XCD-aware pair map of launches in stream order: runs of
 * `run` consecutive pairs per XCD (default 16, so consecutive pairs share
 * their common scan through one L2 while the runs rotate over the XCDs),
 * 0 the identity, -1 the default. */
int slam_icp_set_xcd_map(int run);
int slam_gn_set_stamps(void* dev_buf);
/* GN linear solver (per host thread): 0 auto (block cyclic reduction when the
 * band allows it), 1 band Cholesky, 2 block cyclic reduction (falls back to 1
 * if the band is too wide).  A bordered plan (slam_gn_iteration_bordered_f64)
 * needs the cyclic-reduction solver: with mode 1, or a band too wide for it,
 * that entry point returns SLAM_EINVAL; slamhip.gn plans without a border
 * while mode 1 is set (slam_gn_get_solver). */
int slam_gn_set_solver(int mode);
int slam_gn_get_solver(void);
/* Block rows of the cyclic-reduction solver for (nv, W), 0 = not applicable. */
int slam_gn_bcr_block_rows(int32_t nv, int32_t W);
/* Diagnostics: per-phase s_memtime totals of workgroup 0 into a device buffer of
 * >= 160 uint64 (wave 0's sub-phases in [0, 16), every wave's phase totals in
 * [16 + 8 * wave, 24 + 8 * wave), the pruned search's group iterations, live and
 * visited sub-chunks by active-lane bucket in [96, 120)); NULL turns stamping off. */
int slam_icp_set_stamps(void* dev_buf);
/* Count candidate-distance evaluations performed (all lanes) into a device
 * uint64 (atomic add per wave); NULL turns counting off.  Stamps and the
 * counter run in a separate diagnostics build of the pruned batch kernel
 * (NN mode 2, slam_icp_batch_f64 only); the product kernels carry neither. */
int slam_icp_set_eval_counter(void* dev_u64);
/* Diagnostics: the per-pair phase timeline of slam_icp_batch_f64 into a device
 * buffer of B x 2 x 4 uint64 — per pair and scheduler phase the
 * s_memrealtime (100 MHz) at which its workgroup (part 0) started and ended
 * and where it ran (XCC << 32 | HW_ID); NULL turns it off. */
int slam_icp_set_trace(void* dev_buf);

#ifdef __cplusplus
}
#endif
#endif /* SLAMHIP_H */
