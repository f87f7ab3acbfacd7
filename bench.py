#!/usr/bin/env python3
"""Headline benchmark: batched ICP scan-pairs/s (1081-point scans) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Workload (BASELINE.json configs[2], "Batched ICP: 10k synthetic scan-pairs x
1081 pts, 1->8 GPU sharding"): ONE synthetic scan stream of P+1 scans (P =
10,000 by default; SURVEY.md §8(d) generator, seed 2025) whose P consecutive
pairs (i, i-1) are sharded over the N ranks (``--shard``: contiguous slices,
or cost-balanced by the turn of each pair's initial transform,
slamhip.dist.balanced_shards); each rank holds its shard's scans resident in
HBM and runs ``icp()`` on it with scripts/main.py's
parameters (init = pose_to_mat(odom_i - odom_{i-1}), epsilon 0.05, max_iters
100).  One step = one ``slam_icp_batch_f64`` launch over the rank's shard and,
for N > 1, the RCCL all-gather of the resulting SE(2) edges (the exchange step
of the north star).  Total work is fixed as N grows ("scaling": "strong");
``--weak`` gives every rank its own P-pair stream (seed 2025 + rank) instead.

Printed: ONE JSON line (rank 0) with the driver's contract fields plus
``roofline`` (dominant kernel: the FP32 VALU roofline over the candidate
distances it actually evaluates, the VALU issue fraction from the committed
PMC profile, the HBM rate beside it),
``cpu_baseline`` (NumPy port of the reference, timed on this host) and
secondary pose-graph numbers (``pgo``).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))

FP64_VALU_PEAK_TFLOPS = 78.6     # MI355X vector FP64 (spec), MI355X_MICROARCH.md
FP32_VALU_PEAK_TFLOPS = 157.3    # MI355X vector FP32 (spec)
HBM_PEAK_GBPS = 8000.0
FLOP_PER_EVAL = 5                 # 2 sub, 2 mul, 1 add per candidate distance
# issue-bound candidate rate of the exact scan (~8 VALU
# instructions per candidate): 256 CU x 2.4 GHz x 64 lanes / 8
ISSUE_BOUND_EVALS_PER_S = 4.9e12
DEFAULT_SHARD = "balanced"
KERNEL_SOURCES = ("icp-slam-with-loop-closure_amd/csrc/icp_kernels.hip", "icp-slam-with-loop-closure_amd/csrc/common.hpp")


def kernel_source_sha():
    """sha256 of the ICP kernel sources: ties a committed PMC profile to the
    kernel it measured (tools/collect_profile.py records the same hash)."""
    import hashlib
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(REPO, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--pairs", type=int, default=10000, help="scan pairs in total (default) or per rank (--weak)")
    p.add_argument("--beams", type=int, default=1081)
    p.add_argument("--weak", action="store_true",
                   help="every rank runs its own P-pair stream (weak scaling) instead of a shard of one")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pgo", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=192, help="pairs in the CPU baseline sample")
    p.add_argument("--cpu-workers", type=int, default=0, help="0 = every core this job may use")
    p.add_argument("--instance", type=int, default=-1, help="force a kernel instance (diagnostics)")
    p.add_argument("--sched-probe", type=int, default=-1,
                   help="phase-1 iterations of the batch scheduler (0 = one launch; -1 = library default)")
    p.add_argument("--sched-heads", type=int, default=-1,
                   help="pairs started on CU-exclusive workgroups in phase 2 (-1 = library default)")
    p.add_argument("--sched-gangs", default="",
                   help="G,K: the first G head pairs run as gangs of K workgroups (library default 24,4; 0,2 = off)")
    p.add_argument("--sched-wide", default="",
                   help="W,S: the W slowest-keyed pairs on the wide tier, 1/S of a CU's LDS each (0,1 = off)")
    p.add_argument("--bulk-gangs", default="",
                   help="B,K: batches below B pairs run their bulk as gangs of K workgroups (0,2 = off)")
    p.add_argument("--sched-warm", type=int, default=-1,
                   help="1: phase 2 resumes with the saved search state (library default 0)")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm); gloo only for dry runs")
    p.add_argument("--shard", default=DEFAULT_SHARD, choices=("contiguous", "balanced"),
                   help="strong-scaling split of the pairs over the ranks (slamhip.dist)")
    return p.parse_args()


def init_dist(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # SLAMHIP_ONE_DEVICE=1: every rank on cuda:0 (multi-rank dry run on a 1-GPU box, gloo)
        dev = 0 if os.environ.get("SLAMHIP_ONE_DEVICE") == "1" else local
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def make_workload(args, world, rank):
    """This rank's pairs: (scans it holds, src, dst (local scan indices),
    inits, every rank's pair-index list of the stream)."""
    from slamhip import se2, synthetic
    from slamhip import dist as sd
    seed = 2025 + (rank if args.weak else 0)
    seq = synthetic.make_sequence(args.pairs + 1, seed=seed, n_beams=args.beams)
    odo = seq.odometry
    n = args.pairs
    inits = np.stack([se2.pose_to_mat(odo[i] - odo[i - 1]) for i in range(1, n + 1)]) if n else np.zeros((0, 3, 3))
    if args.weak or world == 1:
        shards = [np.arange(n, dtype=np.int64)]
        idx = shards[0]
    else:
        shards = (sd.balanced_shards(sd.turn_keys(inits), world) if args.shard == "balanced"
                  else sd.contiguous_shards(n, world))
        idx = shards[rank]
    scans, src, dst = sd.local_scans(seq.scans, idx + 1, idx)
    return scans, src, dst, inits[idx], shards


def tier_profile(B):
    """The batch scheduler's automatic tier profile for a batch of B pairs
    (csrc/icp_kernels.hip launch_batch)."""
    if B < 1024:
        return "one launch, one workgroup per pair"
    drain = "; drain tier: phase 2's last 24 running pairs on wide workgroups"
    if B < 2048:
        return ("two-phase (probe 3); turning pairs (<= 40) on the wide pre-tier, 2 query groups per CU-exclusive"
                " workgroup" + drain)
    if B < 4096:
        return ("two-phase (probe 4); turning pairs (<= 64) on the wide pre-tier, 2 query groups per CU-exclusive"
                " workgroup" + drain)
    if B <= 8192:
        return ("two-phase (probe 2); turning pairs (<= 96) as gangs of 4; phase 2: 64 CU-exclusive heads, 24 as"
                " gangs of 4" + drain)
    return "two-phase scheduler (phase 1: 3 iterations per pair; phase 2 slowest-first), no tiers"


def host_cpu():
    """(logical CPUs of the machine, CPUs this process may use, model name)."""
    n_all = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except AttributeError:
        n_aff = n_all
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n_all, n_aff, model


def default_cpu_workers():
    """All host cores this job may use (scripts/main.py:240 uses n_jobs=-1):
    the affinity set, capped by OMP_NUM_THREADS where the launcher sets the
    job's CPU share (the GPU box: 16 per GPU, while os.cpu_count() shows the
    whole machine)."""
    _, n_aff, _ = host_cpu()
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n_aff, int(cap))) if cap and cap.isdigit() else n_aff


def _oracle_pair(pc1, pc2, init, loop):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import icp_oracle
    fn = icp_oracle.correspondences_loop if loop else icp_oracle.correspondences
    h, e = icp_oracle.icp(pc1, pc2, init, 0.05, 100, corr_fn=fn)
    return h[-1], float(e), len(h) - 1


def cpu_baseline(scans, src, dst, inits, sample, workers):
    """The reference's ICP restated in NumPy (oracle/icp_oracle.py, bit-exact
    with src/icp.py) on this host's cores, on bounded samples of this workload:

      ref_loop   the reference's per-query loop (src/icp.py:16-17)
      vectorized the same arithmetic over query blocks (bit-identical results)

    each on 1 core and on `workers` cores through joblib loky, as
    scripts/main.py:240 fans icp() out.  `value` is ref_loop on all cores
    (what scripts/main.py runs).  Returns (baseline dict, {pair index: (tf,
    err, iters)} of the all-core ref_loop sample) — the second feeds the
    parity block."""
    from joblib import Parallel, delayed
    env = {"OMP_NUM_THREADS": "1", "OPENBLAS_NUM_THREADS": "1", "MKL_NUM_THREADS": "1"}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    n_all, n_aff, model = host_cpu()

    def job(i):
        a, b = scans[src[i]], scans[dst[i]]
        return np.c_[a, np.ones(len(a))], np.c_[b, np.ones(len(b))], inits[i].copy()

    def run(idx, loop, n_jobs):
        t0 = time.perf_counter()
        if n_jobs == 1:
            out = [_oracle_pair(*job(i), loop) for i in idx]
        else:
            out = par(delayed(_oracle_pair)(*job(i), loop) for i in idx)
        return out, time.perf_counter() - t0

    try:
        par = Parallel(n_jobs=workers, backend="loky")
        par(delayed(_oracle_pair)(*job(0), False) for _ in range(workers))   # spin the pool up
        modes = {}
        idx_all = np.linspace(0, len(inits) - 1, sample).astype(int)
        res_all, dt = run(idx_all, True, workers)
        modes["ref_loop_all_cores"] = {"pairs": len(idx_all), "s": round(dt, 2), "pairs_per_s": round(len(idx_all) / dt, 3)}
        n1 = max(2, sample // (2 * workers))
        idx1 = idx_all[:n1]
        _, dt = run(idx1, True, 1)
        modes["ref_loop_1_core"] = {"pairs": n1, "s": round(dt, 2), "pairs_per_s": round(n1 / dt, 3)}
        nv = max(4, sample // 12)
        idxv = idx_all[:nv]
        _, dt = run(idxv, False, 1)
        modes["vectorized_1_core"] = {"pairs": nv, "s": round(dt, 2), "pairs_per_s": round(nv / dt, 3)}
        _, dt = run(idx_all, False, workers)
        modes["vectorized_all_cores"] = {"pairs": len(idx_all), "s": round(dt, 2),
                                         "pairs_per_s": round(len(idx_all) / dt, 3)}
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    its = [r[2] for r in res_all]
    base = {"value": modes["ref_loop_all_cores"]["pairs_per_s"], "unit": "scan-pairs/s", "cores": workers,
            "kind": "port",
            "cores_note": f"the job's {workers}-CPU share (n_jobs=-1 within it; OMP_NUM_THREADS caps the share on "
                          "the GPU box), not every CPU of the host",
            "sample": f"{len(idx_all)} evenly spaced pairs of this workload (1081-pt scans, mean {np.mean(its):.1f} "
                      f"ICP iterations): oracle/icp_oracle.py with the reference's per-query loop "
                      f"(src/icp.py:16-17), joblib loky x{workers} (scripts/main.py:240 pattern)",
            "modes": modes, "host": {"os_cpu_count": n_all, "affinity_cpus": n_aff, "workers": workers,
                                     "cpu_model": model},
            # scripts/main.py:240 runs n_jobs=-1 (every CPU it may use).  The GPU box
            # grants this job a 16-CPU share (OMP_NUM_THREADS; worker pools must stay
            # within it), so `value` is n_jobs=-1 inside that share; the per-core
            # rate scaled to every affinity CPU is an (unmeasured, linear) upper
            # bound of the reference on the whole host
            "projection_all_affinity_cpus": {
                "cpus": n_aff, "pairs_per_s": round(modes["ref_loop_1_core"]["pairs_per_s"] * n_aff, 2),
                "vectorized_pairs_per_s": round(modes["vectorized_1_core"]["pairs_per_s"] * n_aff, 2),
                "kind": "linear projection of the 1-core rate, not measured"}}
    return base, {int(i): r for i, r in zip(idx_all, res_all)}


def parity_block(res, ref):
    """GPU results of the timed launches vs the CPU port on the sampled pairs."""
    idx = sorted(ref)
    dtf = max(float(np.abs(res.tf[i] - ref[i][0]).max()) for i in idx)
    derr = max(abs(float(res.err[i]) - ref[i][1]) / max(1.0, abs(ref[i][1])) for i in idx)
    eq = all(int(res.iters[i]) == ref[i][2] for i in idx)
    return {"pairs": len(idx), "max_abs_tf_diff": dtf, "max_rel_err_diff": derr, "iters_equal": eq,
            "tolerance": 1e-9, "ok": bool(eq and dtf <= 1e-9 and derr <= 1e-9),
            "reference": "oracle/icp_oracle.py (bit-exact restatement of src/icp.py)"}


def pgo_bench():
    """Secondary: SGD relaxation step on the C4-size graph (5,000 nodes)."""
    import torch
    from slamhip import pgo, synthetic
    import src.pose_graph as pgm
    poses, loops = synthetic.lap_pose_graph(side_len=3.0, poses_per_side=125, num_loops=10, seed=0,
                                            num_constraints=15000)
    pg = pgm.PoseGraph(poses.copy())
    for a, b in loops:
        pg.add_constraint(a, b, np.eye(3))
    ea, eb, tf = pg.edge_arrays()
    s = pgo.SgdSolver(poses, ea, eb, tf)
    s.step(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 3
    for i in range(k):
        s.step(1.0 / (i + 2))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    # the drop-in call scripts/main.py:325-326 makes 50 times on one graph:
    # host poses in, one step, poses written back in place
    import src.pose_graph_optimization as pgo_drop_in
    pgo_drop_in.pose_graph_optimization_step_sgd(pg, learning_rate=1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        pgo_drop_in.pose_graph_optimization_step_sgd(pg, learning_rate=1.0 / (i + 2))
    dt_drop = (time.perf_counter() - t0) / k
    out = {"sgd_step_ms": round(dt * 1e3, 3), "sgd_dropin_step_ms": round(dt_drop * 1e3, 3),
           "sgd_graph": f"{len(poses)} nodes / {len(ea)} edges"}
    try:
        from slamhip import gn
        out.update(gn.bench_c4())
    except (ImportError, AttributeError):
        pass
    out["cpu_baseline"] = pgo_cpu_baseline(poses, ea, eb, tf)
    return out


def pgo_cpu_baseline(poses, ea, eb, tf):
    """The pose-graph CPU paths timed on this host: the SGD step
    as the vectorised NumPy port of the reference (oracle/pgo_oracle.py,
    src/pose_graph_optimization.py:7-49 restated; one step, 1 core) on the
    same C4-size graph as sgd_step_ms, and the build's float64 SciPy GN
    (oracle/gn_oracle.py) on C4, 1 BLAS thread and every thread of the job's
    share.  The reference's own SGD code is not run here (it stays in the
    build container); its 138.9 s/step is the survey's measurement."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import gn_oracle
    import pgo_oracle
    from threadpoolctl import threadpool_limits
    from slamhip import synthetic
    out = {}
    with threadpool_limits(1):
        t0 = time.perf_counter()
        pgo_oracle.sgd_step(np.array(poses, dtype=np.float64), ea, eb, tf, 1.0)
        out["sgd_port_1core_s_per_step"] = round(time.perf_counter() - t0, 3)
    guess, gea, geb, gtf, _ = synthetic.lap_graph_c4()
    its = 3
    for name, lim in (("gn_oracle_1thread_iters_per_sec", 1), ("gn_oracle_all_threads_iters_per_sec", None)):
        with threadpool_limits(lim):
            t0 = time.perf_counter()
            gn_oracle.optimize(guess.copy(), gea, geb, gtf, iterations=its)
            out[name] = round(its / (time.perf_counter() - t0), 3)
    out.update({"threads_all": default_cpu_workers(), "kind": "port",
                "sgd_reference_s_per_step_survey": 138.9,
                "note": "sgd_port: oracle/pgo_oracle.py (vectorised, bit-exact with the reference) on the "
                        f"{len(poses)}-node / {len(ea)}-edge graph; gn_oracle: SciPy SuperLU GN on C4 "
                        "(5000 nodes / 20000 edges); sgd_reference_s_per_step_survey: the reference's own "
                        "src/pose_graph_optimization.py, 1 core of the build container (SURVEY.md §6), not "
                        "re-run on this box"})
    return out


def c1_bench(reps=20):
    """Config C1 (BASELINE configs[0]): ONE drop-in ``src.icp.icp()`` call on a
    1081-point pair (scripts/test_icp.py shape), host arrays in and out —
    the latency an unchanged caller sees per call (upload, one B = 1 launch
    with the transform history, download)."""
    import torch
    import src.icp as icp
    from slamhip import se2, synthetic
    seq = synthetic.make_sequence(2, seed=0)
    pc1 = np.c_[seq.scans[1], np.ones(len(seq.scans[1]))]
    pc2 = np.c_[seq.scans[0], np.ones(len(seq.scans[0]))]
    init = se2.pose_to_mat(seq.odometry[1] - seq.odometry[0])
    tfs, _ = icp.icp(pc1, pc2, init_transform=init.copy(), epsilon=0.05, max_iters=100)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        tfs, _ = icp.icp(pc1, pc2, init_transform=init.copy(), epsilon=0.05, max_iters=100)
        ts.append(time.perf_counter() - t0)
    its = len(tfs) - 1
    return {"c1_icp_call_ms": round(float(np.median(ts)) * 1e3, 3), "c1_iterations": its,
            "c1_ref_cpu_s_per_call_est": round(0.0318 * its, 3),
            "c1_note": "median of %d drop-in src.icp.icp() calls, host arrays in/out; reference CPU estimate = "
                       "31.8 ms per get_correspondences at 1081^2 (SURVEY.md section 8(a) a2) x iterations" % reps}


def main():
    args = parse()
    import torch
    world, rank, local = init_dist(args)
    if world > 1:
        import torch.distributed as dist
    from slamhip import _abi
    from slamhip import icp as k

    t_gen = time.perf_counter()
    scans, src, dst, inits, shards = make_workload(args, world, rank)
    B = len(inits)
    log(f"[rank {rank}] generated {B} pairs in {time.perf_counter() - t_gen:.1f}s")
    lib = _abi.lib()
    if args.instance >= 0:
        lib.slam_icp_force_instance(args.instance)
    if args.sched_probe >= 0:
        lib.slam_icp_set_schedule(args.sched_probe, 1024)
    if args.sched_heads >= 0:
        lib.slam_icp_set_schedule_heads(args.sched_heads)
    if args.sched_gangs:
        g_, k_ = (int(x) for x in args.sched_gangs.split(","))
        lib.slam_icp_set_schedule_gangs(g_, k_)
    if args.sched_wide:
        w_, s_ = (int(x) for x in args.sched_wide.split(","))
        lib.slam_icp_set_schedule_wide(w_, s_)
    if args.bulk_gangs:
        b_, k_ = (int(x) for x in args.bulk_gangs.split(","))
        lib.slam_icp_set_bulk_gangs(b_, k_)
    if args.sched_warm >= 0:
        lib.slam_icp_set_schedule_warm(args.sched_warm)
    lib.slam_icp_set_screen(int(os.environ.get("SLAMHIP_SCREEN", "2")))
    ss = k.ScanSet(scans)
    batch = k.IcpBatch(ss, src, dst, inits, epsilon=0.05, max_iters=100)
    from slamhip import dist as sd
    gathered = None
    if world > 1:
        # SE(2) edge + error + iteration count of every pair, padded to the largest shard
        Bpad = max(max(len(x) for x in shards) if not args.weak else B, 1)
        gathered = torch.empty((world, Bpad, sd.RESULT_WIDTH), dtype=torch.float64, device=ss.device)
        local_res = torch.zeros((Bpad, sd.RESULT_WIDTH), dtype=torch.float64, device=ss.device)

    stream = torch.cuda.current_stream()

    def exchange():
        sd.pack(batch.out_tf[:B], batch.out_err[:B], batch.out_iters[:B], Bpad, out=local_res)
        sd.all_gather_results(local_res, out=gathered)

    def step():
        batch.launch()
        if world > 1:
            exchange()   # SE(2) edges of every pair -> every rank

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # exchange-tier timeouts (a gang / wide part whose partners were not all
    # co-resident, repaired bit-identically but slow): counted over the timed steps
    lib.slam_icp_gang_timeouts()   # read and clear
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        batch.launch()
        ev[i][1].record(stream)
        if world > 1:
            exchange()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    timeouts = int(lib.slam_icp_gang_timeouts())

    res = batch.result()
    n1 = ss.lens[src]
    n2 = ss.lens[dst]
    evals = float(np.sum(res.iters * n1 * n2))
    t = torch.tensor([dt, evals, float(B), float(res.iters.sum())], dtype=torch.float64,
                     device=ss.device if args.dist_backend == "nccl" else "cpu")
    per_rank = None
    gather_ok = None
    if world > 1 and not args.weak:
        # the gathered SE(2) edges, put back in pair order, hold this rank's own results
        tf_all, _, it_all = sd.unpack_shards(gathered, shards)
        mine_idx = shards[rank]
        gather_ok = bool(np.array_equal(tf_all[mine_idx], res.tf) and np.array_equal(it_all[mine_idx], res.iters))
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        t[0] = tmax[0]
        # every rank's shard and its kernel time (the slowest shard bounds the job)
        mine = torch.tensor([kern_ms, float(B), dt / args.steps * 1e3, float(timeouts), float(res.iters.max())],
                            dtype=torch.float64, device=t.device)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[float(x) for x in r.cpu()] for r in allr]
    dt_max, evals_all, pairs_all, iters_all = [float(x) for x in t.cpu()]
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_per_step = dt_max / args.steps * 1e3
    value = pairs_all * args.steps / dt_max
    # dominant kernel: slam_icp_batch_f64 on rank 0 (its own pairs).  Work is
    # counted as the candidate distances the kernel actually evaluates (exact
    # pruning skips most of the n1*n2 brute-force set): one counting launch,
    # outside the timed region (the search is deterministic).
    mode = int(os.environ.get("SLAMHIP_SCREEN", "2")) if int(ss.lens.max()) <= 4096 else 0
    cnt = torch.zeros(1, dtype=torch.int64, device=ss.device)
    lib.slam_icp_set_eval_counter(cnt.data_ptr())
    batch.launch()
    torch.cuda.synchronize()
    lib.slam_icp_set_eval_counter(None)
    performed = float(cnt.item())
    evals_per_s = performed / (kern_ms * 1e-3)
    flops = FLOP_PER_EVAL * evals_per_s / 1e12
    alg_bytes = 16.0 * float(ss.lens.sum()) + B * (4 + 4 + 72 + 72 + 8 + 4) + 8 * (len(ss.lens) + 1)
    hbm_gbps = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    valu_issue = None
    valu_per_eval = None
    pmc_src = {"file": "profiles/pmc_traffic.json", "kernel_source_sha256": kernel_source_sha()}
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            pmc_src.update({"profile_tag": tj.get("tag"), "profile_commit": tj.get("commit"),
                            "profile_kernel_sha256": tj.get("kernel_source_sha256")})
            pmc_src["current"] = tj.get("kernel_source_sha256") == pmc_src["kernel_source_sha256"]
            # measured on tj["pairs"] pairs of this workload; scale to this launch
            traffic = round(tj["icp_batch_bytes_per_launch"] * B / tj.get("pairs", B))
            # VALU busy fraction of the SIMDs over the kernel's dispatches, measured
            # by counters in the committed profile (tools/gpu_profile.sh busy pass:
            # 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), and
            # the VALU lane-instructions issued per candidate distance evaluated
            if "valu_busy_frac" in tj:
                valu_issue = round(tj["valu_busy_frac"], 4)
            if "valu_insts_per_launch" in tj:
                valu_per_eval = tj["valu_insts_per_launch"] * 64.0 / tj.get("pairs", B)
            if not pmc_src["current"]:
                # the committed counters belong to another build of the kernel:
                # kept for reference under pmc_profile, not reported as this run's
                pmc_src["stale_values"] = {"traffic": traffic, "valu_busy_frac": valu_issue}
                traffic = valu_issue = valu_per_eval = None
        except Exception:
            traffic = None
    sel = lib.slam_icp_selected_instance(int(n1.max()))
    import ctypes
    bb, qq = ctypes.c_int32(), ctypes.c_int32()
    lib.slam_icp_instance_shape(sel, ctypes.byref(bb), ctypes.byref(qq))
    out = {
        "metric": "ICP scan-pairs/sec (1081-pt scans)",
        "value": round(value, 2),
        "unit": "scan-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d) ray-cast room, 1081 beams/270 deg, 0.01 m noise; EECS_3 unavailable offline)",
        "exchange_timeouts": timeouts,
        "config": {"workload": "C3 batched ICP: consecutive scan pairs of a synthetic stream, "
                               "scripts/main.py params (eps 0.05, max_iters 100)",
                   "pairs_per_rank": B, "pairs_total": int(pairs_all), "points_per_scan": int(n1.max()),
                   "mean_icp_iterations": round(iters_all / pairs_all, 3),
                   "kernel_instance": f"{bb.value}x{qq.value}", "parallelism": f"dp{world}",
                   "sharding": "weak (own stream per rank)" if args.weak else args.shard,
                   "tier_profile": tier_profile(B)},
        "roofline": {
            # achieved = candidate evaluations per second against
            # the VALU issue bound 4.9e12 /s (= 24.5 TFLOP/s at 5 flops each)
            "bound": "valu",
            "kernel": "slam_icp_batch_f64 (icp_kernel, %s)" % (
                {2: "fp32 screen with exact pruning + fp64 certification",
                 1: "fp32 screen + fp64 certification", 0: "exact fp64 scan"}[mode]),
            "achieved": round(flops, 3),
            "peak": round(FLOP_PER_EVAL * ISSUE_BOUND_EVALS_PER_S / 1e12, 3),
            "unit": "TFLOP/s",
            "frac": round(evals_per_s / ISSUE_BOUND_EVALS_PER_S, 4),
            "traffic": traffic,
            "kernel_ms": round(kern_ms, 4),
            "candidate_evals_per_s": round(evals_per_s, 1),
            "issue_bound_evals_per_s": ISSUE_BOUND_EVALS_PER_S,
            "candidate_evals_frac_of_issue_bound": round(evals_per_s / ISSUE_BOUND_EVALS_PER_S, 4),
            "fp64_flop_frac": round(flops / FP64_VALU_PEAK_TFLOPS, 4),
            "fp32_flop_frac": round(flops / FP32_VALU_PEAK_TFLOPS, 4),
            "fp64_peak_tflops": FP64_VALU_PEAK_TFLOPS,
            "fp32_peak_tflops": FP32_VALU_PEAK_TFLOPS,
            "candidate_evals_performed_per_launch": performed,
            "brute_force_evals_per_launch": evals,
            "pruning_factor": round(evals / max(performed, 1.0), 2),
            "brute_force_equivalent_evals_per_s": round(evals / (kern_ms * 1e-3), 1),
            "valu_busy_frac": valu_issue,
            "valu_busy_source": "profiles/pmc_traffic.json (rocprofv3 SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE, C3 batch)",
            "pmc_profile": pmc_src,
            "valu_lane_insts_per_candidate_eval": (round(valu_per_eval * B / performed, 2)
                                                   if valu_per_eval and performed else None),
            "brute_force_equivalent_note": "pruning skips candidates exactly; the brute-force-equivalent rate is "
                                           "not a roofline figure",
            "hbm": {"achieved": round(hbm_gbps, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(hbm_gbps / HBM_PEAK_GBPS, 6), "algorithmic_bytes_per_launch": alg_bytes},
        },
    }
    if per_rank is not None:
        out["per_rank"] = {"kernel_ms": [round(r[0], 4) for r in per_rank],
                           "pairs": [int(r[1]) for r in per_rank],
                           "wall_ms_per_step": [round(r[2], 4) for r in per_rank],
                           "max_shard_pairs": int(max(r[1] for r in per_rank)),
                           "slowest_rank": int(np.argmax([r[0] for r in per_rank])),
                           "exchange_timeouts": [int(r[3]) for r in per_rank],
                           "all_gather_unpermuted_ok_rank0": gather_ok,
                           "longest_pair_iterations": [int(r[4]) for r in per_rank],
                           "shard": args.shard if not args.weak else "weak",
                           "note": "kernel_ms: HIP events around batch.launch() on each rank's stream; "
                                   "wall: the rank's timed loop incl. the all-gather; exchange_timeouts: "
                                   "slam_icp_gang_timeouts() over the timed steps (repaired bit-identically)"}
    if world == 1 and not args.no_cpu_baseline:
        try:
            workers = args.cpu_workers or default_cpu_workers()
            out["cpu_baseline"], ref = cpu_baseline(scans, src, dst, inits, args.cpu_sample, workers)
            out["parity"] = parity_block(res, ref)
        except Exception as e:   # keep the GPU line even if the host pool fails
            out["cpu_baseline"] = {"error": repr(e)}
    if "parity" not in out:
        # no CPU baseline run (N > 1 or --no-cpu-baseline): a small vectorised sample
        idx = np.linspace(0, B - 1, min(B, 6)).astype(int) if B else []
        ref = {int(i): _oracle_pair(np.c_[scans[src[i]], np.ones(len(scans[src[i]]))],
                                    np.c_[scans[dst[i]], np.ones(len(scans[dst[i]]))], inits[i].copy(), False)
               for i in idx}
        if ref:
            out["parity"] = parity_block(res, ref)
            out["parity"]["scope"] = "rank 0's shard"
    if world == 1 and not args.no_pgo:
        try:
            out["pgo"] = pgo_bench()
        except Exception as e:
            out["pgo"] = {"error": repr(e)}
        try:
            out["c1"] = c1_bench()
        except Exception as e:
            out["c1"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
