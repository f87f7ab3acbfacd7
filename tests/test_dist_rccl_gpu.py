"""The multi-GPU exchange over RCCL on real hardware: the "nccl" backend
(= RCCL on ROCm) at world size 1 on the box's one GPU — the same
slamhip.dist path bench.py takes at N > 1 (device tensors packed, one
all_gather_into_tensor, the odometry chain from the gathered edges) — with
GPU ICP results of a 200-pair C3 stream, against the single-process chain.
(World sizes 2 and 3 are covered with gloo on the CPU, tests/test_dist_gloo.py;
the 8-GPU run is the driver's.)"""
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_rccl_all_gather_chain_single_rank():
    import torch
    import torch.distributed as dist
    from slamhip import dist as sd
    from slamhip import icp as k
    from slamhip import se2, synthetic
    n = 200
    seq = synthetic.make_sequence(n + 1, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)])
    r = k.icp_batch(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    want = se2.compose_chain(seq.odometry[0], r.tf)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        assert dist.get_backend() == "nccl"
        poses, tf, err, its = sd.sharded_chain(seq.odometry[0], r.tf, n, iters_local=r.iters, err_local=r.err)
        # the device-side exchange itself, as bench.py calls it
        local = sd.pack(torch.as_tensor(r.tf.reshape(n, 9)).cuda(), torch.as_tensor(r.err).cuda(),
                        torch.as_tensor(r.iters).cuda(), n)
        g = sd.all_gather_results(local)
        assert g.is_cuda and g.shape == (1, n, sd.RESULT_WIDTH)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert np.array_equal(tf, r.tf.reshape(n, 3, 3)) and np.array_equal(err, r.err)
    assert np.array_equal(its, r.iters)
    assert np.array_equal(poses, want)
    gt, ge, gi = sd.unpack(g, n)
    assert np.array_equal(gt, r.tf.reshape(n, 3, 3)) and np.array_equal(gi, r.iters)
