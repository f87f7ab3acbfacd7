"""Generate tests/golden/dataloader_ref.npz by running the REFERENCE's
``get_point_cloud`` (:47-55) and ``align_data`` (:83-107, both branches) from
/root/reference/src/dataloader.py, plus
tests/golden/lcm_run/image_timestamps.txt (the camera timestamp file
``get_images`` reads, reference :25-44).

That module imports cv2 and lcm at module level (:1-3), both absent here, and
neither is used by these two functions.  So, as gen_grid.py does, the source
is parsed with ``ast`` and exactly those two function definitions are
executed, in a namespace holding numpy; no stand-in for cv2 or lcm is made.

Inputs: the scans and odometry of tests/golden/lcm_run/run.log as the
reference's own LCM types decoded them (lcm_expected.npz, gen_lcm.py), extra
range/angle vectors for the 0.05 m cut, and camera times before the first
record, on exact record times, between records and past the last one.
Outputs: the point clouds, and per branch the odometry rows and (with images)
the index of each selected point cloud and the images passed through.

Runs only in the build container (the reference never travels to the GPU
box); the .npz holds data only.

    python tests/golden/gen_dataloader.py
"""
import ast
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/src/dataloader.py"
NEEDED = ("get_point_cloud", "align_data")
sys.dont_write_bytecode = True


def reference_functions():
    tree = ast.parse(open(SRC).read(), filename=SRC)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in NEEDED]
    assert sorted(d.name for d in defs) == sorted(NEEDED), [d.name for d in defs]
    ns = {"np": np}
    exec(compile(ast.Module(body=defs, type_ignores=[]), SRC, "exec"), ns)
    return ns


def main():
    ref = reference_functions()
    e = np.load(os.path.join(HERE, "lcm_expected.npz"))
    off = e["off"]
    clouds = [ref["get_point_cloud"](e["ranges"][off[k]:off[k + 1]].tolist(),
                                      e["thetas"][off[k]:off[k + 1]].tolist()) for k in range(len(off) - 1)]
    out = {}
    cl_pts = np.concatenate(clouds)
    cl_off = np.r_[0, np.cumsum([len(c) for c in clouds])]
    out.update(cloud_pts=cl_pts, cloud_off=cl_off)
    # the 0.05 m cut: exactly 0.05 dropped, just above kept, negative and zero dropped
    r = np.array([0.05, 0.0500001, 0.0, -1.0, 3.0, 12.5, 0.049])
    th = np.array([0.1, -0.2, 0.3, 0.0, np.pi, -np.pi / 2, 1.0])
    out.update(cut_ranges=r, cut_thetas=th, cut_cloud=ref["get_point_cloud"](r, th))

    odometry = e["odo"].astype(float)
    odo_t = e["odo_t"].astype(float)
    lid_t = e["lid_t"].astype(float)
    # no-image branch
    o, pcs = ref["align_data"](odometry, odo_t, clouds, lid_t, None, None)
    assert pcs is clouds
    out["noimg_odometry"] = o
    # image branch: camera times (seconds in the text file, microseconds after get_images)
    t0, t1 = min(odo_t[0], lid_t[0]), max(odo_t[-1], lid_t[-1])
    cam_us = np.array([t0 - 5_000.0, odo_t[0], lid_t[0], 0.5 * (odo_t[1] + odo_t[2]), lid_t[3] + 1.0,
                       odo_t[-1], lid_t[-1], t1 + 1.0, t1 + 250_000.0, lid_t[4] - 1.0])
    lines = ["%d, %.6f\n" % (k, t / 1e6) for k, t in enumerate(cam_us)]
    with open(os.path.join(HERE, "lcm_run", "image_timestamps.txt"), "w") as f:
        f.writelines(lines)
    # the timestamps exactly as get_images parses them (:37-42): float(text) * 1E6
    ts = np.array([float(ln.split(", ")[1]) for ln in lines]) * 1E6
    images = np.arange(len(ts) * 2 * 3 * 3, dtype=np.uint8).reshape(len(ts), 2, 3, 3)
    o, pcs, imgs = ref["align_data"](odometry, odo_t, clouds, lid_t, images, ts)
    assert imgs is images
    out["img_timestamps"] = ts
    out["img_odometry"] = o
    out["img_cloud_index"] = np.array([next(k for k, c in enumerate(clouds) if c is p) for p in pcs])
    # a shorter image array than timestamps (align_data loops over images.shape[0])
    o4, pcs4, _ = ref["align_data"](odometry, odo_t, clouds, lid_t, images[:4], ts)
    out["img4_odometry"] = o4
    out["img4_cloud_index"] = np.array([next(k for k, c in enumerate(clouds) if c is p) for p in pcs4])
    np.savez(os.path.join(HERE, "dataloader_ref.npz"), **out)
    print("wrote dataloader_ref.npz and lcm_run/image_timestamps.txt:",
          {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
