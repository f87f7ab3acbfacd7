"""Generate tests/golden/lcm_run/ — a small LCM event log whose messages are
ENCODED BY THE REFERENCE's generated LCM types (src/lcmtypes/lidar_t.py,
odometry_t.py, pure Python, importable here), framed with
slamhip.lcmlog.write_events, plus lcm_expected.npz with the reference
decoder's field values (lidar_t.decode / odometry_t.decode).

Runs only in the build container (the reference stays here).  The point-cloud
conversion and time alignment of src/dataloader.py (:47-55, :83-107) are
restated in tests/test_lcm.py (that module imports cv2 and lcm, absent here).

    python tests/golden/gen_lcm.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = ["/root/reference/src/lcmtypes", os.path.join(REPO, "icp-slam-with-loop-closure_amd")]

from lidar_t import lidar_t  # noqa: E402  (reference generated code)
from odometry_t import odometry_t  # noqa: E402

from slamhip import lcmlog  # noqa: E402


def main():
    rng = np.random.default_rng(11)
    events, exp = [], {"odo": [], "odo_t": [], "lid_t": [], "ranges": [], "thetas": [], "off": [0]}
    t = 1_700_000_000_000_000
    for k in range(9):
        t += int(rng.integers(40_000, 60_000))
        if k % 3 != 2:   # odometry at a different rate than lidar
            m = odometry_t()
            m.utime, m.x, m.y, m.theta = t, *rng.normal(0, 2, 3).tolist()
            events.append((t, "ODOMETRY", m.encode()))
            d = odometry_t.decode(m.encode())
            exp["odo"].append((d.x, d.y, d.theta))
            exp["odo_t"].append(d.utime)
        t += int(rng.integers(5_000, 20_000))
        n = int(rng.integers(20, 60))
        m = lidar_t()
        m.utime, m.num_ranges = t, n
        r = rng.uniform(0.0, 6.0, n)
        r[::7] = 0.01                         # returns below 0.05 m are dropped
        m.ranges = r.tolist()
        m.thetas = np.linspace(-2.3, 2.3, n).tolist()
        m.times = [t + i for i in range(n)]
        m.intensities = rng.uniform(0, 1, n).tolist()
        events.append((t, "LIDAR", m.encode()))
        d = lidar_t.decode(m.encode())
        exp["lid_t"].append(d.utime)
        exp["ranges"].extend(d.ranges)
        exp["thetas"].extend(d.thetas)
        exp["off"].append(exp["off"][-1] + n)
        events.append((t + 1, "OTHER_CHANNEL", b"\x00" * 5))
    os.makedirs(os.path.join(HERE, "lcm_run"), exist_ok=True)
    lcmlog.write_events(os.path.join(HERE, "lcm_run", "run.log"), events)
    np.savez(os.path.join(HERE, "lcm_expected.npz"), **{k: np.asarray(v) for k, v in exp.items()})
    print("wrote", len(events), "events")


if __name__ == "__main__":
    main()
