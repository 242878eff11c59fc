"""Run by tests/test_oracle_asan.py in a child process with libasan + libubsan preloaded: the
oracle's entry points on small cases (edge and interior sources, subgrid 1 and 3, rays, the
local operators on the reference's own neighbourhoods, the band model), built with
-fsanitize=address,undefined (oracle/Makefile: make asan)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
os.environ["ALIFMM_ORACLE_LIB"] = os.path.join(REPO, "oracle", "lib", "liboracle_asan.so")
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as O  # noqa: E402
import workloads as W  # noqa: E402

vt = W.default_table()
n = 61
veln = W.voronoi_small(n, seed=5)
velpn = np.zeros((n, n), dtype=np.int64)
vm = np.ones((n, n))
sd = W.stif_field(n, n)
for x, z in ((0, 0), (30, 20), (60, 60), (0, 45)):
    T = O.travel(1e-3 * x, 1e-3 * z, veln, velpn, vm, sd, vt, vt)
    assert np.all(np.isfinite(T)) and T.max() > 0
T3 = O.travel_finer_grid(1e-3 * 59, 1e-3 * 2, veln, velpn, vm, sd, 3, vt, vt)
assert T3.shape == (3 * (n - 1) + 1,) * 2
rx, ry, t = O.find_ray(1e-3, vt, [5, 50], [30, 20], O.travel(0.030, 0.020, veln, velpn, vm, sd, vt, vt), veln, velpn,
                       vm, sd, 1)
assert t > 0 and len(rx) > 2
assert O.time_between_points(1.0, 50.0, 2.0, 40.0, 1e-3, 1, vt, veln, velpn, vm, sd) > 0
g = np.load(os.path.join(REPO, "tests", "golden", "local_ops.npz"))
for k in range(0, 300, 7):
    a = g["u_args"][k]
    st = np.broadcast_to(g["u_stif"][k], (7, 7, 5))
    v = O.update(np.full((7, 7), g["u_mat"][k, 0]), np.full((7, 7), int(g["u_mat"][k, 1])), np.full((7, 7), g["u_mat"][k, 2]),
                 g["u_nsts"][k], g["u_ttn"][k], int(a[0]), int(a[1]), a[2], int(a[3]), int(a[4]), g["tab_p"], st)
    assert v == g["u_out"][k], k
T, steps = O.band_travel(0.030, 0.020, veln, velpn, vm, sd, vt, vt, 7000.0, cdelta=0.5, exact_init=True, r0=40,
                         exact_r=0)
assert np.all(np.isfinite(T))
print("asan ok")
