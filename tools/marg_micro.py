"""k_marg micro-run: Jacobi sweep counts of the marginal solver (kb_solve_marginal) on a fixed system (repeated calls:
warm starts from the previous V unless KB_MARG_COLD) and along a GN loop, for a 2-camera (C = 22) and an 8-camera
(C = 106) problem.  Run it under rocprofv3 --kernel-trace --stats for the per-call k_marg duration."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from kalibr_amd import capi, synth  # noqa: E402

for name, p in [("c2_100", synth.make_config(2, n_frames=100)), ("c4_24", synth.make_config(4, n_frames=24, p_view=0.7))]:
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.build()
    sw = []
    t0 = time.perf_counter()
    for _ in range(20):
        ok, dx, info = g.solve_marginal()
        sw.append(info["sweeps"])
    t1 = time.perf_counter()
    gl = []
    for _ in range(8):
        g.build()
        ok, dx, info = g.solve_marginal()
        gl.append(info["sweeps"])
        g.apply_update(dx)
    print(f"{name} C={p.cam_cols} fixed-system sweeps {sw} ({(t1 - t0) / 20 * 1e6:.0f} us/call host), "
          f"GN-loop sweeps {gl}, rank {info['rank']}", flush=True)
