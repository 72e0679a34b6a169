"""Diagnostic: configs[2] GN (20 iterations) through the device loop, pipelined build vs k_build vs the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

p = synth.make_config(3)
kw = dict(policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1.0)
st_o, r_o = O.Oracle(p).optimize(p.state_init, nthreads=16, **kw)
print("oracle", r_o["iterations"], r_o["J_final"])
for pipe in ("1", "0"):
    os.environ["KB_BUILD_PIPE"] = pipe
    g = capi.Solver(p)
    g.set_state(p.state_init)
    r = g.optimize(**kw)
    print("pipe", pipe, r["iterations"], r["failed_iterations"], r["linear_solver_failure"], r["J_final"],
          "max|state - oracle|", float(np.abs(g.get_state() - st_o).max()))
    print(r["trace"][:6])
    g.set_state(p.state_init)
    try:
        g.run_gn(8)
        print("run_gn ok")
    except capi.KbError as e:
        print("run_gn:", e)
