"""Wall time of one kb_solve with the direct Schur solver vs the block-Jacobi PCG solvers (on the full system and on
the camera-block Schur complement; LinearSolverPCG defaults, and converged tightly) at full configs[1] / configs[3] sizes on one GPU.  Host-timed around the
C-ABI call (includes the launch and one stream sync); median of `reps` solves of the same built system.

usage: python tools/pcg_bench.py [reps]   -> one JSON line per (config, solver)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kalibr_amd import capi, synth  # noqa: E402


def med_time(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    for idx in (2, 4):
        p = synth.make_config(idx)
        g = capi.Solver(p)
        g.set_state(p.state_init)
        g.build()
        g.set_constant_conditioner(10.0)
        ok, dx_ref = g.solve()
        t_direct = med_time(g.solve, reps)
        print(json.dumps({"config": idx, "frames": p.n_frames, "C": p.cam_cols, "solver": "schur", "ok": ok,
                          "solve_us": round(t_direct * 1e6, 1)}), flush=True)
        for kind, label, kw in (("pcg", "pcg_default", {}),
                                ("pcg", "pcg_tight", dict(tolerance=1e-24, max_iterations=50000, absolute_tolerance=False)),
                                ("pcg_schur", "pcg_schur_default", {}),
                                ("pcg_schur", "pcg_schur_tight", dict(tolerance=1e-24, max_iterations=50000,
                                                                      absolute_tolerance=False))):
            g.set_linear_solver(kind, **kw)
            ok, dx = g.solve()
            it = g.pcg_info()["iterations"]
            t = med_time(lambda: (g.pcg_init(), g.solve()), reps)
            err = float(np.abs(dx - dx_ref).max() / np.abs(dx_ref).max())
            print(json.dumps({"config": idx, "solver": label, "ok": ok, "iterations": it,
                              "solve_us": round(t * 1e6, 1), "us_per_iteration": round(t * 1e6 / max(it, 1), 2),
                              "rel_err_vs_direct": err}), flush=True)
        g.set_linear_solver("schur")
        g.close()


if __name__ == "__main__":
    main()
