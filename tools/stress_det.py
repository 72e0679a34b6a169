"""Determinism stress: repeat builds, solves and LM runs on one handle and report any bitwise difference."""
import sys
import time
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kalibr_amd import capi, synth

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p = synth.make_config(cfg)
g = capi.Solver(p)
t0 = time.time()
# 1. per-call build + solve
g.set_state(p.state_init)
g.build()
B0 = g.normal_blocks()
g.set_constant_conditioner(10.0)
ok0, dx0 = g.solve()
nbad_b = nbad_s = 0
for r in range(reps):
    g.build()
    B = g.normal_blocks()
    bad = [k for k in ("Hff", "Hfc", "gf", "Hcc", "gc") if not np.array_equal(B[k], B0[k])]
    ok, dx = g.solve()
    if bad:
        nbad_b += 1
        print("build differs:", r, bad, flush=True)
    if not np.array_equal(dx, dx0):
        nbad_s += 1
        print("solve differs:", r, np.abs(dx - dx0).max(), flush=True)
print(f"per-call: {reps} reps, {nbad_b} build diffs, {nbad_s} solve diffs ({time.time() - t0:.1f}s)", flush=True)
# 2. LM runs
ref = None
nbad = 0
for r in range(reps):
    g.set_state(p.state_init)
    res = g.optimize(policy="lm")
    st = g.get_state()
    if ref is None:
        ref, rref = st, res
    elif not np.array_equal(st, ref) or res["iterations"] != rref["iterations"]:
        nbad += 1
        print("LM differs:", r, res["iterations"], res["failed_iterations"], res["J_final"], np.abs(st - ref).max(), flush=True)
print(f"LM: {reps} reps, {nbad} diffs, it={rref['iterations']} J={rref['J_final']:.10g} ({time.time() - t0:.1f}s)", flush=True)
# 3. GN runs
ref = None
nbad = 0
for r in range(reps):
    g.set_state(p.state_init)
    g.run_gn(10)
    st = g.get_state()
    if ref is None:
        ref = st
    elif not np.array_equal(st, ref):
        nbad += 1
        print("GN differs:", r, np.abs(st - ref).max(), flush=True)
print(f"GN: {reps} reps, {nbad} diffs ({time.time() - t0:.1f}s)", flush=True)
