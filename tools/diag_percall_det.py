"""Determinism probe of the per-call path (kb_build / kb_solve / kb_apply_update / kb_eval_cost) on two handles of the
same problem: reports the first step whose results differ bitwise, and what differs."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kalibr_amd import capi, synth

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
p = synth.make_config(cfg, n_frames=12, p_view=0.8)
hs = [capi.Solver(p) for _ in range(2)]
for h in hs:
    h.set_state(p.state_init)
lam = 10.0
for it in range(10):
    res = []
    for h in hs:
        J = h.eval_cost()
        h.build()
        B = h.normal_blocks()
        h.set_constant_conditioner(lam)
        ok, dx = h.solve()
        h.apply_update(dx)
        res.append((J, B, ok, dx, h.get_state()))
    (J0, B0, ok0, dx0, s0), (J1, B1, ok1, dx1, s1) = res
    diffs = []
    if J0 != J1:
        diffs.append("cost %.3e" % abs(J0 - J1))
    for k in ("Hff", "Hfc", "gf", "Hcc", "gc"):
        if not np.array_equal(B0[k], B1[k]):
            diffs.append("%s %.3e" % (k, np.abs(B0[k] - B1[k]).max()))
    if not np.array_equal(dx0, dx1):
        C = hs[0].C
        diffs.append("dx_cam %.3e dx_frames %.3e" % (np.abs(dx0[:C] - dx1[:C]).max(), np.abs(dx0[C:] - dx1[C:]).max()))
    if not np.array_equal(s0, s1):
        diffs.append("state %.3e" % np.abs(s0 - s1).max())
    print("iteration", it, "OK" if not diffs else "DIFF " + ", ".join(diffs), flush=True)
