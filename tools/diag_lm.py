"""Diagnostic: LM / GN traces of the device loop (graph and eager) against the oracle on one problem."""
import sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kalibr_amd import capi, synth
from oracle import oracle as O

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 0
pol = sys.argv[3] if len(sys.argv) > 3 else "lm"
p = synth.make_config(cfg, n_frames=nf or None, p_view=0.7 if nf else 1.0)
o = O.Oracle(p)
st_o, r_o = o.optimize(p.state_init, policy=pol, nthreads=16, max_iterations=12)
print("oracle", r_o["iterations"], r_o["failed_iterations"])
print(np.array2string(r_o["trace"][:8], precision=10))
for graph in (True, False):
    g = capi.Solver(p)
    g.set_state(p.state_init)
    r = g.optimize(policy=pol, max_iterations=12, use_graph=graph, sync_every=1)
    print("gpu graph" if graph else "gpu eager", r["iterations"], r["failed_iterations"], np.abs(g.get_state() - st_o).max())
    print(np.array2string(r["trace"][:8], precision=10))
# per-call: build + solve at lambda 10 vs oracle
g = capi.Solver(p)
g.set_state(p.state_init)
g.build()
for lam in (10.0, 1.0):
    g.set_constant_conditioner(lam)
    ok, dx = g.solve()
    A = o.arrow(p.state_init)
    ok_o, dx_o = o.solve(A, lam)
    print("per-call lam", lam, ok, ok_o, np.abs(dx - dx_o).max() / np.abs(dx_o).max())
