"""Diagnostic: repeat the device LM loop with several sync_every / graph settings (determinism check)."""
import sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kalibr_amd import capi, synth

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
p = synth.make_config(cfg)
ref = None
for graph in (True, False):
    for se in (1, 4, 8, 16):
        for rep in range(2):
            g = capi.Solver(p)
            g.set_state(p.state_init)
            r = g.optimize(policy="lm", max_iterations=200, use_graph=graph, sync_every=se)
            st = g.get_state()
            if ref is None:
                ref = st
            print(f"graph={graph} sync_every={se} rep={rep}: it={r['iterations']} failed={r['failed_iterations']} "
                  f"J={r['J_final']:.10g} passes={r['passes']} max|st-ref|={np.abs(st - ref).max():.3e}", flush=True)
            g.close()
