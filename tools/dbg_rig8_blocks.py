"""Diagnostic: per-call build blocks of configs[3] against the oracle, per frame (which frames / blocks differ)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402
from oracle import oracle as om  # noqa: E402

p = synth.make_config(4)
o = om.Oracle(p)
g = capi.Solver(p)
g.set_state(p.state_init)
g.build()
B = g.normal_blocks()
A = o.arrow(p.state_init, nthreads=16)
for k in ("Hff", "Hfc", "gf", "Hcc", "gc"):
    d = np.abs(B[k] - A[k])
    print(k, B[k].shape, "max abs err", d.max(), "max |A|", np.abs(A[k]).max())
    if B[k].ndim >= 2 and B[k].shape[0] == p.n_frames:
        per = d.reshape(p.n_frames, -1).max(axis=1) / (np.abs(A[k]).max() + 1e-300)
        bad = np.nonzero(per > 1e-10)[0]
        print("  bad frames", len(bad), bad[:40], "mod 8:", np.bincount(bad % 8, minlength=8))
        if len(bad) and B[k].ndim == 3:
            f = bad[0]
            e = np.abs(B[k][f] - A[k][f])
            print("  frame", f, "bad entries (row, col):", np.argwhere(e > 1e-10 * np.abs(A[k]).max())[:20].tolist())
