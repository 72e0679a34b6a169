"""Diagnostic: per-phase in-kernel timing (s_memrealtime, 100 MHz) of one GN pass, block 0 / thread 0.
Uses the separate stamp build kalibr_amd/libkalibr_hip_stamps.so (never the product library)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_diag_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
p = synth.make_config(cfg)
g = capi.Solver(p)
g.set_state(p.state_init)
st = np.zeros(64, dtype=np.uint64)
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if warm:
    g.run_gn(warm)
for rep in range(3):
    assert L.kb_diag_stamps(g.h, 3, st.ctypes.data, 64) == 0
    t = st.astype(np.int64)
    us = lambda a, b: (t[b] - t[a]) / 100.0  # noqa: E731
    print(f"config {cfg} rep {rep}")
    print("  k_build  init %.2f  mfma %.2f  bar %.2f  viewsum %.2f  expand+frame %.2f  bar %.2f  chol %.2f  Y %.2f  acc+bar %.2f  write %.2f" % (
        us(16, 17), us(17, 18), us(18, 19), us(19, 20), us(20, 21), us(21, 22), us(22, 23), us(23, 24), us(24, 25), 0.0))
    print("  k_solve  stageA %.2f  camexp %.2f  ldl %.2f  solves %.2f  stats+update %.2f" % (
        us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5)))
    print("  clock in k_solve: %.0f MHz" % ((t[41] - t[40]) / max(1, t[5] - t[0]) * 100.0))
