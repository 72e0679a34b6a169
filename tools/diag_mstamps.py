"""Diagnostic: timeline of k_marg (the marginal Jacobi SVD) through kb_solve_marginal, cold then warm calls, with the
shader clock over the launch (KB_TSM stamps, diagnostic library only): python tools/diag_mstamps.py [frames] [config]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_diag_read_ts.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_int]
nf = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # bit 1: rounds without work, bit 2: without rotations
p = synth.make_config(cfg, n_frames=nf)
g = capi.Solver(p)
g.set_state(p.state_init)
g.build()
buf = (C.c_longlong * 256)()
assert L.kb_diag_read_ts(g.h, buf, 256) == 0
assert L.kb_diag_set_flags(g.h, flags) == 0
names = ["entry", "G", "Omega + b", "warm start", "round-0 setup", "first test", "first round", "first sweep",
         "sweeps done", "sorted", "rank", "end"]
for rep in range(4 if flags == 0 else 1):
    ok, dx, info = g.solve_marginal()
    assert L.kb_diag_read_ts(g.h, buf, 256) == 0
    t0 = buf[200]
    line = ", ".join(f"{names[i]} {(buf[200 + i] - t0) / 100:.2f}" for i in range(12) if buf[200 + i] >= t0)
    clk = 100.0 * (buf[217] - buf[216]) / max(1, buf[211] - buf[200])
    print(f"C={p.cam_cols} call {rep} sweeps {info['sweeps']}: {line} us; shader clock {clk:.0f} MHz, flags {flags}", flush=True)
