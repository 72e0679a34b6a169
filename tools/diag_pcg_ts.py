"""Diagnostic: per-phase timeline of the PCG solve (block 0, KB_PCG_TS stamps, s_memrealtime 100 MHz) at configs[3],
diagnostic library only: python tools/diag_pcg_ts.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_diag_read_ts.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_int]
p = synth.make_config(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
g = capi.Solver(p)
buf = (C.c_longlong * 256)()
assert L.kb_diag_read_ts(g.h, buf, 256) == 0  # allocates the stamp buffer
g.set_state(p.state_init)
g.build()
g.set_constant_conditioner(10.0)
g.set_linear_solver("pcg", tolerance=1e-24, max_iterations=12, absolute_tolerance=False)
for rep in range(2):
    g.pcg_init()
    g.solve()
    assert L.kb_diag_read_ts(g.h, buf, 256) == 0
    names = ["phase A (q_f, partials)", "barrier 1", "q_c column sums", "alpha, updates, M^-1 r, r.s", "barrier 2",
             "phase C + next A start"]
    for it in range(7):
        t = [buf[200 + 6 * it + k] for k in range(6)] + [buf[200 + 6 * (it + 1)]]
        print(f"rep {rep} it {it}: " + "  ".join(f"{names[k]} {(t[k + 1] - t[k]) / 100:.2f}" for k in range(6)))
