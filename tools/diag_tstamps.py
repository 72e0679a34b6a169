"""Diagnostic: timeline of one k_solve launch inside the captured GN passes (KB_TS stamps, s_memrealtime 100 MHz),
diagnostic library only: python tools/diag_tstamps.py [config]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_diag_read_ts.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_int]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
p = synth.make_config(cfg)
g = capi.Solver(p)
g.set_state(p.state_init)
buf = (C.c_longlong * 256)()
assert L.kb_diag_read_ts(g.h, buf, 256) == 0  # allocates the stamp buffer
names = {0: "entry", 1: "staged", 2: "T (+pass end)", 3: "H_cc blocks + grad", 4: "LDL^T", 5: "solves",
         6: "stats + DV update", 7: "chains", 8: "  backsolve done (wave 0)"}
names[47] = "  expansion: intrinsic blocks done (wave 0)"
names[48] = "  expansion: MFMA tiles done (wave 0)"
names[40] = "    p2: lookahead done"
names[41] = "    p2: rows loaded"
names[42] = "    p2: 16 steps done"
for i in range(10, 20):
    names[i] = f"  panel {i - 10}"
for t in range(7):
    names[240 + t] = f"    backsolve tile {t} start"
for q in range(7):
    names[20 + 2 * q] = f"    p{q} factor start (after its MFMA lookahead)"
    names[21 + 2 * q] = f"    p{q} factor end"
for rep in range(3):
    g.set_state(p.state_init)
    g.run_gn(16)
    assert L.kb_diag_read_ts(g.h, buf, 256) == 0
    t0 = buf[0]
    order = sorted((buf[i] - t0, i) for i in names if buf[i] >= t0 and buf[i] - t0 < 10_000_000)
    print(f"k_solve timeline (rep {rep}, us from entry):\n" +
          "\n".join(f"{names[i]:24s} {dt / 100:8.2f}" for dt, i in order))
    print('k_colimg stamps', [buf[i] - t0 for i in range(50, 55)])
    if buf[54] > buf[50]:
        print(f"k_colimg (first image block, thread 0): loads + staging {(buf[51] - buf[50]) / 100:.2f}, barrier "
              f"{(buf[52] - buf[51]) / 100:.2f}, T + barrier {(buf[53] - buf[52]) / 100:.2f}, entry {(buf[54] - buf[53]) / 100:.2f} us;"
              f" k_colimg end -> k_solve entry {(buf[0] - buf[54]) / 100:.2f} us")
    if buf[7] > buf[0]:  # shader clock over the kernel: s_memtime ticks / s_memrealtime (100 MHz) ticks
        print(f"shader clock during k_solve: {100.0 * (buf[61] - buf[60]) / (buf[7] - buf[0]):.0f} MHz")
