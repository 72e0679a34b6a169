"""Diagnostic: timeline of the partitioned spline band solve (KSP_TS stamps, s_memrealtime 100 MHz) of one GN pass
at configs[4], diagnostic library only: KSP_PARTITION=1 python tools/diag_sp_ts.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_sp_diag_read_ts.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_int]
p = synth.make_spline_config()
g = capi.SplineSolver(p)
g.set_state(p.state_init)
buf = (C.c_longlong * 256)()
for rep in range(2):
    g.run_gn(3)
    assert L.kb_sp_diag_read_ts(g.h, buf, 256) == 0
    for lvl in range(3):
        t0 = buf[100 + lvl]
        st = [(buf[64 * lvl + 4 * j + k] - t0) / 100 for j in range(12) for k in range(4)]
        steps = []
        for j in range(12):
            s = st[4 * j:4 * j + 4]
            if s[0] < 0 or s[3] < s[0] or s[3] > 1e5:
                break
            steps.append(s)
        if not steps:
            continue
        print(f"rep {rep} level {lvl} chunk block 0: entry->first step {steps[0][0]:.2f} us")
        for j, s in enumerate(steps):
            nxt = steps[j + 1][0] if j + 1 < len(steps) else float('nan')
            print(f"  step {j}: chol {s[1] - s[0]:6.2f}  forward {s[2] - s[1]:6.2f}  update {s[3] - s[2]:6.2f}  "
                  f"-> next {nxt - s[3]:6.2f} us")
    t0 = buf[104]
    bs = [(buf[200 + 3 * j + k] - t0) / 100 for j in range(12) for k in range(3)]
    print(f"rep {rep} back level 0 block 0: " + "  ".join(
        f"[T {bs[3 * j + 1] - bs[3 * j]:.2f} solve {bs[3 * j + 2] - bs[3 * j + 1]:.2f}]" for j in range(6)))
