"""Diagnostic: timeline of the cyclic reduction of one GN pass at configs[4] (KSP_TSB stamps, s_memrealtime 100 MHz):
k_sp_elim1 (block 1), every k_sp_level (block 1, or 0 when alone) and k_sp_back (block 0), phase by phase, and the
gap from one launch's stamped block end to the next launch's stamped block entry.  Diagnostic library only:
python tools/diag_sp_levels.py"""
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
assert L.kb_sp_diag_read_ts(g.h, buf, 256) == 0  # allocates the stamp buffer
for rep in range(3):
    for q in range(256):
        buf[q] = 0
    g.run_gn(2)
    assert L.kb_sp_diag_read_ts(g.h, buf, 256) == 0
    t0 = buf[112]
    rows = []
    if t0 > 0:
        rows.append(("elim1", [buf[112 + k] for k in range(4)], ["staged", "chol", "fwd+store"]))
    for lv in range(11):
        st = [buf[120 + 6 * lv + k] for k in range(5)]
        if st[0] >= t0 and st[4] >= st[0] and st[0] > 0:
            rows.append((f"level s={1 << lv}", st, ["staged", "products", "chol", "fwd+store"]))
    for lv in reversed(range(11)):
        st = [buf[190 + 4 * lv + k] for k in range(4)]
        if st[0] >= t0 and st[3] >= st[0] and st[0] > 0:
            rows.append((f"back s={1 << lv}", st, ["staged", "T (MFMA)", "solve+store"]))
    print(f"rep {rep}: cyclic reduction of the last GN pass, us from k_sp_elim1 entry")
    prev_end = None
    tot_gap = 0.0
    for name, st, ph in rows:
        gap = (st[0] - prev_end) / 100 if prev_end is not None else 0.0
        tot_gap += gap
        parts = "  ".join(f"{ph[k]} {(st[k + 1] - st[k]) / 100:5.2f}" for k in range(len(ph)))
        print(f"  {name:14s} at {(st[0] - t0) / 100:7.2f}  gap {gap:5.2f} | {parts} | body {(st[-1] - st[0]) / 100:5.2f}")
        prev_end = st[-1]
    if rows:
        print(f"  total {(rows[-1][1][-1] - t0) / 100:.2f} us, of which launch gaps {tot_gap:.2f} us")
    st = [buf[240 + k] for k in range(6)]
    if st[0] > 0:
        print("  products of the last level's stamped block, thread 0 (wave 0): per tile " +
              " ".join(f"{(st[k + 1] - st[k]) / 100:.2f}" for k in range(5) if st[k + 1] >= st[k]) + " us")
