"""Diagnostic: k_sp_assemble timeline of block 500 (KSP_TSB slots 241..252) and k_sp_frames timeline of block 300
(slots 256..270), s_memrealtime 100 MHz, over one GN pass at configs[4], diagnostic library only:
python tools/diag_sp_asm.py"""
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
buf = (C.c_longlong * 320)()
names = ["entry", "frames done", "records staged"] + [f"panel {j} {w}" for j in range(4) for w in ("built", "MFMA done")] + ["end"]
for rep in range(3):
    g.run_gn(2)
    assert L.kb_sp_diag_read_ts(g.h, buf, 320) == 0
    t0 = buf[241]
    print(f"rep {rep} k_sp_assemble block 500:")
    for k, nm in enumerate(names):
        v = (buf[241 + k] - t0) / 100
        if 0 <= v < 1e4:
            print(f"  {nm:20s} {v:8.2f} us")
    t0 = buf[256]
    fn = ["entry", "setup synced"] + [f"f{j} {w}" for j in range(2) for w in
                                       ("pose done", "SYRK done", "Hv synced", "P/Q synced", "FH written",
                                        "frame synced")] + ["summed Q synced"]
    fs = [256, 257] + [258 + 6 * j + k for j in range(2) for k in range(6)] + [271]
    print(f"rep {rep} k_sp_frames block 300:")
    for nm, sl in zip(fn + ["end"], fs + [270]):
        v = (buf[sl] - t0) / 100
        if 0 <= v < 1e4:
            print(f"  {nm:20s} {v:8.2f} us")
    t0 = buf[272]
    print(f"rep {rep} k_sp_bprep block 100 wave 0:")
    for nm, sl in (("entry", 272), ("L, T staged", 273), ("y formed", 274), ("37 columns solved", 275)):
        v = (buf[sl] - t0) / 100
        if 0 <= v < 1e4:
            print(f"  {nm:20s} {v:8.2f} us")
    print(f"  (block 100 entry {(buf[272] - buf[241]) / 100:.2f} us after k_sp_assemble block 500's entry)")
