"""Diagnostic: timeline of block 0 of the last pipelined build (k_buildp) inside GN passes (KB_TSB stamps,
s_memrealtime 100 MHz), diagnostic library only: python tools/diag_bstamps.py [config] [n_frames]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", os.environ.get("KB_STAMPS_LIB", "libkalibr_hip_stamps.so"))
L = capi.lib()
L.kb_diag_read_ts.argtypes = [C.c_void_p, C.POINTER(C.c_longlong), C.c_int]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
p = synth.make_config(cfg, n_frames=int(sys.argv[2])) if len(sys.argv) > 2 else synth.make_config(cfg)
g = capi.Solver(p)
g.set_state(p.state_init)
buf = (C.c_longlong * 256)()
assert L.kb_diag_read_ts(g.h, buf, 256) == 0  # allocates the stamp buffer
names = {0: "entry", 1: "prologue barrier", 63: "end"}
for it in range(8):
    names[2 + 2 * it] = f"view it{it} start"
    names[3 + 2 * it] = f"view it{it} SYRK done"
    names[20 + 4 * it] = f"  frame f{it} start"
    names[21 + 4 * it] = f"  frame f{it} sums done"
    names[22 + 4 * it] = f"  frame f{it} GJ done"
    names[23 + 4 * it] = f"  frame f{it} Schur done"
    names[52 + it] = f"view phase A of f{it} start"
for w, o in (("wave 0", 130), ("last view wave", 160)):
    for ps in range(2):
        names[o + 4 * ps] = f"  [{w}] f2 pass {ps} start"
        names[o + 4 * ps + 1] = f"  [{w}] f2 pass {ps} projected"
        names[o + 4 * ps + 2] = f"  [{w}] f2 pass {ps} u MFMAs done"
        names[o + 4 * ps + 3] = f"  [{w}] f2 pass {ps} v MFMAs done"
    names[o + 8] = f"  [{w}] f2 expansion done"
for w in range(4):
    names[176 + w] = f"    [fw{w}] f2 products done"
    names[184 + w] = f"    [fw{w}] f2 sums done"
names[180] = "    [fw0] f2 products met"
for w in range(8):
    names[144 + w] = f"      [view wave {w}] f3 SYRK done"
    names[152 + w] = f"      [view wave {w}] f3 expansion done"
names[140] = "    [fw0] f2 elimination entry"
names[141] = "    [fw0] f2 6x6 LDL^T done"
names[142] = "    [fw0] f2 column slot 0 solved+stored"
names[143] = "    [fw0] f2 column slot 1 solved+stored"
for rep in range(2):
    g.set_state(p.state_init)
    try:
        g.run_gn(16)
    except capi.KbError as e:  # diagnostic timing variants (wrong results) may fail the solves; the stamps stay
        print("(run_gn:", e, ")")
    assert L.kb_diag_read_ts(g.h, buf, 256) == 0
    t0 = buf[64]
    order = sorted((buf[64 + i] - t0, i) for i in names if buf[64 + i] >= t0 and buf[64 + i] - t0 < 10_000_000)
    print(f"k_buildp block 0 timeline (rep {rep}, us from entry):\n" +
          "\n".join(f"{names[i]:28s} {dt / 100:8.2f}" for dt, i in order))
