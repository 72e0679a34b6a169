"""Diagnostic: cumulative duration of one GN-pass kernel run up to each of its stop points (KB_STAMP), timed
with HIP events over repeated launches.  Uses the separate diagnostic build kalibr_amd/libkalibr_hip_stamps.so
(never the product library): python tools/diag_stamps.py [config] [reps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

capi.LIB_PATH = os.path.join(ROOT, "kalibr_amd", "libkalibr_hip_stamps.so")
L = capi.lib()
L.kb_diag_phase_time.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
p = synth.make_config(cfg)
g = capi.Solver(p)
g.set_state(p.state_init)
KERNELS = {
    "k_build": (0, [(16, "staged"), (26, "pose"), (27, "proj"), (17, "corners+mfma"), (18, "bar"), (19, "viewsum"), (28, "G"), (29, "P,dH"), (20, "expand+frame"),
                    (21, "bar"), (23, "gauss-jordan"), (24, "acc"), (25, "part row"), (-1, "end")]),
    "k_build_gn": (3, [(14, "round2+step f0"), (16, "staged"), (26, "pose"), (27, "proj"), (17, "corners+mfma"), (18, "bar"), (19, "viewsum"), (28, "G"), (29, "P,dH"), (20, "expand+frame"),
                    (21, "bar"), (23, "gauss-jordan"), (24, "acc"), (25, "part row"), (-1, "end")]),
    "k_solve": (1, [(0, "entry"), (1, "stage"), (2, "cam expand"), (40, "diag 0"), (41, "p0 trsm+tile"), (42, "p0 diag 1 | trailing"), (45, "ldl rows"), (46, "ldl factor"), (3, "ldl"), (4, "solves"), (5, "stats+update"),
                    (-1, "end (chains)")]),
    "k_backsub": (2, [(30, "round1"), (31, "dx_f"), (32, "pose"), (33, "cost"), (-1, "end")]),
}
print(f"config {cfg}: cumulative kernel time (us) at each stop point, {reps} launches each")
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
only = sys.argv[4].split(",") if len(sys.argv) > 4 else None
for name, (which, stops) in KERNELS.items():
    if only and name not in only:
        continue
    prev = 0.0
    parts = []
    for stop, label in stops:
        t = C.c_double()
        assert L.kb_diag_phase_time(g.h, which, stop, reps, flags, C.byref(t)) == 0, L.kb_last_error()
        parts.append(f"{label} {t.value:.2f} (+{t.value - prev:.2f})")
        prev = t.value
    print(f"  {name:10s} " + " | ".join(parts))
