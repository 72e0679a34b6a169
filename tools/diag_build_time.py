"""Diagnostic: the build kernel's average time inside GN passes (kb_build_kernel_stats, HIP events) for the library
named by KB_VARIANT_LIB (diagnostic timing variants produce wrong results; only the time is read):
python tools/diag_build_time.py [config] [n_frames]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
p = synth.make_config(cfg, n_frames=int(sys.argv[2])) if len(sys.argv) > 2 else synth.make_config(cfg)
g = capi.Solver(p)
g.set_state(p.state_init)
ts = []
for _ in range(3):
    ms, _, _ = g.build_kernel_stats()
    ts.append(ms * 1e3)
print(f"{os.environ.get('KB_VARIANT_LIB', 'main'):10s} build kernel {min(ts):7.2f} us (runs: {', '.join('%.2f' % t for t in ts)})")
