"""GN iterations/s of the device loop on every BASELINE.json config at full size on one GPU (configs 1-4;
config 4 is the 8-GPU config run here unsharded), plus the build-kernel event timing.  Diagnostic tool;
bench.py is the contract line.  python tools/bench_configs.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kalibr_amd import capi, synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 3, 4]
frames = int(sys.argv[3]) if len(sys.argv) > 3 else None
for cfg in cfgs:
    p = synth.make_config(cfg, n_frames=frames) if frames else synth.make_config(cfg)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.optimize(policy="lm", lambda0=10.0, max_iterations=100, eps_x=1e-3, eps_j=1.0)  # GN from a converged state
    g.run_gn(10)
    t0 = time.perf_counter()
    g.run_gn(steps)
    wall = time.perf_counter() - t0
    ms, by, fl = g.build_kernel_stats()
    print(json.dumps({"config": cfg, "frames": p.n_frames, "cams": p.n_cams, "corners": p.n_corners,
                      "camera_block": p.cam_cols, "gn_it_per_s": steps / wall, "us_per_it": 1e6 * wall / steps,
                      "build_us": 1e3 * ms, "build_GBps": by / (ms * 1e-3) / 1e9}), flush=True)
