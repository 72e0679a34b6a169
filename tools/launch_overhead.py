"""Fixed cost of a timed GN run (kb_gn_prepare + kb_gn_launch) against its pass count, configs[3].

For n passes the wall time of kb_gn_launch is fitted as a + b n: a is the per-run cost outside the passes (graph
launch, the loop's end, the sync), b the pass time.  KB_LAUNCH_DIAG=1 makes the library print the host launch time,
the host total and the HIP-event span of each launch to stderr; KB_SCHED=spin|yield|block selects how the host waits.
Usage: python tools/launch_overhead.py [reps]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kalibr_amd import capi, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    p = synth.make_config(4)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.run_gn(5)
    out = {"sched": os.environ.get("KB_SCHED", "auto"), "runs": {}}
    # bench.py's order first (5 warm-up passes done, one prepared 20-pass launch), then the same launch repeated
    first = []
    for _ in range(4):
        g.gn_prepare(20)
        first.append(g.gn_launch(20))
    out["bench_order_20"] = first
    for n in (1, 2, 4, 8, 16, 20, 32, 64, 200):
        ws = []
        for _ in range(reps):
            g.gn_prepare(n)
            ws.append(g.gn_launch(n))
        out["runs"][n] = float(np.median(ws))
    ns = np.array(sorted(out["runs"]), dtype=float)
    w = np.array([out["runs"][int(n)] for n in ns])
    sel = ns <= 64
    b, a = np.polyfit(ns[sel], w[sel], 1)
    out["fit_fixed_ms"] = 1e3 * a
    out["fit_pass_ms"] = 1e3 * b
    print(json.dumps(out))


if __name__ == "__main__":
    main()
