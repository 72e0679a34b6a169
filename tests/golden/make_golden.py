"""Generates the committed fixtures under tests/golden/.

* quaternion_special_values.json -- the axisAngle2quat known-answer pairs of the reference test
  Schweizer-Messer/sm_kinematics/test/QuaternionTests.cpp:44-59 (axis-angle / pi  ->  JPL quaternion),
  transcribed as data (sqrt(1/2) written out).
* config1_golden.npz -- configs[0] (1x pinhole-radtan, 50 frames) inputs and the oracle's outputs
  (cost, rhs, dx at lambda 10, final LM state): a regression pin for oracle and GPU path alike.
  The reference ships no calibration golden output, so this fixture is produced by
  the oracle, not by the reference.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from kalibr_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

s = float(np.sqrt(0.5))
PAIRS = [
    ([0, 0, 0], [0, 0, 0, 1]),
    ([6.366197723675814e-10, 0, 0], [1e-9, 0, 0, 1]),
    ([0.5, 0, 0], [s, 0, 0, s]),
    ([1, 0, 0], [1, 0, 0, 0]),
    ([1.5, 0, 0], [s, 0, 0, -s]),
    ([2, 0, 0], [0, 0, 0, -1]),
    ([-1, 0, 0], [-1, 0, 0, 0]),
    ([-2, 0, 0], [0, 0, 0, -1]),
    ([0, 0.5, 0], [0, s, 0, s]),
    ([0, 1, 0], [0, 1, 0, 0]),
    ([0, 1.5, 0], [0, s, 0, -s]),
    ([0, 2, 0], [0, 0, 0, -1]),
    ([0, -1, 0], [0, -1, 0, 0]),
    ([0, -2, 0], [0, 0, 0, -1]),
]


def main():
    with open(os.path.join(HERE, "quaternion_special_values.json"), "w") as f:
        json.dump({"source": "Schweizer-Messer/sm_kinematics/test/QuaternionTests.cpp:44-59",
                   "tolerance": "machine epsilon",
                   "pairs": [{"axis_angle_over_pi": a, "quat": q} for a, q in PAIRS]}, f, indent=1)
    p = synth.make_config(1)
    o = O.Oracle(p)
    A = o.arrow(p.state_init)
    ok, dx = o.solve(A, 10.0)
    assert ok
    st, r = o.optimize(p.state_init)
    np.savez_compressed(os.path.join(HERE, "config1_golden.npz"), y=p.y, state_init=p.state_init,
                        cost_init=o.cost(p.state_init), rhs_init=A["rhs"], dx_lambda10=dx, state_lm=st,
                        lm_iterations=r["iterations"])
    print("wrote fixtures; LM iterations", r["iterations"])


if __name__ == "__main__":
    main()
