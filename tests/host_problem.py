"""Writes a synth.Problem in the binary layout read by tests/cpp/test_host.cpp (test helper)."""
import numpy as np

MAGIC = 0x4B424850


def write_problem(path, p):
    hdr = np.array([MAGIC, p.n_cams, p.n_frames, p.n_views, p.n_corners, p.target.shape[0], p.state_init.size],
                   dtype=np.int32)
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(np.ascontiguousarray(p.cam_model, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(p.target, dtype=np.float64).tobytes())
        f.write(np.ascontiguousarray(p.view_frame, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(p.view_cam, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(p.view_offset, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(p.corner_id, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(p.y, dtype=np.float64).tobytes())
        f.write(np.ascontiguousarray(p.state_init, dtype=np.float64).tobytes())
