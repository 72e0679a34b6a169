"""Frame sharding over world_size 2 with the gloo backend on CPU: each rank builds the arrow system of
its frame shard (oracle), the camera-block partials [H_cc | g_c | sum Y^T Y | sum Y^T z | cost] are
all-reduced, every rank solves the camera block redundantly and back-substitutes its own frames.  The
result must equal the unsharded solve -- the exchange the GPU path performs over RCCL."""
import os
import socket

import numpy as np

from kalibr_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lam, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    full = synth.make_config(2, n_frames=12, p_view=0.8, seed_offset=11)
    F = full.n_frames
    f0, f1 = rank * F // world, (rank + 1) * F // world
    sh = full.frame_slice(f0, f1)
    o = O.Oracle(sh)
    A = o.arrow(sh.state_init)
    ok, S_part, b_part = o.schur_partial(A, lam, 0, sh.n_frames)
    C = sh.cam_cols
    packet = torch.from_numpy(np.concatenate([A["Hcc"].ravel(), A["gc"], S_part.ravel(), b_part, [A["cost"]]]))
    dist.all_reduce(packet)
    pk = packet.numpy()
    Hcc = pk[:C * C].reshape(C, C)
    gc = pk[C * C:C * C + C]
    S = Hcc + lam * lam * np.eye(C) - pk[C * C + C:2 * C * C + C].reshape(C, C)
    b = gc - pk[2 * C * C + C:2 * C * C + 2 * C]
    dxc = np.linalg.solve(S, b)
    # back-substitution of this rank's frames
    dxf = []
    for f in range(sh.n_frames):
        Aff = A["Hff"][f] + lam * lam * np.eye(6)
        dxf.append(np.linalg.solve(Aff, A["gf"][f] - A["Hfc"][f] @ dxc))
    out[rank] = (dxc, np.concatenate(dxf), float(pk[-1]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharded_solve():
    # torch is imported inside the tests only: a `pytest -m gpu` process never loads torch's bundled HIP runtime
    import torch.multiprocessing as mp
    from oracle import oracle as O
    mgr = mp.Manager()
    out = mgr.dict()
    lam = 2.0
    mp.spawn(_worker, args=(2, _free_port(), lam, out), nprocs=2, join=True)
    full = synth.make_config(2, n_frames=12, p_view=0.8, seed_offset=11)
    o = O.Oracle(full)
    A = o.arrow(full.state_init)
    ok, dx = o.solve(A, lam)
    assert ok
    C = full.cam_cols
    for r in range(2):
        assert np.abs(out[r][0] - dx[:C]).max() <= 1e-9 * np.abs(dx).max()
        assert abs(out[r][2] - A["cost"]) <= 1e-12 * A["cost"]
    dxf = np.concatenate([out[0][1], out[1][1]])
    assert np.abs(dxf - dx[C:]).max() <= 1e-9 * np.abs(dx).max()
