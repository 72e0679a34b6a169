"""Benchmark: Gauss-Newton iterations/s of the device-resident calibration loop (BASELINE.json metric).

One step = one full Optimizer2 pass with the Gauss-Newton policy: buildSystem (residuals, Jacobians,
arrow normal equations) + solveSystem (frame Schur complement, camera-block Cholesky, back
substitution) + applyStateUpdate + evaluateError, on synthetic AprilGrid data resident in HBM.

Default workload: configs[3], the north-star problem: 8-camera pinhole-radtan rig x 2000 frames, 6x5 AprilGrid
(120 corners), all views visible (1.83 M corners, C = 106 camera-block columns).  It fits one MI355X, so N=1 runs
the whole problem; N>1 shards its frames over the ranks (strong scaling: ceil(2000 / N) frames per rank,
"scaling": "strong"); the stage-1 camera-block rows are all-reduced and the per-frame step rows all-gathered over
RCCL once per pass.  value = GN iterations of the one problem / max-over-ranks wall time.

Other configs behind --config (BASELINE.json configs[i] is --config i+1):
  --config 2: configs[1], 2-camera stereo pinhole-radtan, 500 frames; N>1 is weak scaling (500 frames per rank).
  --config 3: configs[2], 4-camera 2x omni-radtan + 2x EUCM rig, 1000 frames, one GPU.
  --config 5: configs[4], 2-camera rig + IMU on a cubic B-spline pose trajectory, 1200 frames at 20 Hz, 200 Hz
              IMU, 50 knots/s; one step = one GN pass of the spline system.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Gauss-Newton iterations/sec (full J build + solve), N-cam×M-frame AprilGrid"
GN_FUSED = os.environ.get("KB_GN_FUSED", "1") != "0"  # the library's pass variant (kb_create reads the same)


def is_build_kernel(name):
    """The pass's build kernel as rocprofv3 names it: k_build<TW, GNF, MM> or the pipelined k_buildp<TT, GNF, MM>
    (rigs with one wave per camera), with GNF = the GN fused variant (MM = the rig's camera-model set)."""
    name = name.replace("(anonymous namespace)::", "")  # the per-model-set build TUs (kb_build_tu.hip)
    for pre in ("void kb::k_build<", "void kb::k_buildp<"):
        if name.startswith(pre) and name.endswith(">(kb::KbDev, int, int)"):
            args = name[len(pre):-len(">(kb::KbDev, int, int)")].split(", ")
            return len(args) >= 2 and args[1] == ("true" if GN_FUSED else "false")
    return False
FRAMES_PER_RANK = 500
WARM_MS = 30.0  # untimed device warm-up (pass time) before the timed region, beyond the --warmup passes
HBM_PEAK_GBS = 8000.0
# FP64 dense peak of one MI355X (vector FMA and f64 MFMA run at the same rate: 256 CU x 4 SIMD x 32 flop/clk x 2.4 GHz)
FP64_PEAK_TFS = 78.6


def pmc_traffic_bytes(match, config):
    """HBM bytes per launch of the kernel `match(name)` selects, from the newest committed PMC summary of the same
    bench workload (profiles/*/pmc_traffic*.json, written by tools/pmc_traffic.py from two separate rocprofv3 --pmc
    passes of `bench.py --config <config>`, gfx950 FETCH_SIZE correction applied), or None."""
    import glob
    paths = glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic*.json"))
    for path in sorted(paths, key=lambda p: (os.path.basename(os.path.dirname(p)), p), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
            ks = doc["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        if doc.get("bench_config", 2) != config:  # round-1 summaries predate the field: configs[1] (--config 2)
            continue
        for name, k in ks.items():
            if match(name):
                return k["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None


def host_cpu():
    """CPU model and core counts of the host the CPU baseline runs on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "nproc": avail, "os_cpu_count": os.cpu_count()}


def cpu_baseline(prob, seconds_budget=12.0, threads=None, label="configs[1] (full 500-frame problem", state=None):
    """Oracle (our C restatement of the reference CPU flow: threaded per-term evaluation into CCS J^T,
    serial rhs SpMV, J^T J, frame-first sparse Cholesky) timed on host cores, GN passes from `state` (default: the
    problem's initial state)."""
    from oracle import oracle as O
    o = O.Oracle(prob)
    threads = threads or min(16, os.cpu_count() or 1)
    st = prob.state_init if state is None else state
    t1 = o.time_gn(st, 1, threads)  # includes first-touch / warm-up
    n = max(2, min(200, int(seconds_budget / max(t1, 1e-4))))
    t = o.time_gn(st, n, threads)
    return {"value": n / t, "unit": "iterations/s", "cores": threads, "kind": "port", **host_cpu(),
            "sample": f"{n} GN iterations of {label}, {prob.n_corners} corners), "
                      f"oracle/kb_oracle.c kbo_time_gn (restatement, not CHOLMOD), {threads} threads"}


def all_host_cores():
    """every host CPU this process may run on (the strongest CPU configuration of the box)"""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_spline(prob, seconds_budget=15.0, threads=None):
    """configs[4] oracle (oracle/kb_oracle_spline.c: threaded term evaluation into the block-banded normal
    equations, band Cholesky + Schur onto the camera/IMU block) timed on host cores."""
    from oracle import oracle as O
    o = O.SplineOracle(prob)
    threads = threads or min(16, os.cpu_count() or 1)
    t1 = o.time_gn(prob.state_init, 1, threads)
    n = max(2, min(100, int(seconds_budget / max(t1, 1e-4))))
    t = o.time_gn(prob.state_init, n, threads)
    return {"value": n / t, "unit": "iterations/s", "cores": threads, "kind": "port", **host_cpu(),
            "sample": f"{n} GN iterations of configs[4] (full 1200-frame problem, {prob.n_corners} corners, "
                      f"{prob.n_imu} IMU samples), oracle/kb_oracle_spline.c kbo_sp_time_gn, {threads} threads"}


def main_spline(args):
    """configs[4] on one GPU (the spline path does not shard; BASELINE.json quotes it on 1 x MI355X)."""
    from kalibr_amd import build as B
    from kalibr_amd import capi, synth
    if not os.path.exists(B.OUT):
        B.build()
    p = synth.make_spline_config()
    g = capi.SplineSolver(p)
    g.set_state(p.state_init)
    g.run_gn(args.warmup)
    t0 = time.perf_counter()
    g.run_gn(args.steps)
    wall = time.perf_counter() - t0
    ks = g.kernel_stats(10)
    # roofline: the pass's largest single launch, the node assembly (k_sp_assemble); the pass as a whole is bound by
    # the cyclic reduction's dependent chain of small launches
    asm_ms, asm_bytes = g.assemble_stats(10)
    achieved = asm_bytes / (asm_ms * 1e-3) / 1e9
    pmc = pmc_traffic_bytes(lambda n: n.startswith("ksp::k_sp_assemble("), 5)
    value = args.steps / wall
    out = {
        "metric": METRIC, "value": value, "unit": "iterations/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * wall / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "configs[4]: 2-cam + IMU continuous-time B-spline calibration, 1200 frames, 1 GPU",
                   "frames": p.n_frames, "cameras": p.n_cams, "corners": p.n_corners, "imu_samples": p.n_imu,
                   "spline_coefficients": p.n_coeffs, "jacobian_cols": p.total_cols, "camera_block": p.cam_cols,
                   "policy": "gauss_newton", "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "kernel": "k_sp_assemble", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (pmc[0] / (asm_ms * 1e-3) / 1e9) if pmc else None,
                     "traffic_bytes_per_launch": pmc[0] if pmc else None, "traffic_source": pmc[1] if pmc else None,
                     "avg_ms": asm_ms, "algorithmic_bytes": asm_bytes,
                     "frames_kernel": {"avg_ms": ks["frames_ms"], "algorithmic_bytes": ks["frames_bytes"]},
                     # what bounds the pass: the block cyclic reduction (forward levels, Schur sums, the one-column
                     # back substitution) is a chain of dependent small launches, latency- not byte-bound
                     "reduction_chain": {"avg_ms": ks["reduction_ms"], "share_of_pass": ks["reduction_ms"] / ks["pass_ms"],
                                         "bound": "dependent launch chain (per-level latency)"}},
        "pass_breakdown_ms": {k: v for k, v in ks.items() if k.endswith("_ms")},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_spline(p)
        out["speedup_vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=4, choices=[2, 3, 4, 5],
                    help="BASELINE.json configs[i] is --config i+1 (default 4: the north-star 8-cam x 2000-frame rig)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", action="store_true",
                    help="N=1 through the multi-GPU path: rendezvous, a one-rank RCCL communicator, captured RCCL")
    ap.add_argument("--shard-of", type=int, default=0, metavar="K",
                    help="one GPU runs rank 0's shard of a K-way split (configs[3] / configs[2]: ceil(F / K) frames) "
                         "through a one-rank RCCL communicator: the per-rank pass of the K-GPU run (not a headline)")
    args = ap.parse_args()
    if args.config == 5:
        if args.gpus != 1:
            raise SystemExit("configs[4] (--config 5) runs on one GPU")
        return main_spline(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit("for --gpus N>1 launch with torch.distributed.run --nproc-per-node N")
    if args.shard_of and (world != 1 or args.config not in (3, 4)):
        raise SystemExit("--shard-of K: one process, configs[2] / configs[3] (--config 3 | 4)")

    from kalibr_amd import build as B
    from kalibr_amd import capi, rdzv, synth
    if not os.path.exists(B.OUT):
        B.build()

    # host rendezvous over stdlib TCP (RCCL id broadcast, barriers, max of the wall time): no torch in this process,
    # so the library's /opt/rocm HIP runtime and RCCL are the only ones loaded
    use_comm = world > 1 or args.comm or args.shard_of > 0
    grp = rdzv.TcpGroup(rank, world) if use_comm else None
    # the JSON line must be the only stdout output: native banners (RCCL prints its version at init) go to stderr
    sys.stdout.flush()
    stdout_fd = os.dup(1)
    os.dup2(2, 1)

    strong = args.config in (3, 4)
    if strong:  # configs[3] (configs[2]): one problem, frames split over the ranks
        full = synth.make_config(args.config)
        fpr = (full.n_frames + world - 1) // world
    else:  # configs[1] per rank: a 2-camera rig of 500 * world frames, 500 per rank
        full = synth.make_problem(synth.CONFIGS[2]["models"], FRAMES_PER_RANK * world, seed=20261015 + 2,
                                  name=synth.CONFIGS[2]["name"])
        fpr = FRAMES_PER_RANK
    if args.shard_of:  # rank 0's slice of a shard_of-way split, on this one GPU
        fpr = (full.n_frames + args.shard_of - 1) // args.shard_of
    shard = full.frame_slice(rank * fpr, min(full.n_frames, (rank + 1) * fpr)) if (world > 1 or args.shard_of) else full
    g = capi.Solver(shard, device=local)
    g.set_state(shard.state_init)
    if use_comm:  # --comm at N=1: the same launcher + RCCL path with a one-rank communicator
        uid = grp.broadcast(capi.comm_unique_id() if rank == 0 else b"")
        g.comm_init(uid, world, rank)
    gn_start = None
    if args.config == 3:
        # undamped GN diverges from configs[2]'s initial state (the omni xi / focal-length coupling; the oracle does
        # the same): the timed GN passes start from the Kalibr2-default LM solution instead (same pass cost)
        g.optimize(policy="lm", lambda0=10.0, max_iterations=200, eps_x=1e-3, eps_j=1.0)
        gn_start = g.get_state()

    g.run_gn(args.warmup)
    # device warm-up: the GPU's clocks ramp over the first milliseconds of sustained work (measured: a 20-pass run right
    # after 5 warm-up passes takes 2.74 ms, the same run repeated 2.63 ms, tools/launch_overhead.py), so untimed passes
    # run for >= WARM_MS of pass time; the count is the same on every rank (their collectives must match) and is
    # reported in the line
    t8 = g.run_gn(8)
    if grp:
        t8 = grp.max(t8)
    extra = 8 * max(1, int(np.ceil(WARM_MS * 1e-3 / max(t8, 1e-6))))
    if extra > 8:
        g.run_gn(extra - 8)
    graphed = g.gn_prepare(args.steps)  # loop start + every graph the timed passes launch, captured and uploaded
    if grp:
        grp.barrier()
    t0 = time.perf_counter()
    # the library's own clock around the launches and the stream sync that ends them (host launch + device passes +
    # the last step's back-substitution + the sync); the Python wall around the call is reported beside it
    sec = g.gn_launch(args.steps)
    py_wall = time.perf_counter() - t0
    wall = grp.max(sec) if grp else sec

    # dominant kernel (the build) timing with HIP events on the handle's stream, inside GN passes; the per-pass device
    # time of iterations 1..20 from HIP events at every pass start inside one captured graph (the
    # median of iterations 2..20, iteration 1 reported on its own)
    build_ms, bytes_per, flops_per = g.build_kernel_stats()
    kname = g.build_kernel_name()
    pass_ms, _ = g.gn_pass_times(20)
    pass_med = float(np.median(pass_ms[1:]))
    achieved = bytes_per / (build_ms * 1e-3) / 1e9
    useful_tfs = flops_per / (build_ms * 1e-3) / 1e12
    pmc = pmc_traffic_bytes(is_build_kernel, args.config) if (world == 1 and not args.shard_of) else None

    sys.stdout.flush()
    os.dup2(stdout_fd, 1)
    os.close(stdout_fd)
    if rank == 0:
        # weak: every rank iterates its own configs[1]-sized problem; strong: all ranks iterate one problem
        value = (1 if strong else world) * args.steps / wall
        workload = {4: "configs[3]: 8-cam pinhole-radtan rig, 2000 frames (sharded over the GPUs when N>1), 6x5 "
                       "AprilGrid, p_view=1",
                    3: "configs[2]: 4-cam 2x omni-radtan + 2x EUCM rig, 1000 frames (sharded over the GPUs when N>1), "
                       "6x5 AprilGrid, p_view=1",
                    2: "configs[1]: 2-cam stereo pinhole-radtan, 500 frames/GPU, 6x5 AprilGrid, p_view=1"}[args.config]
        if args.shard_of:
            workload = (f"rank 0's shard of a {args.shard_of}-way split of " + workload.split(":")[0] +
                        f" ({shard.n_frames} of {full.n_frames} frames, all-reduce over a one-rank RCCL communicator): "
                        "the per-rank pass of the multi-GPU run, not a headline line")
        out = {
            "metric": METRIC, "value": value, "unit": "iterations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * wall / args.steps, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload,
                       "frames_per_gpu": shard.n_frames, "cameras": full.n_cams, "corners_per_gpu": shard.n_corners,
                       "jacobian_cols": full.total_cols, "camera_block": full.cam_cols, "policy": "gauss_newton",
                       "parallelism": f"frame-sharded x{world}"},
            # the build kernel's arithmetic intensity (SURVEY 8(d) flops / algorithmic bytes: 1.69 GFLOP over 67.6 MB,
            # ~25 flop/B at configs[3]) is above the FP64 ridge (78.6 TF/s / 8 TB/s ~ 9.8 flop/B): its roofline is the
            # FP64 compute pipe, which the f64 MFMAs and the f64 VALU work of one SIMD share (their issue serialises,
            # DESIGN.md 3c), so "mfma" names the compute bound.  The HBM view is kept beside.
            "roofline": {"bound": "mfma", "kernel": kname, "achieved": useful_tfs, "peak": FP64_PEAK_TFS,
                         "unit": "TFLOP/s", "frac": useful_tfs / FP64_PEAK_TFS,
                         "traffic": pmc[0] if pmc else None, "traffic_source": pmc[1] if pmc else None,
                         "avg_ms": build_ms, "algorithmic_flops": flops_per, "algorithmic_bytes": bytes_per,
                         "arithmetic_intensity": flops_per / bytes_per,
                         "limiter": "the SIMD's FP64 pipe (f64 MFMA + f64 VALU issue of the view waves, serialised) "
                                    "and the per-frame dependency chain (SQ counters, DESIGN.md 3c, 6)",
                         "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": achieved / HBM_PEAK_GBS,
                                 "traffic_gbs": (pmc[0] / (build_ms * 1e-3) / 1e9) if pmc else None}},
            "per_pass_median_ms": pass_med, "first_pass_ms": float(pass_ms[0]),
            "per_pass_ms": [round(float(x), 5) for x in pass_ms],
            "useful_fp64_tflops": flops_per / (pass_med * 1e-3) / 1e12,
            "library_seconds": sec, "python_wall_seconds": py_wall,
            "device_warmup": {"warmup_passes": args.warmup, "clock_warmup_passes": extra, "min_ms": WARM_MS},
            "comm": {"rccl": bool(use_comm), "ranks": world, "rendezvous": "stdlib TCP" if use_comm else None,
                     "graphed": int(graphed)},
        }
        if not args.no_cpu_baseline:
            if strong:  # the whole problem on the host cores (configs[3]: ~0.2 s per iteration at 16 threads)
                lab = {4: "configs[3] (full 8-cam 2000-frame problem", 3: "configs[2] (full 4-cam 1000-frame problem"}
                # configs[2]: both sides time GN from the same (post-LM) state
                st = gn_start if (gn_start is not None and world == 1) else None
                out["cpu_baseline"] = cpu_baseline(full, seconds_budget=20.0, label=lab[args.config], state=st)
                allc = all_host_cores()
                if allc != out["cpu_baseline"]["cores"]:
                    out["cpu_baseline_all_cores"] = cpu_baseline(full, seconds_budget=20.0, label=lab[args.config],
                                                                 threads=allc, state=st)
            else:
                out["cpu_baseline"] = cpu_baseline(full if world == 1 else full.frame_slice(0, FRAMES_PER_RANK))
            out["speedup_vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
            if "cpu_baseline_all_cores" in out:
                out["speedup_vs_cpu_baseline_all_cores"] = value / out["cpu_baseline_all_cores"]["value"]
        print(json.dumps(out))
    if grp:
        grp.barrier()
        grp.close()


if __name__ == "__main__":
    main()
