#!/usr/bin/env python3
"""Headline benchmark: Gauss-Newton iterations/s of DeformableMeshToImageFitter (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[1]): one 640x480 synthetic depth frame, a 1500-node warp graph
(50x30, node coverage 0.03, 4 anchors, block-diagonal solve), a 321x241 grid mesh (77,361 vertices, 153,600
triangles). The target depth is the mesh rendered under a smooth ground-truth motion; random-free, seed = rank.

A step = restore a stored mid-motion node state (half the ground-truth motion: non-identity R/t, a deformed mesh) by a
device copy + one full GN iteration through the general kernels (warp, rasterize, residuals, Jacobians, JtJ / Jt r, LM
block solve, Rodrigues update); --graph-steps (default 10, C2's GN iterations per frame) steps are captured as one
hipGraph and replayed as one launch, the way FitToImage replays its iteration loop (the timed step count is rounded up
to a whole number of launches). Every step does the same work, with nothing cached between steps. The reference's own
C2 trajectory cannot be timed as a 10-iteration loop: its block-diagonal GN (A17) raises potrf at iteration 2 on C2, on
the GPU and in the oracle alike (tests/test_gpu_parity.py TRAJECTORIES). --step frame (whole frame fits from the
identity warp, for configs whose trajectory survives, e.g. C2_ARAP) and --step identity (the first iteration of a frame)
are the alternatives.

N > 1: one process per GPU (torchrun), each fitting its own independent sequence (seed = rank) -- replicas, no
collective in the data path; the only collectives are the barrier, the max-over-ranks of the elapsed time and the
end-of-run all-gather of per-rank results. --replicas R: R independent sequences per process, each with
its own fitter, warp field and stream on the one device (seeds rank * R + r); a step launches every replica's iteration
on its stream; value = all sequences' iterations / the slowest rank's time.

Also reported: the dominant kernel's roofline (k_fit_pixels_fused: both pixel passes in one launch, timed in its real
context by nnrt_fitter_time_kernels -- graph-captured prefix sequences of iterations between HIP events on the fitter's
stream, so the figure matches the rocprofv3 kernel trace; every other kernel of the iteration under "kernels"), the once-per-frame setup time, and the CPU baseline (the oracle/ C++
restatement with the reference's binned rasterizer, OpenMP, on a bounded sample of the same workload, rank 0, N = 1: one
socket's physical cores with OMP_PROC_BIND=close and this process's CPU share, the faster as the value; also 1 thread).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM": 8 TB/s spec)
MFMA_F32_PEAK_TFS = 157.3   # dense f32-input MFMA peak (MI355X_MICROARCH.md MFMA table, "F32 (f32 in)")
DEFAULT_CONFIG = "C2"
ROOFLINE_KERNEL = "k_fit_pixels_fused"


# ---------------------------------------------------------------------------------------------------------------------
# distributed helpers (GPU-free; covered by tests/test_distributed_cpu.py with gloo)
# ---------------------------------------------------------------------------------------------------------------------
def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


MIN_WARM_S = 0.05   # seconds of untimed back-to-back GPU work before the timed region (clock ramp-up)


def timed_region(step, launches: int, per_launch: int, world: int, sync, dist_on=None, group=None) -> tuple:
    """The timed protocol: barrier + device sync, `launches` x step(per_launch), device sync, barrier. Returns (OR of
    the step return codes, this rank's elapsed seconds). dist_on: barriers on (default: world > 1); group: the process
    group the barriers run on (default: the world group)."""
    import torch.distributed as dist
    dist_on = world > 1 if dist_on is None else dist_on
    if dist_on:
        dist.barrier(group=group)
    sync()
    t0 = time.perf_counter()
    bad = 0
    for _ in range(launches):
        bad |= step(per_launch)
    sync()
    elapsed = time.perf_counter() - t0
    if dist_on:
        dist.barrier(group=group)
    return bad, elapsed


def exchange_per_rank(steps: int, elapsed: float, update_norm: float, device=None):
    """End-of-run all-gather of per-rank (iterations/s, seconds, final |update|); None at N = 1."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    mine = torch.tensor([steps / elapsed, elapsed, update_norm], dtype=torch.float64, device=device if device is not None else "cpu")
    got = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(got, mine)
    return [dict(rank=i, iters_per_s=float(g[0]), seconds=float(g[1]), update_norm=float(g[2])) for i, g in enumerate(got)]


def aggregate(steps: int, elapsed_s: float, world: int) -> dict:
    """Whole-job throughput: every rank runs `steps` iterations; the job takes the slowest rank's time."""
    return dict(value=world * steps / elapsed_s, ms_per_step=1000.0 * elapsed_s / steps)


# ---------------------------------------------------------------------------------------------------------------------
# algorithmic bytes: SURVEY.md 8(d) "Algorithmic bytes per GN iteration" (compulsory traffic at the reference's stage
# boundaries, fp32 values, int32 indices, 1-byte masks), mode ALL, no ARAP rows for the block-diagonal configs.
# P pixels, V vertices, F faces, N nodes, K anchors, E pixel-node associations (counted from the run).
# ---------------------------------------------------------------------------------------------------------------------
def stage_bytes(P: int, F: int, V: int, N: int, K: int, E: int) -> dict:
    return {
        "warp": V * (48 + 8 * K) + 60 * N,
        "ndc": F * (12 + 36 + 37),
        "raster": F * 72 + P * 24,
        "residual": P * 58 + F * 36,
        "warped_jacobians": V * (24 + 8 * K + 28 * K),
        "rasterized_jacobians": P * 244 + F * 72,
        "pixel_anchor_jacobians": P * 257 + P * 72 * K + 4 * E,
        "jtj_jtr": E * 28 + P * 5 + 168 * N,
        "solve": 144 * N + 48 * N,   # block-diagonal: n0 = N, no wing blocks, no dense corner
    }


# stages fused into each kernel of one GN iteration (block-diagonal configs)
KERNEL_STAGES = {
    "k_warp_mesh_quad": ("warp",),
    "k_raster_scatter_mesh": ("ndc", "raster"),
    # round 4: the warped-surface Jacobians (-wR(v-g), -wRn) are formed per association in pass 2, not stored by the warp
    "k_fit_pixels_fused": ("residual", "rasterized_jacobians", "warped_jacobians", "pixel_anchor_jacobians", "jtj_jtr"),
    "k_solve_update": ("solve",),
}


def arap_stage_bytes(N: int, n0: int, Ee: int) -> dict:
    """SURVEY.md 8(d) ARAP and arrowhead-solve rows (E_e edges, n0 stem nodes, n1 = N - n0 corner nodes)."""
    n1 = N - n0
    return {"arap": Ee * (8 + 20 + 144 + 12) + 288 * N, "solve": 144 * (n0 + 3 * Ee) + 3 * 4 * (6 * n1) ** 2 + 48 * N}


def corner_flops(n1: int, n_rhs: int = 1) -> float:
    """dense corner Cholesky + solve, (6 n1)^3 / 3 + 2 (6 n1)^2 (1 + n_rhs)."""
    m = 6 * n1
    return m ** 3 / 3.0 + 2.0 * m * m * (1 + n_rhs)


def kernel_bytes(kernel: str, sb: dict) -> int:
    return sum(sb[k] for k in KERNEL_STAGES[kernel])


def node_pass_compulsory_bytes(P: int, P_c: int, F: int, V: int, N: int, K: int) -> int:
    """What k_fit_pixels_fused itself must move: per pixel the raster key (8 B read + 8 B reset), the reference
    point (16 B) and the residual / mask / face outputs (9 B); per contributing pixel its 64-B Jacobian record (written
    and re-read by the same wave); each face record once (int4) and its vertices' warped position and normal (2 x
    float4); per vertex its anchors and weights (2 x 4 B x K) and warped-Jacobian rows (24 B x K); per node the fp64 accumulator
    row (27 x 8 B read-modify-write)."""
    return P * (16 + 16 + 9) + P_c * 64 * 2 + F * 16 + V * 32 + V * K * (4 + 4 + 24) + N * 27 * 8 * 2


def count_associations(pixel_faces, residual_mask, faces, anchors) -> int:
    """E = sum over pixels with a residual of the unique anchor nodes of the rasterized face's vertices."""
    import numpy as np
    sel = residual_mask.astype(bool) & (pixel_faces >= 0)
    f = pixel_faces[sel].astype(np.int64)
    nodes = anchors[faces[f]].reshape(len(f), -1)
    nodes = np.sort(nodes, axis=1)
    uniq = (nodes >= 0) & np.concatenate([np.ones((len(f), 1), bool), nodes[:, 1:] != nodes[:, :-1]], axis=1)
    return int(uniq.sum())


# ---------------------------------------------------------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default=DEFAULT_CONFIG, help="synthetic workload (dynamicfuion_python_amd.synthetic.CONFIGS)")
    ap.add_argument("--step", choices=("frame", "snapshot", "identity"), default="snapshot",
                    help="snapshot: one GN iteration per step from a mid-motion node state (general kernels); frame: "
                         "--graph-steps-iteration frame fits from the identity warp (FitToImage's loop; raises potrf on C2, "
                         "as the reference does); identity: the first iteration of a frame per step")
    ap.add_argument("--replicas", type=int, default=1, help="independent sequences per GPU, one stream each (C4's per-rank work)")
    ap.add_argument("--timed-steps", type=int, default=10, help="eager per-stage HIP-event timing steps (association counts, stage_ms)")
    ap.add_argument("--kernel-reps", type=int, default=20, help="iterations per graph of the per-kernel timing (nnrt_fitter_time_kernels)")
    ap.add_argument("--kernel-trials", type=int, default=9, help="interleaved trials of the per-kernel timing (median)")
    ap.add_argument("--graph-steps", type=int, default=10, help="steps per captured graph launch (C2: 10 GN iterations per frame)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU-baseline sample (loop-body seconds)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads for the CPU baseline (0: this process's CPU share, see cpu_threads_default)")
    ap.add_argument("--refine-ratio", type=float, default=None,
                    help="ARAP: upper end of the arrowhead solve's refinement window (default: the library's; inf: refine every solve)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-share-only", action="store_true", help="CPU baseline at this process's CPU share only (large configs: C3)")
    ap.add_argument("--cpu-no-warm", action="store_true", help="CPU baseline without the untimed first call (large configs: C3)")
    ap.add_argument("--traffic-file", default=None,
                    help="PMC-derived HBM bytes per launch of the roofline kernel (tools/pmc_traffic.py output)")
    return ap.parse_args(argv)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def render_target(sc, G, Rr):
    """Target depth = the canonical mesh warped by the ground-truth motion and rasterized (on the GPU, through the same
    C-ABI entry points the fitter exposes); pixels without geometry -> 0."""
    mesh = G.TriangleMesh(sc.points, sc.normals, sc.faces)
    a, w = G.compute_anchors_and_weights_euclidean_fixed_node_weight(sc.points, sc.nodes, 4, 0, sc.coverage)
    warped = G.warp_triangle_mesh(mesh, sc.nodes, sc.gt_rotations, sc.gt_translations, a, w)
    fndc, fm = Rr.get_mesh_ndc_face_vertices_and_clip_mask(warped, sc.K, (sc.H, sc.W), 0.0, 10.0)
    _, dep, _, _ = Rr.rasterize_ndc_triangles(fndc, fm, (sc.H, sc.W), 0.5, 1, -1, -1, True, False, True)
    d = dep[..., 0]
    return (d * (d > 0)).contiguous()


def load_traffic(path, workload: str):
    """PMC traffic file of this workload (tools/pmc_traffic.py): the given path, or else the newest
    profiles/r*_pmc_traffic*.json whose workload matches. Returns (the file's kernels dict, its path relative to the
    repo) or (None, None)."""
    paths = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json")), reverse=True)
    for p in paths:
        try:
            with open(p) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload and t.get("kernels"):
            return t["kernels"], os.path.relpath(p, ROOT)
    return None, None


def host_cpu():
    """CPU model, sockets, physical cores per socket and logical CPUs of this host (/proc/cpuinfo; os.cpu_count() is the
    whole machine)."""
    model, sockets, cores = None, set(), None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    sockets.add(v)
                elif k == "cpu cores" and cores is None and v.isdigit():
                    cores = int(v)
    except OSError:
        pass
    return dict(model=model, sockets=len(sockets) or None, cores_per_socket=cores, logical_cpus=os.cpu_count())


def cpu_baseline(sc, depth_host, share_threads: int, budget_s: float, step: str, iterations: int, R0=None, t0=None,
                 single_thread_s: float = 4.0, share_only: bool = False, warm: bool = True):
    """The oracle (C++/OpenMP restatement of the reference CPU path; test infrastructure, used here only as the
    reported baseline) running the same steps as the GPU: `step` = "frame" -> `iterations`-iteration FitToImage loops from
    the identity warp; "snapshot" -> one GN iteration from the node state (R0, t0); "identity" -> one GN iteration from
    the identity warp. Timed = loop body S1-S12 (DeformableMeshToImageFitter.cpp:111-275), once-per-frame setup
    excluded, as in the GPU step; the rasterizer is the reference's binned one (GridBinNdcTriangles + per-pixel bin loop,
    RasterizeNdcTrianglesImpl.h:187-391), not the oracle's fast K = 1 path. Threads: the physical
    cores of one socket with OMP_PROC_BIND=close and this process's CPU share (16 on the GPU box) -- the faster of the two is
    the value, both are listed under "samples" -- and 1. share_only (large configs, e.g. C3, whose binned raster takes
    minutes per iteration on one thread): the process's CPU share only; warm = False: no untimed first call."""
    os.environ.setdefault("OMP_PROC_BIND", "close")   # read when the oracle's OpenMP runtime initialises (first load)
    os.environ.setdefault("OMP_PLACES", "cores")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    host = host_cpu()
    socket = min(host["cores_per_socket"] or share_threads, len(os.sched_getaffinity(0)))
    refp, refm = O.unproject(depth_host, sc.K, 1.0, 10.0)
    # a progress line every 60 s while the samples run (a single-thread C3 iteration takes minutes)
    import threading
    done = threading.Event()

    def heartbeat():
        t_start = time.perf_counter()
        while not done.wait(60.0):
            log(f"CPU baseline still running ({time.perf_counter() - t_start:.0f} s)")

    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        _cpu_sample.warmed = not warm
        _cpu_sample.no_warm_call = not warm
        if share_only:
            runs = [_cpu_sample(O, sc, refp, refm, share_threads, budget_s, step, iterations, R0, t0)]
            one = None
        else:
            runs = [_cpu_sample(O, sc, refp, refm, socket, budget_s, step, iterations, R0, t0)]
            if share_threads != socket:
                runs.append(_cpu_sample(O, sc, refp, refm, share_threads, budget_s, step, iterations, R0, t0))
            one = _cpu_sample(O, sc, refp, refm, 1, single_thread_s, step, iterations, R0, t0, min_timed=1)
    finally:
        done.set()
    # value: the faster multi-thread sample (the binned raster does not scale to a whole socket on a shared host)
    best = max(runs, key=lambda r: r["value"] or 0.0)
    res = dict(best)
    res["samples"] = [dict(value=r["value"], cores=r["cores"], ms_per_solve=r["ms_per_solve"], sample=r["sample"]) for r in runs]
    res["single_thread"] = (dict(value=one["value"], unit=one["unit"], cores=1, ms_per_solve=one["ms_per_solve"], sample=one["sample"])
                            if one else None)
    res["host"] = host
    res["omp_proc_bind"] = os.environ.get("OMP_PROC_BIND")
    return res


def _cpu_sample(O, sc, refp, refm, threads: int, budget_s: float, step: str, iterations: int, R0, t0, min_timed: int = 1):
    """Timed oracle fits until `budget_s` of loop body has accumulated (at least `min_timed` timed calls); a first
    untimed call warms caches / page-ins unless the process has already run one (the single-thread sample follows the
    multi-thread ones on the same data)."""
    O.set_num_threads(threads)
    N = len(sc.nodes)
    if step != "snapshot" or R0 is None:
        R0 = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1))
        t0 = np.zeros((N, 3), np.float32)
    per_call = iterations if step == "frame" else 1
    h = sc.hierarchy
    hk = {}
    nodes = sc.nodes
    if h:   # the fit runs in virtual node order (the synthetic scenes are pre-sorted: identity permutation)
        nodes = sc.nodes[h["virtual_indices"]]
        hk = dict(edges=h["edges"], edge_layers=h["edge_layers"], radii=h["radii"], first_layer_count=int(h["layer_counts"][0]))
    body = solve = 0.0
    iters = calls = timed = 0
    warm = getattr(_cpu_sample, "warmed", False) and (threads == 1 or getattr(_cpu_sample, "no_warm_call", False))
    wall0 = time.perf_counter()
    while (body < budget_s and time.perf_counter() - wall0 < 3 * budget_s) or timed < min_timed:
        _, _, dg = O.fit(nodes=nodes, rotations=R0, translations=t0, mesh_points=sc.points, mesh_normals=sc.normals, faces=sc.faces,
                         ref_points=refp, ref_mask=refm, H=sc.H, W=sc.W, K=sc.K, max_iterations=per_call, lm_factor=0.001,
                         coverage=sc.coverage, fast_raster=False, **hk)
        if calls > 0 or warm:
            body += dg["stage_seconds"][7]
            solve += dg["stage_seconds"][5]
            iters += per_call
            timed += 1
        calls += 1
    _cpu_sample.warmed = True
    what = {"frame": f"{iters // per_call} {per_call}-iteration frame fits from the identity warp",
            "snapshot": f"{iters} single GN iterations from the mid-motion node state",
            "identity": f"{iters} single GN iterations from the identity warp"}[step]
    return dict(value=iters / body if body > 0 else None, unit="GN iters/s", cores=O.num_threads(), kind="port",
                ms_per_solve=1000.0 * solve / max(iters, 1),
                sample=f"{sc.name}: {what} (loop body timed, setup excluded), oracle/ C++ OpenMP restatement, binned raster "
                       f"(the reference's GridBin + per-pixel bin loop)")


def cpu_threads_default() -> int:
    """The CPU share of this process: its scheduler affinity, capped by OMP_NUM_THREADS when the environment sets it
    (the GPU box sets 16 = one GPU's share of the host, while the affinity mask spans the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff


def check_rank_devices(local_rank: int, world: int, backend: str, device_count: int) -> None:
    """RCCL replicas need one GPU per local rank: fail fast, before any device is touched, instead of mapping two ranks
    onto one device (the gloo rehearsal backend shares devices on purpose)."""
    if backend == "gloo":
        return
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if local_rank >= device_count or local_world > device_count:
        raise SystemExit(f"bench.py: {local_world} local rank(s) on the {backend} backend need one GPU each, but {device_count} "
                         f"device(s) are visible (local rank {local_rank}); launch with --nproc-per-node <= {device_count} "
                         f"(or NNRT_BENCH_BACKEND=gloo for a shared-device rehearsal)")


def main(argv=None):
    args = parse_args(argv)
    rank, local_rank, world = dist_env()
    import torch
    import torch.distributed as dist
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (the MI355X path has no CPU fallback)")
    # NNRT_BENCH_BACKEND=gloo (rehearsal only): several ranks sharing the GPUs of a smaller box (device = local rank
    # modulo the visible devices), their collectives on gloo over host tensors; the default is RCCL, one GPU per rank
    backend = os.environ.get("NNRT_BENCH_BACKEND", "nccl")
    check_rank_devices(local_rank, world, backend, torch.cuda.device_count())
    local_dev = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    # NNRT_BENCH_DIST_ONE_RANK=1: the process group, barriers and collectives also at WORLD_SIZE 1 (a one-GPU box can
    # run the RCCL branch itself: torch.distributed.run --nproc-per-node 1)
    use_dist = world > 1 or os.environ.get("NNRT_BENCH_DIST_ONE_RANK") == "1"
    ctrl_group = None
    if use_dist:
        if backend == "gloo":
            dist.init_process_group(backend="gloo")
        else:
            # RCCL carries the collectives over device tensors (max-over-ranks, the per-rank all-gather). Its communicator
            # is created lazily by the first of them, AFTER the timed region: with the communicator up (and its proxy
            # thread) a one-rank RCCL line ran 0.6-3.7 % slower than the plain line, the graph replay itself 0.8 %
            # (round 6, tools/dev/rccl_overhead.sh; a gloo process group cost 0.5 %). The timed region's two barriers run
            # on a gloo group of the same ranks -- no data-path collective exists to overlap (replicas).
            dist.init_process_group(backend="nccl")
            ctrl_group = dist.new_group(backend="gloo")
    coll_dev = "cpu" if backend == "gloo" else dev

    from dynamicfuion_python_amd import _native as NV
    from dynamicfuion_python_amd import synthetic as S
    from dynamicfuion_python_amd.nnrt import alignment as A
    from dynamicfuion_python_amd.nnrt import geometry as G
    from dynamicfuion_python_amd.nnrt import rendering as Rr

    R = max(1, args.replicas)
    sc = S.make_scene(args.config, seed=rank * R, hierarchy_builder=S.native_hierarchy_builder)
    arap = sc.layer_count > 1
    P, F, V, Nn = sc.H * sc.W, len(sc.faces), len(sc.points), len(sc.nodes)
    solve_kind = f"{sc.layer_count}-layer ARAP arrowhead LM solve" if arap else "block-diagonal LM solve"
    step_desc = {"frame": f"FitToImage loop: {min(args.graph_steps, args.steps)}-iteration frame fits from the identity warp, "
                          f"1 GN iteration per step",
                 "snapshot": "1 GN iteration per step from a mid-motion node state (half the ground-truth motion)",
                 "identity": "1 GN iteration per step from the identity warp"}[args.step]
    workload = f"{sc.name}: {sc.W}x{sc.H} depth, {Nn}-node graph, {V}-vertex/{F}-triangle mesh, {solve_kind}, {step_desc}"
    if R > 1:
        workload += f"; {R} independent sequences per GPU on {R} streams"

    log(f"rank {rank}/{world} on {torch.cuda.get_device_name(dev)}: {workload}")
    lib = NV.lib()
    per_launch = max(1, min(args.graph_steps, args.steps))

    # Step kinds (every one runs the real GN iteration kernels of FitToImage's loop body, :111-275):
    #   frame    -- one launch = one whole frame fit of --graph-steps iterations (C2: the 10-iteration FitToImage loop)
    #               from the identity warp: the motion is restored once per frame, iterations 2..10 run the general
    #               (non-identity R/t) kernels on the deformed mesh; one hipGraph per frame.
    #   snapshot -- every step restores a mid-motion node state (half the ground-truth motion, sc.partial_motion(0.5))
    #               and runs one GN iteration through the general kernels (non-identity R/t, deformed mesh; constant
    #               work per step). The reference's own C2 trajectory cannot serve: its block-diagonal GN (A17) raises
    #               potrf at iteration 2 on C2 (tests/test_gpu_parity.py TRAJECTORIES), so a 10-iteration C2 frame fit
    #               does not exist in the reference either.
    #   identity -- every step is the first GN iteration from the identity warp (identity-specialised warp / update).
    def make_replica(scene, stream):
        depth_r = render_target(scene, G, Rr)
        wf_r = G.HierarchicalGraphWarpField(scene.nodes, scene.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE,
                                            scene.layer_count)
        ft_r = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=A.GRAPH_ALWAYS)
        if args.refine_ratio is not None:
            ft_r.set_refine_ratio(args.refine_ratio)
        mesh_r = G.TriangleMesh(scene.points, scene.normals, scene.faces)
        if args.step == "snapshot":
            R_mid, t_mid = scene.partial_motion(0.5)
            wf_r.set_node_rotations(R_mid)
            wf_r.set_node_translations(t_mid)
        ft_r.prepare(wf_r, mesh_r, depth_r, None, scene.K, stream=stream)
        ft_r.snapshot_motion(wf_r, stream=stream)   # the state every step (snapshot) or every frame (frame) restarts from
        return dict(sc=scene, depth=depth_r, wf=wf_r, ft=ft_r, mesh=mesh_r, stream=stream, s_ptr=NV.stream_ptr(stream))

    reps = [make_replica(sc, torch.cuda.current_stream(dev))]
    for r in range(1, R):
        reps.append(make_replica(S.make_scene(args.config, seed=rank * R + r, hierarchy_builder=S.native_hierarchy_builder),
                                 torch.cuda.Stream(dev)))
    torch.cuda.synchronize(dev)
    depth, wf, ft, mesh = reps[0]["depth"], reps[0]["wf"], reps[0]["ft"], reps[0]["mesh"]
    R1, t1 = wf.get_node_rotations(True), wf.get_node_translations(True)   # (virtual order) for the CPU baseline

    def step_one(rp, n):
        if args.step == "frame":
            return lib.nnrt_fitter_fit_from_snapshot(rp["ft"]._h, rp["wf"].handle, n, rp["s_ptr"])
        if args.step == "snapshot":
            return lib.nnrt_fitter_iterate_from_snapshot(rp["ft"]._h, rp["wf"].handle, 0, n, rp["s_ptr"])
        return lib.nnrt_fitter_iterate_from_identity(rp["ft"]._h, rp["wf"].handle, 0, n, rp["s_ptr"])

    def step(n):   # every replica's iterations, each on its own stream
        bad = 0
        for rp in reps:
            bad |= step_one(rp, n)
        return bad

    # warmup (graphs are captured on first use: use_hip_graph = 2): the requested W steps, and at least MIN_WARM_S of
    # back-to-back GPU work -- the GPU's clocks ramp up from idle: a 20-step timed region after 10 warmup steps measured
    # 14,300 GN it/s at C2, after 200 warmup steps 15,500 (round-3 A/B r3_warm, in git history)
    for _ in range(max(1, args.warmup // per_launch)):
        if step(per_launch):
            NV.check(1)
    torch.cuda.synchronize(dev)
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < MIN_WARM_S:
        for _ in range(4):
            if step(per_launch):
                NV.check(1)
        torch.cuda.synchronize(dev)
    for rp in reps:
        rp["ft"].check(stream=rp["stream"])

    launches = -(-args.steps // per_launch)
    args.steps = launches * per_launch   # whole graphs only: the timed step count is rounded up to a multiple
    bad, elapsed = timed_region(step, launches, per_launch, world, lambda: torch.cuda.synchronize(dev), dist_on=use_dist, group=ctrl_group)
    if bad:
        NV.check(bad)
    per_replica = []
    for r, rp in enumerate(reps):
        rp["ft"].check(stream=rp["stream"])   # solver failure flag (potrf) -> raises
        final_t = rp["wf"].get_node_translations()
        if not np.isfinite(final_t).all():
            raise SystemExit(f"non-finite node motion after the timed steps (replica {r})")
        per_replica.append(dict(replica=r, seed=rank * R + r,
                                update_norm=float(np.linalg.norm(rp["ft"].diagnostics(stream=rp["stream"])["updates"]))))
    elapsed_max = max_over_ranks(elapsed, coll_dev)
    agg = aggregate(args.steps * R, elapsed_max, world)
    agg["ms_per_step"] = 1000.0 * elapsed_max / args.steps   # one step = every replica's iteration

    # per-kernel device time, each kernel in its real context: prefix sequences of graph-captured iterations from the
    # snapshot state, replayed between HIP events on the fitter's stream (nnrt_fitter_time_kernels); these are the
    # numbers the rocprofv3 kernel trace of the same command reports (profiles/r04_bench_kernel_stats.csv)
    ft.restore_motion(wf)
    ft.snapshot_motion(wf)   # "frame": the frame's start state; otherwise the restored mid-motion state
    ktimes = ft.time_kernels(wf, reps=args.kernel_reps, trials=args.kernel_trials)
    ft.restore_motion(wf)
    # kernel times are differences of medians: a short kernel can come out <= 0. Such a difference is not a
    # time: it is reported as None and no fraction is priced on it (the roofline falls back to the whole iteration's time,
    # a conservative lower bound on the kernel's rate)
    ktimes = {k: (v if v > 0 else None) for k, v in ktimes.items()}
    # per-stage eager event timing over the same iterations as the timed steps (a frame's iterations for "frame", the
    # restored iteration otherwise), one iteration at a time so that each iteration's algorithmic bytes use its own
    # association count E (the stage times themselves carry launch / event overhead and are reported as stage_ms only)
    anchors, _ = ft.anchors(V, 4)
    stages = {k: 0.0 for k in A.TIMED_STAGES}
    samples = []   # (E, contributing pixels) per timed iteration
    while len(samples) < args.timed_steps:
        if args.step == "identity":
            wf.reset_motion()
            its = [0]
        elif args.step == "snapshot":
            ft.restore_motion(wf)
            its = [0]
        else:
            ft.restore_motion(wf)
            its = list(range(per_launch))
        for it in its:
            r = ft.iterate_timed(wf, it, 1)
            for k in stages:
                stages[k] += r[k]
            dg = ft.diagnostics()
            if not (np.isfinite(dg["updates"]).all() and np.abs(dg["updates"]).max() > 0):
                raise SystemExit(f"non-finite or empty GN update at iteration {it + 1} of the timed configuration")
            samples.append((count_associations(dg["pixel_faces"], dg["residual_mask"], sc.faces, anchors), int(dg["residual_mask"].sum())))
    for k in stages:
        stages[k] /= len(samples)
    ft.check()

    E = int(round(np.mean([e for e, _ in samples])))
    P_c = int(round(np.mean([p for _, p in samples])))
    sb = stage_bytes(P, F, V, Nn, 4, E)
    kernels = {}
    for kname in KERNEL_STAGES:
        if arap and kname == "k_solve_update":
            continue
        kb = kernel_bytes(kname, sb)
        ms = ktimes[kname if kname != "k_solve_update" else "solve"]
        kernels[kname] = dict(ms=round(ms, 5) if ms else None, algorithmic_bytes=kb, frac=kb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ms else None)
    corner = None
    if arap:
        counts = wf.get_layer_node_counts()
        n0 = int(counts[0])
        Ee = len(wf.get_edges())
        ab = arap_stage_bytes(Nn, n0, Ee)
        sb.update(ab)
        # the ARAP edge terms run in extra workgroups of the fused pixel launch: charged to it
        kp = kernels[ROOFLINE_KERNEL]
        kp["algorithmic_bytes"] += ab["arap"]
        kp["frac"] = kp["algorithmic_bytes"] / (kp["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS if kp["ms"] else None
        kernels["k_arap_edges"] = dict(ms=None, fused_into=ROOFLINE_KERNEL, algorithmic_bytes=ab["arap"], frac=None)
        fl = corner_flops(Nn - n0)
        solve_ms = ktimes["solve"] or ktimes["iteration"]
        # headline: the MFMA flops the tile-sparse plan executes per solve (update-term tile products + rank-32
        # products) over the whole solve stage's time; the reference's dense-corner count of
        # SURVEY.md 8(d), about ten times that work, is kept beside it under "dense"
        work = ft.corner_work()
        xfl = float(work["mfma_flops"])
        corner = dict(kernel="arrowhead solve stage (stem Schur update + tile-sparse corner Cholesky + substitutions + update)",
                      bound="mfma", achieved=xfl / (solve_ms * 1e-3) / 1e12, peak=MFMA_F32_PEAK_TFS, unit="TFLOP/s",
                      frac=xfl / (solve_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS, traffic=None, flops=xfl, kernel_ms=solve_ms,
                      kernel_ms_source="solve" if ktimes["solve"] else "iteration (the solve's prefix difference was not positive)",
                      n0=n0, n1=Nn - n0, corner_size=6 * (Nn - n0), edges=Ee,
                      flops_formula="MFMA flops of the executed tile-sparse plan per solve (nnrt_fitter_corner_work: "
                                    "update-term tile products + rank-32 products), over the solve stage's time",
                      dense=dict(flops=fl, achieved=fl / (solve_ms * 1e-3) / 1e12, frac=fl / (solve_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
                                 flops_formula="SURVEY.md 8(d): (6 n1)^3 / 3 + 2 (6 n1)^2 (1 + n_rhs), n_rhs = 1 (the reference's "
                                               "dense corner)"),
                      plan=ft.corner_info(), refinement=ft.refine_info(), executed=work)
    kbytes = kernels[ROOFLINE_KERNEL]["algorithmic_bytes"]
    k_ms = ktimes[ROOFLINE_KERNEL] or ktimes["iteration"]
    achieved = kbytes / (k_ms * 1e-3) / 1e9
    it_bytes = sum(sb.values())
    pmc, traffic_src = load_traffic(args.traffic_file, workload)
    traffic = (pmc or {}).get(ROOFLINE_KERNEL, {}).get("hbm_bytes_per_launch")
    if pmc:   # every kernel the PMC passes measured: its HBM bytes per launch and that traffic's fraction of peak
        for kname, kd in kernels.items():
            pk = pmc.get(kname) or pmc.get(kname + "_lanes")
            if pk and kd.get("ms"):
                kd["traffic"] = pk["hbm_bytes_per_launch"]
                kd["traffic_frac"] = pk["hbm_bytes_per_launch"] / (kd["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS

    # once-per-frame setup (DeformableMeshToImageFitter.cpp:96-106: anchors, reference point cloud, buffers), timed
    # on a repeated prepare() of the same frame
    torch.cuda.synchronize(dev)
    t_setup = time.perf_counter()
    ft.prepare(wf, mesh, depth, None, sc.K)
    torch.cuda.synchronize(dev)
    setup_ms = (time.perf_counter() - t_setup) * 1000.0

    # end-of-run exchange of per-rank results: iterations/s, seconds, final |update|
    per_rank = exchange_per_rank(args.steps * R, elapsed, float(np.linalg.norm(dg["updates"])), coll_dev)

    out = {
        "metric": "GN iters/sec (640x480, 1.5k-node graph)" if args.config == "C2" else f"GN iters/sec ({args.config})",
        "value": agg["value"],
        "unit": "GN iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": agg["ms_per_step"],
        "ms_per_solve": ktimes["solve"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (smooth grid mesh + GT node motion rendered to depth; seed = rank)",
        "config": {"workload": workload, "config": args.config, "frame": [sc.H, sc.W], "nodes": Nn, "vertices": V, "triangles": F,
                   "anchors": 4, "iteration_mode": "ALL", "lm_damping": 0.001, "hip_graph": True, "steps_per_graph": per_launch, "step": args.step,
                   "parallelism": f"replicas{world * R}" if world * R > 1 else "single", "replicas_per_gpu": R,
                   **({"collectives": "rccl (max-over-ranks, per-rank all-gather; timed-region barriers on a gloo group)" if backend == "nccl" else f"{backend} (rehearsal: {world} ranks on "
                                                                       f"{torch.cuda.device_count()} visible GPU(s))"}
                      if use_dist else {})},
        "setup_ms": round(setup_ms, 3),
        "kernel_ms": {k: (round(v, 5) if v else None) for k, v in ktimes.items()},
        "kernel_ms_note": f"nnrt_fitter_time_kernels: per-iteration device time of each kernel in its real context, by differences "
                          f"of graph-captured prefix sequences ({args.kernel_reps} iterations per graph, median of {args.kernel_trials} "
                          f"interleaved trials); 'solve' = {'the arrowhead chain' if arap else 'k_solve_update'}; kernels.*.ms and "
                          f"roofline.kernel_ms are these",
        "stage_ms": {k: round(v, 5) for k, v in stages.items()},
        "stage_note": "single eager launches between HIP events (include launch / event overhead; not used for any fraction); "
                      "pixel_jacobians is back-to-back event overhead only: both pixel passes run in the one launch node_reduce "
                      "times (k_fit_pixels_fused)"
                      + ("; so is arap: the ARAP edge terms run in extra workgroups of that launch" if arap else ""),
        "roofline": {"kernel": ROOFLINE_KERNEL, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "algorithmic_bytes": kbytes, "kernel_ms": k_ms,
                     "bytes_formula": "SURVEY.md 8(d): residuals + rasterized Jacobians + warped-surface Jacobians (formed in pass 2 since "
                                      "round 4) + pixel-anchor Jacobians + JtJ/Jtr rows (P*58 + F*36 + P*244 + F*72 + V*(24+36K) + P*257 "
                                      "+ P*72K + 4E + E*28 + P*5 + 168N)"
                                      + (" + ARAP edge rows (E_e*184 + 288N, fused into the launch)" if arap else ""),
                     "associations_E": E, "contributing_pixels": P_c,
                     "associations_note": "E and contributing pixels averaged over the timed iterations", "traffic_source": traffic_src,
                     "compulsory_bytes": node_pass_compulsory_bytes(P, P_c, F, V, Nn, 4),
                     # the same launch against the bytes it really moves (PMC) and must move (compulsory): frac prices the
                     # reference's stage-boundary tensors, which the fused launch never materialises
                     "traffic_frac": (traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                     "compulsory_frac": node_pass_compulsory_bytes(P, P_c, F, V, Nn, 4) / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "iteration_algorithmic_bytes": it_bytes,
                     "iteration_frac": it_bytes / (agg["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "kernels": kernels,
        "hbm_roofline": None,
        "per_rank": per_rank,
        "per_replica": per_replica if R > 1 else None,
        "cpu_baseline": None,
    }
    if corner is not None and pmc:   # the solve stage's kernels as the PMC passes measured them (bytes per launch)
        corner["traffic_per_launch"] = {k: v["hbm_bytes_per_launch"] for k, v in pmc.items()
                                        if k in ("k_corner_factor", "k_corner_flow", "k_corner_invert", "k_stem_schur_rhs", "k_arrow_prepare",
                                                 "k_init_stem")}
        corner["traffic_source"] = traffic_src
        tpl = corner["traffic_per_launch"]
        if "k_corner_factor" in tpl and corner.get("kernel_ms"):
            # the solve stage's HBM bytes per iteration (every launch of it: the factor once per level) against the HBM peak
            # over the stage's time: how far from memory-bound this MFMA-priced stage runs
            per_iter = sum(v * (corner.get("plan", {}).get("factor_launches", 1) if k == "k_corner_factor" else 1) for k, v in tpl.items())
            corner["traffic"] = per_iter
            corner["traffic_frac"] = per_iter / (corner["kernel_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
    if corner is not None:   # ARAP configs: the dense corner (MFMA-bound) is the dominant stage; the HBM one moves aside
        out["hbm_roofline"] = out["roofline"]
        out["roofline"] = corner
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or cpu_threads_default()
        log(f"GPU: {agg['value']:.1f} it/s; running the CPU baseline samples (~{args.cpu_seconds:.0f} s each: one socket's physical "
            f"cores, {threads} threads, 1 thread)")
        out["cpu_baseline"] = cpu_baseline(sc, depth.cpu().numpy(), threads, args.cpu_seconds, args.step, per_launch, R1, t1,
                                           share_only=args.cpu_share_only, warm=not args.cpu_no_warm)
        out["cpu_baseline"]["host"]["sched_affinity"] = len(os.sched_getaffinity(0))
        out["cpu_baseline"]["host"]["omp_num_threads_env"] = os.environ.get("OMP_NUM_THREADS")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
