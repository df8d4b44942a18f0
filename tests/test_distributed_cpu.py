"""N > 1 path of bench.py on CPU (gloo, world_size 2): replicas with no data-path collective -- each rank fits its own
independent sequence (seed = rank) and the only cross-rank steps are the barrier and the max-over-ranks of the elapsed
time that the whole-job throughput is computed from."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, lr, w = bench.dist_env()
        elapsed = 1.0 + 0.5 * rank            # rank 1 is the slow one
        m = bench.max_over_ranks(elapsed)
        agg = bench.aggregate(100, m, w)
        from dynamicfuion_python_amd import synthetic as S
        sc = S.make_scene("S1", seed=r)
        dist.barrier()
        q.put((rank, r, lr, w, m, agg["value"], agg["ms_per_step"], float(sc.gt_translations.sum())))
    finally:
        dist.destroy_process_group()


def test_two_rank_replica_aggregation():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    results.sort()
    for rank, r, lr, w, m, value, ms, _ in results:
        assert r == rank and lr == rank and w == world
        assert m == pytest.approx(1.5)                       # max over ranks
        assert value == pytest.approx(world * 100 / 1.5)     # whole-job iterations / slowest rank's time
        assert ms == pytest.approx(15.0)
    # independent sequences: different ground-truth motion per rank
    assert results[0][-1] != results[1][-1]


def _protocol_worker(rank, world, port, q):
    """bench.main's N > 1 control path with a stubbed fitter step: timed_region (barrier + sync + launches + sync +
    barrier), max_over_ranks, aggregate and the end-of-run all_gather of per-rank results, over gloo."""
    import time

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def step(n):                            # stub fitter launch: rank 1 is twice as slow
            time.sleep(0.01 * (1 + rank))
            calls.append(n)
            return 0

        syncs = []
        bad, elapsed = bench.timed_region(step, 5, 10, world, lambda: syncs.append(1))
        m = bench.max_over_ranks(elapsed)
        agg = bench.aggregate(50, m, world)
        per_rank = bench.exchange_per_rank(50, elapsed, 1.0 + rank)
        q.put((rank, bad, calls, len(syncs), elapsed, m, agg["value"], per_rank))
    finally:
        dist.destroy_process_group()


def test_two_rank_bench_protocol():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_protocol_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    slowest = max(r[4] for r in results)
    for rank, bad, calls, nsync, elapsed, m, value, per_rank in results:
        assert bad == 0 and calls == [10] * 5 and nsync == 2
        assert m == pytest.approx(slowest)                   # every rank sees the slowest rank's time
        assert value == pytest.approx(world * 50 / slowest)
        assert [p["rank"] for p in per_rank] == [0, 1]
        assert [p["update_norm"] for p in per_rank] == [1.0, 2.0]
        assert per_rank[rank]["seconds"] == pytest.approx(elapsed)
        assert per_rank[rank]["iters_per_s"] == pytest.approx(50 / elapsed)
    assert results[1][4] > results[0][4]                     # rank 1's stub is slower
    assert slowest >= 5 * 0.02


def test_single_process_helpers():
    assert bench.max_over_ranks(3.0) == 3.0
    assert bench.exchange_per_rank(10, 1.0, 0.0) is None
    bad, el = bench.timed_region(lambda n: 0, 3, 2, 1, lambda: None)
    assert bad == 0 and el >= 0
    agg = bench.aggregate(10, 0.5, 1)
    assert agg["value"] == pytest.approx(20.0) and agg["ms_per_step"] == pytest.approx(50.0)


def test_algorithmic_bytes_c2():
    # SURVEY.md 8(d) worked example: C2 (P = 307,200, V = 77,361, F = 153,600, K = 4, E ~ 1.4 M, N = 1500) ~ 374 MB
    sb = bench.stage_bytes(640 * 480, 153600, 77361, 1500, 4, 1_400_000)
    total = sum(sb.values())
    assert 330e6 < total < 400e6
    assert sb["pixel_anchor_jacobians"] == 307200 * 257 + 307200 * 72 * 4 + 4 * 1_400_000
    # round 4: the fused pixel launch also forms the warped-surface Jacobians (the warp stores positions / normals only)
    assert bench.kernel_bytes("k_fit_pixels_fused", sb) == (sb["residual"] + sb["rasterized_jacobians"] + sb["warped_jacobians"]
                                                            + sb["pixel_anchor_jacobians"] + sb["jtj_jtr"])
    assert bench.kernel_bytes("k_warp_mesh_quad", sb) == sb["warp"]
    # every stage of the block-diagonal iteration except the ARAP rows is covered by exactly one kernel
    covered = [st for k in bench.KERNEL_STAGES.values() for st in k]
    assert sorted(covered) == sorted(sb)
    # every kernel the bytes are charged to has a per-kernel time (nnrt_fitter_time_kernels order)
    from dynamicfuion_python_amd.nnrt.alignment import KERNEL_TIMES
    assert set(bench.KERNEL_STAGES) - {"k_solve_update"} <= set(KERNEL_TIMES) and "solve" in KERNEL_TIMES


def test_association_count():
    import numpy as np
    faces = np.array([[0, 1, 2], [1, 2, 3]])
    anchors = np.array([[0, 1, 2, 3], [0, 1, 2, 4], [0, 5, -1, -1], [6, 6, 7, 8]], np.int32)
    pixel_faces = np.array([0, 1, -1, 0])
    mask = np.array([1, 1, 1, 0])
    # pixel 0: face 0 -> {0,1,2,3,4,5} = 6 ; pixel 1: face 1 -> {0,1,2,4,5,6,7,8} = 8 ; pixel 2: no face ; pixel 3: masked
    assert bench.count_associations(pixel_faces, mask, faces, anchors) == 14


def test_more_ranks_than_devices_fails_fast(monkeypatch):
    """bench.main under the default (RCCL) backend with more local ranks than visible GPUs stops with a clear message
    before touching a device or the process group (no silent device mis-mapping)."""
    import torch
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)

    def no_device(*a, **k):
        raise AssertionError("a device was selected before the rank/device check")

    monkeypatch.setattr(torch.cuda, "set_device", no_device)
    monkeypatch.delenv("NNRT_BENCH_BACKEND", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    for rank in (0, 1):
        monkeypatch.setenv("RANK", str(rank))
        monkeypatch.setenv("LOCAL_RANK", str(rank))
        monkeypatch.setenv("WORLD_SIZE", "2")
        with pytest.raises(SystemExit, match="need one GPU each, but 1 device"):
            bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    # the gloo rehearsal shares devices on purpose; one rank per device passes
    bench.check_rank_devices(1, 2, "gloo", 1)
    bench.check_rank_devices(0, 1, "nccl", 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    bench.check_rank_devices(3, 16, "nccl", 8)   # two nodes of 8: local ranks 0..7 on 8 devices


def test_refinement_window_constants_agree():
    """The refinement window the GPU tests assume (tests/test_gpu_parity.py REFINE_FLOOR) is the one the kernels are
    built with (csrc/fitter_kernels.hpp NNRT_REFINE_PIVOT_FLOOR / NNRT_REFINE_PIVOT_RATIO), and the documented default
    threshold (include/nnrt_mi355x.h) is the built one."""
    import re
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hpp = open(os.path.join(ROOT, "dynamicfuion_python_amd", "csrc", "fitter_kernels.hpp")).read()
    floor = float(re.search(r"#define NNRT_REFINE_PIVOT_FLOOR ([0-9.e+-]+)f", hpp).group(1))
    upper = float(re.search(r"#define NNRT_REFINE_PIVOT_RATIO ([0-9.e+-]+)f", hpp).group(1))
    src = open(os.path.join(ROOT, "tests", "test_gpu_parity.py")).read()
    assert float(re.search(r"^REFINE_FLOOR = ([0-9.e+-]+)", src, re.M).group(1)) == floor
    hdr = open(os.path.join(ROOT, "include", "nnrt_mi355x.h")).read()
    assert float(re.search(r"refinement gate \(default ([0-9.e+-]+)\)", hdr).group(1)) == upper
    assert float(re.search(r"and is at least ([0-9.e+-]+)\)", hdr).group(1)) == floor
    assert floor < upper
