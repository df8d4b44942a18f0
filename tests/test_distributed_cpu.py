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


def test_single_process_helpers():
    assert bench.max_over_ranks(3.0) == 3.0
    agg = bench.aggregate(10, 0.5, 1)
    assert agg["value"] == pytest.approx(20.0) and agg["ms_per_step"] == pytest.approx(50.0)


def test_algorithmic_bytes_c2():
    # C2: 640x480, 153,600 triangles, 77,361 vertices, 1500 nodes, 4 anchors
    b = bench.fit_pixels_bytes(640 * 480, 153600, 77361, 1500, 4)
    assert b == 307200 * 29 + 153600 * 16 + 77361 * 176 + 1500 * 216
    assert bench.iteration_bytes(640 * 480, 153600, 77361, 1500, 4) > b
