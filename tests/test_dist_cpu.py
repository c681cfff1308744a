"""The N>1 path on CPU: world_size-2 gloo ranks each render their interleaved
row shard (the oracle stands in for the per-rank GPU render here, it is the
checker) and gather_canvas must rebuild exactly the single-rank canvas."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, out_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from conftest import load_scene
    from fast_ray_tracer_amd.dist import gather_canvas, rows_of, shard_capacity
    scene = load_scene(name)
    rows = rows_of(rank, world, scene.height)
    cap = shard_capacity(world, scene.height)
    shard = torch.zeros((cap, scene.width, 4), dtype=torch.float64)
    for i, r in enumerate(rows):
        shard[i] = torch.from_numpy(oracle.render(scene, r, r + 1, threads=1)[0])
    canvas = gather_canvas(shard, rank, world, scene.height)
    if rank == 0:
        np.save(out_path, canvas.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_interleaved_split_gathers_bit_identical(built, tmp_path, world):
    import oracle
    from conftest import load_scene
    name = "group_test_150x50"
    out = str(tmp_path / "canvas.npy")
    mp.start_processes(_worker, args=(world, _free_port(), name, out), nprocs=world, join=True, start_method="spawn")
    full = oracle.render(load_scene(name), threads=2)
    assert np.array_equal(np.load(out), full)
