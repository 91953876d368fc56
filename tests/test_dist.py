"""Multi-process frame sharding on CPU: world_size 2 (and 3) over gloo.

Each rank takes its interleaved row stripes of a frame rendered by the CPU oracle (stand-in
for its GPU tile — the GPU tile itself is checked bit-exactly against the full frame in
test_gpu_parity.py::test_tiles_assemble_to_full_frame), pads to max_tile_rows and the root
gathers with pathtracer_cl_amd.dist.gather_frame — the same code path bench.py runs over RCCL.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, stripe, frame_path, result_path):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ptload

    pdist = ptload.submodule("dist")
    full = np.load(frame_path)
    rows = pdist.tile_rows(H, stripe, world, rank)
    rmax = pdist.max_tile_rows(H, stripe, world)
    local = torch.zeros(rmax * W * 4, dtype=torch.float32)
    local[: len(rows) * W * 4] = torch.from_numpy(full[rows].reshape(-1))
    frame = pdist.gather_frame(local, H, W, stripe)
    if rank == 0:
        np.save(result_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe", [(2, 8), (3, 5)])
def test_gather_frame_gloo(world, stripe, tmp_path, oracle, pt):
    sc = pt.scenes
    W, H = 40, 29
    Wp, Hp = sc.padded_dims(W, H)
    verts, idx = sc.make_mesh(1500)
    cam = sc.camera_spherical(W, **sc.PLY_CAMERA)
    out = np.zeros(W * H * 4, np.float32)
    oracle.render_tris(out, cam, sc.ply_scene(), W, H, Wp, Hp, 1, 6, 0, sc.default_seeds(Wp, Hp), verts, idx)
    full = out.reshape(H, W, 4)
    fp = tmp_path / "frame.npy"
    rp = tmp_path / "result.npy"
    np.save(fp, full)
    mp.spawn(_worker, args=(world, _free_port(), H, W, stripe, str(fp), str(rp)), nprocs=world, join=True)
    got = np.load(rp)
    np.testing.assert_array_equal(got.view(np.uint32), full.view(np.uint32))
