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


def _worker(rank, world, port, H, W, stripe, frame_path, result_path, owner=None):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ptload

    pdist = ptload.submodule("dist")
    full = np.load(frame_path)
    rows = pdist.tile_rows(H, stripe, world, rank, owner)
    rmax = pdist.max_tile_rows(H, stripe, world, owner)
    local = torch.zeros(rmax * W * 4, dtype=torch.float32)
    local[: len(rows) * W * 4] = torch.from_numpy(full[rows].reshape(-1))
    frame = pdist.gather_frame(local, H, W, stripe, owner=owner)
    if rank == 0:
        np.save(result_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe,balanced", [(2, 8, False), (3, 5, False), (2, 4, True), (3, 3, True)])
def test_gather_frame_gloo(world, stripe, balanced, tmp_path, oracle, pt):
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
    owner = None
    if balanced:  # an owner map like rt_partition_stripes': LPT over a cost per stripe (here: its brightness)
        ns = (H + stripe - 1) // stripe
        cost = [int(full[s * stripe:(s + 1) * stripe].sum() * 1000) for s in range(ns)]
        owner = pdist_module().lpt_owner(cost, world)
    mp.spawn(_worker, args=(world, _free_port(), H, W, stripe, str(fp), str(rp), owner), nprocs=world, join=True)
    got = np.load(rp)
    np.testing.assert_array_equal(got.view(np.uint32), full.view(np.uint32))


def pdist_module():
    import ptload

    return ptload.submodule("dist")


# ---- seed-row halo for tiled progressive sphere frames (raytracer.cl:20-30) ----------------

def _halo_schedule():
    """Progression sequence with a restart (camera move resets progression to 0)."""
    return [0, 1, 2, 3, 4, 5, 0, 1, 2, 9, 10]


def _write_value(row, frame_no):
    return (row * 7919 + frame_no * 104729 + 1) & 0x7FFFFFFF


@pytest.mark.parametrize("H,hpad,stripe,n", [(29, 32, 4, 2), (45, 48, 8, 3), (64, 64, 8, 4), (17, 24, 3, 2)])
def test_seed_halo_plan_keeps_every_read_current(pt, H, hpad, stripe, n):
    """Single-process model of N ranks: each rank reads seed rows (y+s)%Hpad of its pixel
    rows, which must hold the latest value written by any rank, then writes them."""
    import ptload

    pdist = ptload.submodule("dist")
    halo = pdist.SeedHalo(H, hpad, stripe, n)
    truth = np.arange(hpad, dtype=np.int64) * 3 + 11  # initial seeds, replicated
    local = [truth.copy() for _ in range(n)]
    moved = 0
    for f, s in enumerate(_halo_schedule()):
        for (src, dst), rows in halo.plan(s).items():
            local[dst][rows] = local[src][rows]
            moved += len(rows)
        for y in range(H):
            r = (y + s) % hpad
            k = halo.row_rank[y]
            assert local[k][r] == truth[r], (f, s, y, r)
            truth[r] = local[k][r] = _write_value(r, f)
        halo.commit(s)
    assert moved > 0


def _halo_worker(rank, world, port, H, hpad, wpad, stripe, result_path):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ptload

    pdist = ptload.submodule("dist")
    halo = pdist.SeedHalo(H, hpad, stripe, world)
    seeds = np.zeros((2, hpad, wpad), np.int32)
    seeds[0] = (np.arange(hpad)[:, None] * 5 + np.arange(wpad)[None, :]) & 0xFFFF
    seeds[1] = seeds[0] ^ 0x5A5A
    truth = seeds.copy()  # every rank replays all writes to know the expected state
    ok = True
    received = 0

    def pack(rows):
        return torch.from_numpy(np.ascontiguousarray(seeds[:, rows.astype(np.int64), :]))

    def unpack(rows, buf):
        seeds[:, rows.astype(np.int64), :] = buf.numpy()

    for f, s in enumerate(_halo_schedule()):
        received += pdist.exchange_seed_rows(halo.plan(s), pack, unpack, wpad)
        for y in range(H):
            r = (y + s) % hpad
            if halo.row_rank[y] == rank:
                ok &= bool(np.array_equal(seeds[:, r, :], truth[:, r, :]))
                seeds[:, r, :] = _write_value(r, f) + np.arange(wpad)[None, :]
            truth[:, r, :] = _write_value(r, f) + np.arange(wpad)[None, :]
        halo.commit(s)
    flags = torch.tensor([int(ok), received], dtype=torch.int64)
    dist.all_reduce(flags[:1], op=dist.ReduceOp.MIN)
    dist.all_reduce(flags[1:], op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(result_path, flags.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,hpad,stripe", [(2, 29, 32, 4), (3, 45, 48, 8)])
def test_seed_halo_exchange_gloo(world, H, hpad, stripe, tmp_path):
    rp = tmp_path / "flags.npy"
    mp.spawn(_halo_worker, args=(world, _free_port(), H, hpad, 32, stripe, str(rp)), nprocs=world, join=True)
    ok, received = np.load(rp)
    assert ok == 1 and received > 0


def _frames_worker(rank, world, port, result_path):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ptload

    pdist = ptload.submodule("dist")
    local = torch.full((6 * 5 * 4,), float(rank) + 0.5)
    frames = pdist.gather_frames(local)
    if rank == 0:
        np.save(result_path, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gather_frames_gloo(tmp_path):
    """Frame-parallel (weak-scaling) mode: one full frame per rank, gathered in rank order."""
    rp = tmp_path / "frames.npy"
    mp.spawn(_frames_worker, args=(3, _free_port(), str(rp)), nprocs=3, join=True)
    got = np.load(rp)
    assert got.shape == (3, 120)
    for r in range(3):
        assert np.all(got[r] == r + 0.5)


@pytest.mark.parametrize("H,hpad,stripe,n", [(53, 56, 8, 2), (45, 48, 4, 3), (64, 64, 8, 8), (30, 32, 16, 4)])
def test_native_halo_plan_equals_python(pt, H, hpad, stripe, n):
    """rt_seed_halo_plan (the native host's halo planner, csrc/rt_comm.hip) makes the same
    moves as dist.SeedHalo over a progression with restarts, and commits the same writers."""
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    halo = dist.SeedHalo(H, hpad, stripe, n)
    writer = np.full(hpad, -1, np.int32)
    total = 0
    for s in [0, 1, 2, 3, 7, 0, 1, 5, hpad - 1, hpad + 3, 2]:
        plan = halo.plan(s)
        src, dst, rows = dist.seed_halo_plan_native(writer, H, hpad, stripe, n, s)
        exp = [(a, b, int(r)) for (a, b), rr in plan.items() for r in rr]
        got = list(zip(src.tolist(), dst.tolist(), rows.tolist()))
        assert got == exp, f"shift {s}"
        total += len(got)
        halo.commit(s)
        np.testing.assert_array_equal(writer, halo.writer)
    assert total > 0


@pytest.mark.parametrize("H,hpad,stripe,n", [(53, 56, 8, 2), (45, 48, 4, 3), (64, 64, 8, 8), (1080, 1080, 8, 8)])
def test_halo_moves_rows_whose_stripe_changed_owner(pt, H, hpad, stripe, n):
    """rt_comm_render under the balanced partition: each view brings its own owner map
    (rt_partition_stripes), so between triangle frames (unshifted seed rows) a stripe may change
    owner.  rt_seed_halo_plan must equal SeedHalo.plan under the new map, and after the moves every
    row a rank reads holds the latest write — the seeds follow their stripes."""
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    ns = (H + stripe - 1) // stripe
    rng = np.random.default_rng(H + n)
    maps = [None] + [dist.lpt_owner(rng.integers(1, 100, ns), n) for _ in range(4)] + [None]
    halo = dist.SeedHalo(H, hpad, stripe, n)
    writer = np.full(hpad, -1, np.int32)
    truth = np.arange(hpad, dtype=np.int64) * 3 + 11
    local = [truth.copy() for _ in range(n)]
    moved = 0
    for f, own in enumerate(maps + maps[1:3]):  # (a map used again later)
        halo.set_owner(own)
        plan = halo.plan(0)
        src, dst, rows = dist.seed_halo_plan_native(writer, H, hpad, stripe, n, 0, own)
        exp = [(a, b, int(r)) for (a, b), rr in plan.items() for r in rr]
        assert list(zip(src.tolist(), dst.tolist(), rows.tolist())) == exp, f
        for a, b, r in exp:
            local[b][r] = local[a][r]
        moved += len(exp)
        for y in range(H):
            k = halo.row_rank[y]
            assert local[k][y] == truth[y], (f, y)
            truth[y] = local[k][y] = _write_value(y, f)
        halo.commit(0)
        np.testing.assert_array_equal(writer, halo.writer)
    assert moved > 0


# (kernel, progression) sequences of rt_comm_render calls: progressive sphere frames with
# restarts, interleaved with raytrace_ss / raytrace_tris frames (unshifted seed rows)
_COMM_SEQUENCE = [(0, 0), (0, 1), (0, 2), (0, 3), (2, 0), (0, 4), (0, 5), (1, 0), (0, 0), (0, 1), (2, 0),
                  (2, 0), (0, 1), (0, 9), (1, 0), (0, 2)]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("H,hpad,stripe", [(61, 64, 8), (45, 48, 4)])
def test_native_comm_render_block_plan_replay(pt, n, H, hpad, stripe):
    """rt_comm_render's halo step, replayed on the host for N ranks (csrc/rt_comm.hip): every rank
    plans with rt_seed_halo_plan, splits the plan into per-peer blocks with
    rt_seed_halo_peer_blocks and packs its send block to each peer; peer p unpacks what it
    receives from rank q in the order of its own receive block.  The blocks must pair up (q's
    block to p lists exactly p's rows from q, in the same order, so the packed buffers match
    word for word), every row a rank reads must then hold the latest write of any rank
    (dist.SeedHalo's contract), and the plan must equal SeedHalo.plan — for raytrace frames
    (rows shifted by the progression) and for the unshifted kernels after them."""
    from importlib import import_module

    dist = import_module("pathtracer_cl_amd.dist")
    halo = dist.SeedHalo(H, hpad, stripe, n)
    writer = np.full(hpad, -1, np.int32)
    truth = np.arange(hpad, dtype=np.int64) * 3 + 11
    local = [truth.copy() for _ in range(n)]
    moved = 0
    for f, (kernel, prog) in enumerate(_COMM_SEQUENCE):
        shift = prog if kernel == 0 else 0
        if f > 0:  # the first frame on a communicator is "fresh": identical seeds everywhere
            plan = halo.plan(shift)
            src, dst, rows = dist.seed_halo_plan_native(writer, H, hpad, stripe, n, shift)
            exp = [(a, b, int(r)) for (a, b), rr in plan.items() for r in rr]
            assert list(zip(src.tolist(), dst.tolist(), rows.tolist())) == exp, (f, kernel, prog)
            blocks = [dist.seed_halo_peer_blocks(src, dst, rows, n, me) for me in range(n)]
            inbox = {}
            for q in range(n):
                send, _ = blocks[q]
                for p_ in range(n):
                    if len(send[p_]):
                        inbox[(q, p_)] = (send[p_].copy(), local[q][send[p_].astype(np.int64)].copy())
            for p_ in range(n):
                _, recv = blocks[p_]
                for q in range(n):
                    if len(recv[q]) == 0:
                        assert (q, p_) not in inbox
                        continue
                    rows_sent, packed = inbox.pop((q, p_))
                    np.testing.assert_array_equal(rows_sent, recv[q])
                    local[p_][recv[q].astype(np.int64)] = packed
                    moved += len(recv[q])
            assert not inbox
        else:
            # the native planner still records the first frame's writes (rt_comm_render commits)
            dist.seed_halo_plan_native(writer, H, hpad, stripe, n, shift)
        for y in range(H):
            r = (y + shift) % hpad
            k = halo.row_rank[y]
            assert local[k][r] == truth[r], (f, kernel, prog, y, r)
            truth[r] = local[k][r] = _write_value(r, f)
        halo.commit(shift)
        np.testing.assert_array_equal(writer, halo.writer)
    assert moved > 0


# ---- NativeComm.from_torch: the ranks agree before ncclCommInitRank ------------

def _from_torch_worker(rank, world, port, mode, result_path):
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ptload

    pdist = ptload.submodule("dist")
    made = []

    def fake_init(self, n_ranks, r, device, uid):  # stands in for rt_comm_create (RCCL needs GPUs)
        made.append((n_ranks, r, device, len(uid)))

    pdist.NativeComm.__init__ = fake_init
    if mode == "ok":
        pdist.NativeComm.unique_id = staticmethod(lambda: bytes(range(128)))
    else:  # rank 0 cannot make the id: every rank must raise, none may wait in a collective
        def boom():
            raise RuntimeError("no id")
        pdist.NativeComm.unique_id = staticmethod(boom)
    try:
        pdist.NativeComm.from_torch(0)
        res = "made" if made == [(world, rank, 0, 128)] else f"bad {made}"
    except RuntimeError as e:
        res = "raised" if not made and "not created on any rank" in str(e) else f"bad {e}"
    dist.barrier()  # every rank got here: nobody is stuck in a collective
    with open(f"{result_path}.{rank}", "w") as f:
        f.write(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,want", [("ok", "made"), ("fail", "raised")])
def test_native_comm_from_torch_agrees_before_init(mode, want, tmp_path, pt):
    world = 3
    rp = tmp_path / "res"
    mp.spawn(_from_torch_worker, args=(world, _free_port(), mode, str(rp)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"res.{r}").read_text() == want
