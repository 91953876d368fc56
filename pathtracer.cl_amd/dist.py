"""Multi-GPU frame sharding: one process per GPU, interleaved row stripes, RCCL gather.

Every pixel of raytrace_tris is independent (its own seed slot, its own read-modify-write
of its output pixel — raytracer.cl:207-242), so a frame splits into row stripes dealt
round-robin over ranks (load balance: the mesh sits mid-frame).  Each rank keeps a full
scene/BVH replica and the full seed planes, renders its rows into a compact local
framebuffer (rt_tile), and the frame is assembled on the root with ONE collective: a
gather of the compact tiles over RCCL (torch.distributed backend "nccl" = RCCL on ROCm),
which over xGMI is one point-to-point transfer per sender.

Progressive accumulation stays local (each rank mixes into its own rows), so the gather is
only needed when the root wants to display/store the frame.

The sphere kernel (raytrace) is the exception: pixel row y reads and writes seed row
(y + progressive) % Hpad (get_seed / put_seed, raytracer.cl:20-30), so between progressive
frames one seed row per stripe boundary migrates to the neighbouring rank.  `SeedHalo`
plans those moves (it tracks the last writer of every seed row) and `exchange_seed_rows`
performs them with point-to-point sends (RCCL over xGMI, 2 * Wpad * 4 B per row).
"""
from __future__ import annotations

import numpy as np


def tile_rows(height: int, stripe: int, n_ranks: int, rank: int) -> np.ndarray:
    """Global row indices owned by `rank`, in the order they are stored (rt_tile_rows)."""
    y = np.arange(height)
    return y[(y // stripe) % n_ranks == rank]


def max_tile_rows(height: int, stripe: int, n_ranks: int) -> int:
    return max(len(tile_rows(height, stripe, n_ranks, r)) for r in range(n_ranks))


def assemble(tiles, height: int, width: int, stripe: int):
    """Scatter gathered compact tiles (rank order; each [>=rows_r, W, 4]) into a full
    [H, W, 4] frame.  Works on numpy arrays or torch tensors."""
    n = len(tiles)
    first = tiles[0]
    if isinstance(first, np.ndarray):
        full = np.empty((height, width, 4), first.dtype)
    else:
        import torch

        full = torch.empty((height, width, 4), dtype=first.dtype, device=first.device)
    for r, t in enumerate(tiles):
        rows = tile_rows(height, stripe, n, r)
        if len(rows) == 0:
            continue
        t = t.reshape(-1, width, 4)[: len(rows)]
        if isinstance(full, np.ndarray):
            full[rows] = t
        else:
            import torch

            full[torch.as_tensor(rows, device=full.device)] = t
    return full


def gather_frame(local, height: int, width: int, stripe: int, group=None, root: int = 0):
    """Gather every rank's compact tile to `root` with one torch.distributed.gather
    (RCCL over xGMI for CUDA tensors; gloo on CPU).  `local` is the rank's framebuffer
    padded to max_tile_rows rows.  Returns the assembled [H, W, 4] frame on root, else None."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":  # CPU rehearsal of the RCCL path
        local = local.cpu()
    rows_max = max_tile_rows(height, stripe, world)
    local = local.reshape(-1)[: rows_max * width * 4]
    if local.numel() != rows_max * width * 4:
        raise ValueError("local framebuffer must hold max_tile_rows rows")
    gathered = [torch.empty_like(local) for _ in range(world)] if rank == root else None
    dist.gather(local, gathered, dst=root, group=group)
    if rank != root:
        return None
    return assemble([g.reshape(rows_max, width, 4) for g in gathered], height, width, stripe)


def gather_frames(local, group=None, root: int = 0):
    """Frame-parallel mode: every rank rendered its own full frame; gather them to `root`
    with one torch.distributed.gather (RCCL for CUDA tensors).  Returns the list of frames
    (rank order) on root, else None."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        local = local.cpu()
    gathered = [torch.empty_like(local) for _ in range(world)] if rank == root else None
    dist.gather(local, gathered, dst=root, group=group)
    return gathered


class SeedHalo:
    """Seed-row bookkeeping for tiled progressive sphere frames.

    Every rank holds the full seed planes; a rank's copy of a row is current only if it
    wrote it last (or nobody has: the initial seeds are identical everywhere).  Before a
    frame with row shift s, rank j needs rows (y + s) % Hpad for its pixel rows y < H;
    `plan(s)` lists, per (src, dst) rank pair, the rows dst must receive from their last
    writer src.  `commit(s)` records the frame's writes."""

    def __init__(self, height: int, hpad: int, stripe: int, n_ranks: int):
        if hpad < height:
            raise ValueError("Hpad < H")
        self.height, self.hpad, self.stripe, self.n_ranks = height, hpad, stripe, n_ranks
        y = np.arange(height)
        self.row_rank = (y // stripe) % n_ranks
        self.writer = np.full(hpad, -1, np.int64)

    def _rows(self, shift: int) -> np.ndarray:
        return (np.arange(self.height) + int(shift)) % self.hpad

    def plan(self, shift: int) -> dict:
        r = self._rows(shift)
        src = self.writer[r]
        dst = self.row_rank
        need = (src >= 0) & (src != dst)
        out = {}
        for s_, d_, row in zip(src[need], dst[need], r[need]):
            out.setdefault((int(s_), int(d_)), []).append(int(row))
        return {k: np.asarray(v, np.uint32) for k, v in sorted(out.items())}

    def commit(self, shift: int) -> None:
        self.writer[self._rows(shift)] = self.row_rank


def exchange_seed_rows(plan: dict, pack, unpack, n_words_per_row: int, device=None, group=None) -> int:
    """Carry out a SeedHalo plan on this rank: `pack(rows) -> tensor` ([2, n, Wpad] uint32)
    for rows this rank sends, `unpack(rows, tensor)` for rows it receives, moved with
    point-to-point sends (torch.distributed: RCCL for CUDA tensors, gloo on CPU).
    Returns the number of rows this rank received."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    ops, recvs = [], []
    for (src, dst), rows in plan.items():
        if src == rank:
            ops.append(dist.P2POp(dist.isend, pack(rows), dst, group))
        elif dst == rank:
            buf = torch.empty((2, len(rows), n_words_per_row), dtype=torch.int32, device=device)
            ops.append(dist.P2POp(dist.irecv, buf, src, group))
            recvs.append((rows, buf))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for rows, buf in recvs:
        unpack(rows, buf)
    return sum(len(r) for r, _ in recvs)
