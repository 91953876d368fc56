"""Multi-GPU frame sharding: one process per GPU, row stripes, RCCL gather.

Every pixel of raytrace_tris is independent (its own seed slot, its own read-modify-write
of its output pixel — raytracer.cl:207-242), so a frame splits into row stripes dealt
over ranks: round-robin (interleaved), or by an owner map that balances the stripes'
probed cost (RayTracer.partitionStripes, rt_partition_stripes: the long serial chains of
the box pixels crowd the top of the dragon frame).  Every function below takes the
partition as (stripe, n_ranks[, owner]).  Each rank keeps a full
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

`NativeComm` drives the same protocol inside librtmi (csrc/rt_comm.hip: its own RCCL
communicator, grouped ncclSend/ncclRecv, device-side assembly): the path a C++ host
without Python uses; torch.distributed only carries its 128-byte id to every rank.
"""
from __future__ import annotations

import numpy as np


def row_owner(height: int, stripe: int, n_ranks: int, owner=None) -> np.ndarray:
    """Owner rank of every frame row: owner[y // stripe], or (y // stripe) % n_ranks."""
    s = np.arange(height) // stripe
    return s % n_ranks if owner is None else np.asarray(owner, np.int64)[s]


def tile_rows(height: int, stripe: int, n_ranks: int, rank: int, owner=None) -> np.ndarray:
    """Global row indices owned by `rank`, in the order they are stored (rt_tile_rows)."""
    y = np.arange(height)
    return y[row_owner(height, stripe, n_ranks, owner) == rank]


def max_tile_rows(height: int, stripe: int, n_ranks: int, owner=None) -> int:
    return max(len(tile_rows(height, stripe, n_ranks, r, owner)) for r in range(n_ranks))


def lpt_owner(costs, n_ranks: int) -> np.ndarray:
    """The stripes dealt costliest first to the least-loaded rank (ties: the lower stripe index, the
    lower rank) — the rule rt_partition_stripes applies to its probed costs."""
    c = np.asarray(costs)
    order = sorted(range(len(c)), key=lambda s: -c[s])  # stable: ties keep the lower index first
    load = [0] * n_ranks
    own = np.zeros(len(c), np.uint32)
    for s in order:
        r = min(range(n_ranks), key=lambda k: (load[k], k))
        own[s] = r
        load[r] += c[s]
    return own


def assemble(tiles, height: int, width: int, stripe: int, owner=None):
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
        rows = tile_rows(height, stripe, n, r, owner)
        if len(rows) == 0:
            continue
        t = t.reshape(-1, width, 4)[: len(rows)]
        if isinstance(full, np.ndarray):
            full[rows] = t
        else:
            import torch

            full[torch.as_tensor(rows, device=full.device)] = t
    return full


def gather_frame(local, height: int, width: int, stripe: int, group=None, root: int = 0, owner=None):
    """Gather every rank's compact tile to `root` with one torch.distributed.gather
    (RCCL over xGMI for CUDA tensors; gloo on CPU).  `local` is the rank's framebuffer
    padded to max_tile_rows rows.  Returns the assembled [H, W, 4] frame on root, else None."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":  # CPU rehearsal of the RCCL path
        local = local.cpu()
    rows_max = max_tile_rows(height, stripe, world, owner)
    local = local.reshape(-1)[: rows_max * width * 4]
    if local.numel() != rows_max * width * 4:
        raise ValueError("local framebuffer must hold max_tile_rows rows")
    gathered = [torch.empty_like(local) for _ in range(world)] if rank == root else None
    dist.gather(local, gathered, dst=root, group=group)
    if rank != root:
        return None
    return assemble([g.reshape(rows_max, width, 4) for g in gathered], height, width, stripe, owner)


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
    writer src.  `commit(s)` records the frame's writes.  `set_owner` changes the partition:
    the next plan moves the rows whose stripe changed owner since they were written."""

    def __init__(self, height: int, hpad: int, stripe: int, n_ranks: int, owner=None):
        if hpad < height:
            raise ValueError("Hpad < H")
        self.height, self.hpad, self.stripe, self.n_ranks = height, hpad, stripe, n_ranks
        self.set_owner(owner)
        self.writer = np.full(hpad, -1, np.int64)

    def set_owner(self, owner=None) -> None:
        self.row_rank = row_owner(self.height, self.stripe, self.n_ranks, owner)

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


def seed_halo_plan_native(writer: np.ndarray, height: int, hpad: int, stripe: int, n_ranks: int, shift: int,
                          owner=None):
    """rt_seed_halo_plan (librtmi, host only): the moves of SeedHalo.plan(shift) as
    (src, dst, row) arrays, then SeedHalo.commit(shift) applied to `writer` in place."""
    from . import _abi

    lib = _abi.load()
    w = np.ascontiguousarray(writer, np.int32)
    src = np.empty(height, np.uint32)
    dst = np.empty(height, np.uint32)
    rows = np.empty(height, np.uint32)
    k = _abi.ctypes.c_uint32(0)
    o = None if owner is None else np.ascontiguousarray(owner, np.uint32)
    st = lib.rt_seed_halo_plan(_abi.ptr(w), height, hpad, stripe, n_ranks, _abi.ptr(o), shift, _abi.ptr(src),
                               _abi.ptr(dst), _abi.ptr(rows), _abi.ctypes.byref(k))
    if st != _abi.RT_OK:
        raise _abi.RtError(st, "rt_seed_halo_plan")
    writer[...] = w
    n = k.value
    return src[:n], dst[:n], rows[:n]


def seed_halo_peer_blocks(src, dst, rows, n_ranks: int, me: int):
    """rt_seed_halo_peer_blocks (librtmi, host only): rank `me`'s side of a halo plan — the rows
    it sends to and receives from each peer, one block per peer in peer order.  Returns
    (send: list of per-peer row arrays, recv: list of per-peer row arrays)."""
    from . import _abi

    lib = _abi.load()
    k = len(src)
    s_ = np.ascontiguousarray(src, np.uint32)
    d_ = np.ascontiguousarray(dst, np.uint32)
    r_ = np.ascontiguousarray(rows, np.uint32)
    send_rows = np.empty(max(k, 1), np.uint32)
    recv_rows = np.empty(max(k, 1), np.uint32)
    send_cnt = np.empty(n_ranks, np.uint32)
    recv_cnt = np.empty(n_ranks, np.uint32)
    st = lib.rt_seed_halo_peer_blocks(_abi.ptr(s_), _abi.ptr(d_), _abi.ptr(r_), k, n_ranks, me, _abi.ptr(send_rows),
                                      _abi.ptr(send_cnt), _abi.ptr(recv_rows), _abi.ptr(recv_cnt))
    if st != _abi.RT_OK:
        raise _abi.RtError(st, "rt_seed_halo_peer_blocks")
    send, recv, so, ro = [], [], 0, 0
    for p in range(n_ranks):
        send.append(send_rows[so:so + send_cnt[p]].copy())
        recv.append(recv_rows[ro:ro + recv_cnt[p]].copy())
        so += int(send_cnt[p])
        ro += int(recv_cnt[p])
    return send, recv


class NativeComm:
    """librtmi's RCCL communicator (rt_comm_*; one per rank and GPU).

    `uid` (RT_COMM_ID_BYTES bytes) comes from `NativeComm.unique_id()` on rank 0 and is
    handed to every rank by any channel; `from_torch` uses torch.distributed for that."""

    def __init__(self, n_ranks: int, rank: int, device: int, uid: bytes):
        from . import _abi

        self._abi = _abi
        self._lib = _abi.load()
        if len(uid) != _abi.RT_COMM_ID_BYTES:
            raise ValueError("bad communicator id")
        self._uid = (_abi.ctypes.c_uint8 * _abi.RT_COMM_ID_BYTES).from_buffer_copy(uid)
        h = _abi.ctypes.c_void_p()
        st = self._lib.rt_comm_create(_abi.ctypes.addressof(self._uid), n_ranks, rank, device, _abi.ctypes.byref(h))
        if st != _abi.RT_OK:
            raise _abi.RtError(st, "rt_comm_create")
        self._h = h
        self.n_ranks, self.rank, self.device = n_ranks, rank, device

    @staticmethod
    def unique_id() -> bytes:
        from . import _abi

        buf = (_abi.ctypes.c_uint8 * _abi.RT_COMM_ID_BYTES)()
        st = _abi.load().rt_comm_get_unique_id(_abi.ctypes.addressof(buf))
        if st != _abi.RT_OK:
            raise _abi.RtError(st, "rt_comm_get_unique_id")
        return bytes(buf)

    @classmethod
    def from_torch(cls, device: int, group=None):
        """Collective over a torch.distributed group: rank 0 makes the id, a broadcast carries it.

        Every rank takes the same collective steps whatever fails where: each checks that the library
        and its rt_comm_* entry points load; rank 0 ALWAYS joins the broadcast, sending None (the
        error marker) when it could not make the id; then one all_reduce (MIN) agrees on the
        outcome, and only if every rank is ready does any rank enter ncclCommInitRank
        (rt_comm_create).  Otherwise every rank raises, none of them waiting in a collective the
        others never reach."""
        import torch
        import torch.distributed as dist

        from . import _abi

        rank = dist.get_rank(group)
        err = None
        try:
            lib = _abi.load()
            for sym in ("rt_comm_get_unique_id", "rt_comm_create", "rt_comm_render", "rt_comm_destroy"):
                getattr(lib, sym)
        except Exception as e:  # noqa: BLE001 - agreed on below
            err = f"{type(e).__name__}: {e}"
        uid = None
        if rank == 0 and err is None:
            try:
                uid = cls.unique_id()
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
        obj = [uid if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        if obj[0] is None and err is None:
            err = "rank 0 could not make the communicator id"
        dev = torch.device("cuda", device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
        ready = torch.tensor([0 if err else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(ready, op=dist.ReduceOp.MIN, group=group)
        if not int(ready.item()):
            raise RuntimeError(f"native communicator not created on any rank ({err or 'a peer was not ready'})")
        return cls(dist.get_world_size(group), rank, device, obj[0])

    def _check(self, st: int, what: str):
        if st != self._abi.RT_OK:
            raise self._abi.RtError(st, f"{what}: {self._lib.rt_comm_last_error(self._h).decode()}")

    def gather(self, tile, frame, width: int, height: int, stripe: int = 8, root: int = 0, owner=None) -> None:
        """rt_comm_gather_frame: device tile (this rank's rows) -> device frame on root."""
        p = self._abi.ptr
        o = None if owner is None else np.ascontiguousarray(owner, np.uint32)
        self._check(self._lib.rt_comm_gather_frame(self._h, p(tile), p(frame), width, height, stripe, p(o), root),
                    "rt_comm_gather_frame")

    def set_partition(self, balanced: bool) -> None:
        """rt_comm_set_partition: rt_comm_render's triangle frames by the cost-balanced owner map
        (rt_partition_stripes, the default) or interleaved stripes."""
        mode = self._abi.RT_PARTITION_BALANCED if balanced else self._abi.RT_PARTITION_INTERLEAVED
        self._check(self._lib.rt_comm_set_partition(self._h, mode), "rt_comm_set_partition")

    def last_partition(self):
        """rt_comm_last_partition: the owner map of the last rt_comm_render frame (None: interleaved)."""
        n = self._abi.ctypes.c_uint32(0)
        self._check(self._lib.rt_comm_last_partition(self._h, None, 0, self._abi.ctypes.byref(n)),
                    "rt_comm_last_partition")
        if not n.value:
            return None
        out = np.empty(n.value, np.uint32)
        self._check(self._lib.rt_comm_last_partition(self._h, self._abi.ptr(out), n.value, self._abi.ctypes.byref(n)),
                    "rt_comm_last_partition")
        return out

    def render(self, rt, frame, width: int, height: int, progression: int, kernel: int, stripe: int = 8,
               root: int = 0) -> None:
        """rt_comm_render: this rank's stripes (+ the seed-row halo for raytrace) -> frame on root."""
        rt._sync_scene()
        self._check(self._lib.rt_comm_render(self._h, rt._h, self._abi.ptr(frame), width, height, progression, kernel,
                                             stripe, root), "rt_comm_render")

    def reset_halo(self) -> None:
        self._check(self._lib.rt_comm_reset_halo(self._h), "rt_comm_reset_halo")

    def count(self) -> int:
        """ncclCommCount: the ranks RCCL sees in this communicator."""
        n = self._abi.ctypes.c_int(0)
        self._check(self._lib.rt_comm_count(self._h, self._abi.ctypes.byref(n)), "rt_comm_count")
        return n.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.rt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def assemble_native(tiles, height: int, width: int, stripe: int, frame, device: int = 0, owner=None) -> None:
    """rt_assemble_tiles: the root's device-side scatter of compact tiles (device tensors,
    rank order) into `frame` (device, H*W*4 floats)."""
    from . import _abi

    arr = (_abi.ctypes.c_void_p * len(tiles))(*[t.data_ptr() for t in tiles])
    o = None if owner is None else np.ascontiguousarray(owner, np.uint32)
    st = _abi.load().rt_assemble_tiles(_abi.ctypes.addressof(arr), len(tiles), width, height, stripe, _abi.ptr(o),
                                       _abi.ptr(frame), device)
    if st != _abi.RT_OK:
        raise _abi.RtError(st, "rt_assemble_tiles")
