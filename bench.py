#!/usr/bin/env python3
"""Benchmark: Mrays/s + frames/s of raytrace_tris on the dragon-class config.

Workload (BASELINE.json configs[3], the metric's config): 871,414-triangle
synthetic mesh (dragon class), 1920x1080, sampleRate 16 (256 spp, one launch,
progression 0), maxDepth 6, plymain.cpp lights and camera, BVH traversal.
One step = one full frame: every rank renders its row stripes (rt_tile; dealt by their probed
cost, rt_partition_stripes, unless --partition interleaved) and,
for N > 1, the frame is gathered to rank 0 over RCCL — by librtmi's own communicator
(rt_comm_render: seed-row halo, grouped ncclSend/ncclRecv, device-side assembly; the
default, `--comm native`) or by torch.distributed (`--comm torch`, also the gloo rehearsal).
At N > 1 the line carries `gathered_bit_exact`: the frame gathered through the same path from
fixed seeds, compared on rank 0 with a single-GPU render of the same seeds (and every rank's
seed rows with the single render's).
A ray = one closest-hit or one any-hit (shadow) query, counted on the device.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0 (contract in the task statement), with a `roofline` object for
the triangle kernel (algorithmic bytes from the device traversal counters / HIP-event kernel
time) and a `cpu_baseline` object (the CPU oracle, bit-identical restatement of the reference
kernel, on a bounded pixel sample, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mrays/sec + frames/sec at 1920×1080, 871k-tri PLY, 1/2/4/8 MI355X"
# the other BASELINE configurations (configs[1], [2], [4]) under their own names
CONFIG_METRIC = {"bunny": "Mrays/sec + frames/sec at 1024×1024, 69k-tri PLY (bunny class), 1 spp",
                 "spheres": "Mrays/sec + frames/sec, built-in sphere scene 1024×1024 progressive",
                 "lucy": "Mrays/sec + frames/sec at 4096×4096, 28M-tri PLY (Lucy class), 16 spp, row-stripe tiles"}
# --scaling weak renders one whole frame per rank: a different quantity, never reported as METRIC
METRIC_WEAK = "Mrays/sec + frames/sec, one 1920×1080 frame per MI355X (weak scaling, not tile-parallel)"
N_SIMD, N_CU = 1024, 256  # MI355X: 256 CUs x 4 SIMD-32 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2 (per XCD, 32 MiB aggregate) ~34.5 TB/s
NODE_BYTES = {"bvh": 64, "bvh4f": 112, "linear": 0}  # bytes read per node visit, csrc/rt_internal.h + rt_quant.h
# bytes read per triangle test: the whole 48-B record (one-record steps of the compressed traversal), else
# v0+orig (16), e1 (12), e2 (12); csrc/rt_internal.h
TRI_BYTES = {"bvh": 48, "bvh4f": 40, "linear": 40}
TRI_BYTES_8D = 36  # the reference's triangle_t per test
PIXEL_BYTES = 16 + 8 + 8  # RGBA32F store + seed read + seed write per pixel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="dragon", choices=["dragon", "bunny", "lucy", "spheres"])
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--sample-rate", type=int, default=None)
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--partition", default="balanced", choices=["balanced", "interleaved"],
                    help="N > 1 strong scaling: the row stripes dealt to ranks by their probed cost (rt_partition_stripes, "
                         "LPT; the default) or round-robin")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="N > 1: strong (default) = one frame split into row-stripe tiles across ranks, gathered "
                         "to rank 0 over RCCL; weak = one full frame per rank (turntable views 3 degrees apart), "
                         "reported under its own metric name (METRIC_WEAK)")
    ap.add_argument("--comm", default="native", choices=["native", "torch"],
                    help="N > 1 strong scaling: native = librtmi's own RCCL communicator (rt_comm_render: "
                         "seed-row halo + grouped ncclSend/ncclRecv gather + device-side assembly, the C++ "
                         "host's path); torch = torch.distributed gather (also the gloo rehearsal)")
    ap.add_argument("--linear", action="store_true", help="reference linear traversal instead of the BVH")
    ap.add_argument("--traversal", default="bvh", choices=["bvh", "bvh4f", "linear"],
                    help="bvh: 4-wide compressed BVH (default); bvh4f: full-precision nodes; linear: the reference loop")
    ap.add_argument("--builder", default="host", choices=["host", "gpu"],
                    help="BVH builder: host binned SAH (default) or the GPU LBVH build")
    ap.add_argument("--ply", default=None, help="render this PLY mesh (normalised, SURVEY §8d) instead of "
                    "the synthetic mesh of the config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-linear-leg", action="store_true", help="skip the GPU linear-traversal leg (N = 1)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N fresh child processes of this script
    (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; nothing here has touched the GPU:
    counting devices does not initialise it on this image), relay their output (rank 0 prints the
    line) and return non-zero if any rank fails — then the others, which would wait in a collective
    for it, are stopped.  With RCCL (the default) the node must have N devices; the gloo rehearsal
    (BENCH_DIST_BACKEND=gloo) may share one."""
    import signal
    import subprocess

    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend == "nccl":
        import torch

        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: this node has {have} GPU(s); one rank per GPU needs {n} "
                  "(BENCH_DIST_BACKEND=gloo rehearses the N > 1 path on fewer)", file=sys.stderr)
            return 2
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.2)
            if rc:
                deadline = time.time() + 20
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        # one process per GPU; BENCH_DIST_BACKEND=gloo rehearses the N>1 path on one device
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        dev = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    device = (local_rank % max(torch.cuda.device_count(), 1)) if world > 1 else 0
    torch.cuda.set_device(device)

    import ptload

    pt = ptload.load()
    sc = pt.scenes
    ptdist = ptload.submodule("dist")

    cfg = args.config
    if cfg == "spheres":
        W, H, sr, kernel = 1024, 1024, 1, pt.RayTracer.KERNEL_SPHERES
        n_tris = 0
    else:
        W, H = (1920, 1080) if cfg == "dragon" else ((1024, 1024) if cfg == "bunny" else (4096, 4096))
        sr = 16 if cfg == "dragon" else (1 if cfg == "bunny" else 4)
        n_tris = sc.MESH_CONFIGS[cfg]
        kernel = pt.RayTracer.KERNEL_TRIS
    W = args.width or W
    H = args.height or H
    sr = args.sample_rate or sr

    frames_per_rank = world > 1 and args.scaling == "weak"

    rt = pt.RayTracer(device)
    S = sc.ply_scene() if kernel == pt.RayTracer.KERNEL_TRIS else sc.main_scene()
    rt.setSpheres(S)
    cam_setup = sc.PLY_CAMERA if kernel == pt.RayTracer.KERNEL_TRIS else sc.MAIN_CAMERA
    # weak scaling: rank r renders the view r arrow-key steps (3 degrees, GlutCLWindow.cpp:228-262)
    # around the turntable; rank 0's frame is the single-GPU frame
    azimuth = cam_setup["azimuth"] + (3.0 * rank if frames_per_rank else 0.0)
    rt.setCameraSpherical(cam_setup["target"], cam_setup["elevation"], azimuth, cam_setup["distance"])
    rt.setFoVAngle(sc.DEFAULT_FOV)
    rt.setSampleRate(sr)
    rt.setMaxPathDepth(6)
    if args.linear:
        args.traversal = "linear"
    args.linear = args.traversal == "linear"
    rt.setTraversal(args.traversal)
    rt.setBuilder(args.builder)
    mesh_info = {}
    if args.ply and kernel == pt.RayTracer.KERNEL_TRIS:
        t0 = time.time()
        verts, idx = sc.load_ply(args.ply)
        t1 = time.time()
        n_tris = len(idx)
        cfg = f"PLY {Path(args.ply).name}"
        rt.setMesh(verts, idx)
        mesh_info = rt.meshInfo()
        mesh_info["load_seconds"] = round(t1 - t0, 3)
    elif n_tris:
        t0 = time.time()
        verts, idx = sc.make_mesh(n_tris)
        t1 = time.time()
        rt.setMesh(verts, idx)
        mesh_info = rt.meshInfo()
        mesh_info["gen_seconds"] = round(t1 - t0, 3)

    n_ranks = 1 if frames_per_rank else world  # ranks sharing one frame
    # the stripes' owners: by probed cost (every rank computes the same map from the same view) for
    # triangle frames, round-robin for the progressive sphere frames (their seed-row halo)
    owner = None
    if n_ranks > 1 and args.partition == "balanced" and kernel == pt.RayTracer.KERNEL_TRIS:
        owner = rt.partitionStripes(W, H, args.stripe, n_ranks)
    tile = (args.stripe, n_ranks, rank, owner) if n_ranks > 1 else None
    rows = ptdist.max_tile_rows(H, args.stripe, n_ranks, owner) if n_ranks > 1 else H
    out = torch.zeros(rows * W * 4, dtype=torch.float32, device=f"cuda:{device}")

    Wp, Hp = sc.padded_dims(W, H)
    # sphere config: progressive frames (progression 0, 1, 2, ...: row-shifted seeds); on a
    # tile the seed rows that cross stripe boundaries move between ranks every frame
    progressive = kernel != pt.RayTracer.KERNEL_TRIS
    halo = ptdist.SeedHalo(H, Hp, args.stripe, n_ranks) if (progressive and n_ranks > 1) else None
    frame_no = [0]

    # halo buffers live on the GPU for RCCL; the gloo rehearsal moves them through host memory
    halo_dev = f"cuda:{device}" if (dist and dist.get_backend() == "nccl") else "cpu"

    def pack(rows):
        buf = torch.empty((2, len(rows), Wp), dtype=torch.int32, device=halo_dev)
        rt.packSeedRows(rows, buf)
        return buf

    # native sharding (csrc/rt_comm.hip): librtmi's RCCL communicator renders the rank's
    # stripes, moves the seed-row halo and assembles the frame on rank 0's GPU
    comm = None
    comm_note = None
    if n_ranks > 1 and args.comm == "native" and dist.get_backend() == "nccl":
        # every rank must take the same path: the communicator is created collectively and the
        # outcome agreed on, so a failure anywhere sends all ranks to the torch.distributed gather
        err = None
        try:
            comm = ptdist.NativeComm.from_torch(device)
            comm.set_partition(args.partition == "balanced")
        except Exception as e:  # noqa: BLE001 - reported in the line
            err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if err else 1], dtype=torch.int64, device=f"cuda:{device}")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()):
            if comm is not None:
                comm.close()
            comm = None
            comm_note = f"native communicator unavailable ({err or 'on another rank'}): torch.distributed gather"
        else:
            frame_full = torch.zeros((W * H * 4) if rank == 0 else 4, dtype=torch.float32, device=f"cuda:{device}")

    def step():
        p = frame_no[0] if progressive else 0
        if comm is not None:
            comm.render(rt, frame_full, W, H, p, kernel, stripe=args.stripe)
            frame_no[0] += 1
            c = rt.counters()
            return c["rays_closest"] + c["rays_shadow"]
        if halo is not None:
            ptdist.exchange_seed_rows(halo.plan(p), pack, rt.unpackSeedRows, Wp, device=halo_dev)
        rt.rayTrace(out, W, H, p, kernel=kernel, tile=tile, halo=halo is not None)
        if halo is not None:
            halo.commit(p)
        frame_no[0] += 1
        c = rt.counters()
        if n_ranks > 1:
            ptdist.gather_frame(out, H, W, args.stripe, owner=owner)
        elif frames_per_rank:
            ptdist.gather_frames(out)
        return c["rays_closest"] + c["rays_shadow"]

    # first render creates the seed layout; snapshot it so the counting launch and the
    # first timed frame see the same seeds
    step()
    seeds0 = rt.getSeeds()
    # counting launch (untimed): traversal node / triangle-test counts for the roofline
    rt.setCounting(True)
    rt.setSeeds(Wp, Hp, seeds0)
    rt.rayTrace(out, W, H, 0, kernel=kernel, tile=tile)
    cnt = rt.counters()
    rt.setCounting(False)
    # the whole frame's query counts: at N > 1 (strong scaling) every rank's counting launch
    # covers its own stripes, so the frame's totals are the sum over ranks (the roofline below
    # stays rank 0's: its tile's counts against its own kernel time)
    cnt_frame = {k: int(cnt.get(k, 0)) for k in ("rays_closest", "rays_shadow", "rays_skipped")}
    if dist and n_ranks > 1:
        v = torch.tensor([cnt_frame[k] for k in ("rays_closest", "rays_shadow", "rays_skipped")],
                         dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        cnt_frame = dict(zip(("rays_closest", "rays_shadow", "rays_skipped"), (int(x) for x in v.tolist())))
    chain = None
    if world == 1 and kernel == pt.RayTracer.KERNEL_TRIS and not args.linear:
        chain = critical_chain(rt, pt, W, H, Wp, Hp, seeds0, kernel)
    # the plain (timed) kernel's frame from seeds0, kept for the bit-exact check against the
    # reference kernel's CPU render of the same pixels (cpu_baseline)
    rt.setSeeds(Wp, Hp, seeds0)
    rt.rayTrace(out, W, H, 0, kernel=kernel, tile=tile)
    frame0 = out.cpu().numpy().copy() if world == 1 else None
    seeds_after0 = rt.getSeeds() if world == 1 else None
    rt.setSeeds(Wp, Hp, seeds0)

    # W warmup steps, then more (untimed) until the launch time has settled: the first
    # process on a freshly taken box has been seen running 4-17x slower for its first
    # seconds. At most 30 s / 40 extra steps; the count is reported (extra_warmup_steps).
    warm_ms = []
    for _ in range(args.warmup):
        step()
        warm_ms.append(rt.lastKernelMs())
    extra_warm = 0
    t_w = time.perf_counter()
    while True:
        want = (args.warmup > 0 and extra_warm < 40 and time.perf_counter() - t_w < 30.0
                and (len(warm_ms) < 2 or abs(warm_ms[-1] - warm_ms[-2]) > 0.03 * min(warm_ms[-1], warm_ms[-2])))
        if dist:  # one decision for all ranks: step() holds collectives
            w = torch.tensor([1 if want else 0], dtype=torch.int64, device=f"cuda:{device}")
            dist.all_reduce(w, op=dist.ReduceOp.MAX)
            want = bool(w.item())
        if not want:
            break
        step()
        warm_ms.append(rt.lastKernelMs())
        extra_warm += 1
    print(f"warmup kernel ms: {[round(x, 2) for x in warm_ms]}", file=sys.stderr)

    kernel_ms, split_ms = [], []
    # One GPU, whole frames: the K frames are enqueued back to back on the library's stream
    # (rt_render_async) and the host never waits between them, so a short frame's launch and host
    # work overlap the previous frame's kernels (bunny class: ~40 us of a 0.5-ms frame); each
    # frame is the same full render, its seeds carried on the device from the one before. The
    # per-frame kernel times for the roofline come from a synchronous pass after the timed one.
    pipelined = world == 1 and halo is None and comm is None and not frames_per_rank
    rays_warm = None  # the last warm frame's count (same view), reported beside the measured mean
    if pipelined:
        rays_warm = step()
        rt.counterTotals(reset=True)  # the timed frames' own counts accumulate on the device from here
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    for _ in range(args.steps):
        if pipelined:
            pnum = frame_no[0] if progressive else 0
            rt.rayTrace(out, W, H, pnum, kernel=kernel, tile=tile, sync=False)  # the library's own stream
            frame_no[0] += 1
        else:
            rays += step()
            kernel_ms.append(rt.lastKernelMs())
            split_ms.append(rt.lastKernelSplitMs())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    counted = None
    if pipelined:
        rt.synchronize()  # the render's own completion checks (guard words) for the last frame
        # every timed frame's own queries, summed on the device by the counter hand-back kernel
        # (raises if a defect guard fired in any of them)
        tot = rt.counterTotals(reset=True)
        if tot["renders"] != args.steps:
            raise RuntimeError(f"counter totals cover {tot['renders']} renders, {args.steps} were timed")
        rays = tot["rays_closest"] + tot["rays_shadow"]
        counted = {"rays_skipped": tot["rays_skipped"], "renders": tot["renders"]}
        for _ in range(min(args.steps, 5)):  # untimed: each frame's kernel time (HIP events)
            step()
            kernel_ms.append(rt.lastKernelMs())
            split_ms.append(rt.lastKernelSplitMs())
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    info = rt.renderInfo()
    # a frame right after a camera change (the reference restarts refinement on every arrow
    # key or drag, GlutCLWindow.cpp:229-279): wall clock including the host work of the new
    # schedule (cost probe, LPT order, pixel classes), against the next frame with the camera
    # unchanged
    cold = interactive_cost(rt, step, cam_setup, azimuth, device, dist)

    sharded = None
    if n_ranks > 1:
        sharded = verify_sharded(rt, pt, sc, ptdist, comm, dist, W, H, Wp, Hp, kernel, args.stripe, n_ranks, rank,
                                 device, out, frame_full if comm is not None else None, owner)

    if rank != 0:
        if comm is not None:
            comm.close()
        if dist:
            dist.destroy_process_group()
        return

    steps = args.steps
    mrays = rays / elapsed / 1e6
    ms_step = elapsed / steps * 1e3
    frame_ms = float(np.mean(kernel_ms))  # all of a frame's kernels (rank 0), HIP events
    # the dominant kernel's launches alone: the frame less the camera-ray candidate-list pre-pass
    pre_ms = float(np.mean([p for p, _ in split_ms]))
    k_ms = float(np.mean([m for _, m in split_ms]))
    rays_cnt = cnt["rays_closest"] + cnt["rays_shadow"]
    workload = workload_name(cfg, n_tris, W, H, sr, args.traversal, args.builder)
    pix = W * (len(ptdist.tile_rows(H, args.stripe, n_ranks, 0, owner)) if n_ranks > 1 else H)
    roofline = roofline_block(pt, kernel, cnt, args.traversal, pix, k_ms, workload, n_ranks, chain, rays_cnt,
                              frame_ms, pre_ms)

    cpu = gpu_linear = None
    if world == 1 and not args.no_cpu_baseline:
        print("cpu baseline", file=sys.stderr, flush=True)
        cpu = cpu_baseline(pt, sc, W, H, sr, S, seeds0, Wp, Hp, kernel, args.cpu_seconds,
                           verts if n_tris else None, idx if n_tris else None, frame0, seeds_after0)
        if kernel == pt.RayTracer.KERNEL_TRIS and not args.linear and not args.no_linear_leg:
            # every query tests every triangle: ~3 queries per pixel at sampleRate 1, ~4e11 tests/s
            # (r03: the dragon frame in 9.5 s); a leg past ~50 s (the Lucy class: ~1 h) is skipped
            est_s = 3.0 * W * H * n_tris / 4e11
            if est_s <= 50.0:
                print(f"gpu linear leg (~{est_s:.0f} s)", file=sys.stderr, flush=True)
                gpu_linear = gpu_linear_leg(rt, pt, W, H, Wp, Hp, seeds0, cpu)
            else:
                gpu_linear = {"skipped": f"~{est_s:.0f} s estimated for {W}x{H} x {n_tris} triangles per query"}

    frame_rays = cnt_frame["rays_closest"] + cnt_frame["rays_shadow"]
    traversed_share = (frame_rays - cnt_frame["rays_skipped"]) / max(frame_rays, 1)
    if counted is not None:  # the timed frames' own share (one GPU, pipelined frames)
        traversed_share = (rays - counted["rays_skipped"]) / max(rays, 1)
    line = {
        "metric": (METRIC_WEAK if frames_per_rank else METRIC) if cfg == "dragon" else CONFIG_METRIC.get(
            cfg, f"Mrays/sec + frames/sec, {cfg}"),
        "value": round(mrays, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "extra_warmup_steps": extra_warm,
        "ms_per_step": round(ms_step, 3),
        # one GPU: the timed frames enqueued back to back on one stream, no host wait between them
        "frames_pipelined": bool(pipelined),
        "frames_per_sec": round(steps * (world if frames_per_rank else 1) / elapsed, 4),
        # the same frames counting only the queries that ran a traversal (rank 0's counting
        # launch share; DESIGN.md §5: shadow rays answered without one are still rays)
        "mrays_traversed_per_sec": round(mrays * traversed_share, 2),
        "value_traversed": round(mrays * traversed_share, 2),
        "value_rule": ("value counts the reference's queries (closest-hit + shadow, equal to the oracle's counts) "
                       "of the timed frames themselves, summed on the device (rt_counter_totals); "
                       "value_traversed leaves out the shadow rays answered without a traversal (tmax <= tmin, or "
                       "cos(wi) <= 0, whose term rtcommon.h:93-95 drops after the visibility test)"),
        "rays_counted": ("device totals over the timed frames" if counted is not None
                         else "per frame, read after each timed step"),
        "higher_is_better": True,
        "scaling": "weak" if frames_per_rank else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": workload,
                   "W": W, "H": H, "spp": sr * sr, "n_tris": n_tris,
                   "parallelism": ((f"frames x{world} (one turntable view per rank)" if frames_per_rank
                                    else f"row-stripes({args.stripe}, {args.partition if owner is not None or comm else 'interleaved'})x{world}")
                                   + ((" + librtmi rt_comm (RCCL send/recv gather)" if comm is not None
                                       else " + rccl gather (torch.distributed)"
                                       if os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl"
                                       else " + gloo gather") if world > 1 else "")),
                   "rays_per_frame": int(rays / steps / (world if frames_per_rank else 1)),
                   # one untimed warm frame of the same view (seeds carried on, so each frame's count differs)
                   "rays_warm_frame": int(rays_warm) if rays_warm is not None else None,
                   # rays = the reference's queries (oracle-equal counts); shadow rays whose answer
                   # cannot change the pixel are answered without a traversal
                   "rays_traversed_per_frame": int(cnt_frame["rays_closest"] + cnt_frame["rays_shadow"]
                                                   - cnt_frame["rays_skipped"]),
                   "mesh": mesh_info},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if kernel == pt.RayTracer.KERNEL_TRIS and info:
        line["config"]["candidate_lists"] = {"on": bool(info["lists"]), "capacity_records": int(info["list_capacity"]),
                                             "records": int(info["list_records"]),
                                             "pixels_on_tree": int(info["list_pixels_tree"])}
        line["config"]["sample_split"] = {"chunks_per_pixel": int(info.get("split_chunks", 0)),
                                          "long_chains": int(info.get("pixels_long", 0))}
    line.update(cold)
    if comm_note:
        line["comm_note"] = comm_note
    if sharded is not None:
        line.update(sharded)
        if sharded["ranks"] != world:
            print(f"bench.py: {world} ranks launched but the communicator has {sharded['ranks']}", file=sys.stderr)
            sys.exit(3)
    if cpu is not None and "gpu_vs_reference_bit_exact" in cpu:
        line["gpu_vs_reference_bit_exact"] = cpu["gpu_vs_reference_bit_exact"]
        line["gpu_vs_reference_pixels"] = cpu["gpu_vs_reference_pixels"]
    if gpu_linear is not None:
        line["gpu_linear"] = gpu_linear
    print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist:
        dist.destroy_process_group()


def interactive_cost(rt, step, cam_setup, azimuth, device, dist):
    """Wall time of a step right after a 3-degree camera move (one arrow key: the schedule and,
    from sampleRate 4, the candidate lists are rebuilt), of the next step and of the one after
    (the view's steady state); max over ranks.  Restores the camera afterwards."""
    import torch

    def timed():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    res = {}
    for k, az in (("cold", azimuth + 3.0), ("restore", azimuth)):
        rt.setCameraSpherical(cam_setup["target"], cam_setup["elevation"], az, cam_setup["distance"])
        c_ms = timed()
        info = rt.renderInfo()
        s_ms = timed()  # below sampleRate 4 the second frame of a view builds the candidate lists
        w_ms = timed()
        if k == "cold":
            res = {"cold_frame_ms": c_ms, "second_frame_ms": s_ms, "warm_frame_ms": w_ms,
                   "cold_schedule_host_ms": info.get("schedule_host_ms", 0.0)}
    if dist:
        keys = ("cold_frame_ms", "second_frame_ms", "warm_frame_ms")
        t = torch.tensor([res[k] for k in keys], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        for i, k in enumerate(keys):
            res[k] = float(t[i])
    return {k: round(v, 3) for k, v in res.items()}


def verify_sharded(rt, pt, sc, ptdist, comm, dist, W, H, Wp, Hp, kernel, stripe, n_ranks, rank, device, out,
                   frame_full, owner=None):
    """The N > 1 line checks itself (collective; untimed, after the timed steps): every rank
    takes the same seed planes (the glibc rand() stream from its start), renders its stripes and
    the frame is gathered through the same path as the timed step (rt_comm_render, or the
    torch.distributed gather); rank 0 then renders the whole frame from the same seeds on its own
    GPU and compares the two bit for bit, and every rank's seed rows (gathered to rank 0) with
    the single render's.  Returns the fields for the line on rank 0."""
    import torch

    s0 = sc.default_seeds(Wp, Hp)
    rt.setSeeds(Wp, Hp, s0)
    if comm is not None:
        comm.reset_halo()
        comm.render(rt, frame_full, W, H, 0, kernel, stripe=stripe)
        gathered = frame_full.cpu().numpy().reshape(-1) if rank == 0 else None
        ranks = comm.count()
        owner = comm.last_partition()
    else:
        rt.rayTrace(out, W, H, 0, kernel=kernel, tile=(stripe, n_ranks, rank, owner))
        g = ptdist.gather_frame(out, H, W, stripe, owner=owner)
        gathered = g.cpu().numpy().reshape(-1) if rank == 0 else None
        ranks = dist.get_world_size()
    seeds = torch.from_numpy(rt.getSeeds().view(np.int32).copy())
    if dist.get_backend() == "nccl":
        seeds = seeds.to(f"cuda:{device}")
    bucket = [torch.empty_like(seeds) for _ in range(n_ranks)] if rank == 0 else None
    dist.gather(seeds, bucket, dst=0)
    if rank != 0:
        return None
    rt.setSeeds(Wp, Hp, s0)
    full = np.zeros(W * H * 4, np.float32)
    rt.rayTrace(full, W, H, 0, kernel=kernel)
    single = rt.getSeeds()
    seeds_ok = True
    plane = Wp * Hp
    for r in range(n_ranks):
        got = bucket[r].cpu().numpy().view(np.uint32)
        rows = ptdist.tile_rows(H, stripe, n_ranks, r, owner)
        sl = (rows[:, None] * Wp + np.arange(W)[None, :]).reshape(-1)
        seeds_ok &= bool(np.array_equal(got[sl], single[sl]) and np.array_equal(got[plane + sl], single[plane + sl]))
    return {"gathered_bit_exact": bool(np.array_equal(gathered.view(np.uint32), full.view(np.uint32))),
            "gathered_seeds_bit_exact": bool(seeds_ok), "ranks": int(ranks),
            "partition": ("owner map (rt_partition_stripes: probed stripe costs, LPT), rows per rank "
                          + str([len(ptdist.tile_rows(H, stripe, n_ranks, r, owner)) for r in range(n_ranks)])
                          if owner is not None else "interleaved stripes"),
            "gathered_check": "frame from the initial glibc rand() seeds gathered through the timed path == "
                              "rank 0's single-GPU render of the same seeds (bits), seed rows per rank likewise"}


def critical_chain(rt, pt, W, H, Wp, Hp, seeds0, kernel):
    """The frame's longest serial chain, timed with the chip to itself: a counting launch with
    per-pixel clocks (RT_PIXEL_STATS) finds the pixel that took longest, then the row holding it
    is rendered alone (tile = that row: 30 waves on 256 CUs), so the launch time is that chain's
    latency.  Its share of the frame time is the roofline's critical-path fraction."""
    import tempfile

    path = os.path.join(tempfile.gettempdir(), f"bench_pixel_stats_{os.getpid()}.bin")
    os.environ["RT_PIXEL_STATS"] = path
    try:
        rt.setCounting(True)
        rt.setSeeds(Wp, Hp, seeds0)
        out = np.zeros(W * H * 4, np.float32)
        rt.rayTrace(out, W, H, 0, kernel=kernel)
        rt.setCounting(False)
        st = np.fromfile(path, np.uint32).reshape(H, W, 8).astype(np.int64)
    finally:
        os.environ.pop("RT_PIXEL_STATS", None)
        if os.path.exists(path):
            os.remove(path)
    dur = (st[..., 1] - st[..., 0]) & 0xFFFFFFFF  # s_memrealtime ticks (100 MHz), low 32 bits
    y, x = np.unravel_index(int(np.argmax(dur)), dur.shape)
    row = np.zeros(W * 4, np.float32)
    best = 1e9
    for _ in range(2):
        rt.setSeeds(Wp, Hp, seeds0)
        rt.rayTrace(row, W, H, 0, kernel=kernel, tile=(1, H, int(y)))
        best = min(best, rt.lastKernelMs())
    return {"pixel": [int(x), int(y)], "queries": int(st[y, x, 2]), "steps": int(st[y, x, 3]),
            "in_frame_ms": round(float(dur[y, x]) / 1e5, 2), "alone_ms": round(best, 2)}


def roofline_block(pt, kernel, cnt, traversal, pix, k_ms, workload, n_ranks, chain, rays_cnt, frame_ms=None,
                   pre_ms=0.0):
    """The dominant kernel against the HBM roofline, SURVEY.md §8(d): algorithmic bytes per launch =
    nodes visited x 64 B (the compressed node) + triangle tests x 36 B (the reference's triangle_t)
    + 32 B of pixel I/O per pixel, from the device counters of a counting launch of the same frame,
    over the live (HIP-event) kernel time, against 8 TB/s.  `traffic` = the PMC HBM bytes per launch
    (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) of the committed profile of this workload.

    `fractions` adds every resource the kernel could be bound by, each <= 1, each recomputable from
    the committed profile alone (its own kernel time and clock, profiles/pmc_roofline.json <-
    profiles/<run>/pmc_summary.json):
      hbm_pmc        PMC HBM bytes / the profiled launch time, vs 8 TB/s;
      valu_issue     SQ_INSTS_VALU wave-instructions, 2 cycles each on 1024 SIMD-32s, over the
                     profiled kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs);
      salu_issue     SQ_INSTS_SALU on 256 scalar units over those cycles;
      vmem_address   TA busy cycles / those cycles (the gather address path);
    and, measured live: record_gather (node + triangle records per second vs the best random 64-B
    record rate measured on a table of the scene's size, profiles/gather_ceiling.json) and
    critical_path (the frame's longest pixel chain rendered alone / the frame time).
    `limiter` = the largest of them."""
    is_tris = kernel == pt.RayTracer.KERNEL_TRIS
    records = (cnt["nodes_visited"] + cnt["tris_tested"]) if is_tris else 0
    alg_bytes = (cnt["nodes_visited"] * NODE_BYTES[traversal] + cnt["tris_tested"] * TRI_BYTES_8D
                 if is_tris else 0) + pix * PIXEL_BYTES
    fetched = (cnt["nodes_visited"] * NODE_BYTES[traversal] + cnt["tris_tested"] * TRI_BYTES[traversal]
               if is_tris else 0) + pix * PIXEL_BYTES
    sec = k_ms * 1e-3
    fr = {}
    pm = None
    tp = ROOT / "profiles" / "pmc_roofline.json"
    if tp.exists() and n_ranks == 1:
        pm = json.loads(tp.read_text()).get(workload)
    if pm:
        sec_p = pm["avg_kernel_ms_rocprof"] * 1e-3
        f_ghz = pm["effective_clock_ghz"]
        fr["hbm_pmc"] = {"achieved": pm["hbm_bytes_per_launch"] / sec_p / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
        fr["valu_issue"] = {"achieved": pm["valu_issue_frac"] * N_SIMD * f_ghz / 2, "peak": N_SIMD * f_ghz / 2,
                            "unit": "G wave-instr/s", "frac_exact": pm["valu_issue_frac"]}
        if pm.get("salu_issue_frac"):
            fr["salu_issue"] = {"achieved": pm["salu_issue_frac"] * N_CU * f_ghz, "peak": N_CU * f_ghz,
                                "unit": "G instr/s", "frac_exact": pm["salu_issue_frac"]}
        if pm.get("ta_busy_frac"):
            fr["vmem_address"] = {"achieved": pm["ta_busy_frac"] * f_ghz, "peak": f_ghz,
                                  "unit": "G busy cycles/s per TA", "frac_exact": pm["ta_busy_frac"]}
        for v in fr.values():
            v["time_base"] = f"profiled launch {pm['avg_kernel_ms_rocprof']:.3f} ms at {f_ghz:.3f} GHz ({pm['source']})"
    gp = ROOT / "profiles" / "gather_ceiling.json"
    if is_tris and gp.exists() and traversal != "linear":
        g = json.loads(gp.read_text())
        fr["record_gather"] = {"achieved": records / sec / 1e9, "peak": g["best_grec_per_s"], "unit": "G records/s",
                               "ceiling": g["source"], "time_base": "live kernel time"}
    if chain:
        fr["critical_path"] = {"achieved": chain["alone_ms"], "peak": round(frame_ms or k_ms, 3),
                               "unit": "ms (chain alone / frame)", "time_base": "live", **chain}
    for v in fr.values():
        v["frac"] = round(v.pop("frac_exact", v["achieved"] / v["peak"]), 4)
        v["achieved"] = round(v["achieved"], 3)
        v["peak"] = round(v["peak"], 3)
    limiter = max(fr, key=lambda k: fr[k]["frac"]) if fr else None
    alg_gbps = alg_bytes / sec / 1e9
    out = {"bound": "hbm", "achieved": round(alg_gbps, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(alg_gbps / HBM_PEAK_GBS, 4),
           # the same algorithmic bytes over the committed steady-state profile's kernel time
           # (profiles/<run>/pmc_summary.json: rocprofv3 over the steady-state frames only)
           "frac_profiled": (round(pm["algorithmic_frac_of_hbm_peak"], 4)
                             if pm and pm.get("algorithmic_frac_of_hbm_peak") else None),
           "traffic": pm["hbm_bytes_per_launch"] if pm else None,
           "traffic_unit": "HBM bytes/launch (2*FETCH_SIZE + WRITE_SIZE, PMC)" if pm else None,
           "traffic_source": pm["source"] if pm else None,
           "achieved_def": "SURVEY 8(d) algorithmic bytes per launch (nodes x 64 B + triangle tests x 36 B + pixels x "
                           "32 B, device counters) / live HIP-event kernel time",
           "algorithmic_bytes_per_launch": int(alg_bytes),
           "fetched_record_bytes_per_launch": int(fetched),
           "limiter": limiter,
           "fractions": fr,
           "kernel": (f"k_tris<{traversal.upper()}>" if is_tris else "k_spheres"),
           "kernel_ms": round(k_ms, 3),
           "prepass_ms": round(pre_ms, 3),
           "frame_kernels_ms": round(frame_ms or k_ms, 3)}
    if is_tris:
        out["nodes_per_ray"] = round(cnt["nodes_visited"] / max(rays_cnt, 1), 2)
        out["tris_per_ray"] = round(cnt["tris_tested"] / max(rays_cnt, 1), 2)
    if cnt.get("lane_slots"):
        out["simd_efficiency"] = round((cnt["nodes_visited"] + cnt["leaves_visited"]) / cnt["lane_slots"], 4)
    return out


def host_cpus():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota (a GPU box's
    share is a quota over a larger machine), with nproc and the CPU model for the report."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": min(aff, quota) if quota else aff, "nproc": os.cpu_count(), "affinity": aff,
            "cgroup_quota_cpus": quota, "cpu_model": model}


TRAVERSAL_NAMES = {"bvh": "4-wide compressed BVH", "bvh4f": "4-wide BVH", "linear": "linear (reference)"}


def workload_name(cfg, n_tris, W, H, sr, traversal, builder="host"):
    name = _workload_name(cfg, n_tris, W, H, sr, traversal)
    return name + (" (GPU-built BVH)" if (builder == "gpu" and n_tris) else "")


def _workload_name(cfg, n_tris, W, H, sr, traversal):
    if n_tris and cfg.startswith("PLY "):
        return (f"raytrace_tris {cfg[4:]} ({n_tris} tris, normalised), {W}x{H}, sampleRate {sr} "
                f"({sr * sr} spp, one launch), maxDepth 6, {TRAVERSAL_NAMES[traversal]} traversal")
    if n_tris:
        return (f"raytrace_tris {cfg}-class synthetic mesh {n_tris} tris, {W}x{H}, sampleRate {sr} "
                f"({sr * sr} spp, one launch), maxDepth 6, {TRAVERSAL_NAMES[traversal]} traversal")
    return f"raytrace spheres main.cpp scene {W}x{H}, sampleRate {sr}, progressive frames (row-shifted seeds)"


def cpu_baseline(pt, sc, W, H, sr, S, seeds, Wp, Hp, kernel, target_s, verts, idx, frame0, seeds_after0):
    """The reference's own kernel (clrt/ocl/raytracer.cl compiled for x86-64 from its source,
    oracle/_ref/libptref.so: kind "reference") on the host cores, on a bounded sample of the
    same frame: whole pixels (all sr*sr samples) strided over the frame.  Rays are counted by
    the oracle (oracle/pt_oracle.c, the bit-identical restatement) on the same pixels, untimed.
    Checks: the two CPU renders agree bit for bit, and the GPU's plain-kernel frame from the same
    seeds (frame0, seeds_after0) equals the reference on every sampled pixel and seed slot
    (gpu_vs_reference_bit_exact).  Without oracle/_ref (built in the container from
    /root/reference) the oracle itself is timed (kind "port")."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from oracle import LIBREF, Oracle, Reference

    orc = Oracle()
    ref = Reference(build_if_missing=False) if LIBREF.exists() else None
    hc = host_cpus()
    threads = hc["threads"]
    cam = sc.camera_spherical(W, **(sc.PLY_CAMERA if kernel == 2 else sc.MAIN_CAMERA))
    out = np.zeros(W * H * 4, np.float32)
    out_o = np.zeros_like(out)
    sd = seeds.copy()
    sd_o = seeds.copy()
    closest = shadow = 0
    dt = 0.0
    batches = 0
    sampled = []
    if kernel != 2:  # sphere scene: one full frame (a few seconds on the host cores)
        t0 = time.perf_counter()
        if ref is not None:
            ref.launch(0, out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, nthreads=threads)
        else:
            orc.render_spheres(out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, nthreads=threads)
        dt = time.perf_counter() - t0
        closest, shadow = orc.render_spheres(out_o, cam, S, W, H, Wp, Hp, sr, 6, 0, sd_o, nthreads=threads)
        batches = 1
        sampled = np.arange(W * H, dtype=np.int64)
    # batches of whole pixels, strided over the frame with a different phase per batch, until
    # the timed renders have taken target_s seconds (bounded)
    n_px = threads
    stride = W * H // n_px
    while kernel == 2 and dt < target_s and batches < 64:
        phase = (batches * 7919 + stride // 2) % stride
        pix = (np.arange(n_px, dtype=np.uint64) * stride + phase).astype(np.uint32)
        t0 = time.perf_counter()
        if ref is not None:
            ref.launch_pixels(2, out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, pix, verts, idx, nthreads=threads)
        else:
            orc.render_tris(out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, verts, idx, pixels=pix, nthreads=threads)
        dt += time.perf_counter() - t0
        c, s = orc.render_tris(out_o, cam, S, W, H, Wp, Hp, sr, 6, 0, sd_o, verts, idx, pixels=pix, nthreads=threads)
        closest += c
        shadow += s
        batches += 1
        sampled.append(pix.astype(np.int64))
    if kernel == 2:
        sampled = np.unique(np.concatenate(sampled))
    exact = True
    if ref is not None:
        exact = bool(np.array_equal(out.view(np.uint32), out_o.view(np.uint32)) and np.array_equal(sd, sd_o))
    rays = closest + shadow
    if kernel == 2:
        sample = (f"{batches * n_px} whole pixels x {sr * sr} samples ({batches} strided batches over the frame), "
                  "linear traversal (the reference algorithm)")
    else:
        sample = f"full {W}x{H} frame"
    res = {"value": round(rays / dt / 1e6, 6), "unit": "Mrays/s", "cores": threads,
           "kind": "reference" if ref is not None else "port", "sample": sample, "seconds": round(dt, 2),
           "rays": int(rays), **{k: v for k, v in hc.items() if k != "threads"}}
    if ref is not None:
        res["source"] = "clrt/ocl/raytracer.cl compiled for x86-64 (oracle/Makefile ref), one work-item per pixel"
        res["bit_exact_vs_oracle"] = exact
    if frame0 is not None:
        # the GPU frame (plain kernel, same seeds) against the CPU render, on the sampled pixels
        # and their seed slots (both planes; raytrace_tris reads unshifted slots, the sphere
        # frame is progression 0, so slot = y * Wpad + x either way)
        g = frame0.reshape(-1, 4)[sampled].view(np.uint32)
        r = out.reshape(-1, 4)[sampled].view(np.uint32)
        slots = (sampled // W) * Wp + (sampled % W)
        plane = Wp * Hp
        ok = (np.array_equal(g, r) and np.array_equal(seeds_after0[slots], sd[slots])
              and np.array_equal(seeds_after0[plane + slots], sd[plane + slots]))
        res["gpu_vs_reference_bit_exact"] = bool(ok)
        res["gpu_vs_reference_pixels"] = int(len(sampled))
    return res


def gpu_linear_leg(rt, pt, W, H, Wp, Hp, seeds0, cpu):
    """The same algorithm as the CPU baseline on the GPU: the reference's linear
    loop over every triangle (RT_TRAVERSAL_LINEAR) on the whole frame at sampleRate 1 (a 256-spp
    linear frame would take tens of minutes; a partial frame is bound by its longest pixel
    chain rather than by throughput)."""
    sr0 = rt.getSampleRate()
    rt.setTraversal("linear")
    rt.setSampleRate(1)
    buf = np.zeros(W * H * 4, np.float32)
    rt.setSeeds(Wp, Hp, seeds0)
    rt.rayTrace(buf, W, H, 0, kernel=2)
    ms = rt.lastKernelMs()
    c = rt.counters()
    rt.setTraversal("bvh")
    rt.setSampleRate(sr0)
    rt.setSeeds(Wp, Hp, seeds0)
    rays = c["rays_closest"] + c["rays_shadow"]
    v = rays / (ms * 1e-3) / 1e6
    res = {"value": round(v, 4), "unit": "Mrays/s", "kernel_ms": round(ms, 1), "rays": int(rays),
           "sample": f"the full {W}x{H} frame at sampleRate 1, linear traversal (every triangle per query)"}
    if cpu and cpu.get("value"):
        res["vs_cpu_baseline"] = round(v / cpu["value"], 2)
    return res


if __name__ == "__main__":
    main()
