#!/usr/bin/env python3
"""Benchmark: Mrays/s + frames/s of raytrace_tris on the dragon-class config.

Workload (BASELINE.json configs[3], the metric's config): 871,414-triangle
synthetic mesh (dragon class), 1920x1080, sampleRate 16 (256 spp, one launch,
progression 0), maxDepth 6, plymain.cpp lights and camera, BVH traversal.
One step = one full frame: every rank renders its interleaved row stripes (rt_tile) and,
for N > 1, the frame is gathered to rank 0 over RCCL (torch.distributed "nccl").
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
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2 (per XCD, 32 MiB aggregate) ~34.5 TB/s
NODE_BYTES = {"bvh": 64, "bvh4f": 112, "linear": 0}  # bytes read per node visit, csrc/rt_internal.h + rt_quant.h
# bytes read per triangle test: the whole 48-B record (one-record steps of the compressed traversal), else
# v0+orig (16), e1 (12), e2 (12); csrc/rt_internal.h
TRI_BYTES = {"bvh": 48, "bvh4f": 40, "linear": 40}
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
    ap.add_argument("--scaling", default="auto", choices=["auto", "strong", "weak"],
                    help="N > 1: strong = one frame split into row-stripe tiles across ranks; weak = one full "
                         "frame per rank (turntable views 3 degrees apart), frames gathered to rank 0. auto: weak "
                         "for the dragon config (its 256-spp pixels are serial chains: DESIGN.md), else strong")
    ap.add_argument("--linear", action="store_true", help="reference linear traversal instead of the BVH")
    ap.add_argument("--traversal", default="bvh", choices=["bvh", "bvh4f", "linear"],
                    help="bvh: 4-wide compressed BVH (default); bvh4f: full-precision nodes; linear: the reference loop")
    ap.add_argument("--builder", default="host", choices=["host", "gpu"],
                    help="BVH builder: host binned SAH (default) or the GPU LBVH build")
    ap.add_argument("--ply", default=None, help="render this PLY mesh (normalised, SURVEY §8d) instead of "
                    "the synthetic mesh of the config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
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

    scaling = args.scaling
    if scaling == "auto":
        scaling = "weak" if (cfg == "dragon" and world > 1) else "strong"
    frames_per_rank = world > 1 and scaling == "weak"

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
    tile = (args.stripe, n_ranks, rank) if n_ranks > 1 else None
    rows = ptdist.max_tile_rows(H, args.stripe, n_ranks) if n_ranks > 1 else H
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

    def step():
        p = frame_no[0] if progressive else 0
        if halo is not None:
            ptdist.exchange_seed_rows(halo.plan(p), pack, rt.unpackSeedRows, Wp, device=halo_dev)
        rt.rayTrace(out, W, H, p, kernel=kernel, tile=tile, halo=halo is not None)
        if halo is not None:
            halo.commit(p)
        frame_no[0] += 1
        c = rt.counters()
        if n_ranks > 1:
            ptdist.gather_frame(out, H, W, args.stripe)
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

    kernel_ms = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    for _ in range(args.steps):
        rays += step()
        kernel_ms.append(rt.lastKernelMs())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    steps = args.steps
    mrays = rays / elapsed / 1e6
    ms_step = elapsed / steps * 1e3
    # roofline of the dominant kernel, per launch (rank 0's launches)
    k_ms = float(np.mean(kernel_ms))
    rays_cnt = cnt["rays_closest"] + cnt["rays_shadow"]
    pix = W * (len(ptdist.tile_rows(H, args.stripe, n_ranks, 0)) if n_ranks > 1 else H)
    if kernel == pt.RayTracer.KERNEL_TRIS:
        alg_bytes = cnt["nodes_visited"] * NODE_BYTES[args.traversal] + cnt["tris_tested"] * TRI_BYTES[args.traversal] + pix * PIXEL_BYTES
    else:
        alg_bytes = pix * PIXEL_BYTES
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                # the BVH + triangles are L2/MALL-resident (PMC traffic << algorithmic bytes), so
                # the algorithmic rate is also stated against the aggregate L2 bandwidth
                "l2_peak": L2_PEAK_GBS, "frac_of_l2": round(achieved / L2_PEAK_GBS, 4),
                "kernel": f"k_tris<{args.traversal.upper()}>" if kernel == 2 else "k_spheres",
                "kernel_ms": round(k_ms, 3), "algorithmic_bytes_per_launch": int(alg_bytes),
                "nodes_per_ray": round(cnt["nodes_visited"] / max(rays_cnt, 1), 2),
                "tris_per_ray": round(cnt["tris_tested"] / max(rays_cnt, 1), 2)}
    if cnt.get("lane_slots"):
        # share of lanes doing a node or leaf step per traversal round (resumable BVH queries)
        roofline["simd_efficiency"] = round((cnt["nodes_visited"] + cnt["leaves_visited"]) / cnt["lane_slots"], 4)
    if cnt.get("clocks_total"):
        # share of the waves' time spent in traversal rounds (counting launch, s_memtime)
        roofline["traversal_time_frac"] = round(cnt["clocks_traversal"] / cnt["clocks_total"], 4)
        roofline["shade_time_frac"] = round(cnt.get("clocks_shade", 0) / cnt["clocks_total"], 4)

    # HBM traffic per launch from the PMC passes (profiles/run_profile.sh + summarize_pmc.py),
    # when they were taken on this exact workload and kernel variant
    tp = ROOT / "profiles" / "pmc_traffic.json"
    workload = workload_name(cfg, n_tris, W, H, sr, args.traversal, args.builder)
    if tp.exists() and kernel == pt.RayTracer.KERNEL_TRIS and not args.linear and n_ranks == 1:
        t = json.loads(tp.read_text())
        if t.get("workload") == workload:
            roofline["traffic"] = t["hbm_bytes_per_launch"]
            roofline["traffic_unit"] = "bytes/launch (2*FETCH_SIZE + WRITE_SIZE)"
            roofline["traffic_source"] = t["source"]

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(pt, sc, cfg, W, H, sr, S, seeds0, Wp, Hp, kernel, args.cpu_seconds,
                           verts if n_tris else None, idx if n_tris else None)

    line = {
        "metric": METRIC,
        "value": round(mrays, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "extra_warmup_steps": extra_warm,
        "ms_per_step": round(ms_step, 3),
        "frames_per_sec": round(steps * (world if frames_per_rank else 1) / elapsed, 4),
        # the same frames counting only the queries that ran a traversal (rank 0's counting
        # launch share; DESIGN.md §5: shadow rays answered without one are still rays)
        "mrays_traversed_per_sec": round(mrays * (rays_cnt - cnt.get("rays_skipped", 0)) / max(rays_cnt, 1), 2),
        "higher_is_better": True,
        "scaling": "weak" if frames_per_rank else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": workload,
                   "W": W, "H": H, "spp": sr * sr, "n_tris": n_tris,
                   "parallelism": ((f"frames x{world} (one turntable view per rank)" if frames_per_rank
                                    else f"row-stripes({args.stripe})x{world}")
                                   + ((" + rccl gather" if os.environ.get("BENCH_DIST_BACKEND", "nccl") == "nccl"
                                       else " + gloo gather") if world > 1 else "")),
                   "rays_per_frame": int(rays / steps / (world if frames_per_rank else 1)),
                   # rays = the reference's queries (oracle-equal counts); shadow rays whose answer
                   # cannot change the pixel are answered without a traversal
                   "rays_traversed_per_frame": int(rays_cnt - cnt.get("rays_skipped", 0)),
                   "mesh": mesh_info},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


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


def cpu_baseline(pt, sc, cfg, W, H, sr, S, seeds, Wp, Hp, kernel, target_s, verts, idx):
    """The reference's own kernel (clrt/ocl/raytracer.cl compiled for x86-64 from its source,
    oracle/_ref/libptref.so: kind "reference") on the host cores, on a bounded sample of the
    same frame: whole pixels (all sr*sr samples) strided over the frame.  Rays are counted by
    the oracle (oracle/pt_oracle.c, the bit-identical restatement) on the same pixels, untimed,
    and the two renders of the sample are compared bit for bit.  Without oracle/_ref (it is
    built in the container from /root/reference), the oracle itself is timed (kind "port")."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from oracle import LIBREF, Oracle, Reference

    orc = Oracle()
    ref = Reference(build_if_missing=False) if LIBREF.exists() else None
    threads = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))
    cam = sc.camera_spherical(W, **(sc.PLY_CAMERA if kernel == 2 else sc.MAIN_CAMERA))
    out = np.zeros(W * H * 4, np.float32)
    out_o = np.zeros_like(out)
    sd = seeds.copy()
    sd_o = seeds.copy()
    closest = shadow = 0
    dt = 0.0
    batches = 0
    exact = True
    # batches of whole pixels, strided over the frame with a different phase per batch, until
    # the timed renders have taken target_s seconds (bounded)
    if kernel != 2:  # sphere scene: one full frame (a few seconds on the host cores)
        t0 = time.perf_counter()
        if ref is not None:
            ref.launch(0, out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, nthreads=threads)
        else:
            orc.render_spheres(out, cam, S, W, H, Wp, Hp, sr, 6, 0, sd, nthreads=threads)
        dt = time.perf_counter() - t0
        closest, shadow = orc.render_spheres(out_o, cam, S, W, H, Wp, Hp, sr, 6, 0, sd_o, nthreads=threads)
        batches = 1
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
           "rays": int(rays)}
    if ref is not None:
        res["source"] = "clrt/ocl/raytracer.cl compiled for x86-64 (oracle/Makefile ref), one work-item per pixel"
        res["bit_exact_vs_oracle"] = exact
    return res


if __name__ == "__main__":
    main()
