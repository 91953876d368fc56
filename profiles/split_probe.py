import sys, json
sys.path.insert(0, '/root/repo')
import torch, ptload
pt = ptload.load(); sc = pt.scenes
W, H, sr = 1920, 1080, 16
rt = pt.RayTracer(0)
rt.setSpheres(sc.ply_scene()); c = sc.PLY_CAMERA
rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
rt.setSampleRate(sr); rt.setMaxPathDepth(6); rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
out = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda:0")
for tile in ((8, 8, 0), (8, 8, 0), (8, 2, 0)):
    rt.rayTrace(out, W, H, 0, kernel=2, tile=tile)
    print(tile, round(rt.lastKernelMs(), 2), [round(x, 2) for x in rt.lastKernelSplitMs()], flush=True)
