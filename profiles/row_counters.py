import sys, json
sys.path.insert(0, "/root/repo")
import torch, ptload
pt = ptload.load(); sc = pt.scenes
rt = pt.RayTracer(0)
rt.setSpheres(sc.ply_scene()); c = sc.PLY_CAMERA
rt.setCameraSpherical(c["target"], c["elevation"], c["azimuth"], c["distance"])
rt.setSampleRate(16); rt.setMaxPathDepth(6)
rt.setMesh(*sc.make_mesh(sc.MESH_CONFIGS["dragon"]))
out = torch.zeros(1920*1080*4, dtype=torch.float32, device="cuda:0")
for row in (81, 486, 918):
    rt.setCounting(True)
    rt.rayTrace(out, 1920, 1080, 0, kernel=2, tile=(1, 1080, row))
    print(row, rt.lastKernelMs(), json.dumps(rt.counters()), flush=True)
    rt.setCounting(False)
