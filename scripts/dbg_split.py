import os, sys
sys.path.insert(0, "/root/repo")
os.environ["RT_SPLIT"] = "1"
os.environ["RT_DEBUG_LAUNCH"] = "1"
import numpy as np
import ptload
pt = ptload.load()
sc = pt.scenes
W, H, sr = 72, 40, 2
Wp, Hp = sc.padded_dims(W, H)
verts, idx = sc.make_mesh(20_000)
rt = pt.RayTracer(0)
rt.setSpheres(sc.ply_scene()); rt.setCamera(sc.camera_spherical(W, **sc.PLY_CAMERA)); rt.setSampleRate(sr); rt.setMaxPathDepth(6); rt.setMesh(verts, idx)
rt.setSeeds(Wp, Hp, sc.default_seeds(Wp, Hp, skip=3))
got = np.zeros(W * H * 4, np.float32)
rt.rayTrace(got, W, H, 0, kernel=2)
print(rt.renderInfo(), flush=True)
