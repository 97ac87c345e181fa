"""Render fixed frames with the library SPTR_LIB names and dump the accumulation bits, for comparing two
builds (e.g. a kernel variant against the default build): python tools/micro/render_dump.py out.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "simple-path-tracer_amd"))
import sptr  # noqa: E402
import workloads  # noqa: E402

r = sptr.Renderer(0)
out = {}
for name, scene, p0, p1, W, H, S in (("mesh300", "sphere_mesh", 300, 600, 160, 120, 16),
                                     ("mesh60", "sphere_mesh", 60, 120, 128, 96, 8)):
    sptr.setup_default(r, scene, p0, p1)
    cam = sptr.camera_lookat(aspect=W / H)
    st = r.render(cam, W, H, spp=S)
    out[name] = r.read_accum().view(np.uint32).copy()
    out[name + "_counts"] = np.array([st.rays_closest, st.rays_shadow], np.uint64)
for name, W, H, S in (("c2", 320, 180, 32), ("c3", 320, 180, 32), ("c5", 320, 180, 8)):
    wl = workloads.WORKLOADS[name]
    workloads.setup(r, wl)
    cam = workloads.camera(wl)
    st = r.render(cam, W, H, spp=S)
    out[name] = r.read_accum().view(np.uint32).copy()
    out[name + "_counts"] = np.array([st.rays_closest, st.rays_shadow], np.uint64)
np.savez(sys.argv[1], **out)
print("dumped", sys.argv[1], {k: v.shape for k, v in out.items()})
