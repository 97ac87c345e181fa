import sys, os
sys.path.insert(0, "simple-path-tracer_amd")
import faulthandler; faulthandler.enable()
import sptr
r = sptr.Renderer(0)
p0, p1 = int(os.environ.get("P0", 60)), int(os.environ.get("P1", 120))
sptr.setup_default(r, "sphere_mesh", p0, p1)
W, H = 160, 96
cam = sptr.camera_lookat(aspect=W / H)
for mode in (int(a) for a in sys.argv[1:]):
    r.set_launch_mode(mode)
    for i in range(3):
        print("mode", mode, "call", i, flush=True)
        st = r.render(cam, W, H, spp=int(os.environ.get("SPP", 16)), frame_begin=1)
        print("  ok", st.waves, st.rays_closest, flush=True)
