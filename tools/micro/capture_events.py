"""Run the stream-capture state probe (capture_events.hip) against torch's libamdhip64 (--torch) or
ROCm's.  usage: python tools/micro/capture_events.py [--torch] [iters] [--topo N]
Without --topo: the shared-event probe (probe_run), then each capture topology in a child process
(a topology that crashes the runtime must not take the others with it)."""
import ctypes
import os
import subprocess
import sys

if "--torch" in sys.argv:
    import torch  # noqa: F401  (loads torch's libamdhip64 first; the probe then binds to it)
    torch.cuda.init()
nums = [a for a in sys.argv[1:] if a.isdigit()]
iters = int(nums[0]) if nums else 4
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcapture_events.so"))
if "--topo" in sys.argv:
    topo = int(sys.argv[sys.argv.index("--topo") + 1])
    sys.exit(min(lib.probe_topo(topo, iters), 100))
with open("/proc/self/maps") as fh:
    print(sorted({l.split()[-1] for l in fh if "libamdhip64" in l}))
for mode in (0, 1):
    sys.stdout.flush()
    rc = lib.probe_run(mode, iters, 1 if iters <= 2 else 0)
    sys.stdout.flush()
    print("mode", mode, "stale", rc)
for topo in (1, 2, 3, 4):
    args = [sys.executable, "-u", __file__, str(iters), "--topo", str(topo)] + (["--torch"] if "--torch" in sys.argv else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=60)
    print(r.stdout[-3000:])
    print("topo", topo, "exit code", r.returncode, r.stderr[-300:] if r.returncode else "")
    sys.stdout.flush()
