"""Run the graph event-node probe (graph_events.hip) under torch's HIP runtime (--torch) or ROCm's."""
import ctypes
import os
import sys

if "--torch" in sys.argv:
    import torch  # noqa: F401  (torch's libamdhip64 first; the probe binds to it)
    torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgraph_events.so"))
sys.stdout.flush()
rc = lib.probe_graph_events()
sys.stdout.flush()
print("rc", rc)
