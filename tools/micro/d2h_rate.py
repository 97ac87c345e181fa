"""D2H copy rate of a 1080p RGB8 frame (6.2 MB) into pinned and pageable host memory (torch's copy path)."""
import time

import torch

n = 1920 * 1080 * 3
src = torch.empty(n, dtype=torch.uint8, device="cuda")
for name, dst in (("pinned", torch.empty(n, dtype=torch.uint8, pin_memory=True)), ("pageable", torch.empty(n, dtype=torch.uint8))):
    for _ in range(5):
        dst.copy_(src)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        dst.copy_(src)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 100
    print(f"{name}: {dt * 1e3:.3f} ms per copy, {n / dt / 1e9:.1f} GB/s")
