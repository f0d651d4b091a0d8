"""H2D / D2H link rate on this box: pageable vs page-locked host memory (torch copies, 1 GB)."""
import time

import torch


def rate(src, dst, reps=5):
    dst.copy_(src, non_blocking=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=False)
    torch.cuda.synchronize()
    return src.numel() * reps / (time.perf_counter() - t) / 1e9


n = 1 << 30
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
for pinned in (False, True):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h.fill_(1)
    print(f"{'pinned' if pinned else 'pageable'}: H2D {rate(h, dev):.1f} GB/s, D2H {rate(dev, h):.1f} GB/s", flush=True)
