"""D2H copy path probe: pinned-host <- device copies of 4 MiB chunks on a side
stream while a compute kernel runs; prints the achieved copy rate.  Run under
rocprofv3 --kernel-trace to see whether the runtime used blit kernels."""
import time
import torch

torch.cuda.set_device(0)
n = 1 << 20                                     # words per chunk (SHUF_CHUNK)
chunks = 64
dev = torch.randint(0, 2**31 - 1, (chunks * n,), dtype=torch.int32, device="cuda")
host = torch.empty(chunks * n, dtype=torch.int32).pin_memory()
side = torch.cuda.Stream()
a = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()
for busy in (False, True):
    if busy:
        for _ in range(20):
            a = a @ a.T * 1e-4                  # keep the CUs busy on the default stream
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        for c in range(chunks):
            host[c * n:(c + 1) * n].copy_(dev[c * n:(c + 1) * n], non_blocking=True)
    side.synchronize()
    dt = time.perf_counter() - t0
    print(f"busy={busy} {chunks * n * 4 / dt / 1e9:.1f} GB/s over {chunks * 4} MiB")
torch.cuda.synchronize()
assert torch.equal(host[:16], dev[:16].cpu())
