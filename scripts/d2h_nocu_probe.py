"""Device -> host word copies without compute units?  Copies 256 MiB in 4 MiB chunks
from device memory into pinned host memory on a side stream, with each hipMemcpyKind
(D2H = 2, Default = 4, DeviceToDeviceNoCU = 1024 onto the host buffer's device alias),
while a GEMM loop keeps the CUs busy on the default stream; prints the copy rate and
checks the bytes.  Run under rocprofv3 --kernel-trace --stats: a blit copy shows up as
__amd_rocclr_copyBuffer kernels, an SDMA copy does not."""
import ctypes as C
import time

import torch

hip = C.CDLL("libamdhip64.so")
torch.cuda.set_device(0)
n = 1 << 20                       # words per chunk
chunks = 64
dev = torch.randint(0, 2**31 - 1, (chunks * n,), dtype=torch.int32, device="cuda")
host = torch.zeros(chunks * n, dtype=torch.int32).pin_memory()
hptr = C.c_void_p(host.data_ptr())
dalias = C.c_void_p()
rc = hip.hipHostGetDevicePointer(C.byref(dalias), hptr, 0)
print("hipHostGetDevicePointer rc", rc, "alias == host ptr:", dalias.value == hptr.value)
side = torch.cuda.Stream()
s = C.c_void_p(side.cuda_stream)
a = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()
for kind, dst in ((2, hptr.value), (4, hptr.value), (1024, dalias.value)):
    for busy in (False, True):
        host.zero_()
        torch.cuda.synchronize()
        if busy:
            for _ in range(30):
                a = a @ a.T * 1e-4
        t0 = time.perf_counter()
        err = 0
        for ci in range(chunks):
            err |= hip.hipMemcpyAsync(C.c_void_p(dst + ci * n * 4), C.c_void_p(dev.data_ptr() + ci * n * 4),
                                      C.c_size_t(n * 4), C.c_int(kind), s)
        side.synchronize()
        dt = time.perf_counter() - t0
        ok = torch.equal(host[::4099], dev[::4099].cpu())
        print(f"kind={kind:5d} busy={busy}: rc={err} {chunks * n * 4 / dt / 1e9:6.1f} GB/s  bytes ok={ok}")
        torch.cuda.synchronize()
