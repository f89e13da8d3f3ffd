"""Data-parallel plumbing for libbppo.

One process per GPU. Each rank owns its own envs (global env index
rank * N + i, seeds `seed + rank * N + i`) and its own main-RNG ChaCha stream
(stream id = rank).  The only exchange step is the SUM all-reduce of the flat
gradient (+ metric partials) once per minibatch; libbppo divides by world
size before clip + Adam, so all ranks apply the same step and stay in sync.

`make_allreduce` builds the callback libbppo invokes (bppo_set_allreduce):
  mode "device": the buffer is HIP device memory; all-reduce a torch CUDA
                 tensor (backend "nccl" = RCCL over xGMI) staged by D2D copy;
  mode "device_async": stream-ordered (bppo_set_allreduce_async): D2D copy,
                 RCCL all-reduce and D2D copy all enqueued on the context's
                 stream (torch.cuda.ExternalStream); the host never waits;
  mode "host_staged": D2H copy, CPU all-reduce (gloo), H2D copy — lets several
                 ranks share one GPU in tests;
  mode "host":   the pointer is host memory (CPU-only tests of the plumbing).
"""
import ctypes as C

import numpy as np

_HIP = None
_H2D, _D2H, _D2D = 1, 2, 3


def _hip():
    global _HIP
    if _HIP is None:
        lib = C.CDLL("libamdhip64.so")
        lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        lib.hipMemcpy.restype = C.c_int
        _HIP = lib
    return _HIP


def _memcpy(dst, src, nbytes, kind):
    st = _hip().hipMemcpy(dst, src, nbytes, kind)
    if st != 0:
        raise RuntimeError(f"hipMemcpy failed ({st})")


def _memcpy_async(dst, src, nbytes, stream):
    lib = _hip()
    if not hasattr(lib, "_async"):
        lib.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        lib.hipMemcpyAsync.restype = C.c_int
        lib._async = True
    st = lib.hipMemcpyAsync(dst, src, nbytes, _D2D, stream)
    if st != 0:
        raise RuntimeError(f"hipMemcpyAsync failed ({st})")


def make_allreduce(dist, mode="device", max_elems=1 << 20, stream=None, reduce=None):
    """Return fn(ptr:int, n:int) that leaves the sum over ranks in place.
    device_async needs the context's stream; `reduce(tensor)` replaces
    dist.all_reduce (tests)."""
    import torch
    if mode == "device_async":
        buf = torch.zeros(max_elems, device="cuda")
        ext = torch.cuda.ExternalStream(stream)
        red = reduce or (lambda t: dist.all_reduce(t))

        def fn(ptr, n):
            _memcpy_async(buf.data_ptr(), ptr, n * 4, stream)
            with torch.cuda.stream(ext):
                red(buf[:n])
            _memcpy_async(ptr, buf.data_ptr(), n * 4, stream)
        return fn
    if mode == "device":
        buf = torch.zeros(max_elems, device="cuda")

        def fn(ptr, n):
            _memcpy(buf.data_ptr(), ptr, n * 4, _D2D)
            dist.all_reduce(buf[:n])
            torch.cuda.synchronize()
            _memcpy(ptr, buf.data_ptr(), n * 4, _D2D)
        return fn
    if mode == "host_staged":
        host = np.zeros(max_elems, np.float32)
        t = torch.from_numpy(host)

        def fn(ptr, n):
            _memcpy(host.ctypes.data, ptr, n * 4, _D2H)
            dist.all_reduce(t[:n])
            _memcpy(ptr, host.ctypes.data, n * 4, _H2D)
        return fn
    if mode == "host":
        def fn(ptr, n):
            arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_float)), shape=(n,))
            dist.all_reduce(torch.from_numpy(arr))
        return fn
    raise ValueError(mode)


def shard(cfg, rank, world, envs_per_rank):
    """Per-rank config fields: (env_seed_base, rng_stream) — SURVEY.md 8(e)."""
    seed = cfg["seed"]
    return seed + rank * envs_per_rank, (rank if world > 1 else 0)
