// Device -> host copies on the SDMA engines (hsa_amd_memory_async_copy, no compute
// units) while a kernel occupies every CU: can the shuffle engine get its host words
// from the GPU's copy without blit kernels?  256 MiB in 4 MiB chunks into locked
// 2 MB-page host memory (as the engine's word buffer), idle GPU vs busy GPU.
// Build: hipcc -O2 --offload-arch=gfx950 scripts/sdma_probe.cpp -o scripts/sdma_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdint>

__global__ void fill(uint32_t *d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        d[i] = (uint32_t)(i * 2654435761u);
}
__global__ void busy(float *o, int iters) {
    float a = threadIdx.x * 1e-3f;
    for (int i = 0; i < iters; i++) a = __builtin_fmaf(a, 0.999999f, 1e-7f);
    if (a == 12345.0f) o[0] = a;
}
static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t agent_cb(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}
#define CK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { printf("FAIL %s = %d\n", #x, (int)s_); return 1; } } while (0)
int main() {
    hipSetDevice(0);
    const size_t chunk = (size_t)1 << 20, nch = 64, n = chunk * nch, bytes = n * 4;
    uint32_t *d = nullptr;
    float *o = nullptr;
    hipMalloc(&d, bytes);
    hipMalloc(&o, 64);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, n);
    hipDeviceSynchronize();
    void *h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(h, bytes, MADV_HUGEPAGE);
    memset(h, 0, bytes);
    CK(hsa_init());
    CK(hsa_iterate_agents(agent_cb, nullptr));
    void *hg = nullptr;
    CK(hsa_amd_memory_lock(h, bytes, &g_gpu, 1, &hg));
    uint32_t mask = 0;
    hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask);
    printf("agents gpu=%llx cpu=%llx; sdma engines free (gpu->cpu) mask=0x%x; locked alias %s\n",
           (unsigned long long)g_gpu.handle, (unsigned long long)g_cpu.handle, mask, hg == h ? "== host ptr" : "differs");
    hsa_signal_t sig;
    CK(hsa_signal_create(1, 0, nullptr, &sig));
    hipStream_t st;
    hipStreamCreate(&st);
    for (int mode = 0; mode < 4; mode++) {
        memset(h, 0, bytes);
        if (mode > 0) hipLaunchKernelGGL(busy, dim3(256 * 16), dim3(1024), 0, st, o, 4000000);
        auto t0 = std::chrono::steady_clock::now();
        hsa_signal_store_relaxed(sig, (hsa_signal_value_t)nch);
        for (size_t c = 0; c < nch; c++) {
            char *dst = (char *)hg + c * chunk * 4;
            const char *src = (const char *)d + c * chunk * 4;
            if (mode == 3) {
                uint32_t e[4], ne = 0;
                for (int b = 0; b < 32 && ne < 4; b++) if (mask & (1u << b)) e[ne++] = 1u << b;
                CK(hsa_amd_memory_async_copy_on_engine(dst, g_cpu, src, g_gpu, chunk * 4, 0, nullptr, sig,
                                                       (hsa_amd_sdma_engine_id_t)e[c % ne], false));
            } else if (mode < 2) {
                CK(hsa_amd_memory_async_copy(dst, g_cpu, src, g_gpu, chunk * 4, 0, nullptr, sig));
            } else {
                CK(hsa_amd_memory_async_copy_on_engine(dst, g_cpu, src, g_gpu, chunk * 4, 0, nullptr, sig,
                                                       HSA_AMD_SDMA_ENGINE_0, true));
            }
        }
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        hipError_t q = hipStreamQuery(st);
        size_t bad = 0;
        for (size_t i = 0; i < n; i += 4093) bad += ((uint32_t *)h)[i] != (uint32_t)(i * 2654435761u);
        printf("mode %d (%s): %.1f GB/s over %zu MiB, busy kernel %s at copy end, mismatches %zu\n", mode,
               mode == 0 ? "idle GPU, async_copy" : mode == 1 ? "busy GPU, async_copy" : mode == 2 ? "busy GPU, on_engine SDMA0" : "busy GPU, 4 engines round-robin",
               bytes / dt / 1e9, bytes >> 20, q == hipSuccess ? "DONE (copy not overlapped)" : "still running", bad);
        hipStreamSynchronize(st);
    }
    hsa_signal_destroy(sig);
    hsa_amd_memory_unlock(h);
    return 0;
}
