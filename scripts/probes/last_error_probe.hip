// What hipGetLastError returns after calls whose non-success status the caller handled
// ("gae launch failed" came from launch_gae_1p's hipGetLastError).
// Each case: one or more calls, then hipGetLastError, printed.  Build:
//   hipcc --offload-arch=gfx950 -O2 -o scripts/probes/last_error_probe scripts/probes/last_error_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

// a bounded busy kernel (~50 ms on the 100 MHz constant clock, at most 2^26 polls)
__global__ void busy(unsigned long long ticks, int *out) {
    const unsigned long long t0 = wall_clock64();
    unsigned int it = 0;
    while (wall_clock64() - t0 < ticks && ++it < (1u << 26)) {}
    if (threadIdx.x == 0) out[0] = (int)it;
}
__global__ void noop(int *out) { if (threadIdx.x == 0) out[1] = 1; }

static const char *nm(hipError_t e) { return hipGetErrorName(e); }

int main() {
    hipStream_t s;
    int *d;
    hipEvent_t a, b;
    if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&d, 8) != hipSuccess ||
        hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        printf("setup failed\n");
        return 1;
    }
    auto pending = [&]() {   // a, b around a busy kernel; b not complete yet
        (void)hipEventRecord(a, s);
        hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, 5000000ull, d);
        (void)hipEventRecord(b, s);
        (void)hipGetLastError();
    };
    float ms = 0;
    hipError_t r, l;

    pending();
    r = hipEventQuery(b); l = hipGetLastError();
    printf("A hipEventQuery(incomplete)=%s -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);

    pending();
    r = hipEventQuery(b);
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, d);
    l = hipGetLastError();
    printf("B hipEventQuery(incomplete)=%s, ok launch -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);

    pending();
    r = hipEventElapsedTime(&ms, a, b); l = hipGetLastError();
    printf("C hipEventElapsedTime(incomplete)=%s -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);

    pending();
    r = hipEventElapsedTime(&ms, a, b);
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, d);
    l = hipGetLastError();
    printf("D hipEventElapsedTime(incomplete)=%s, ok launch -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);

    pending();
    r = hipEventElapsedTime(&ms, a, b);
    const hipError_t rec = hipEventRecord(a, s);
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, d);
    l = hipGetLastError();
    printf("E hipEventElapsedTime(incomplete)=%s, ok record=%s, ok launch -> hipGetLastError=%s\n", nm(r), nm(rec),
           nm(l));
    (void)hipStreamSynchronize(s);

    r = hipEventElapsedTime(&ms, a, b); l = hipGetLastError();
    printf("F hipEventElapsedTime(complete)=%s (%.3f ms) -> hipGetLastError=%s\n", nm(r), ms, nm(l));

    pending();
    r = hipStreamQuery(s); l = hipGetLastError();
    printf("G hipStreamQuery(busy)=%s -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);
    hipEvent_t never;
    (void)hipEventCreate(&never);
    r = hipEventElapsedTime(&ms, never, b); l = hipGetLastError();
    printf("H hipEventElapsedTime(never recorded)=%s -> hipGetLastError=%s\n", nm(r), nm(l));
    r = hipEventElapsedTime(&ms, never, b);
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, d);
    l = hipGetLastError();
    printf("I hipEventElapsedTime(never recorded)=%s, ok launch -> hipGetLastError=%s\n", nm(r), nm(l));
    r = hipSetDevice(4096);
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, d);
    const hipError_t r2 = hipEventRecord(a, s);
    l = hipGetLastError();
    printf("J hipSetDevice(4096)=%s, ok launch, ok record=%s -> hipGetLastError=%s\n", nm(r), nm(r2), nm(l));
    r = hipFree((void *)0x1234);
    l = hipGetLastError();
    printf("K hipFree(bad)=%s -> hipGetLastError=%s\n", nm(r), nm(l));
    (void)hipStreamSynchronize(s);
    printf("done\n");
    return 0;
}
