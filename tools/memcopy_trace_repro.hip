// memcopy_trace_repro.hip — the host leg's HIP call pattern without the library, for the
// exit-time SIGSEGV under rocprofv3 --memory-copy-trace (round 4's gpurun_out/r4_hostprof.err,
// profiles/r05_hostprof_sigsegv.err): a page-locked host block (hipHostMalloc), a non-blocking
// stream of its own, DMA copies to HBM on it, an event polled for completion; then everything
// destroyed and freed before main returns, as tcpcsum_ctx_destroy / tcpcsum_host_free do.
//   hipcc --offload-arch=gfx950 -O2 tools/memcopy_trace_repro.hip -o tools/memcopy_trace_repro
//   rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o t -- tools/memcopy_trace_repro [keep]
// "keep": leave the stream, event and buffers alive at exit instead.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const bool keep = argc > 1 && !strcmp(argv[1], "keep");
    const size_t n = 256u << 20;
    void *h = nullptr, *d = nullptr;
    hipStream_t s;
    hipEvent_t ev;
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    memset(h, 1, n);
    CK(hipMalloc(&d, n));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int i = 0; i < 20; ++i) {
        CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
        CK(hipEventRecord(ev, s));
        while (hipEventQuery(ev) == hipErrorNotReady) usleep(20);
    }
    CK(hipMemcpyAsync(h, d, 1 << 20, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (!keep) {
        CK(hipEventDestroy(ev));
        CK(hipStreamDestroy(s));
        CK(hipFree(d));
        CK(hipHostFree(h));
    }
    printf("copies done (%s)\n", keep ? "kept" : "freed");
    fflush(stdout);   // on record before the exit-time teardown
    return 0;
}
