// waitvalue_probe.hip — round 3: can a staged wire batch queue its kernel
// BEFORE the CPU copies are done, released by a flag the copy threads set
// (hipStreamWaitValue64), so the launch latency and the GPU's PCIe reads of
// block j overlap the copy of block j+1?
//
// For each flag memory kind (hipHostMalloc pinned; hipExtMallocWithFlags
// hipMallocSignalMemory) it queues  wait(flag >= g) -> tiny kernel -> event,
// sleeps `delay` us on the CPU, sets the flag, and reports how long after the
// store the event completes (the release latency). The CPU always sets the
// flag, so every wait is satisfied; a wait the GPU never sees released is
// reported as a timeout after 1 s (and the process exits: the queue goes with it).
//   hipcc -O2 --offload-arch=gfx950 -o tools/waitvalue_probe tools/waitvalue_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_touch(uint32_t* out, uint32_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = v;
}

static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static int probe(const char* kind, volatile uint64_t* flag, hipStream_t st, uint32_t* dout, int delay_us) {
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<double> lat;
    for (int r = 0; r < 50; ++r) {
        const uint64_t g = (uint64_t)r + 1;
        CK(hipStreamWaitValue64(st, (void*)flag, g, hipStreamWaitValueGte, ~0ull));
        hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, st, dout, (uint32_t)g);
        CK(hipGetLastError());
        CK(hipEventRecord(ev, st));
        const uint64_t t0 = now_ns();
        while (now_ns() - t0 < (uint64_t)delay_us * 1000u) {
        }
        if (hipEventQuery(ev) == hipSuccess) {   // ran before the flag: the wait did not hold
            std::printf("{\"kind\": \"%s\", \"error\": \"event done before the flag was set\", \"round\": %d}\n", kind, r);
            return 1;
        }
        std::atomic_thread_fence(std::memory_order_seq_cst);
        *flag = g;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        const uint64_t t1 = now_ns();
        while (hipEventQuery(ev) != hipSuccess) {
            if (now_ns() - t1 > 1000000000ull) {
                std::printf("{\"kind\": \"%s\", \"error\": \"timeout: wait never released\", \"round\": %d}\n", kind, r);
                std::fflush(stdout);
                *flag = ~0ull;   // release whatever still waits before the process goes
                return 2;
            }
        }
        lat.push_back((now_ns() - t1) / 1e3);
    }
    std::sort(lat.begin(), lat.end());
    std::printf("{\"kind\": \"%s\", \"delay_us\": %d, \"release_us_median\": %.1f, \"release_us_min\": %.1f, "
                "\"release_us_max\": %.1f}\n",
                kind, delay_us, lat[lat.size() / 2], lat[0], lat.back());
    std::fflush(stdout);
    CK(hipEventDestroy(ev));
    return 0;
}

int main() {
    int can = 0;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("{\"can_use_stream_wait_value\": %d}\n", can);
    if (!can) return 0;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t* dout;
    CK(hipMalloc(&dout, 64));
    uint64_t* pinned;
    CK(hipHostMalloc((void**)&pinned, 4096, hipHostMallocDefault));
    *pinned = 0;
    int rc = probe("hipHostMalloc", pinned, st, dout, 50);
    if (rc) return rc;
    uint64_t* sig = nullptr;
    if (hipExtMallocWithFlags((void**)&sig, 4096, hipMallocSignalMemory) == hipSuccess) {
        hipPointerAttribute_t a;
        const bool host_ok = hipPointerGetAttributes(&a, sig) == hipSuccess && a.hostPointer != nullptr;
        std::printf("{\"signal_memory_host_pointer\": %s}\n", host_ok ? "true" : "false");
        if (host_ok) {
            volatile uint64_t* hs = (volatile uint64_t*)a.hostPointer;
            *hs = 0;
            rc = probe("hipMallocSignalMemory", hs, st, dout, 50);
            if (rc) return rc;
        }
    }
    CK(hipStreamSynchronize(st));
    std::printf("{\"done\": true}\n");
    return 0;
}
