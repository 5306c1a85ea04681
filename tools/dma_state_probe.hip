// dma_state_probe.hip — why the chunked host pipelines slow down after a large device
// allocation ("Order in the bench process"). Pure HIP, no library: the same
// 1.5 GB of page-locked host memory goes to HBM by DMA in several shapes, before and after
// one 16 GiB hipMalloc that is written once and freed (what bench.py's 64k config does).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/dma_state_probe tools/dma_state_probe.hip
//   tools/dma_state_probe [big_gib=16] [reps=5]
//
// Shapes (each timed `reps` times, GiB/s of host bytes moved, best and median):
//   one        one 1.5 GB hipMemcpyAsync into one 1.5 GB buffer
//   chunks1    16 MiB chunks, one stream, into consecutive parts of one 1.5 GB buffer
//   slots2     16 MiB chunks alternating over two 16 MiB slots on two streams (the context's
//              pinned-input pipeline without its kernels; a slot's next copy stays behind its
//              last one on the same stream)
//   slots2_new the same with two slots allocated after the big allocation was freed
//   slots2_1s  16 MiB chunks alternating over the two slots, every copy on ONE stream
//   pipe2s     the pipeline with its kernels: copy k into slot k%2 and kernel k over it, both on
//              stream k%2 (the context's layout through round 4)
//   pipe1c     copies on one copy stream, kernels on a compute stream, events between them
//              (copy k waits for kernel k-2, kernel k for copy k)
//   pipe1s_M   ONE stream, chunks of M MiB into one M MiB slot, each copy followed by its
//              kernel (in-stream order is the only synchronisation)
// Prints one JSON line per phase.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const size_t kBytes = (size_t)1500 * 1048576;   // the 1M x 1500 shard
static const size_t kChunk = (size_t)16 << 20;

__global__ void k_read(const uint4* p, size_t n16, unsigned long long* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) out[threadIdx.x] = acc;   // keeps the loads; practically never taken
}

struct Bufs {
    unsigned char* host;
    unsigned char* dst;       // 1.5 GB
    unsigned char* slot[2];   // 16 MiB each
    hipStream_t st[2];
    hipEvent_t cev[2], kev[2];
    unsigned long long* sink;
};

template <class F>
static void timed(const char* name, int reps, F&& f, const Bufs& b, bool first_field) {
    std::vector<double> r;
    f();   // warm
    CK(hipDeviceSynchronize());
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_s();
        f();
        CK(hipStreamSynchronize(b.st[0]));
        CK(hipStreamSynchronize(b.st[1]));
        r.push_back(kBytes / (now_s() - t0) / (1u << 30));
    }
    std::sort(r.begin(), r.end());
    printf("%s\"%s\": {\"best\": %.2f, \"median\": %.2f}", first_field ? "" : ", ", name, r.back(), r[r.size() / 2]);
}

static void phase(const char* label, Bufs& b, int reps, unsigned char* slot_new[2]) {
    printf("{\"phase\": \"%s\"", label);
    timed("one", reps, [&] { CK(hipMemcpyAsync(b.dst, b.host, kBytes, hipMemcpyHostToDevice, b.st[0])); }, b, false);
    timed("chunks1", reps, [&] {
        for (size_t o = 0; o < kBytes; o += kChunk)
            CK(hipMemcpyAsync(b.dst + o, b.host + o, std::min(kChunk, kBytes - o), hipMemcpyHostToDevice, b.st[0]));
    }, b, false);
    auto slots = [&](unsigned char* const* sl) {
        size_t k = 0;
        for (size_t o = 0; o < kBytes; o += kChunk, ++k)
            CK(hipMemcpyAsync(sl[k & 1], b.host + o, std::min(kChunk, kBytes - o), hipMemcpyHostToDevice, b.st[k & 1]));
    };
    timed("slots2", reps, [&] { slots(b.slot); }, b, false);
    if (slot_new) timed("slots2_new", reps, [&] { slots(slot_new); }, b, false);
    timed("slots2_1s", reps, [&] {
        size_t k = 0;
        for (size_t o = 0; o < kBytes; o += kChunk, ++k)
            CK(hipMemcpyAsync(b.slot[k & 1], b.host + o, std::min(kChunk, kBytes - o), hipMemcpyHostToDevice, b.st[0]));
    }, b, false);
    timed("pipe2s", reps, [&] {
        size_t k = 0;
        for (size_t o = 0; o < kBytes; o += kChunk, ++k) {
            const size_t n = std::min(kChunk, kBytes - o);
            CK(hipMemcpyAsync(b.slot[k & 1], b.host + o, n, hipMemcpyHostToDevice, b.st[k & 1]));
            hipLaunchKernelGGL(k_read, dim3(1024), dim3(256), 0, b.st[k & 1], (const uint4*)b.slot[k & 1], n / 16, b.sink);
        }
    }, b, false);
    timed("pipe1c", reps, [&] {
        size_t k = 0;
        for (size_t o = 0; o < kBytes; o += kChunk, ++k) {
            const size_t n = std::min(kChunk, kBytes - o);
            const int s = (int)(k & 1);
            if (k >= 2) CK(hipStreamWaitEvent(b.st[0], b.kev[s], 0));
            CK(hipMemcpyAsync(b.slot[s], b.host + o, n, hipMemcpyHostToDevice, b.st[0]));
            CK(hipEventRecord(b.cev[s], b.st[0]));
            CK(hipStreamWaitEvent(b.st[1], b.cev[s], 0));
            hipLaunchKernelGGL(k_read, dim3(1024), dim3(256), 0, b.st[1], (const uint4*)b.slot[s], n / 16, b.sink);
            CK(hipEventRecord(b.kev[s], b.st[1]));
        }
    }, b, false);
    for (size_t mib : {16, 64, 256}) {
        const size_t ch = mib << 20;
        char nm[32];
        snprintf(nm, sizeof nm, "pipe1s_%zu", mib);
        timed(nm, reps, [&] {
            for (size_t o = 0; o < kBytes; o += ch) {
                const size_t n = std::min(ch, kBytes - o);
                CK(hipMemcpyAsync(b.dst, b.host + o, n, hipMemcpyHostToDevice, b.st[0]));
                hipLaunchKernelGGL(k_read, dim3(1024), dim3(256), 0, b.st[0], (const uint4*)b.dst, n / 16, b.sink);
            }
        }, b, false);
    }
    printf("}\n");
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t big_gib = argc > 1 ? (size_t)atoi(argv[1]) : 16;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    Bufs b;
    CK(hipHostMalloc((void**)&b.host, kBytes, hipHostMallocDefault));
    for (size_t i = 0; i < kBytes; i += 4096) b.host[i] = (unsigned char)i;
    CK(hipMalloc((void**)&b.dst, kBytes));
    CK(hipMalloc((void**)&b.slot[0], kChunk));
    CK(hipMalloc((void**)&b.slot[1], kChunk));
    CK(hipStreamCreateWithFlags(&b.st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b.st[1], hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        CK(hipEventCreateWithFlags(&b.cev[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&b.kev[i], hipEventDisableTiming));
    }
    CK(hipMalloc((void**)&b.sink, 256 * sizeof(unsigned long long)));

    phase("fresh", b, reps, nullptr);

    unsigned char* big = nullptr;
    CK(hipMalloc((void**)&big, big_gib << 30));
    CK(hipMemsetAsync(big, 1, big_gib << 30, b.st[0]));
    CK(hipStreamSynchronize(b.st[0]));
    CK(hipFree(big));

    unsigned char* slot_new[2];
    CK(hipMalloc((void**)&slot_new[0], kChunk));
    CK(hipMalloc((void**)&slot_new[1], kChunk));
    char label[64];
    snprintf(label, sizeof label, "after %zu GiB alloc+memset+free", big_gib);
    phase(label, b, reps, slot_new);

    CK(hipFree(slot_new[0]));
    CK(hipFree(slot_new[1]));
    CK(hipFree(b.slot[0]));
    CK(hipFree(b.slot[1]));
    CK(hipFree(b.dst));
    CK(hipHostFree(b.host));
    CK(hipStreamDestroy(b.st[0]));
    CK(hipStreamDestroy(b.st[1]));
    return 0;
}
