// pin_cache_probe.cpp — does a HIP copy from pageable memory leave the user
// pages page-locked (a cached pin-in-place) after it returns? For each size:
// malloc a pageable buffer, query hipPointerGetAttributes, hipMemcpy it to the
// device, query again, then try hipHostRegister on it (which fails when HIP
// already holds the pages). Also times the copy (first and repeated). Reads
// only; no kernel runs. One JSON line per size.
//   hipcc -O2 -o tools/pin_cache_probe tools/pin_cache_probe.cpp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static int attr_type(const void* p, void** dev) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        *dev = nullptr;
        return -1;
    }
    *dev = a.devicePointer;
    return (int)a.type;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t sizes[] = {1u << 20, 4u << 20, 16u << 20, 32u << 20, 64u << 20};
    void* d = nullptr;
    if (hipMalloc(&d, 64u << 20) != hipSuccess) return 1;
    for (size_t n : sizes) {
        uint8_t* h = (uint8_t*)malloc(n + 4096);
        uint8_t* p = h + 64;   // not page-aligned, like a heap object
        memset(h, 1, n + 4096);
        void* dv0;
        void* dv1;
        const int t0 = attr_type(p, &dv0);
        double a = now_us();
        hipError_t e1 = hipMemcpy(d, p, n, hipMemcpyHostToDevice);
        const double first = now_us() - a;
        const int t1 = attr_type(p, &dv1);
        a = now_us();
        for (int k = 0; k < 5; ++k) (void)hipMemcpy(d, p, n, hipMemcpyHostToDevice);
        const double again = (now_us() - a) / 5;
        void* dv2;
        const int t2 = attr_type(p, &dv2);
        const int mid_t = attr_type(p + n / 2, &dv2);
        // would our registry's hipHostRegister of these pages succeed?
        uint8_t* lo = (uint8_t*)(((uintptr_t)p + 4095) & ~(uintptr_t)4095);
        hipError_t er = hipHostRegister(lo, 4096, hipHostRegisterMapped);
        if (er == hipSuccess) (void)hipHostUnregister(lo);
        else (void)hipGetLastError();
        // our own pin-in-place: register the page hull, DMA, unregister (5 reps)
        uint8_t* hl = (uint8_t*)((uintptr_t)p & ~(uintptr_t)4095);
        const size_t hn = (((uintptr_t)p + n + 4095) & ~(uintptr_t)4095) - (uintptr_t)hl;
        double reg_us = 0, dma_us = 0, unreg_us = 0;
        int rrc = 0;
        for (int k = 0; k < 5; ++k) {
            a = now_us();
            hipError_t r = hipHostRegister(hl, hn, hipHostRegisterMapped);
            const double b1 = now_us();
            if (r != hipSuccess) { rrc = (int)r; (void)hipGetLastError(); break; }
            (void)hipMemcpy(d, p, n, hipMemcpyHostToDevice);
            const double b2 = now_us();
            (void)hipHostUnregister(hl);
            const double b3 = now_us();
            reg_us += (b1 - a) / 5; dma_us += (b2 - b1) / 5; unreg_us += (b3 - b2) / 5;
        }
        std::printf("{\"bytes\": %zu, \"copy_rc\": %d, \"type_before\": %d, \"type_after_copy\": %d, "
                    "\"type_after_6_copies\": %d, \"type_mid\": %d, \"dev_after\": \"%p\", \"register_rc\": %d, "
                    "\"first_copy_us\": %.1f, \"repeat_copy_us\": %.1f, \"own_pin_rc\": %d, \"own_register_us\": %.1f, "
                    "\"own_dma_us\": %.1f, \"own_unregister_us\": %.1f}\n",
                    n, (int)e1, t0, t1, t2, mid_t, dv1, (int)er, first, again, rrc, reg_us, dma_us, unreg_us);
        std::fflush(stdout);
        free(h);
    }
    (void)hipFree(d);
    return 0;
}
