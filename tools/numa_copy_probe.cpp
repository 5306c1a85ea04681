// numa_copy_probe.cpp — round 3: why does one core write 1.5 MB into pinned staging
// (hipHostMalloc) in ~35 us but into pageable memory in ~22 us (tools/hostpath_sweep.py)?
// For every NUMA node with CPUs this process may use, pin the thread to one of them and
// time memcpy of a 1.5 MB pageable source (first touched on that CPU) into (a) pinned
// memory from hipHostMalloc and (b) pageable memory first touched on that CPU. Also prints
// the GPU's NUMA node (sysfs, by PCI bus id). JSON lines.
//   hipcc -O2 --offload-arch=gfx950 -o tools/numa_copy_probe tools/numa_copy_probe.cpp
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int read_int(const std::string& path) {
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return -1;
    int v = -1;
    if (fscanf(f, "%d", &v) != 1) v = -1;
    fclose(f);
    return v;
}

static std::vector<int> node_cpus(int node) {
    std::vector<int> cpus;
    FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return cpus;
    char buf[4096] = {0};
    if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
    fclose(f);
    for (char* tok = strtok(buf, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        if (sscanf(tok, "%d-%d", &a, &b) == 2) {
            for (int c = a; c <= b; ++c) cpus.push_back(c);
        } else if (sscanf(tok, "%d", &a) == 1) {
            cpus.push_back(a);
        }
    }
    return cpus;
}

static double best_copy(void* dst, const void* src, size_t n) {
    double best = 1e30;
    for (int r = 0; r < 200; ++r) {
        const double t0 = now_us();
        memcpy(dst, src, n);
        best = std::min(best, now_us() - t0);
    }
    return best;
}

int main() {
    const size_t n = 1536000;
    char bus[64] = {0};
    int gpu_node = -1;
    if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) == hipSuccess) {
        std::string b(bus);
        for (auto& ch : b) ch = (char)tolower(ch);
        gpu_node = read_int("/sys/bus/pci/devices/" + b + "/numa_node");
    }
    std::printf("{\"gpu_pci\": \"%s\", \"gpu_numa_node\": %d}\n", bus, gpu_node);
    cpu_set_t allowed;
    sched_getaffinity(0, sizeof allowed, &allowed);
    for (int node = 0; node < 16; ++node) {
        std::vector<int> cpus = node_cpus(node);
        int cpu = -1;
        for (int c : cpus)
            if (CPU_ISSET(c, &allowed)) { cpu = c; break; }
        if (cpu < 0) continue;
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpu, &one);
        sched_setaffinity(0, sizeof one, &one);
        std::vector<char> src(n, 1), dst_pg(n, 0);   // first touched here
        void* pin = nullptr;
        if (hipHostMalloc(&pin, n, hipHostMallocDefault) != hipSuccess) return 1;
        memset(pin, 0, n);
        const double t_pin = best_copy(pin, src.data(), n), t_pg = best_copy(dst_pg.data(), src.data(), n);
        std::printf("{\"node\": %d, \"cpu\": %d, \"us_best_into_pinned\": %.1f, \"us_best_into_pageable\": %.1f}\n",
                    node, cpu, t_pin, t_pg);
        std::fflush(stdout);
        (void)hipHostFree(pin);
    }
    return 0;
}
