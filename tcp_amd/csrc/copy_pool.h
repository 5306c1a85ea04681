// copy_pool.h — the host side's copy threads (tcpcsum_host.hip): a small
// pool that runs one data-parallel job at a time over [0, n) in pieces, plus
// the streaming-store memcpy the uniform staging uses. Host-only C++ (no HIP),
// so tests/c/copy_pool_test.cpp runs it under ThreadSanitizer on the CPU.
#pragma once

#include <ctype.h>
#include <emmintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tcpcsum {

// Set on the library's own threads (the copy pool's workers) for their whole life:
// tcpcsum_on_library_thread() reports it, so the interposer's arena never serves a
// packet block to an allocation the library makes.
inline thread_local int t_library_thread = 0;

inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A few host threads for the copies into pinned staging: one core's memcpy
// (≈10-20 GB/s) is below the PCIe rate the kernel reads staging at
// (≈50 GiB/s), and the copy of chunk k+1 must keep pace with the kernel on
// chunk k. The calling thread works too; workers that wake late find the job
// done and go back to sleep (nobody waits for a sleeper to wake).
//
// `cpus` (nullable): the CPUs the workers run on — the GPU's NUMA node, where
// the pinned staging lives: one core writes 1.5 MB into it in 17 us from that
// node and in 31 us from the other (tools/numa_copy_probe.cpp on the MI355X
// box). The calling thread is left where it is.
class CopyPool {
public:
    CopyPool(int workers, uint64_t spin_ns, const cpu_set_t* cpus = nullptr)
        : nw_(workers < 0 ? 0 : workers), spin_ns_(spin_ns) {
        if (cpus) {
            cpus_ = *cpus;
            pin_ = true;
        }
    }
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int threads() const { return nw_ + 1; }

    // CPU time the workers have used since they started (copies, the spin after
    // each job, wake-ups), from their per-thread CPU clocks. Call from the thread
    // that runs jobs (the workers are started there).
    uint64_t worker_cpu_ns() const {
        uint64_t ns = 0;
        for (const auto& t : th_) {
            clockid_t cid;
            timespec ts;
            if (pthread_getcpuclockid(const_cast<std::thread&>(t).native_handle(), &cid) == 0 &&
                clock_gettime(cid, &ts) == 0)
                ns += (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
        }
        return ns;
    }

    // body(lo, hi) over [0, n) in pieces of `grain`; returns when every piece is done.
    // max_threads: at most this many threads work on it, the caller included
    // (0 = every worker; 1 = the caller alone, no worker is woken).
    void run(size_t n, size_t grain, const std::function<void(size_t, size_t)>& body, int max_threads = 0) {
        if (n == 0) return;
        if (grain == 0) grain = 1;
        const int helpers = max_threads <= 0 ? nw_ : std::min(nw_, max_threads - 1);
        if (helpers <= 0 || n <= grain) {
            body(0, n);
            return;
        }
        start();
        auto job = std::make_shared<Job>(&body, n, grain, helpers);
        {
            std::lock_guard<std::mutex> lk(m_);
            cur_ = job;
            ++gen_;
        }
        if (helpers >= nw_)
            cv_.notify_all();
        else
            for (int i = 0; i < helpers; ++i) cv_.notify_one();
        job->drain();
        while (job->done.load(std::memory_order_acquire) < n) std::this_thread::yield();
        std::lock_guard<std::mutex> lk(m_);
        if (cur_ == job) cur_.reset();
    }

private:
    struct Job {
        Job(const std::function<void(size_t, size_t)>* b, size_t n_, size_t g, int helpers)
            : body(b), n(n_), grain(g), seats(helpers) {}
        const std::function<void(size_t, size_t)>* body;   // valid while done < n
        size_t n, grain;
        std::atomic<size_t> next{0}, done{0};
        std::atomic<int> seats;   // workers that may still join
        void drain() {
            for (;;) {
                const size_t i = next.fetch_add(grain, std::memory_order_relaxed);
                if (i >= n) return;
                const size_t e = std::min(n, i + grain);
                (*body)(i, e);
                done.fetch_add(e - i, std::memory_order_release);
            }
        }
    };
    void start() {
        if (started_) return;
        started_ = true;
        try {
            for (int i = 0; i < nw_; ++i) {
                th_.emplace_back([this] { loop(); });
                if (pin_) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof cpus_, &cpus_);
            }
        } catch (...) {   // fewer threads than asked: the caller still does all the work it must
        }
    }
    // A worker spins briefly after each job before it sleeps: a staged wire
    // batch hands the pool three jobs (header reads, copies; after the kernel,
    // the FILL write-back), microseconds apart, and a condition-variable
    // wake-up costs about as long as one of them.
    void loop() {
        t_library_thread = 1;
        uint64_t seen = 0;
        for (;;) {
            const uint64_t t0 = now_ns();
            while (gen_.load(std::memory_order_acquire) == seen && !quit_.load(std::memory_order_relaxed) &&
                   now_ns() - t0 < spin_ns_)
                _mm_pause();
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_.load() || gen_.load() != seen; });
                if (quit_) return;
                seen = gen_.load();
                job = cur_;
            }
            if (job && job->seats.fetch_sub(1, std::memory_order_relaxed) > 0) job->drain();
        }
    }
    int nw_;
    uint64_t spin_ns_;
    cpu_set_t cpus_;
    bool pin_ = false;
    bool started_ = false;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::shared_ptr<Job> cur_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> quit_{false};
};

// Host threads for staging copies: TCPCSUM_HOST_THREADS, else from the CPUs this
// process may use (the affinity mask, capped by a cgroup CPU quota): half of them
// (1..8) for a process alone on its node; when LOCAL_WORLD_SIZE (torch.distributed.run's
// ranks on this node, which share that quota) is k > 1, the rank's 1/k share of them
// (1..8), so k ranks copying at once fit the CPUs the job has instead of
// oversubscribing the quota and being throttled.
inline int default_copy_threads() {
    if (const char* e = getenv("TCPCSUM_HOST_THREADS")) {
        const int v = atoi(e);
        if (v >= 1) return std::min(v, 64);
    }
    int cpus = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = std::max(1, CPU_COUNT(&set));
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long per = 0;
        if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
            const long long quota = atoll(q);
            if (quota > 0) cpus = std::min<long long>(cpus, std::max<long long>(1, (quota + per - 1) / per));
        }
        fclose(f);
    }
    int ranks = 1;
    if (const char* e = getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, atoi(e));
    if (ranks > 1) return std::max(1, std::min(8, cpus / ranks));
    return std::max(1, std::min(8, cpus / 2));
}

// The CPUs of `device_pci_bus`'s NUMA node (sysfs, "0000:8e:00.0" style) that
// this process may run on, and the node (nullable); false when unknown or none.
inline bool numa_node_cpus(const char* device_pci_bus, cpu_set_t* out, int* node_out = nullptr) {
    char path[256], buf[4096];
    std::string bus(device_pci_bus);
    for (auto& ch : bus) ch = (char)tolower((unsigned char)ch);
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus.c_str());
    int node = -1;
    if (FILE* f = fopen(path, "r")) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    if (node < 0) return false;
    if (node_out) *node_out = node;
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE* f = fopen(path, "r");
    if (!f) return false;
    const bool got = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!got) return false;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
    CPU_ZERO(out);
    int count = 0;
    for (char* save = nullptr, *tok = strtok_r(buf, ",\n", &save); tok; tok = strtok_r(nullptr, ",\n", &save)) {
        int a = 0, b = 0;
        const int k = sscanf(tok, "%d-%d", &a, &b);
        if (k < 1) continue;
        if (k == 1) b = a;
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &allowed)) {
                CPU_SET(c, out);
                ++count;
            }
    }
    return count > 0;
}

// memcpy into staging with non-temporal (streaming) stores: the kernel reads
// the staging over PCIe, not the CPU, so the copy should not first read the
// destination lines into the cache (read-for-ownership) nor evict the source
// stream's own working set. Ends with sfence: streaming stores are weakly
// ordered, and the piece must be globally visible before the launch.
inline void copy_stream(uint8_t* d, const uint8_t* s, size_t n);
inline void copy_nt(uint8_t* d, const uint8_t* s, size_t n) {
    copy_stream(d, s, n);
    _mm_sfence();
}

// copy_nt without the closing sfence, for a thread that copies many pieces and
// fences once after the last.
inline void copy_stream(uint8_t* d, const uint8_t* s, size_t n) {
    size_t h = (16u - ((uintptr_t)d & 15u)) & 15u;
    if (h > n) h = n;
    memcpy(d, s, h);
    d += h;
    s += h;
    n -= h;
    const size_t k = n & ~(size_t)63;
    for (size_t i = 0; i < k; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(s + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(s + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32));
        const __m128i e = _mm_loadu_si128((const __m128i*)(s + i + 48));
        _mm_stream_si128((__m128i*)(d + i), a);
        _mm_stream_si128((__m128i*)(d + i + 16), b);
        _mm_stream_si128((__m128i*)(d + i + 32), c);
        _mm_stream_si128((__m128i*)(d + i + 48), e);
    }
    memcpy(d + k, s + k, n - k);
}

}  // namespace tcpcsum
