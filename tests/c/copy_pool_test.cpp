// copy_pool_test.cpp — the host copy threads (tcp_amd/csrc/copy_pool.h) under
// ThreadSanitizer: every piece of every job runs exactly once, run() returns
// only after all of them, back-to-back jobs of every size (the staged wire
// batch hands the pool three per batch) and idle gaps longer than the
// workers' spin (so they sleep and are woken), a job whose body writes shared
// per-block counters, the streaming-store copy, and teardown with idle and
// with never-started workers.
//   g++ -std=c++17 -O1 -g -fsanitize=thread copy_pool_test.cpp -lpthread
#include "../../tcp_amd/csrc/copy_pool.h"

#include <cstdio>
#include <set>
#include <string>
#include <vector>

static int fails = 0;
#define EXPECT(c)                                                       \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            ++fails;                                                    \
        }                                                               \
    } while (0)

static void exactly_once(tcpcsum::CopyPool& pool, size_t n, size_t grain, int max_threads = 0) {
    std::vector<std::atomic<uint32_t>> hit(n);
    for (auto& h : hit) h.store(0, std::memory_order_relaxed);
    std::mutex m;
    std::set<std::thread::id> who;
    pool.run(n, grain, [&](size_t lo, size_t hi) {
        EXPECT(lo < hi && hi <= n);
        for (size_t i = lo; i < hi; ++i) hit[i].fetch_add(1, std::memory_order_relaxed);
        std::lock_guard<std::mutex> lk(m);
        who.insert(std::this_thread::get_id());
    }, max_threads);
    for (size_t i = 0; i < n; ++i) EXPECT(hit[i].load(std::memory_order_relaxed) == 1u);
    if (max_threads > 0) EXPECT(who.size() <= (size_t)max_threads);   // never more threads than allowed
    if (max_threads == 1 && n) EXPECT(who.size() == 1 && *who.begin() == std::this_thread::get_id());
}

int main() {
    {
        tcpcsum::CopyPool pool(3, 20000);   // three workers + the caller, 20 us spin
        const size_t sizes[] = {0, 1, 15, 16, 17, 64, 1000, 1024, 4096, 100003};
        for (int rep = 0; rep < 20; ++rep)
            for (size_t n : sizes)
                for (size_t g : {(size_t)1, (size_t)16, (size_t)64, (size_t)4096}) exactly_once(pool, n, g);
        // at most max_threads participants (the caller included); 1 = the caller alone
        for (int rep = 0; rep < 10; ++rep)
            for (int mt : {1, 2, 3, 4, 9}) exactly_once(pool, 20000, 16, mt);
        EXPECT(pool.worker_cpu_ns() > 0);   // the workers ran and their CPU clocks are read
        // idle longer than the spin: the workers sleep on the condition variable and are woken
        for (int rep = 0; rep < 5; ++rep) {
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            exactly_once(pool, 4096, 16);
        }
        // plain (non-atomic) writes to disjoint pieces, read by the caller after run()
        std::vector<uint32_t> out(50000, 0);
        pool.run(out.size(), 64, [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; ++i) out[i] = (uint32_t)(i * 2654435761u);
        });
        for (size_t i = 0; i < out.size(); ++i) EXPECT(out[i] == (uint32_t)(i * 2654435761u));
        // the workers are the library's threads for life (tcpcsum_on_library_thread: the
        // interposer's arena never serves them), the caller is not
        std::atomic<int> marked{0}, unmarked{0};
        const std::thread::id me = std::this_thread::get_id();
        for (int rep = 0; rep < 20; ++rep)
            pool.run(4096, 1, [&](size_t, size_t) {
                if (std::this_thread::get_id() != me) (tcpcsum::t_library_thread ? marked : unmarked)++;
            });
        EXPECT(marked.load() > 0 && unmarked.load() == 0);
        EXPECT(tcpcsum::t_library_thread == 0);
        // the streaming-store copy, every destination head / tail alignment, source at
        // an aligned and an odd offset (wire staging: 64-B destination starts, packets
        // anywhere in the caller's buffers)
        std::vector<uint8_t> src(4096 + 64), dst(4096 + 64);
        for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 7 + 3);
        for (size_t b : {(size_t)0, (size_t)5})
            for (size_t a = 0; a < 16; ++a)
                for (size_t len : {(size_t)0, (size_t)1, (size_t)63, (size_t)64, (size_t)65, (size_t)1500, (size_t)4000}) {
                    std::fill(dst.begin(), dst.end(), 0);
                    pool.run(len, 256, [&](size_t lo, size_t hi) {
                        if (lo & 1024) tcpcsum::copy_nt(dst.data() + a + lo, src.data() + b + lo, hi - lo);
                        else tcpcsum::copy_stream(dst.data() + a + lo, src.data() + b + lo, hi - lo);
                        _mm_sfence();
                    });
                    EXPECT(std::equal(src.begin() + b, src.begin() + b + len, dst.begin() + a));
                    EXPECT(std::all_of(dst.begin(), dst.begin() + a, [](uint8_t v) { return v == 0; }));
                    EXPECT(std::all_of(dst.begin() + a + len, dst.end(), [](uint8_t v) { return v == 0; }));
                }
    }   // teardown with idle workers
    {
        tcpcsum::CopyPool unused(4, 0);   // workers never started
        tcpcsum::CopyPool serial(0, 0);   // caller only
        exactly_once(serial, 1000, 7);
    }
    {   // workers pinned to a CPU set (the GPU's NUMA node on the box): the allowed set here
        cpu_set_t cpus;
        EXPECT(sched_getaffinity(0, sizeof cpus, &cpus) == 0);
        tcpcsum::CopyPool pinned(3, 1000, &cpus);
        for (int rep = 0; rep < 10; ++rep) exactly_once(pinned, 10000, 16);
        cpu_set_t none;
        EXPECT(!tcpcsum::numa_node_cpus("no-such-bus", &none));   // no device: no pinning
    }
    {   // copy threads per context: TCPCSUM_HOST_THREADS, else half the usable CPUs (1..8) alone,
        // or the rank's 1/LOCAL_WORLD_SIZE share of them (1..8) beside co-located ranks
        unsetenv("TCPCSUM_HOST_THREADS");
        unsetenv("LOCAL_WORLD_SIZE");
        const int alone = tcpcsum::default_copy_threads();
        EXPECT(alone >= 1 && alone <= 8);
        cpu_set_t set;
        EXPECT(sched_getaffinity(0, sizeof set, &set) == 0);
        const int cpus = CPU_COUNT(&set);   // this container has no cgroup quota below its mask
        for (int k : {2, 4, 8, 64}) {
            setenv("LOCAL_WORLD_SIZE", std::to_string(k).c_str(), 1);
            const int share = tcpcsum::default_copy_threads();
            EXPECT(share >= 1 && share <= 8 && share <= std::max(1, cpus / k));
        }
        setenv("LOCAL_WORLD_SIZE", "1", 1);
        EXPECT(tcpcsum::default_copy_threads() == alone);
        setenv("TCPCSUM_HOST_THREADS", "3", 1);   // explicit: wins over the share
        setenv("LOCAL_WORLD_SIZE", "8", 1);
        EXPECT(tcpcsum::default_copy_threads() == 3);
        unsetenv("TCPCSUM_HOST_THREADS");
        unsetenv("LOCAL_WORLD_SIZE");
    }
    std::printf(fails ? "copy_pool_test: %d failures\n" : "copy_pool_test: OK\n", fails);
    return fails ? 1 : 0;
}
