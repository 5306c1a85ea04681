// registry_test.cpp — CPU unit test of tcp_amd/csrc/host_registry.h (the page
// lookup behind tcpcsum_ipv4_batch_ptrs_host) against a fake backend that
// models a host: every resolved packet must lie entirely in pages someone else
// page-locked, under ONE device mapping; everything else is refused (the caller
// copies it). The fake backend has no lock or unlock at all — the lookup cannot
// change any page's state, which is the point of the round-4 design.
//
//   registry_test [seed]   exit 0 when every check holds
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../tcp_amd/csrc/host_registry.h"

static int fails = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            if (fails++ < 20) std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
        }                                                                   \
    } while (0)

using tcpcsum::kHostPage;

struct Alloc {
    uintptr_t lo, hi;   // as the owner allocated / registered it (maybe unaligned)
    intptr_t delta;
};

struct FakeHost {
    std::vector<Alloc> pinned;   // page-locked by someone else (tcpcsum_host_alloc, hipHostRegister)
    uint64_t extent_calls = 0;
    bool pinned_extent(uintptr_t p, uintptr_t* lo, uintptr_t* hi, intptr_t* delta) {
        ++extent_calls;
        for (const auto& f : pinned)
            if (f.lo <= p && p < f.hi) { *lo = f.lo; *hi = f.hi; *delta = f.delta; return true; }
        return false;
    }
    // the mapping that holds byte a, or nullptr (device mappings are page granular:
    // the rest of an allocation's first and last page is mapped too)
    const Alloc* holder(uintptr_t a) const {
        for (const auto& f : pinned)
            if ((f.lo & ~(kHostPage - 1)) <= a && a < ((f.hi + kHostPage - 1) & ~(kHostPage - 1))) return &f;
        return nullptr;
    }
};

using Lookup = tcpcsum::PinnedLookup<FakeHost>;

// [p, p+len) -> dev is safe: every byte's page is mapped by ONE allocation, and
// dev + k is where byte p + k lives.
static bool mapped_by_one(const FakeHost& h, uintptr_t p, size_t len, intptr_t* delta) {
    const Alloc* first = h.holder(p);
    if (!first) return false;
    for (uintptr_t a = p; a < p + len; a = (a | (kHostPage - 1)) + 1) {
        const Alloc* l = h.holder(a);
        if (!l || l->delta != first->delta) return false;
    }
    const Alloc* last = h.holder(p + len - 1);
    if (!last || last->delta != first->delta) return false;
    *delta = first->delta;
    return true;
}

static void scenario(bool flat, uint64_t seed) {
    FakeHost h;
    std::mt19937_64 r(seed * 7 + 3);
    Lookup reg(h);
    // a heap: buffers laid end to end with 16-B headers, like malloc; some are
    // page-locked allocations (page-aligned, locked by their owner)
    struct Buf { uintptr_t p; size_t n; bool pinned; };
    std::vector<Buf> bufs;
    uintptr_t cur = 0x7f0000001010ull;
    for (int i = 0; i < 600; ++i) {
        const int kind = (int)(r() % 10);
        if (kind == 0) {
            cur = (cur + kHostPage - 1) & ~(kHostPage - 1);
            const size_t n = (r() % 8 + 1) * kHostPage;
            h.pinned.push_back({cur, cur + n, flat ? 0 : (intptr_t)((r() % 1000 + 1) << 24)});
            bufs.push_back({cur, n, true});
            cur += n + kHostPage;
        } else {
            const size_t n = kind < 4 ? 32768 : kind < 8 ? 4096 : (size_t)(r() % 3000 + 64);
            bufs.push_back({cur, n, false});
            cur += n + 16;
        }
    }
    for (int round = 0; round < 6; ++round) {
        reg.begin_batch();
        for (int k = 0; k < 1500; ++k) {
            const Buf& b = bufs[r() % bufs.size()];
            const size_t len = 20 + r() % (b.n - 20 < 1500 ? b.n - 20 : 1500);
            const size_t off = r() % (b.n - len + 1);
            uintptr_t dev = 0;
            const int rc = reg.resolve(b.p + off, len, &dev);
            intptr_t delta = 0;
            const bool want = mapped_by_one(h, b.p + off, len, &delta);
            CHECK((rc == 0) == want);   // in place exactly when one page-locked allocation covers it
            CHECK(rc == 0 || rc == Lookup::kUnmappable);
            if (rc == 0) CHECK((intptr_t)dev - (intptr_t)(b.p + off) == delta);
            if (b.pinned) CHECK(rc == 0);
        }
    }
}

// Memory pinned by someone else is freed between two batches (its pages reused
// as pageable memory): after begin_batch() the lookup never hands out its old
// mapping — the packet is refused (copied).
static void stale_foreign() {
    FakeHost h;
    Lookup reg(h);
    const uintptr_t base = 0x7d0000000000ull;
    h.pinned.push_back({base, base + 8 * kHostPage, (intptr_t)(77ull << 24)});
    uintptr_t dev = 0;
    reg.begin_batch();
    CHECK(reg.resolve(base + 100, 1500, &dev) == 0 && dev == base + 100 + (77ull << 24));
    CHECK(reg.extents() == 1);
    h.pinned.clear();   // the owner frees it
    reg.begin_batch();
    CHECK(reg.extents() == 0);
    CHECK(reg.resolve(base + 100, 1500, &dev) == Lookup::kUnmappable);
}

// A pageable page is asked about once, not once per packet per batch; the memo
// is dropped every kMemoBatches batches, so memory page-locked later at those
// addresses is read in place again (it used to stay copied for good).
static void memo(uint64_t seed) {
    FakeHost h;
    std::mt19937_64 r(seed);
    Lookup reg(h);
    const uintptr_t heap = 0x7c0000001010ull, pinned = 0x7c0100000000ull;
    h.pinned.push_back({pinned, pinned + 64 * kHostPage, 0});
    uintptr_t dev = 0;
    for (uint32_t batch = 0; batch < 2 * Lookup::kMemoBatches + 3; ++batch) {
        reg.begin_batch();
        const uint64_t before = h.extent_calls;
        for (int k = 0; k < 64; ++k) {
            const uintptr_t p = heap + (uintptr_t)k * (32768 + 16);
            CHECK(reg.resolve(p, 1500, &dev) == Lookup::kUnmappable);
        }
        // one lookup per buffer on the memo's first batch, none after
        const bool fresh = batch == 0 || (batch + 1) % Lookup::kMemoBatches == 0;
        CHECK(h.extent_calls - before == (fresh ? 64u : 0u));
        for (int k = 0; k < 16; ++k) {
            const uintptr_t p = pinned + (uintptr_t)k * kHostPage + r() % 2000;
            CHECK(reg.resolve(p, 1500, &dev) == 0 && dev == p);
        }
        // a packet running off the end of the allocation is refused (copied), never extended
        CHECK(reg.resolve(pinned + 64 * kHostPage - 100, 1500, &dev) == Lookup::kUnmappable);
    }
    // the application page-locks the heap buffers now: within kMemoBatches batches they are in place
    h.pinned.push_back({heap & ~(kHostPage - 1), heap + 64 * (32768 + 16) + kHostPage, 0});
    int batches = 0;
    for (;; ++batches) {
        reg.begin_batch();
        if (reg.resolve(heap, 1500, &dev) == 0) break;
        if (batches > (int)Lookup::kMemoBatches) break;
    }
    CHECK(batches <= (int)Lookup::kMemoBatches);
    reg.forget_pageable();
    CHECK(reg.memo_pages() == 0);
}

// An allocation whose reported size is not a page multiple: its last
// page is mapped whole, so a packet crossing the allocation's last byte into that
// page resolves through it; one running on into the next page does not.
static void unaligned_foreign() {
    FakeHost h;
    Lookup reg(h);
    const uintptr_t base = 0x7b0000000000ull;
    h.pinned.push_back({base, base + 5000, 0});
    uintptr_t dev = 0;
    reg.begin_batch();
    CHECK(reg.resolve(base + 4900, 200, &dev) == 0 && dev == base + 4900);
    CHECK(reg.resolve(base + 8000, 100, &dev) == 0);
    CHECK(reg.resolve(base + 8000, 1000, &dev) == Lookup::kUnmappable);   // into page 2: nobody's mapping
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
    for (uint64_t s = seed; s < seed + 4; ++s) {
        scenario(true, s);
        scenario(false, s);
        memo(s);
    }
    stale_foreign();
    unaligned_foreign();
    std::printf(fails ? "FAIL (%d)\n" : "OK\n", fails);
    return fails ? 1 : 0;
}
