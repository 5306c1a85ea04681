// host_registry.h — which host packets a context may hand to its kernels in
// place, and where the GPU sees them.
//
// tcpcsum_ipv4_batch_ptrs_host takes one pointer per packet (the reference's
// separately malloc'd out-buffers, loop.c:180-183). The kernel may only touch
// host pages that are page-locked and mapped for the device, so every packet
// [p, p + len) is resolved here to a device address — or to "not mappable",
// and then the caller copies the packet into its own pinned staging instead.
// A packet is used in place when ONE page-locked allocation covers all of it:
// memory its owner page-locked (tcpcsum_host_alloc / hipHostMalloc, the
// application's own hipHostRegister), looked up afresh every batch — its owner
// may free it between two batches.
//
// The library never page-locks or unlocks memory it did not allocate (round 4,
// DESIGN.md §7): GPU mappings of host pages are per page, HIP pins pageable
// copy buffers in place behind its own back (invisible to
// hipPointerGetAttributes), and a page a malloc'd buffer shares with its heap
// neighbours can be under such a pin; locking or unlocking it from here is what
// left a later pageable HIP copy faulting in rounds 2 and 3. So this is a
// lookup only: nothing here changes any page's state.
//
// Header-only and templated on the backend, so the bookkeeping runs under a CPU
// unit test with a fake backend (tests/c/registry_test.cpp) exactly as it runs
// over HIP.
//
// Backend interface:
//   bool pinned_extent(uintptr_t p, uintptr_t* lo, uintptr_t* hi, intptr_t* delta)
//          p lies in memory page-locked by someone else: the extent of that
//          allocation / registration (as HIP reports it, not necessarily
//          page-aligned) and its device offset (device address = host + delta).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <unordered_set>
#include <vector>

namespace tcpcsum {

constexpr uintptr_t kHostPage = 4096;

struct HostRange {
    uintptr_t lo, hi;   // page-aligned
    intptr_t delta;     // device address = host address + delta
};

template <class Backend>
class PinnedLookup {
public:
    static constexpr int kUnmappable = -1000;
    // Pages remembered as "nobody has page-locked these" (a packet starting there
    // cannot lie in a page-locked allocation), so a pageable buffer costs one
    // lookup (three HIP calls), not one per batch. The memo is dropped past this
    // many pages, and every kMemoBatches batches: memory the application
    // page-locks later at addresses seen pageable before is read in place again
    // within that many batches (until then it is copied — slower, never wrong).
    static constexpr size_t kPageableMemo = 1u << 16;
    static constexpr uint32_t kMemoBatches = 256;

    explicit PinnedLookup(Backend& b) : b_(b) {}
    PinnedLookup(const PinnedLookup&) = delete;
    PinnedLookup& operator=(const PinnedLookup&) = delete;

    // Called at the start of every batch: forget the extents found so far (their
    // owners may free or unregister them between two batches) and age the memo.
    void begin_batch() {
        if (!regs_.empty()) {
            regs_.clear();
            view_.clear();
            finger_ = 0;
        }
        if (++batches_ >= kMemoBatches) {
            batches_ = 0;
            forget_pageable();
        }
    }

    // Device address of the host bytes [p, p + len), len > 0, or kUnmappable.
    int resolve(uintptr_t p, size_t len, uintptr_t* dev) {
        const uintptr_t e = p + len;
        if (find(p, e, dev)) return 0;
        const uintptr_t pg = p & ~(kHostPage - 1);
        if (pageable_.count(pg)) return kUnmappable;
        uintptr_t rs = 0, re = 0;
        intptr_t delta = 0;
        if (!b_.pinned_extent(p, &rs, &re, &delta)) {
            if (pageable_.size() >= kPageableMemo) forget_pageable();
            pageable_.insert(pg);
            return kUnmappable;
        }
        add(rs, re, delta);
        // a packet running on past its allocation is copied: the pages beyond
        // are someone else's business, and nothing here locks them
        return find(p, e, dev) ? 0 : kUnmappable;
    }

    // Drop the pageable-page memo: every kMemoBatches batches, when it is full,
    // and on demand (a test that page-locks memory it used pageable before and
    // wants it read in place at once).
    void forget_pageable() { pageable_.clear(); }

    size_t extents() const { return regs_.size(); }
    size_t memo_pages() const { return pageable_.size(); }

private:
    // Someone else's page-locked allocation. HIP reports its extent as
    // allocated (e.g. an unaligned hipHostRegister); the device mapping is page
    // granular, so it is recorded rounded out to whole pages — otherwise a
    // packet crossing the allocation's last byte into the rest of that page
    // would fall between this range and the next.
    void add(uintptr_t rs, uintptr_t re, intptr_t delta) {
        rs &= ~(kHostPage - 1);
        re = (re + kHostPage - 1) & ~(kHostPage - 1);
        for (const auto& r : regs_)
            if (r.lo == rs && r.hi == re && r.delta == delta) return;
        regs_.push_back({rs, re, delta});
        rebuild();
    }

    // Lookup view: ranges sorted by address, touching ranges of equal offset merged.
    void rebuild() {
        std::sort(regs_.begin(), regs_.end(), [](const HostRange& a, const HostRange& b) { return a.lo < b.lo; });
        view_.clear();
        for (const auto& r : regs_) {
            if (!view_.empty() && view_.back().hi >= r.lo && view_.back().delta == r.delta)
                view_.back().hi = std::max(view_.back().hi, r.hi);
            else
                view_.push_back(r);
        }
        finger_ = 0;
    }

    // [p, e) inside one interval of the view. `finger_` is the last hit: packets of a
    // batch mostly come in pool order, so the next one is usually there or one on.
    bool find(uintptr_t p, uintptr_t e, uintptr_t* dev) {
        if (view_.empty()) return false;
        auto hit = [&](size_t j) { return j < view_.size() && view_[j].lo <= p && e <= view_[j].hi; };
        size_t k = finger_;
        if (!hit(k)) {
            if (hit(k + 1)) {
                k = k + 1;
            } else {   // the last interval starting at or before p
                size_t lo = 0, hi = view_.size();
                while (hi - lo > 1) {
                    const size_t mid = (lo + hi) / 2;
                    if (view_[mid].lo <= p) lo = mid; else hi = mid;
                }
                // extents of different offsets may overlap (rounded to pages): look a few back
                size_t j = lo;
                while (!hit(j) && j > 0 && lo - j < 8) --j;
                if (!hit(j)) return false;
                k = j;
            }
        }
        finger_ = k;
        *dev = (uintptr_t)((intptr_t)p + view_[k].delta);
        return true;
    }

    Backend& b_;
    std::vector<HostRange> regs_;   // sorted by lo
    std::vector<HostRange> view_;
    std::unordered_set<uintptr_t> pageable_;
    size_t finger_ = 0;
    uint32_t batches_ = 0;
};

}  // namespace tcpcsum
