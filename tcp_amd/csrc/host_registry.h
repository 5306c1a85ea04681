// host_registry.h — which host pages a context may hand to its kernels in
// place, and where the GPU sees them.
//
// tcpcsum_ipv4_batch_ptrs_host takes one pointer per packet (the reference's
// separately malloc'd out-buffers, loop.c:180-183). The kernel may only touch
// host pages that are page-locked and mapped for the device, so every packet
// [p, p + len) is resolved here to a device address — or to "not mappable",
// and then the caller copies the packet into its own pinned staging instead.
// A packet is used in place when ONE mapping covers all of it:
//   * pages this registry locked (tcpcsum_ctx_register_host, or on first use
//     when the context opted in to auto-registration), or
//   * memory page-locked by someone else (hipHostMalloc, the application's own
//     registration): looked up afresh every batch (forget_foreign), its owner
//     may free it between two batches.
// The registry never unlocks anything during a lookup, and it locks pages only
// when asked to (may_lock), never pages someone else already holds.
//
// Header-only and templated on the backend that does the locking, so the
// bookkeeping runs under a CPU unit test with a fake backend
// (tests/c/registry_test.cpp) exactly as it runs over HIP.
//
// Backend interface:
//   int  lock(uintptr_t lo, size_t bytes, intptr_t* delta)
//          page-lock [lo, lo + bytes) (whole pages); device address = host + *delta.
//          0 on success, else a backend error.
//   void unlock(uintptr_t lo)                      undo one lock() by its start.
//   bool pinned_extent(uintptr_t p, uintptr_t* lo, uintptr_t* hi, intptr_t* delta)
//          p lies in memory page-locked by someone else (or by us): the extent
//          of that allocation / registration (as HIP reports it, not necessarily
//          page-aligned) and its device offset.
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
    bool owned;         // locked by this registry (unlocked by it)
};

template <class Backend>
class HostRegistry {
public:
    static constexpr int kUnmappable = -1000;
    // pages remembered as "nobody has locked these" (a packet starting there
    // cannot lie in someone else's page-locked allocation); dropped wholesale
    // past this many, so the set stays small
    static constexpr size_t kPageableMemo = 1u << 16;

    explicit HostRegistry(Backend& b) : b_(b) {}
    HostRegistry(const HostRegistry&) = delete;
    HostRegistry& operator=(const HostRegistry&) = delete;

    // Device address of the host bytes [p, p + len), len > 0, or kUnmappable.
    // may_lock: page-lock the packet's pages when nobody holds them (and the
    // registry would stay within max_owned bytes). A failed lock is
    // kUnmappable too (its backend error is kept in last_lock_error()).
    int resolve(uintptr_t p, size_t len, bool may_lock, uint64_t max_owned, uintptr_t* dev) {
        const uintptr_t e = p + len;
        if (find(p, e, dev)) return 0;
        const uintptr_t pg = p & ~(kHostPage - 1);
        // (a packet that starts in pages of ours and runs on past them needs no
        // lookup: the backend would only report our own registration)
        if (!owns(pg) && !pageable_.count(pg)) {
            uintptr_t rs = 0, re = 0;
            intptr_t delta = 0;
            if (b_.pinned_extent(p, &rs, &re, &delta)) {
                add_foreign(rs, re, delta);
                if (find(p, e, dev)) return 0;
                // p's page is held by someone else but the packet runs on past that
                // allocation: with may_lock the pages nobody holds are locked below
                // (never the other owner's), and the view joins the two mappings
                if (!may_lock) return kUnmappable;
            } else {
                if (pageable_.size() >= kPageableMemo) pageable_.clear();
                pageable_.insert(pg);
            }
        }
        if (!may_lock) return kUnmappable;
        const uintptr_t lo = pg, hi = (e + kHostPage - 1) & ~(kHostPage - 1);
        if (bytes_ + (hi - lo) > max_owned) return kUnmappable;
        if (lock_pages(lo, hi)) return kUnmappable;
        return find(p, e, dev) ? 0 : kUnmappable;
    }

    // Page-lock [p, p + bytes) ahead of use (tcpcsum_ctx_register_host).
    int lock_range(uintptr_t p, size_t bytes) {
        const uintptr_t lo = p & ~(kHostPage - 1), hi = (p + bytes + kHostPage - 1) & ~(kHostPage - 1);
        return lock_pages(lo, hi);
    }

    // Forget every range overlapping [p, p + bytes) (p == 0: all), unlocking the owned ones.
    void release(uintptr_t p, size_t bytes) {
        const uintptr_t lo = p, hi = p ? p + bytes : UINTPTR_MAX;
        std::vector<HostRange> keep;
        for (const auto& r : regs_) {
            if (r.lo < hi && r.hi > lo) {
                if (r.owned) {
                    b_.unlock(r.lo);
                    bytes_ -= r.hi - r.lo;
                }
            } else {
                keep.push_back(r);
            }
        }
        regs_.swap(keep);
        rebuild();
    }

    // Forget the mappings of memory page-locked by someone else (kept, they could
    // go stale: their owner may free or unregister them between two batches).
    // Called at the start of every batch. The pageable-page memo stays: a page
    // that was pageable and has since been locked by someone else is only
    // copied instead of read in place — slower, never wrong.
    void forget_foreign() {
        bool any = false;
        for (const auto& r : regs_) any = any || !r.owned;
        if (!any) return;
        std::vector<HostRange> keep;
        for (const auto& r : regs_)
            if (r.owned) keep.push_back(r);
        regs_.swap(keep);
        rebuild();
    }

    // Drop the pageable-page memo (the application locked memory the registry
    // had seen as pageable, and wants it read in place from now on).
    void forget_pageable() { pageable_.clear(); }

    uint64_t owned_ranges() const {
        uint64_t k = 0;
        for (const auto& r : regs_) k += r.owned ? 1u : 0u;
        return k;
    }
    uint64_t owned_bytes() const { return bytes_; }
    int last_lock_error() const { return last_error_; }
    const std::vector<HostRange>& ranges() const { return regs_; }

private:
    bool owns(uintptr_t pg) const {
        for (const auto& r : regs_)
            if (r.owned && r.lo <= pg && pg < r.hi) return true;
        return false;
    }

    // Someone else's page-locked allocation. HIP reports its extent as
    // allocated (e.g. an unaligned hipHostRegister); the device mapping is page
    // granular, so it is recorded rounded out to whole pages — otherwise a
    // packet crossing the allocation's last byte into the rest of that page
    // would fall between this range and the next.
    void add_foreign(uintptr_t rs, uintptr_t re, intptr_t delta) {
        rs &= ~(kHostPage - 1);
        re = (re + kHostPage - 1) & ~(kHostPage - 1);
        for (const auto& r : regs_)
            if (r.lo == rs && r.hi == re && r.delta == delta) return;
        regs_.push_back({rs, re, delta, false});
        rebuild();
    }

    // Lock the pages of [lo, hi) (page-aligned) that no known range covers. A
    // page already locked by someone else — another context of this process, the
    // application — is taken as theirs (recorded, never locked twice, never
    // unlocked here): HIP keeps one registration per page, so a second lock and a
    // second unlock would undo the first owner's.
    int lock_pages(uintptr_t lo, uintptr_t hi) {
        std::vector<std::pair<uintptr_t, uintptr_t>> gaps;
        uintptr_t cur = lo;
        for (const auto& r : regs_) {   // sorted by lo
            if (r.hi <= cur) continue;
            if (r.lo >= hi) break;
            if (r.lo > cur) gaps.push_back({cur, r.lo});
            if (r.hi > cur) cur = r.hi;
            if (cur >= hi) break;
        }
        if (cur < hi) gaps.push_back({cur, hi});
        int rc = 0;
        for (const auto& g : gaps) {
            uintptr_t pg = g.first;
            while (pg < g.second && !rc) {
                uintptr_t rs = 0, re = 0;
                intptr_t delta = 0;
                if (b_.pinned_extent(pg, &rs, &re, &delta)) {
                    const uintptr_t end = (re + kHostPage - 1) & ~(kHostPage - 1);
                    add_foreign(rs, re, delta);   // someone else's pages
                    pg = std::min<uintptr_t>(std::max<uintptr_t>(end, pg + kHostPage), g.second);
                    continue;
                }
                uintptr_t run = pg + kHostPage;   // the run of pages nobody has locked
                while (run < g.second && !b_.pinned_extent(run, &rs, &re, &delta)) run += kHostPage;
                rc = b_.lock(pg, run - pg, &delta);
                if (rc) {
                    last_error_ = rc;
                    break;
                }
                regs_.push_back({pg, run, delta, true});
                bytes_ += run - pg;
                pg = run;
            }
            if (rc) break;
        }
        rebuild();
        return rc;
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
                // ranges locked by someone else may overlap ours: look a few back
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
    uint64_t bytes_ = 0;
    int last_error_ = 0;
};

}  // namespace tcpcsum
