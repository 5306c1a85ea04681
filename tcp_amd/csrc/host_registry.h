// host_registry.h — which host pages a context has page-locked, and where the
// GPU sees them.
//
// tcpcsum_ipv4_batch_ptrs_host takes one pointer per packet (the reference's
// separately malloc'd out-buffers, loop.c:180-183). The kernel may only touch
// host pages that are page-locked and mapped for the device, so every packet
// [p, p + len) is resolved here to a device address, page-locking the pages
// nobody has locked yet. Header-only and templated on the backend that does
// the locking, so the bookkeeping runs under a CPU unit test with a fake
// backend (tests/c/registry_test.cpp) exactly as it runs over HIP.
//
// Backend interface:
//   int  lock(uintptr_t lo, size_t bytes, intptr_t* delta)
//          page-lock [lo, lo + bytes) (whole pages); device address = host + *delta.
//          0 on success, else a backend error (returned to the caller as is).
//   void unlock(uintptr_t lo)                      undo one lock() by its start.
//   bool pinned_extent(uintptr_t p, uintptr_t* lo, uintptr_t* hi, intptr_t* delta)
//          p lies in memory page-locked by someone else (or by us): the extent
//          of that allocation / registration and its device offset.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace tcpcsum {

constexpr uintptr_t kHostPage = 4096;

struct HostRange {
    uintptr_t lo, hi;
    intptr_t delta;   // device address = host address + delta
    bool owned;       // locked by this registry (unlocked by it)
};

template <class Backend>
class HostRegistry {
public:
    explicit HostRegistry(Backend& b) : b_(b) {}
    HostRegistry(const HostRegistry&) = delete;
    HostRegistry& operator=(const HostRegistry&) = delete;

    // Device address of the host bytes [p, p + len), len > 0; page-locks them on first use.
    // Returns 0, a backend error, or kUnmappable when no single mapping can cover them.
    static constexpr int kUnmappable = -1000;
    int resolve(uintptr_t p, size_t len, uintptr_t* dev) {
        const uintptr_t e = p + len;
        if (find(p, e, dev)) return 0;
        // memory page-locked by someone else: use that mapping, but only when the
        // allocation it belongs to covers the whole range — p may sit in a page
        // locked for a neighbouring buffer while the range runs on into pages
        // nobody has locked
        uintptr_t rs = 0, re = 0;
        intptr_t delta = 0;
        if (b_.pinned_extent(p, &rs, &re, &delta) && rs <= p && e <= re) {
            bool known = false;
            for (const auto& r : regs_) known = known || (r.lo == rs && r.hi == re);
            if (!known) {
                regs_.push_back({rs, re, delta, false});
                rebuild();
            }
            if (find(p, e, dev)) return 0;
        }
        const uintptr_t lo = p & ~(kHostPage - 1), hi = (e + kHostPage - 1) & ~(kHostPage - 1);
        int rc = lock_pages(lo, hi);
        if (rc) return rc;
        if (find(p, e, dev)) return 0;
        // the range spans locks mapped at unrelated device offsets (a host whose
        // registrations are not mapped at their host address): replace the owned
        // ones under it by a single lock of their union
        uintptr_t ulo = lo, uhi = hi;
        std::vector<HostRange> keep;
        for (const auto& r : regs_) {
            if (r.owned && r.lo < hi && r.hi > lo) {
                ulo = std::min(ulo, r.lo);
                uhi = std::max(uhi, r.hi);
                b_.unlock(r.lo);
                bytes_ -= r.hi - r.lo;
            } else {
                keep.push_back(r);
            }
        }
        regs_.swap(keep);
        rebuild();
        rc = lock_pages(ulo, uhi);
        if (rc) return rc;
        return find(p, e, dev) ? 0 : kUnmappable;
    }

    // Page-lock [p, p + bytes) ahead of use.
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
    // Called at the start of every batch; the first packet of a batch in such
    // memory looks its mapping up again.
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

    uint64_t owned_ranges() const {
        uint64_t k = 0;
        for (const auto& r : regs_) k += r.owned ? 1u : 0u;
        return k;
    }
    uint64_t owned_bytes() const { return bytes_; }
    const std::vector<HostRange>& ranges() const { return regs_; }

private:
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
                if (b_.pinned_extent(pg, &rs, &re, &delta) && rs <= pg && re > pg) {
                    bool known = false;
                    for (const auto& r : regs_) known = known || (r.lo == rs && r.hi == re);
                    if (!known) regs_.push_back({rs, re, delta, false});   // someone else's pages
                    pg = std::min<uintptr_t>((re + kHostPage - 1) & ~(kHostPage - 1), g.second);
                    continue;
                }
                uintptr_t run = pg + kHostPage;   // the run of pages nobody has locked
                while (run < g.second && !b_.pinned_extent(run, &rs, &re, &delta)) run += kHostPage;
                rc = b_.lock(pg, run - pg, &delta);
                if (rc) break;
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
            if (!view_.empty() && view_.back().hi == r.lo && view_.back().delta == r.delta)
                view_.back().hi = r.hi;
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
    size_t finger_ = 0;
    uint64_t bytes_ = 0;
};

}  // namespace tcpcsum
