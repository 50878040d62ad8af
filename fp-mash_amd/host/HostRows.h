// HostRows.h — page-populated host arrays for device results and uploads (sketch rows,
// packed reference matrices: tens of MB).
#pragma once

#include <algorithm>
#include <cstddef>
#include <new>
#include <sys/mman.h>

namespace fpmhost {

// Host array for device rows (C2's sketch rows or packed matrix: 80 MB): anonymous pages
// (zero, no memset), huge pages where the kernel allows them, populated up front in one call
// instead of ~20k first-touch page faults (a value-initialised std::vector paid both).
template <typename T>
struct HostRows {
    T *p = nullptr;
    size_t bytes = 0;
    // populate = false: the caller runs populate() later (e.g. on a thread beside device work)
    explicit HostRows(size_t n, bool populateNow = true) : bytes(std::max<size_t>(n * sizeof(T), 1))
    {
        void *q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(q, bytes, MADV_HUGEPAGE);
        p = static_cast<T *>(q);
        if (populateNow) populate();
    }
    void populate()
    {
#ifdef MADV_POPULATE_WRITE
        (void)madvise(p, bytes, MADV_POPULATE_WRITE);   // best effort (Linux >= 5.14)
#endif
    }
    ~HostRows() { munmap(p, bytes); }
    HostRows(const HostRows &) = delete;
    HostRows &operator=(const HostRows &) = delete;
    T *data() { return p; }
    T *begin() { return p; }
};

}  // namespace fpmhost
