// Small-object allocator for the native shard executor (replaces global operator new/delete).
//
// The executor's hot path is allocation-heavy (JSON DOM nodes, strings, coroutine frames) and runs on
// one thread, so glibc malloc's general-purpose paths are most of its user time.  Requests up to 16 KiB
// are served from per-size-class free lists carved out of one reserved virtual region: 16-byte classes up
// to 512 bytes, then four classes per doubling (640, 768, 896, 1024, 1280 ... 16384: request and response
// bodies, raw payloads, HTTP buffers); everything larger, and anything once the region is exhausted, goes
// to malloc.  A pointer is
// ours iff it lies inside the region, so unsized deletes work too; each 64 KiB chunk of the region holds
// one size class (a side table maps chunk -> class).  Free lists are thread-local (OpenSSL and glibc may
// allocate from other threads through malloc, never through here; a block freed on another thread simply
// joins that thread's list).  Memory is kept for reuse, never returned to the OS: the executor's working
// set is bounded by its caches.
#pragma once

#include <sys/mman.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <new>

namespace ncc::alloc {

constexpr std::size_t kMaxSmall = 512;
constexpr std::size_t kMaxPooled = 16384;
constexpr std::size_t kSmallClasses = kMaxSmall / 16;
constexpr std::size_t kClasses = kSmallClasses + 4 * 5;  // 512 -> 16384: five doublings, four steps each
constexpr std::size_t kChunk = 64 * 1024;

// size class of a request of n (1 <= n <= kMaxPooled) bytes, and a class's block size
inline std::size_t class_of(std::size_t n) {
    if (n <= kMaxSmall) return (n - 1) >> 4;
    int hb = 63 - __builtin_clzll(static_cast<unsigned long long>(n - 1));  // n - 1 in [2^hb, 2^(hb+1))
    // (n - 1) >> (hb - 2) is 4..7: which quarter of the doubling
    return kSmallClasses + 4 * static_cast<std::size_t>(hb - 9) + ((n - 1) >> (hb - 2)) - 4;
}
inline std::size_t class_size(std::size_t cls) {
    if (cls < kSmallClasses) return (cls + 1) << 4;
    std::size_t j = cls - kSmallClasses, hb = 9 + j / 4;
    return (std::size_t(1) << hb) + ((j % 4) + 1) * (std::size_t(1) << (hb - 2));
}
constexpr std::size_t kRegion = std::size_t(64) << 30;  // 64 GiB of address space, committed lazily

struct Region {
    char* base = nullptr;
    std::atomic<std::size_t> used{0};
    uint8_t* chunk_class = nullptr;  // (class + 1) per chunk; 0 = unused
    Region() {
        void* p = mmap(nullptr, kRegion, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (p == MAP_FAILED) return;
        void* t = mmap(nullptr, kRegion / kChunk, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                       -1, 0);
        if (t == MAP_FAILED) {
            munmap(p, kRegion);
            return;
        }
        base = static_cast<char*>(p);
        chunk_class = static_cast<uint8_t*>(t);
    }
    bool owns(const void* q) const {
        return base != nullptr && static_cast<const char*>(q) >= base && static_cast<const char*>(q) < base + kRegion;
    }
};

inline Region& region() {
    static Region r;  // constructed on first allocation, before main; never destroyed
    return r;
}

struct FreeBlock {
    FreeBlock* next;
};

struct ThreadCache {
    FreeBlock* free[kClasses] = {};
    char* cur[kClasses] = {};  // bump pointer inside the class's current chunk
    char* end[kClasses] = {};
};

inline ThreadCache& cache() {
    static thread_local ThreadCache c;
    return c;
}

inline void* allocate(std::size_t n) {
    if (n == 0) n = 1;
    if (n <= kMaxPooled) {
        std::size_t cls = class_of(n);
        ThreadCache& tc = cache();
        if (FreeBlock* b = tc.free[cls]) {
            tc.free[cls] = b->next;
            __builtin_prefetch(b->next);  // the next pop of this class reads it: start the miss now
            return b;
        }
        std::size_t size = class_size(cls);
        if (tc.cur[cls] + size > tc.end[cls]) {
            Region& r = region();
            std::size_t off = r.base ? r.used.fetch_add(kChunk, std::memory_order_relaxed) : kRegion;
            if (off + kChunk <= kRegion) {
                tc.cur[cls] = r.base + off;
                tc.end[cls] = tc.cur[cls] + kChunk;
                r.chunk_class[off / kChunk] = static_cast<uint8_t>(cls + 1);
            } else {
                tc.cur[cls] = tc.end[cls] = nullptr;
            }
        }
        if (tc.cur[cls] != nullptr) {
            void* p = tc.cur[cls];
            tc.cur[cls] += size;
            return p;
        }
    }
    void* p = std::malloc(n);
    if (p == nullptr) throw std::bad_alloc();
    return p;
}

inline void release(void* p) noexcept {
    if (p == nullptr) return;
    Region& r = region();
    if (r.owns(p)) {
        std::size_t cls = r.chunk_class[(static_cast<char*>(p) - r.base) / kChunk] - 1u;
        FreeBlock* b = static_cast<FreeBlock*>(p);
        ThreadCache& tc = cache();
        b->next = tc.free[cls];
        tc.free[cls] = b;
        return;
    }
    std::free(p);
}

}  // namespace ncc::alloc

// Global replacements (this header is included by exactly one translation unit: executor.cpp).
void* operator new(std::size_t n) { return ncc::alloc::allocate(n); }
void* operator new[](std::size_t n) { return ncc::alloc::allocate(n); }
void* operator new(std::size_t n, const std::nothrow_t&) noexcept {
    try {
        return ncc::alloc::allocate(n);
    } catch (...) {
        return nullptr;
    }
}
void* operator new[](std::size_t n, const std::nothrow_t&) noexcept {
    try {
        return ncc::alloc::allocate(n);
    } catch (...) {
        return nullptr;
    }
}
void operator delete(void* p) noexcept { ncc::alloc::release(p); }
void operator delete[](void* p) noexcept { ncc::alloc::release(p); }
void operator delete(void* p, std::size_t) noexcept { ncc::alloc::release(p); }
void operator delete[](void* p, std::size_t) noexcept { ncc::alloc::release(p); }
