// native/executor/strmap.hpp — the executor's string-keyed caches (shard stores, controller-side objects, write
// memos, dependent → template index) as one open-addressing table.
//
// std::unordered_map keeps every entry in its own heap node behind a bucket array, and libstdc++ maps a hash to
// a bucket with an integer division by a prime: a lookup is the division, the bucket load, the node load and
// the key's own buffer — three dependent cache misses on a cache of 10^5 objects.  The executor's sampling
// profile put 15 % of its CPU there (profiles/r6/r6h/executor_profile.txt: _M_find_before_node, the hash-code
// compare, _Mod_range_hashing, _Hash_bytes and the key memcmp).  Here the entries sit in one power-of-two
// array with their 64-bit hash beside them (linear probing from the hash's top bits, at most 70 % full): a
// lookup is a shift, a walk over adjacent slots comparing hashes, and one key compare on the match.
//
// Not a drop-in for every use: a rehash moves the entries, so a pointer or reference into the table does not
// survive an insertion into the same table (the work queue, which hands out references to its nodes, stays on
// std::unordered_map).  Erasing leaves a tombstone, so erasing during iteration is fine and iterators to other
// entries stay valid until the next insertion.  Lookups take std::string_view (no key string built to find).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <string_view>
#include <tuple>
#include <type_traits>
#include <utility>

namespace ncc {

inline uint64_t strmap_hash(std::string_view s) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    uint64_t h = 0x2545F4914F6CDD1DULL ^ (s.size() * m);
    const char* p = s.data();
    size_t n = s.size();
    while (n >= 8) {
        uint64_t k;
        std::memcpy(&k, p, 8);
        k *= m;
        k ^= k >> 47;
        k *= m;
        h ^= k;
        h *= m;
        p += 8;
        n -= 8;
    }
    uint64_t tail = 0;
    for (size_t i = 0; i < n; ++i) tail |= static_cast<uint64_t>(static_cast<unsigned char>(p[i])) << (8 * i);
    h ^= tail;
    h *= m;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    return h;
}

template <class V>
class StrMap {
  public:
    using key_type = std::string;
    using mapped_type = V;
    using value_type = std::pair<const std::string, V>;

  private:
    static constexpr uint64_t kEmpty = 0, kDeleted = 1;
    struct Slot {
        uint64_t tag;  // kEmpty, kDeleted, or the key's hash with bit 1 set (never 0 or 1)
        alignas(value_type) unsigned char buf[sizeof(value_type)];
        value_type& kv() { return *std::launder(reinterpret_cast<value_type*>(buf)); }
        const value_type& kv() const { return *std::launder(reinterpret_cast<const value_type*>(buf)); }
    };
    static uint64_t tag_of(uint64_t h) { return h | 2; }
    size_t home(uint64_t tag) const { return static_cast<size_t>(tag >> shift_); }  // the high bits: kept in the tag

    template <bool Const>
    class Iter {
        using S = std::conditional_t<Const, const Slot, Slot>;
        S* p_ = nullptr;
        S* e_ = nullptr;
        void skip() {
            while (p_ != e_ && p_->tag <= kDeleted) ++p_;
        }
        friend class StrMap;

      public:
        using reference = std::conditional_t<Const, const value_type&, value_type&>;
        using pointer = std::conditional_t<Const, const value_type*, value_type*>;
        Iter() = default;
        Iter(S* p, S* e, bool at_entry) : p_(p), e_(e) {
            if (!at_entry) skip();
        }
        template <bool C = Const, class = std::enable_if_t<C>>
        Iter(const Iter<false>& o) : p_(o.p_), e_(o.e_) {}  // iterator -> const_iterator
        reference operator*() const { return p_->kv(); }
        pointer operator->() const { return &p_->kv(); }
        Iter& operator++() {
            ++p_;
            skip();
            return *this;
        }
        bool operator==(const Iter& o) const { return p_ == o.p_; }
        bool operator!=(const Iter& o) const { return p_ != o.p_; }
        template <bool> friend class Iter;
    };

  public:
    using iterator = Iter<false>;
    using const_iterator = Iter<true>;

    StrMap() = default;
    StrMap(const StrMap&) = delete;
    StrMap& operator=(const StrMap&) = delete;
    StrMap(StrMap&& o) noexcept { steal(o); }
    StrMap& operator=(StrMap&& o) noexcept {
        if (this != &o) {
            release();
            steal(o);
        }
        return *this;
    }
    ~StrMap() { release(); }

    size_t size() const { return size_; }
    bool empty() const { return size_ == 0; }
    iterator begin() { return iterator(slots_, slots_ + cap_, false); }
    iterator end() { return iterator(slots_ + cap_, slots_ + cap_, true); }
    const_iterator begin() const { return const_iterator(slots_, slots_ + cap_, false); }
    const_iterator end() const { return const_iterator(slots_ + cap_, slots_ + cap_, true); }

    iterator find(std::string_view k) {
        Slot* s = locate(k, strmap_hash(k));
        return s ? iterator(s, slots_ + cap_, true) : end();
    }
    const_iterator find(std::string_view k) const {
        const Slot* s = const_cast<StrMap*>(this)->locate(k, strmap_hash(k));
        return s ? const_iterator(s, slots_ + cap_, true) : end();
    }
    size_t count(std::string_view k) const { return find(k) != end() ? 1 : 0; }

    template <class K, class... Args>
    std::pair<iterator, bool> try_emplace(K&& key, Args&&... args) {
        std::string_view kv(key);
        uint64_t h = strmap_hash(kv);
        if (Slot* s = locate(kv, h)) return {iterator(s, slots_ + cap_, true), false};
        Slot* s = insert_slot(h);
        ::new (static_cast<void*>(s->buf)) value_type(std::piecewise_construct,
                                                        std::forward_as_tuple(std::forward<K>(key)),
                                                        std::forward_as_tuple(std::forward<Args>(args)...));
        s->tag = tag_of(h);
        ++size_;
        return {iterator(s, slots_ + cap_, true), true};
    }
    template <class K, class M>
    std::pair<iterator, bool> emplace(K&& key, M&& value) {
        return try_emplace(std::forward<K>(key), std::forward<M>(value));
    }
    V& operator[](const std::string& k) { return try_emplace(k).first->second; }
    V& operator[](std::string&& k) { return try_emplace(std::move(k)).first->second; }

    iterator erase(iterator it) {
        Slot* s = const_cast<Slot*>(it.p_);
        s->kv().~value_type();
        s->tag = kDeleted;
        --size_;
        ++it;
        return it;
    }
    size_t erase(std::string_view k) {
        Slot* s = locate(k, strmap_hash(k));
        if (s == nullptr) return 0;
        erase(iterator(s, slots_ + cap_, true));
        return 1;
    }
    void clear() {
        for (size_t i = 0; i < cap_; ++i) {
            if (slots_[i].tag > kDeleted) slots_[i].kv().~value_type();
            slots_[i].tag = kEmpty;
        }
        size_ = used_ = 0;
    }
    void reserve(size_t n) {
        size_t want = 16;
        while (want * 7 < n * 10) want <<= 1;
        if (want > cap_) rehash(want);
    }

  private:
    Slot* slots_ = nullptr;
    size_t cap_ = 0;   // 0 or a power of two
    size_t size_ = 0;  // live entries
    size_t used_ = 0;  // live entries + tombstones (what stops a probe)
    int shift_ = 64;   // 64 - log2(cap_): a slot's home is the top log2(cap_) bits of its hash

    Slot* locate(std::string_view k, uint64_t h) {
        if (cap_ == 0) return nullptr;
        const uint64_t t = tag_of(h), mask = cap_ - 1;
        for (size_t i = home(t);; i = (i + 1) & mask) {
            Slot& s = slots_[i];
            if (s.tag == kEmpty) return nullptr;
            if (s.tag == t && s.kv().first == k) return &s;
        }
    }
    // a free slot for a key known to be absent (the table grown or cleaned first if need be)
    Slot* insert_slot(uint64_t h) {
        if ((used_ + 1) * 10 > cap_ * 7)  // past 70 % full: double, or only drop the tombstones when they are most of it
            rehash(cap_ == 0 ? 16 : (size_ + 1) * 20 > cap_ * 7 ? cap_ * 2 : cap_);
        const uint64_t mask = cap_ - 1;
        for (size_t i = home(tag_of(h));; i = (i + 1) & mask) {
            Slot& s = slots_[i];
            if (s.tag == kDeleted) return &s;
            if (s.tag == kEmpty) {
                ++used_;
                return &s;
            }
        }
    }
    void rehash(size_t cap) {
        Slot* old = slots_;
        size_t old_cap = cap_;
        slots_ = new Slot[cap];
        for (size_t i = 0; i < cap; ++i) slots_[i].tag = kEmpty;
        cap_ = cap;
        shift_ = 64 - __builtin_ctzll(static_cast<unsigned long long>(cap));
        used_ = size_;
        const uint64_t mask = cap_ - 1;
        for (size_t i = 0; i < old_cap; ++i) {
            Slot& o = old[i];
            if (o.tag <= kDeleted) continue;
            size_t j = home(o.tag);
            while (slots_[j].tag != kEmpty) j = (j + 1) & mask;
            ::new (static_cast<void*>(slots_[j].buf))
                value_type(std::move(const_cast<std::string&>(o.kv().first)), std::move(o.kv().second));
            slots_[j].tag = o.tag;
            o.kv().~value_type();
        }
        delete[] old;
    }
    void release() {
        if (slots_ == nullptr) return;
        for (size_t i = 0; i < cap_; ++i)
            if (slots_[i].tag > kDeleted) slots_[i].kv().~value_type();
        delete[] slots_;
        slots_ = nullptr;
        cap_ = size_ = used_ = 0;
        shift_ = 64;
    }
    void steal(StrMap& o) {
        slots_ = o.slots_;
        cap_ = o.cap_;
        size_ = o.size_;
        used_ = o.used_;
        shift_ = o.shift_;
        o.slots_ = nullptr;
        o.cap_ = o.size_ = o.used_ = 0;
        o.shift_ = 64;
    }
};

}  // namespace ncc
