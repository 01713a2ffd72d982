// JSON byte scanning shared by the C++ shard executor (native/executor/json.hpp) and the Python extension
// (native/ncc_native.cpp): SSE2 (part of every x86-64) searches for quotes and brackets, and a container skip
// that goes 64 bytes per step; other targets get the same functions a byte at a time.  Only valid JSON text
// is expected; a skipped container is not validated.
#pragma once

#include <cstdint>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif

namespace ncc {

// ------------------------------------------------------------------------------------ byte search
// 16 bytes per step (SSE2, part of every x86-64): JSON text is mostly string content and structure-free runs.
// The first '"' or '\\' in [p, e), or e.
inline const char* find_quote(const char* p, const char* e) {
#if defined(__SSE2__)
    const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\');
    while (e - p >= 16) {
        __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
        int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, b)));
        if (m) return p + __builtin_ctz(static_cast<unsigned>(m));
        p += 16;
    }
#endif
    while (p < e && *p != '"' && *p != '\\') ++p;
    return p;
}
// The first '"', '{', '}', '[' or ']' in [p, e), or e ('[' | 0x20 == '{', ']' | 0x20 == '}').
inline const char* find_structural(const char* p, const char* e) {
#if defined(__SSE2__)
    const __m128i q = _mm_set1_epi8('"'), lo = _mm_set1_epi8(0x20), open = _mm_set1_epi8('{'),
                  close = _mm_set1_epi8('}');
    while (e - p >= 16) {
        __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
        __m128i f = _mm_or_si128(x, lo);
        int m = _mm_movemask_epi8(
            _mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_or_si128(_mm_cmpeq_epi8(f, open), _mm_cmpeq_epi8(f, close))));
        if (m) return p + __builtin_ctz(static_cast<unsigned>(m));
        p += 16;
    }
#endif
    while (p < e && *p != '"' && (*p | 0x20) != '{' && (*p | 0x20) != '}') ++p;
    return p;
}
// Past the string whose opening quote is at p (escapes skipped, not checked); nullptr when unterminated.
inline const char* skip_string_text(const char* p, const char* e) {
    ++p;
    while (true) {
        p = find_quote(p, e);
        if (p >= e) return nullptr;
        if (*p == '"') return p + 1;
        p += 2;  // the escaped character
    }
}
// 64 bytes as bit masks: bit i of each mask describes p[i]
struct Block64 {
    uint64_t quote, backslash, open, close;
    explicit Block64(const char* p) {
        quote = backslash = open = close = 0;
#if defined(__SSE2__)
        const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), lo = _mm_set1_epi8(0x20),
                      op = _mm_set1_epi8('{'), cl = _mm_set1_epi8('}');
        for (int i = 0; i < 4; ++i) {
            __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * i));
            __m128i f = _mm_or_si128(x, lo);  // '[' | 0x20 == '{', ']' | 0x20 == '}'
            int sh = 16 * i;
            quote |= static_cast<uint64_t>(static_cast<uint16_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(x, q)))) << sh;
            backslash |= static_cast<uint64_t>(static_cast<uint16_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(x, bs)))) << sh;
            open |= static_cast<uint64_t>(static_cast<uint16_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(f, op)))) << sh;
            close |= static_cast<uint64_t>(static_cast<uint16_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(f, cl)))) << sh;
        }
#else  // portable: the same masks a byte at a time
        for (int i = 0; i < 64; ++i) {
            char c = p[i], f = static_cast<char>(c | 0x20);
            uint64_t bit = 1ULL << i;
            if (c == '"') quote |= bit;
            if (c == '\\') backslash |= bit;
            if (f == '{') open |= bit;
            if (f == '}') close |= bit;
        }
#endif
    }
};
inline uint64_t prefix_xor(uint64_t x) {
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    return x;
}
// Past the object or array whose bracket is at p; nullptr when unbalanced.  64 bytes per step while a block
// has no backslash: the in-string mask is the prefix XOR of the quote bits, brackets outside strings move the
// depth, and only a block where the depth could reach zero has its brackets walked one by one.  A block with
// a backslash (or a string escape carried into it) is read byte by byte.  The last, short block is copied
// into a zero-padded one (NUL is no JSON structure), so a container ending near the end of its buffer — a
// watch line's object, a response body — does not fall back to bytes.
struct ContainerSkip {
    int depth = 0;
    bool in_str = false, esc = false;
    // the `n` bytes of `blk` (64 readable): the offset just past the closing bracket, or -1
    int block(const char* blk, int n) {
        Block64 b(blk);
        if (b.backslash == 0 && !esc) {
            uint64_t str = prefix_xor(b.quote) ^ (in_str ? ~0ULL : 0ULL);  // 1 = inside a string (open quote incl.)
            uint64_t op = b.open & ~str, cl = b.close & ~str;
            int ncl = __builtin_popcountll(cl);
            if (depth > ncl) {
                depth += __builtin_popcountll(op) - ncl;
            } else {
                uint64_t br = op | cl;
                while (br) {
                    int i = __builtin_ctzll(br);
                    br &= br - 1;
                    if ((op >> i) & 1) {
                        ++depth;
                    } else if (--depth == 0) {
                        return i + 1;
                    }
                }
            }
            in_str = (str >> 63) & 1;
            return -1;
        }
        for (int i = 0; i < n; ++i) {
            char c = blk[i];
            if (in_str) {
                if (esc) {
                    esc = false;
                } else if (c == '\\') {
                    esc = true;
                } else if (c == '"') {
                    in_str = false;
                }
            } else if (c == '"') {
                in_str = true;
            } else if ((c | 0x20) == '{') {
                ++depth;
            } else if ((c | 0x20) == '}') {
                if (--depth == 0) return i + 1;
            }
        }
        return -1;
    }
};
inline const char* skip_container_text(const char* p, const char* e) {
    ContainerSkip st;
    while (e - p >= 64) {
        int r = st.block(p, 64);
        if (r >= 0) return p + r;
        p += 64;
    }
    if (p < e) {
        char tail[64] = {};
        const int n = static_cast<int>(e - p);
        __builtin_memcpy(tail, p, static_cast<unsigned long>(n));
        int r = st.block(tail, n);
        if (r >= 0) return p + r;
    }
    return nullptr;
}

// The first '"', '\\' or control byte (< 0x20, invalid inside a JSON string) in [p, e), or e.
inline const char* find_quote_or_ctl(const char* p, const char* e) {
#if defined(__SSE2__)
    const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\'), c = _mm_set1_epi8(0x1F);
    while (e - p >= 16) {
        __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
        __m128i ctl = _mm_cmpeq_epi8(_mm_max_epu8(x, c), c);  // x <= 0x1F, unsigned
        int m = _mm_movemask_epi8(_mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, b)), ctl));
        if (m) return p + __builtin_ctz(static_cast<unsigned>(m));
        p += 16;
    }
#endif
    while (p < e && *p != '"' && *p != '\\' && static_cast<unsigned char>(*p) >= 0x20) ++p;
    return p;
}

}  // namespace ncc
