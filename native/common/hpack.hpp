// HPACK, the header compression of HTTP/2 (RFC 7541): integer and string primitives, the static table, the
// canonical Huffman code, a decoder with its dynamic table, and a stateless encoder.
//
// Shared by the C++ shard executor's HTTP/2 client (native/executor/h2.hpp, C++20) and the extension
// (native/ncc_native.cpp, C++17), which hands the decoder to the fake apiserver's HTTP/2 server
// (ncc/fakeapi/h2.py) — so the two ends of every HTTP/2 test share no code path by accident but the table.
//
// The encoder never inserts into the peer's dynamic table: every field is a literal "without indexing"
// (a static-table name index where there is one), so the encoder has no state to keep in step with the
// peer and a SETTINGS_HEADER_TABLE_SIZE change needs no size update from us.  The decoder implements all
// of RFC 7541 §6: indexed fields, the three literal forms with static or dynamic name indexes, Huffman
// strings, dynamic table size updates at the start of a block, eviction.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace ncc {
namespace hpack {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Code length of each symbol (0..255, 256 = EOS) of the HPACK Huffman code (RFC 7541 Appendix B).  The code is
// canonical — codes of one length are consecutive and ordered by symbol, each length's first code follows
// the previous length's last — so the lengths determine every code (HuffTables).  Checked against the RFC's
// Appendix C examples in tests/test_http2.py.
inline constexpr unsigned char kHuffLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,
    6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15, 6, 12, 10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5, 6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28,
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, 19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,
    30};

struct HuffTables {
    static constexpr int kMaxLen = 30;
    uint32_t code[257] = {};
    uint32_t first[kMaxLen + 1] = {};   // the first (lowest) code of each length
    uint16_t count[kMaxLen + 1] = {};   // codes of each length
    uint16_t offset[kMaxLen + 1] = {};  // index of that first code's symbol in `sorted`
    uint16_t sorted[257] = {};          // symbols by (length, symbol)

    HuffTables() {
        for (int s = 0; s < 257; ++s) ++count[kHuffLen[s]];
        uint16_t at = 0;
        for (int l = 1; l <= kMaxLen; ++l) {
            offset[l] = at;
            at = static_cast<uint16_t>(at + count[l]);
        }
        uint16_t fill[kMaxLen + 1];
        std::memcpy(fill, offset, sizeof fill);
        for (int s = 0; s < 257; ++s) sorted[fill[kHuffLen[s]]++] = static_cast<uint16_t>(s);
        uint32_t c = 0;
        int prev = 0;
        for (int l = 1; l <= kMaxLen; ++l) {
            c <<= (l - prev);
            prev = l;
            first[l] = c;
            for (int k = 0; k < count[l]; ++k) code[sorted[offset[l] + k]] = c++;
        }
    }
};

inline const HuffTables& huff() {
    static const HuffTables t;
    return t;
}

inline std::string huffman_encode(std::string_view s) {
    const HuffTables& h = huff();
    std::string out;
    out.reserve(s.size());
    uint64_t bits = 0;
    int nb = 0;
    for (unsigned char ch : s) {
        bits = (bits << kHuffLen[ch]) | h.code[ch];
        nb += kHuffLen[ch];
        while (nb >= 8) {
            nb -= 8;
            out.push_back(static_cast<char>((bits >> nb) & 0xff));
        }
    }
    if (nb > 0) out.push_back(static_cast<char>(((bits << (8 - nb)) | ((1u << (8 - nb)) - 1)) & 0xff));  // EOS prefix
    return out;
}

inline size_t huffman_length(std::string_view s) {
    size_t bits = 0;
    for (unsigned char ch : s) bits += kHuffLen[ch];
    return (bits + 7) / 8;
}

inline void huffman_decode(const uint8_t* p, size_t n, std::string& out) {
    const HuffTables& h = huff();
    uint32_t v = 0;
    int len = 0;
    for (size_t i = 0; i < n; ++i) {
        for (int b = 7; b >= 0; --b) {
            v = (v << 1) | ((p[i] >> b) & 1u);
            ++len;
            if (len > HuffTables::kMaxLen) throw Error("invalid Huffman code");
            if (h.count[len] != 0 && v >= h.first[len] && v - h.first[len] < h.count[len]) {
                uint16_t sym = h.sorted[h.offset[len] + (v - h.first[len])];
                if (sym == 256) throw Error("EOS in a Huffman string");
                out.push_back(static_cast<char>(sym));
                v = 0;
                len = 0;
            }
        }
    }
    // padding: fewer than 8 bits, all ones (a prefix of EOS)
    if (len > 7 || v != (len == 0 ? 0u : ((1u << len) - 1))) throw Error("invalid Huffman padding");
}

// ---- the static table (RFC 7541 Appendix A); index 1..61
struct Field {
    const char* name;
    const char* value;
};
inline constexpr Field kStatic[62] = {
    {"", ""},
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""}, {"cache-control", ""},
    {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""}, {"content-length", ""},
    {"content-location", ""}, {"content-range", ""}, {"content-type", ""}, {"cookie", ""}, {"date", ""},
    {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""}, {"if-match", ""},
    {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""}, {"if-unmodified-since", ""},
    {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""}, {"proxy-authenticate", ""},
    {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""}, {"retry-after", ""},
    {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""}, {"transfer-encoding", ""},
    {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};
inline constexpr int kStaticCount = 61;

// the static index of `name` (the first entry with it), or 0
inline int static_name_index(std::string_view name) {
    for (int i = 1; i <= kStaticCount; ++i)
        if (name == kStatic[i].name) return i;
    return 0;
}

// ---- primitives (RFC 7541 §5)
inline void encode_int(std::string& out, uint64_t v, int prefix, uint8_t high_bits) {
    const uint64_t max = (uint64_t{1} << prefix) - 1;
    if (v < max) {
        out.push_back(static_cast<char>(high_bits | v));
        return;
    }
    out.push_back(static_cast<char>(high_bits | max));
    v -= max;
    while (v >= 128) {
        out.push_back(static_cast<char>((v & 0x7f) | 0x80));
        v >>= 7;
    }
    out.push_back(static_cast<char>(v));
}

inline uint64_t decode_int(const uint8_t*& p, const uint8_t* end, int prefix) {
    if (p >= end) throw Error("truncated integer");
    const uint64_t max = (uint64_t{1} << prefix) - 1;
    uint64_t v = *p++ & max;
    if (v < max) return v;
    for (int shift = 0;; shift += 7) {
        if (p >= end) throw Error("truncated integer");
        if (shift > 56) throw Error("integer overflow");
        uint8_t b = *p++;
        v += static_cast<uint64_t>(b & 0x7f) << shift;
        if ((b & 0x80) == 0) return v;
    }
}

inline void encode_string(std::string& out, std::string_view s, bool huffman = false) {
    if (huffman) {
        size_t hl = huffman_length(s);
        if (hl < s.size()) {
            encode_int(out, hl, 7, 0x80);
            out += huffman_encode(s);
            return;
        }
    }
    encode_int(out, s.size(), 7, 0x00);
    out.append(s.data(), s.size());
}

inline std::string decode_string(const uint8_t*& p, const uint8_t* end) {
    if (p >= end) throw Error("truncated string");
    bool huffman = (*p & 0x80) != 0;
    uint64_t n = decode_int(p, end, 7);
    if (n > static_cast<uint64_t>(end - p)) throw Error("truncated string");
    std::string out;
    if (huffman) {
        out.reserve(static_cast<size_t>(n) * 8 / 5);
        huffman_decode(p, static_cast<size_t>(n), out);
    } else {
        out.assign(reinterpret_cast<const char*>(p), static_cast<size_t>(n));
    }
    p += n;
    return out;
}

// ---- encoder (stateless: literals without indexing)
inline void encode_indexed(std::string& out, int index) { encode_int(out, static_cast<uint64_t>(index), 7, 0x80); }

inline void encode_literal(std::string& out, std::string_view name, std::string_view value, bool huffman = false) {
    int ni = static_name_index(name);
    if (ni != 0) {
        encode_int(out, static_cast<uint64_t>(ni), 4, 0x00);
    } else {
        out.push_back(0x00);
        encode_string(out, name, huffman);
    }
    encode_string(out, value, huffman);
}

// A literal without indexing whose name is static-table entry `name_index` (no lookup: the caller knows it).
inline void encode_literal_indexed_name(std::string& out, int name_index, std::string_view value) {
    encode_int(out, static_cast<uint64_t>(name_index), 4, 0x00);
    encode_string(out, value, false);
}

// A field from the static table when it holds (name, value) exactly, else a literal.
inline void encode_field(std::string& out, std::string_view name, std::string_view value, bool huffman = false) {
    for (int i = 1; i <= kStaticCount; ++i)
        if (kStatic[i].value[0] != '\0' && name == kStatic[i].name && value == kStatic[i].value) {
            encode_indexed(out, i);
            return;
        }
    encode_literal(out, name, value, huffman);
}

// ---- decoder
class Decoder {
public:
    using Header = std::pair<std::string, std::string>;

    explicit Decoder(size_t max_table = 4096) : limit_(max_table), max_(max_table) {}

    // The most the peer may size the table to (our SETTINGS_HEADER_TABLE_SIZE).
    void set_limit(size_t limit) {
        limit_ = limit;
        if (max_ > limit_) {
            max_ = limit_;
            evict(0);
        }
    }
    size_t table_size() const { return size_; }
    size_t table_entries() const { return table_.size(); }

    // Decode one complete header block (HEADERS + CONTINUATION payloads, concatenated).
    void decode(const uint8_t* p, size_t n, std::vector<Header>& out) {
        const uint8_t* end = p + n;
        bool start = true;
        while (p < end) {
            uint8_t b = *p;
            if (b & 0x80) {  // indexed field
                uint64_t i = decode_int(p, end, 7);
                out.push_back(lookup(i));
            } else if ((b & 0xc0) == 0x40) {  // literal with incremental indexing
                Header h = literal(p, end, 6);
                add(h);
                out.push_back(std::move(h));
            } else if ((b & 0xe0) == 0x20) {  // dynamic table size update
                if (!start) throw Error("table size update after the first field of a block");
                uint64_t sz = decode_int(p, end, 5);
                if (sz > limit_) throw Error("table size update above the limit");
                max_ = static_cast<size_t>(sz);
                evict(0);
                continue;  // more updates may follow at the start
            } else {  // literal without indexing (0000) or never indexed (0001)
                out.push_back(literal(p, end, 4));
            }
            start = false;
        }
    }

private:
    std::deque<Header> table_;  // newest first: dynamic index 62 is table_[0]
    size_t size_ = 0, limit_, max_;

    Header lookup(uint64_t i) const {
        if (i == 0) throw Error("index 0");
        if (i <= static_cast<uint64_t>(kStaticCount)) return {kStatic[i].name, kStatic[i].value};
        uint64_t d = i - kStaticCount - 1;
        if (d >= table_.size()) throw Error("index past the dynamic table");
        return table_[static_cast<size_t>(d)];
    }
    Header literal(const uint8_t*& p, const uint8_t* end, int prefix) {
        uint64_t ni = decode_int(p, end, prefix);
        Header h;
        if (ni == 0)
            h.first = decode_string(p, end);
        else
            h.first = lookup(ni).first;
        h.second = decode_string(p, end);
        return h;
    }
    static size_t entry_size(const Header& h) { return h.first.size() + h.second.size() + 32; }
    void evict(size_t room) {
        while (!table_.empty() && size_ + room > max_) {
            size_ -= entry_size(table_.back());
            table_.pop_back();
        }
    }
    void add(const Header& h) {
        size_t sz = entry_size(h);
        if (sz > max_) {  // larger than the whole table: empties it (RFC 7541 §4.4)
            table_.clear();
            size_ = 0;
            return;
        }
        evict(sz);
        table_.push_front(h);
        size_ += sz;
    }
};

}  // namespace hpack
}  // namespace ncc
