// The msgpack subset spoken on the coordinator <-> executor socketpair (ncc/controller/ipc.py):
// frames are a 4-byte big-endian length (high bit: the body is an array of messages) followed by
// one msgpack value; messages are maps with string keys.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace ncc::mp {

struct Obj {
    enum Type : uint8_t { NIL, BOOL, INT, FLOAT, STR, BIN, ARR, MAP };
    Type t = NIL;
    bool b = false;
    long long i = 0;
    double d = 0;
    std::string s;  // STR and BIN payloads
    std::vector<Obj> a;
    std::vector<std::pair<Obj, Obj>> m;

    const Obj* get(std::string_view key) const {
        if (t != MAP) return nullptr;
        for (const auto& kv : m)
            if (kv.first.t == STR && kv.first.s == key) return &kv.second;
        return nullptr;
    }
    std::string_view sget(std::string_view key) const {
        const Obj* o = get(key);
        return (o != nullptr && (o->t == STR || o->t == BIN)) ? std::string_view(o->s) : std::string_view();
    }
    long long iget(std::string_view key, long long dflt = 0) const {
        const Obj* o = get(key);
        return (o != nullptr && o->t == INT) ? o->i : dflt;
    }
};

struct Decoder {
    const unsigned char* p;
    const unsigned char* e;

    [[noreturn]] static void fail() { throw std::runtime_error("msgpack: malformed frame"); }
    void need(size_t n) {
        if (static_cast<size_t>(e - p) < n) fail();
    }
    uint64_t be(int n) {
        need(static_cast<size_t>(n));
        uint64_t v = 0;
        for (int k = 0; k < n; ++k) v = (v << 8) | p[k];
        p += n;
        return v;
    }
    void bytes(std::string& out, size_t n) {
        need(n);
        out.assign(reinterpret_cast<const char*>(p), n);
        p += n;
    }
    void decode(Obj& o, int depth = 0) {
        if (depth > 64) fail();
        need(1);
        unsigned c = *p++;
        if (c <= 0x7f) {
            o.t = Obj::INT;
            o.i = c;
        } else if (c >= 0xe0) {
            o.t = Obj::INT;
            o.i = static_cast<int8_t>(c);
        } else if ((c & 0xf0) == 0x80) {
            map(o, c & 0x0f, depth);
        } else if ((c & 0xf0) == 0x90) {
            arr(o, c & 0x0f, depth);
        } else if ((c & 0xe0) == 0xa0) {
            o.t = Obj::STR;
            bytes(o.s, c & 0x1f);
        } else {
            switch (c) {
                case 0xc0: o.t = Obj::NIL; break;
                case 0xc2: o.t = Obj::BOOL; o.b = false; break;
                case 0xc3: o.t = Obj::BOOL; o.b = true; break;
                case 0xc4: o.t = Obj::BIN; bytes(o.s, be(1)); break;
                case 0xc5: o.t = Obj::BIN; bytes(o.s, be(2)); break;
                case 0xc6: o.t = Obj::BIN; bytes(o.s, be(4)); break;
                case 0xca: {
                    uint32_t u = static_cast<uint32_t>(be(4));
                    float f;
                    std::memcpy(&f, &u, 4);
                    o.t = Obj::FLOAT;
                    o.d = f;
                    break;
                }
                case 0xcb: {
                    uint64_t u = be(8);
                    o.t = Obj::FLOAT;
                    std::memcpy(&o.d, &u, 8);
                    break;
                }
                case 0xcc: o.t = Obj::INT; o.i = static_cast<long long>(be(1)); break;
                case 0xcd: o.t = Obj::INT; o.i = static_cast<long long>(be(2)); break;
                case 0xce: o.t = Obj::INT; o.i = static_cast<long long>(be(4)); break;
                case 0xcf: o.t = Obj::INT; o.i = static_cast<long long>(be(8)); break;
                case 0xd0: o.t = Obj::INT; o.i = static_cast<int8_t>(be(1)); break;
                case 0xd1: o.t = Obj::INT; o.i = static_cast<int16_t>(be(2)); break;
                case 0xd2: o.t = Obj::INT; o.i = static_cast<int32_t>(be(4)); break;
                case 0xd3: o.t = Obj::INT; o.i = static_cast<long long>(be(8)); break;
                case 0xd9: o.t = Obj::STR; bytes(o.s, be(1)); break;
                case 0xda: o.t = Obj::STR; bytes(o.s, be(2)); break;
                case 0xdb: o.t = Obj::STR; bytes(o.s, be(4)); break;
                case 0xdc: arr(o, be(2), depth); break;
                case 0xdd: arr(o, be(4), depth); break;
                case 0xde: map(o, be(2), depth); break;
                case 0xdf: map(o, be(4), depth); break;
                default: fail();
            }
        }
    }
    void arr(Obj& o, uint64_t n, int depth) {
        o.t = Obj::ARR;
        if (n > static_cast<uint64_t>(e - p)) fail();
        o.a.resize(n);
        for (auto& x : o.a) decode(x, depth + 1);
    }
    void map(Obj& o, uint64_t n, int depth) {
        o.t = Obj::MAP;
        if (n > static_cast<uint64_t>(e - p)) fail();
        o.m.resize(n);
        for (auto& kv : o.m) {
            decode(kv.first, depth + 1);
            decode(kv.second, depth + 1);
        }
    }
};

inline Obj decode(std::string_view body) {
    Decoder d{reinterpret_cast<const unsigned char*>(body.data()),
              reinterpret_cast<const unsigned char*>(body.data()) + body.size()};
    Obj o;
    d.decode(o);
    return o;
}

// ------------------------------------------------------------------------------------ encode
struct Encoder {
    std::string out;

    void put_be(uint64_t v, int n) {
        for (int k = n - 1; k >= 0; --k) out.push_back(static_cast<char>((v >> (8 * k)) & 0xff));
    }
    void nil() { out.push_back(static_cast<char>(0xc0)); }
    void boolean(bool b) { out.push_back(static_cast<char>(b ? 0xc3 : 0xc2)); }
    void integer(long long v) {
        if (v >= 0 && v <= 0x7f) {
            out.push_back(static_cast<char>(v));
        } else if (v < 0 && v >= -32) {
            out.push_back(static_cast<char>(static_cast<int8_t>(v)));
        } else {
            out.push_back(static_cast<char>(0xd3));
            put_be(static_cast<uint64_t>(v), 8);
        }
    }
    void str(std::string_view s) {
        size_t n = s.size();
        if (n < 32) {
            out.push_back(static_cast<char>(0xa0 | n));
        } else if (n < 256) {
            out.push_back(static_cast<char>(0xd9));
            put_be(n, 1);
        } else if (n < 65536) {
            out.push_back(static_cast<char>(0xda));
            put_be(n, 2);
        } else {
            out.push_back(static_cast<char>(0xdb));
            put_be(n, 4);
        }
        out.append(s.data(), n);
    }
    void map(size_t n) {
        if (n < 16) {
            out.push_back(static_cast<char>(0x80 | n));
        } else {
            out.push_back(static_cast<char>(0xde));
            put_be(n, 2);
        }
    }
    void array(size_t n) {
        if (n < 16) {
            out.push_back(static_cast<char>(0x90 | n));
        } else if (n < 65536) {
            out.push_back(static_cast<char>(0xdc));
            put_be(n, 2);
        } else {
            out.push_back(static_cast<char>(0xdd));
            put_be(n, 4);
        }
    }
};

}  // namespace ncc::mp
