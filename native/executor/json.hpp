// JSON DOM for the native shard executor: parse, serialise, structural 64-bit fingerprints.
//
// The executor keeps every controller-side object it needs (templates, workgroups, Secrets,
// ConfigMaps) and a slim copy of every shard object as `Value` trees.  Members keep their wire
// order (a PUT re-sends shard metadata exactly as read); numbers keep their text.  Fingerprints
// are order-independent for objects and number-canonical (1 == 1.0), so "is the shard copy's spec
// the template's spec" — reflect.DeepEqual in the reference (controller.go:795-802) — is one
// integer compare.
#pragma once

#include <cmath>
#include <initializer_list>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>
#include <charconv>
#include <system_error>
#include "../common/byte_scan.hpp"

namespace ncc {

struct JsonError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct Value {
    enum Type : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ };
    Type t = NUL;
    bool b = false;
    std::string s;  // string value, or the number's text
    std::vector<Value> a;
    std::vector<std::pair<std::string, Value>> o;

    Value() = default;
    static Value str(std::string v) {
        Value x;
        x.t = STR;
        x.s = std::move(v);
        return x;
    }
    static Value object() {
        Value x;
        x.t = OBJ;
        return x;
    }
    static Value array() {
        Value x;
        x.t = ARR;
        return x;
    }
    static Value boolean(bool v) {
        Value x;
        x.t = BOOL;
        x.b = v;
        return x;
    }
    static Value number(long long v) {
        Value x;
        x.t = NUM;
        x.s = std::to_string(v);
        return x;
    }

    bool is_obj() const { return t == OBJ; }
    bool is_arr() const { return t == ARR; }
    bool is_str() const { return t == STR; }
    bool is_null() const { return t == NUL; }

    const Value* get(std::string_view k) const {
        if (t != OBJ) return nullptr;
        for (const auto& kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    Value* get(std::string_view k) {
        if (t != OBJ) return nullptr;
        for (auto& kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    // string member or "" (absent / not a string)
    std::string_view sget(std::string_view k) const {
        const Value* v = get(k);
        return (v != nullptr && v->t == STR) ? std::string_view(v->s) : std::string_view();
    }
    Value& set(std::string_view k, Value v) {
        if (t != OBJ) {
            t = OBJ;
            o.clear();
        }
        for (auto& kv : o)
            if (kv.first == k) {
                kv.second = std::move(v);
                return kv.second;
            }
        o.emplace_back(std::string(k), std::move(v));
        return o.back().second;
    }
    void erase(std::string_view k) {
        if (t != OBJ) return;
        for (auto it = o.begin(); it != o.end(); ++it)
            if (it->first == k) {
                o.erase(it);
                return;
            }
    }
    bool empty_container() const { return (t == OBJ && o.empty()) || (t == ARR && a.empty()); }
};

// ------------------------------------------------------------------------------------ parse
class Parser {
public:
    Parser(const char* p, size_t n) : p_(p), e_(p + n) {}

    Value parse() {
        Value v;
        value(v, 0);
        ws();
        if (p_ != e_) throw JsonError("trailing characters");
        return v;
    }

    // A top-level object whose members named in `keys` are kept as raw JSON text (`raw[i]`, empty when
    // absent) instead of being decoded: the payloads (spec, data, ...) the executor only fingerprints
    // and re-sends verbatim.  Returns the object without them.
    Value parse_split(const std::string_view* keys, size_t n, std::string_view* raw) {
        Value v;
        object_split(v, keys, n, raw);
        ws();
        if (p_ != e_) fail("trailing characters");
        return v;
    }
    // A watch event {"type": ..., "object": {...}} with the object split as in parse_split.
    Value parse_event_split(std::string& type, const std::string_view* keys, size_t n, std::string_view* raw) {
        Value obj;
        bool have_obj = false;
        ws();
        if (p_ >= e_ || *p_ != '{') fail("expected an event object");
        ++p_;
        while (true) {
            ws();
            if (p_ >= e_ || *p_ != '"') fail("expected key");
            std::string key;
            string(key);
            ws();
            if (p_ >= e_ || *p_ != ':') fail("expected ':'");
            ++p_;
            ws();
            if (key == "type") {
                if (p_ >= e_ || *p_ != '"') fail("expected the event type");
                type.clear();
                string(type);
            } else if (key == "object" && p_ < e_ && *p_ == '{') {
                object_split(obj, keys, n, raw);
                have_obj = true;
            } else {
                skip(0);
            }
            ws();
            if (p_ < e_ && *p_ == ',') {
                ++p_;
                continue;
            }
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                break;
            }
            fail("expected ',' or '}'");
        }
        ws();
        if (p_ != e_) fail("trailing characters");
        if (!have_obj) obj = Value();
        return obj;
    }
    // A top-level object with only the members named in `keys` decoded (the rest skipped).
    Value parse_only(const std::string_view* keys, size_t n) {
        Value v;
        ws();
        if (p_ >= e_ || *p_ != '{') fail("expected an object");
        ++p_;
        v.t = Value::OBJ;
        ws();
        if (p_ < e_ && *p_ == '}') {
            ++p_;
            return v;
        }
        while (true) {
            ws();
            if (p_ >= e_ || *p_ != '"') fail("expected key");
            std::string key;
            string(key);
            ws();
            if (p_ >= e_ || *p_ != ':') fail("expected ':'");
            ++p_;
            size_t i = 0;
            while (i < n && keys[i] != key) ++i;
            if (i < n) {
                v.o.emplace_back(std::move(key), Value());
                value(v.o.back().second, 1);
            } else {
                skip(0);
            }
            ws();
            if (p_ < e_ && *p_ == ',') {
                ++p_;
                continue;
            }
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                break;
            }
            fail("expected ',' or '}'");
        }
        ws();
        if (p_ != e_) fail("trailing characters");
        return v;
    }
    // fingerprint() of the value at the start of the text; `end` gets the position just past it
    uint64_t fingerprint_prefix(const char** end) {
        uint64_t h = fp(0);
        *end = p_;
        return h;
    }
    // fingerprint() of the JSON text without building it (same decoding, same hash)
    uint64_t fingerprint_text() {
        uint64_t h = fp(0);
        ws();
        if (p_ != e_) fail("trailing characters");
        return h;
    }

private:
    const char* p_;
    const char* e_;
    std::string tmp_;

    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    [[noreturn]] void fail(const char* what) { throw JsonError(what); }

    void object_split(Value& v, const std::string_view* keys, size_t n, std::string_view* raw) {
        for (size_t i = 0; i < n; ++i) raw[i] = std::string_view();
        ws();
        if (p_ >= e_ || *p_ != '{') fail("expected an object");
        ++p_;
        v.t = Value::OBJ;
        ws();
        if (p_ < e_ && *p_ == '}') {
            ++p_;
            return;
        }
        while (true) {
            ws();
            if (p_ >= e_ || *p_ != '"') fail("expected key");
            std::string key;
            string(key);
            ws();
            if (p_ >= e_ || *p_ != ':') fail("expected ':'");
            ++p_;
            ws();
            size_t i = 0;
            while (i < n && keys[i] != key) ++i;
            if (i < n) {
                const char* s = p_;
                skip(0);
                raw[i] = std::string_view(s, static_cast<size_t>(p_ - s));
            } else {
                v.o.emplace_back(std::move(key), Value());
                value(v.o.back().second, 1);
            }
            ws();
            if (p_ < e_ && *p_ == ',') {
                ++p_;
                continue;
            }
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                return;
            }
            fail("expected ',' or '}'");
        }
    }
    // Skip one value (strings decoded into tmp_, which also validates their escapes).
    void skip(int depth) {
        if (depth > 200) fail("nesting too deep");
        ws();
        if (p_ >= e_) fail("unexpected end");
        char c = *p_;
        if (c == '"') {
            str_view();  // validates escapes only when there are any
            return;
        }
        if (c == '{' || c == '[') {
            char close = c == '{' ? '}' : ']';
            ++p_;
            ws();
            if (p_ < e_ && *p_ == close) {
                ++p_;
                return;
            }
            while (true) {
                if (c == '{') {
                    ws();
                    if (p_ >= e_ || *p_ != '"') fail("expected key");
                    tmp_.clear();
                    string(tmp_);
                    ws();
                    if (p_ >= e_ || *p_ != ':') fail("expected ':'");
                    ++p_;
                }
                skip(depth + 1);
                ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == close) {
                    ++p_;
                    return;
                }
                fail("expected ',' or a closing bracket");
            }
        }
        Value scalar;
        value(scalar, depth);
    }
    uint64_t fp(int depth) {
        if (depth > 200) fail("nesting too deep");
        ws();
        if (p_ >= e_) fail("unexpected end");
        char c = *p_;
        if (c == '"') return hash_str(str_view());
        if (c == '{') {
            ++p_;
            uint64_t acc = 0, count = 0;
            ws();
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                return fp_object(acc, 0);
            }
            while (true) {
                ws();
                if (p_ >= e_ || *p_ != '"') fail("expected key");
                uint64_t kh = hash_key(str_view());
                ws();
                if (p_ >= e_ || *p_ != ':') fail("expected ':'");
                ++p_;
                acc += fp_member(kh, fp(depth + 1));
                ++count;
                ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == '}') {
                    ++p_;
                    return fp_object(acc, count);
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++p_;
            uint64_t h = kArraySeed, count = 0;
            ws();
            if (p_ < e_ && *p_ == ']') {
                ++p_;
                return fp_array_end(h, 0);
            }
            while (true) {
                h = fp_array_step(h, fp(depth + 1));
                ++count;
                ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == ']') {
                    ++p_;
                    return fp_array_end(h, count);
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == 't' && e_ - p_ >= 4 && std::memcmp(p_, "true", 4) == 0) {
            p_ += 4;
            return fp_bool(true);
        }
        if (c == 'f' && e_ - p_ >= 5 && std::memcmp(p_, "false", 5) == 0) {
            p_ += 5;
            return fp_bool(false);
        }
        if (c == 'n' && e_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
            p_ += 4;
            return kNullFp;
        }
        const char* s = p_;
        while (p_ < e_ && (*p_ == '-' || *p_ == '+' || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                           (*p_ >= '0' && *p_ <= '9')))
            ++p_;
        if (p_ == s || !(c == '-' || (c >= '0' && c <= '9'))) fail("unexpected character");
        return fp_number(std::string_view(s, static_cast<size_t>(p_ - s)));
    }
    // the next string's content: a view of the text when it has no escape sequence, else decoded into tmp_
    std::string_view str_view() {
        const char* s = p_ + 1;
        const char* q = find_quote(s, e_);
        if (q < e_ && *q == '"') {
            p_ = q + 1;
            return std::string_view(s, static_cast<size_t>(q - s));
        }
        tmp_.clear();
        string(tmp_);
        return tmp_;
    }
    static uint64_t hash_str(std::string_view s);
public:
    // the pieces fingerprint() composes (a caller walking an object itself combines its members with them)
    static uint64_t hash_key(std::string_view s);
    static uint64_t fp_member(uint64_t key_hash, uint64_t value_fp);
    static uint64_t fp_object(uint64_t acc, uint64_t count);
    static constexpr uint64_t kArraySeed = 0x6666ULL;
    static constexpr uint64_t kNullFp = 0x9e3779b97f4a7c15ULL;
    static uint64_t fp_array_step(uint64_t h, uint64_t item);
    static uint64_t fp_array_end(uint64_t h, uint64_t count);
    static uint64_t fp_bool(bool b);
    static uint64_t fp_number(std::string_view text);

private:

    void value(Value& v, int depth) {
        if (depth > 200) fail("nesting too deep");
        ws();
        if (p_ >= e_) fail("unexpected end");
        char c = *p_;
        if (c == '{') {
            ++p_;
            v.t = Value::OBJ;
            ws();
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                return;
            }
            while (true) {
                ws();
                if (p_ >= e_ || *p_ != '"') fail("expected key");
                std::string key;
                string(key);
                ws();
                if (p_ >= e_ || *p_ != ':') fail("expected ':'");
                ++p_;
                v.o.emplace_back(std::move(key), Value());
                value(v.o.back().second, depth + 1);
                ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == '}') {
                    ++p_;
                    return;
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++p_;
            v.t = Value::ARR;
            ws();
            if (p_ < e_ && *p_ == ']') {
                ++p_;
                return;
            }
            while (true) {
                v.a.emplace_back();
                value(v.a.back(), depth + 1);
                ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == ']') {
                    ++p_;
                    return;
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.t = Value::STR;
            string(v.s);
            return;
        }
        if (c == 't' && e_ - p_ >= 4 && std::memcmp(p_, "true", 4) == 0) {
            p_ += 4;
            v.t = Value::BOOL;
            v.b = true;
            return;
        }
        if (c == 'f' && e_ - p_ >= 5 && std::memcmp(p_, "false", 5) == 0) {
            p_ += 5;
            v.t = Value::BOOL;
            v.b = false;
            return;
        }
        if (c == 'n' && e_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
            p_ += 4;
            v.t = Value::NUL;
            return;
        }
        if (c == '-' || (c >= '0' && c <= '9')) {
            const char* s = p_;
            ++p_;
            while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                               *p_ == '+' || *p_ == '-'))
                ++p_;
            v.t = Value::NUM;
            v.s.assign(s, static_cast<size_t>(p_ - s));
            return;
        }
        fail("unexpected character");
    }

    static int hex(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    unsigned u4() {
        if (e_ - p_ < 4) fail("short \\u escape");
        unsigned v = 0;
        for (int i = 0; i < 4; ++i) {
            int h = hex(p_[i]);
            if (h < 0) fail("bad \\u escape");
            v = (v << 4) | static_cast<unsigned>(h);
        }
        p_ += 4;
        return v;
    }
    static void utf8(std::string& out, unsigned cp) {
        if (cp < 0x80) {
            out.push_back(static_cast<char>(cp));
        } else if (cp < 0x800) {
            out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
        } else {
            out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
        }
    }
    void string(std::string& out) {
        ++p_;  // opening quote
        const char* run = p_;
        while (true) {
            if (p_ >= e_) fail("unterminated string");
            char c = *p_;
            if (c == '"') {
                out.append(run, static_cast<size_t>(p_ - run));
                ++p_;
                return;
            }
            if (c == '\\') {
                out.append(run, static_cast<size_t>(p_ - run));
                ++p_;
                if (p_ >= e_) fail("bad escape");
                char x = *p_++;
                switch (x) {
                    case '"': out.push_back('"'); break;
                    case '\\': out.push_back('\\'); break;
                    case '/': out.push_back('/'); break;
                    case 'b': out.push_back('\b'); break;
                    case 'f': out.push_back('\f'); break;
                    case 'n': out.push_back('\n'); break;
                    case 'r': out.push_back('\r'); break;
                    case 't': out.push_back('\t'); break;
                    case 'u': {
                        unsigned cp = u4();
                        if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                            p_ += 2;
                            unsigned lo = u4();
                            if (lo >= 0xDC00 && lo < 0xE000) {
                                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                            } else {
                                utf8(out, 0xFFFD);
                                cp = lo;
                            }
                        }
                        utf8(out, cp);
                        break;
                    }
                    default: fail("bad escape");
                }
                run = p_;
                continue;
            }
            p_ = find_quote(p_, e_);
        }
    }
};

inline Value parse(std::string_view text) { return Parser(text.data(), text.size()).parse(); }

// ------------------------------------------------------------------------------------ serialise
inline void write_string(std::string& out, std::string_view s) {
    static const char* hexd = "0123456789abcdef";
    out.push_back('"');
    const char* run = s.data();
    const char* end = s.data() + s.size();
    for (const char* p = run; p < end; ++p) {
        unsigned char c = static_cast<unsigned char>(*p);
        if (c >= 0x20 && c != '"' && c != '\\') continue;
        out.append(run, static_cast<size_t>(p - run));
        switch (c) {
            case '"': out.append("\\\""); break;
            case '\\': out.append("\\\\"); break;
            case '\n': out.append("\\n"); break;
            case '\r': out.append("\\r"); break;
            case '\t': out.append("\\t"); break;
            case '\b': out.append("\\b"); break;
            case '\f': out.append("\\f"); break;
            default:
                out.append("\\u00");
                out.push_back(hexd[c >> 4]);
                out.push_back(hexd[c & 15]);
        }
        run = p + 1;
    }
    out.append(run, static_cast<size_t>(end - run));
    out.push_back('"');
}

inline void dump(std::string& out, const Value& v) {
    switch (v.t) {
        case Value::NUL: out.append("null"); break;
        case Value::BOOL: out.append(v.b ? "true" : "false"); break;
        case Value::NUM: out.append(v.s); break;
        case Value::STR: write_string(out, v.s); break;
        case Value::ARR: {
            out.push_back('[');
            bool first = true;
            for (const auto& x : v.a) {
                if (!first) out.push_back(',');
                first = false;
                dump(out, x);
            }
            out.push_back(']');
            break;
        }
        case Value::OBJ: {
            out.push_back('{');
            bool first = true;
            for (const auto& kv : v.o) {
                if (!first) out.push_back(',');
                first = false;
                write_string(out, kv.first);
                out.push_back(':');
                dump(out, kv.second);
            }
            out.push_back('}');
            break;
        }
    }
}

inline std::string dumps(const Value& v) {
    std::string out;
    out.reserve(256);
    dump(out, v);
    return out;
}

// ------------------------------------------------------------------------------------ scanning
// type / metadata.namespace / .name / .resourceVersion of a raw watch line without building a DOM, so
// the echo of the executor's own write (already cached from the write's response) costs one scan.  Any
// escape in the strings read, or anything unexpected, returns false (the caller parses the line).
class EventScanner {
public:
    EventScanner(std::string_view line) : p_(line.data()), e_(line.data() + line.size()) {}
    // non-null: also collect metadata.ownerReferences[*].name (the partition of a shard dependent)
    std::vector<std::string_view>* owners = nullptr;
    bool scan(std::string_view& type, std::string_view& ns, std::string_view& name, std::string_view& rv) {
        if (!expect('{')) return false;
        bool have_type = false, have_meta = false;
        while (true) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            if (key == "type") {
                if (!str(type)) return false;
                have_type = true;
            } else if (key == "object") {
                if (!object_meta(ns, name, rv)) return false;
                have_meta = true;
            } else if (!skip()) {
                return false;
            }
            if (have_type && have_meta) return true;
            if (!expect(',')) return false;
        }
    }

private:
    const char* p_;
    const char* e_;
    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    bool expect(char c) {
        ws();
        if (p_ >= e_ || *p_ != c) return false;
        ++p_;
        return true;
    }
    bool str(std::string_view& out) {
        ws();
        if (p_ >= e_ || *p_ != '"') return false;
        const char* s = p_ + 1;
        const char* q = find_quote(s, e_);
        if (q >= e_ || *q != '"') return false;
        out = std::string_view(s, static_cast<size_t>(q - s));
        p_ = q + 1;
        return true;
    }
    bool skip_str() {
        const char* q = skip_string_text(p_, e_);
        if (q == nullptr) return false;
        p_ = q;
        return true;
    }
    bool skip() {
        ws();
        if (p_ >= e_) return false;
        if (*p_ == '"') return skip_str();
        if (*p_ == '{' || *p_ == '[') {
            const char* q = skip_container_text(p_, e_);
            if (q == nullptr) return false;
            p_ = q;
            return true;
        }
        const char* s = p_;
        while (p_ < e_ && *p_ != ',' && *p_ != '}' && *p_ != ']' && *p_ != ' ' && *p_ != '\n') ++p_;
        return p_ > s;
    }
    bool owner_names() {
        ws();
        if (e_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
            p_ += 4;
            return true;
        }
        if (!expect('[')) return false;
        ws();
        if (p_ < e_ && *p_ == ']') {
            ++p_;
            return true;
        }
        while (true) {
            if (!expect('{')) return false;
            while (true) {
                std::string_view k, v;
                if (!str(k) || !expect(':')) return false;
                if (k == "name") {
                    if (!str(v)) return false;
                    owners->push_back(v);
                } else if (!skip()) {
                    return false;
                }
                if (expect(',')) continue;
                if (!expect('}')) return false;
                break;
            }
            if (expect(',')) continue;
            return expect(']');
        }
    }
    bool object_meta(std::string_view& ns, std::string_view& name, std::string_view& rv) {
        if (!expect('{')) return false;
        while (true) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            if (key == "metadata") {
                if (!expect('{')) return false;
                bool have_name = false, have_rv = false;
                while (true) {
                    std::string_view k;
                    if (!str(k) || !expect(':')) return false;
                    if (k == "name") {
                        if (!str(name)) return false;
                        have_name = true;
                    } else if (k == "namespace") {
                        if (!str(ns)) return false;
                    } else if (k == "resourceVersion") {
                        if (!str(rv)) return false;
                        have_rv = true;
                    } else if (owners != nullptr && k == "ownerReferences") {
                        if (!owner_names()) return false;
                    } else if (!skip()) {
                        return false;
                    }
                    if (expect(',')) continue;
                    return expect('}') && have_name && have_rv;
                }
            }
            if (!skip() || !expect(',')) return false;
        }
    }
};

// ------------------------------------------------------------------------------------ raw members
// A cursor over JSON text for reading a few members without building a DOM.  Strings are returned as views
// of the text, so one with an escape sequence is refused (`str` returns false) and the caller falls back to
// the parser.
struct RawCursor {
    const char* p;
    const char* e;
    RawCursor(std::string_view t) : p(t.data()), e(t.data() + t.size()) {}
    void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool at(char c) {
        ws();
        return p < e && *p == c;
    }
    bool expect(char c) {
        if (!at(c)) return false;
        ++p;
        return true;
    }
    bool str(std::string_view& out) {
        ws();
        if (p >= e || *p != '"') return false;
        const char* s = p + 1;
        const char* q = find_quote(s, e);
        if (q >= e || *q != '"') return false;
        out = std::string_view(s, static_cast<size_t>(q - s));
        p = q + 1;
        return true;
    }
    bool skip_str() {
        const char* q = skip_string_text(p, e);
        if (q == nullptr) return false;
        p = q;
        return true;
    }
    // skip one value; `span` gets its text
    bool value(std::string_view& span) {
        ws();
        if (p >= e) return false;
        const char* s = p;
        if (*p == '"') {
            if (!skip_str()) return false;
        } else if (*p == '{' || *p == '[') {
            const char* q = skip_container_text(p, e);
            if (q == nullptr) return false;
            p = q;
        } else {
            while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' &&
                   *p != '\t')
                ++p;
            if (p == s) return false;
        }
        span = std::string_view(s, static_cast<size_t>(p - s));
        return true;
    }
    // the members of an object (the cursor at its '{'): fn(key, value text) for each; false when malformed
    // or a key carries an escape
    template <class Fn>
    bool members(Fn&& fn) {
        if (!expect('{')) return false;
        if (expect('}')) return true;
        while (true) {
            std::string_view k, v;
            if (!str(k) || !expect(':') || !value(v)) return false;
            if (!fn(k, v)) return false;
            if (expect(',')) continue;
            return expect('}');
        }
    }
    // members() reading in place: fn(key, *this) consumes the member's value itself (value(), str(), a
    // nested walk()...), so a member the caller descends into is not skipped first
    template <class Fn>
    bool walk(Fn&& fn) {
        if (!expect('{')) return false;
        if (expect('}')) return true;
        while (true) {
            std::string_view k;
            if (!str(k) || !expect(':')) return false;
            if (!fn(k, *this)) return false;
            if (expect(',')) continue;
            return expect('}');
        }
    }
    template <class Fn>
    bool elements(Fn&& fn) {
        if (!expect('[')) return false;
        if (expect(']')) return true;
        while (true) {
            std::string_view v;
            if (!value(v)) return false;
            if (!fn(v)) return false;
            if (expect(',')) continue;
            return expect(']');
        }
    }
};

// `{...}` text of a JSON object with the given members appended (each as raw JSON; an empty text adds
// nothing).  For objects kept as text without those members (the shard cache), this is dumps_with.
inline std::string splice_members(std::string_view obj, std::initializer_list<std::pair<std::string_view, std::string_view>> add) {
    std::string out;
    out.reserve(obj.size() + 64);
    size_t end = obj.rfind('}');
    if (end == std::string_view::npos) end = obj.size();
    out.append(obj.substr(0, end));
    size_t i = end;
    while (i > 0 && (obj[i - 1] == ' ' || obj[i - 1] == '\n' || obj[i - 1] == '\r' || obj[i - 1] == '\t')) --i;
    bool empty = i > 0 && obj[i - 1] == '{';
    for (const auto& m : add) {
        if (m.second.empty()) continue;
        if (!empty) out.push_back(',');
        empty = false;
        write_string(out, m.first);
        out.push_back(':');
        out.append(m.second);
    }
    out.push_back('}');
    return out;
}

// ------------------------------------------------------------------------------------ fingerprints
inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

inline uint64_t hash_bytes(std::string_view s, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    uint64_t h = seed ^ (s.size() * m);
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
    return fmix64(h);
}

// fingerprint of a JSON number's text: integral values (1 == 1.0) hash as integers
inline uint64_t fp_number_text(std::string_view text) {
    long long iv = 0;
    auto [ip, iec] = std::from_chars(text.data(), text.data() + text.size(), iv);
    if (iec == std::errc() && ip == text.data() + text.size() && iv > -9000000000000000LL && iv < 9000000000000000LL)
        return fmix64(static_cast<uint64_t>(iv) ^ 0x3333ULL);
    double d = 0;
    std::string z(text);
    d = std::strtod(z.c_str(), nullptr);
    if (std::isfinite(d) && d == std::floor(d) && std::fabs(d) < 9.0e15)
        return fmix64(static_cast<uint64_t>(static_cast<long long>(d)) ^ 0x3333ULL);
    uint64_t bits;
    std::memcpy(&bits, &d, 8);
    return fmix64(bits ^ 0x4444ULL);
}

inline uint64_t fingerprint(const Value& v) {
    switch (v.t) {
        case Value::NUL: return Parser::kNullFp;
        case Value::BOOL: return Parser::fp_bool(v.b);
        case Value::NUM: return fp_number_text(v.s);
        case Value::STR: return hash_bytes(v.s, 0x5555ULL);
        case Value::ARR: {
            uint64_t h = Parser::kArraySeed;
            for (const auto& x : v.a) h = Parser::fp_array_step(h, fingerprint(x));
            return Parser::fp_array_end(h, v.a.size());
        }
        case Value::OBJ: {
            uint64_t acc = 0x7777ULL + v.o.size();
            for (const auto& kv : v.o)  // commutative: member order does not matter
                acc += fmix64(hash_bytes(kv.first, 0x8888ULL) ^ (fingerprint(kv.second) * 0x9E3779B97F4A7C15ULL));
            return fmix64(acc);
        }
    }
    return 0;
}

// The streaming form (Parser::fingerprint_text) composes the same pieces.
inline uint64_t Parser::hash_str(std::string_view s) { return hash_bytes(s, 0x5555ULL); }
inline uint64_t Parser::hash_key(std::string_view s) { return hash_bytes(s, 0x8888ULL); }
inline uint64_t Parser::fp_member(uint64_t kh, uint64_t vf) { return fmix64(kh ^ (vf * 0x9E3779B97F4A7C15ULL)); }
inline uint64_t Parser::fp_object(uint64_t acc, uint64_t count) { return fmix64(acc + 0x7777ULL + count); }
inline uint64_t Parser::fp_array_step(uint64_t h, uint64_t item) { return fmix64(h * 31 + item); }
inline uint64_t Parser::fp_array_end(uint64_t h, uint64_t count) { return fmix64(h ^ (count * 0xA0761D6478BD642FULL)); }
inline uint64_t Parser::fp_bool(bool b) { return fmix64(b ? 0x1234567ULL : 0x7654321ULL); }
inline uint64_t Parser::fp_number(std::string_view text) { return fp_number_text(text); }

inline uint64_t fingerprint_text(std::string_view text) { return Parser(text.data(), text.size()).fingerprint_text(); }

// fp_opt of raw text: absent, null and empty maps/arrays are one value (a nil Go map == an empty one)
inline bool raw_is_empty(std::string_view raw) {
    size_t i = 0, n = raw.size();
    while (i < n && (raw[i] == ' ' || raw[i] == '\n' || raw[i] == '\r' || raw[i] == '\t')) ++i;
    if (i >= n) return true;
    if (raw.substr(i, 4) == "null") return true;
    if (raw[i] != '{' && raw[i] != '[') return false;
    char close = raw[i] == '{' ? '}' : ']';
    ++i;
    while (i < n && (raw[i] == ' ' || raw[i] == '\n' || raw[i] == '\r' || raw[i] == '\t')) ++i;
    return i < n && raw[i] == close;
}
inline uint64_t fp_opt_text(std::string_view raw) {
    return raw_is_empty(raw) ? fingerprint(Value()) : fingerprint_text(raw);
}

// dumps(base) with the members named in `over` written as the given raw JSON text (replacing a member of
// that name, or appended after base's members); an empty text drops the member.
inline std::string dumps_with(const Value& base, std::initializer_list<std::pair<std::string_view, std::string_view>> over) {
    std::string out;
    out.reserve(512);
    out.push_back('{');
    bool first = true;
    auto member = [&](std::string_view k) {
        if (!first) out.push_back(',');
        first = false;
        write_string(out, k);
        out.push_back(':');
    };
    std::vector<bool> done(over.size(), false);
    if (base.t == Value::OBJ)
        for (const auto& kv : base.o) {
            size_t i = 0;
            bool replaced = false;
            for (const auto& ov : over) {
                if (ov.first == kv.first) {
                    done[i] = true;
                    replaced = true;
                    if (!ov.second.empty()) {
                        member(kv.first);
                        out.append(ov.second);
                    }
                    break;
                }
                ++i;
            }
            if (replaced) continue;
            member(kv.first);
            dump(out, kv.second);
        }
    size_t i = 0;
    for (const auto& ov : over) {
        if (!done[i] && !ov.second.empty()) {
            member(ov.first);
            out.append(ov.second);
        }
        ++i;
    }
    out.push_back('}');
    return out;
}

// fingerprint(x or None): absent, null and empty maps are one value (a nil Go map == an empty one)
inline uint64_t fp_opt(const Value* v) {
    static const Value null_value;
    if (v == nullptr || v->t == Value::NUL || v->empty_container()) return fingerprint(null_value);
    return fingerprint(*v);
}

}  // namespace ncc
