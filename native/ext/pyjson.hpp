// native/ext/pyjson.hpp — JSON <-> CPython objects: the encoder, the decoder and the coordinator's slim template decode.
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// ----------------------------------------------------------------------------- JSON encoder
// dumps(obj) -> bytes: compact JSON (separators "," and ":") of a JSON-shaped Python value, key order
// preserved.  Non-ASCII text is emitted as UTF-8 (valid JSON; json.loads reads it back identically),
// so strings need only the quote/backslash/control-character escapes.  Used for request bodies and the
// fake apiserver's responses and watch lines, where json.dumps was the largest single per-object cost.
class JsonWriter {
  public:
    std::string out;

    void value(PyObject* o, int depth) {
        if (depth > 512) throw py::value_error("dumps: nesting too deep");
        if (o == Py_None) {
            out.append("null", 4);
        } else if (o == Py_True) {
            out.append("true", 4);
        } else if (o == Py_False) {
            out.append("false", 5);
        } else if (PyUnicode_Check(o)) {
            str(o);
        } else if (PyLong_Check(o)) {
            int overflow = 0;
            long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
            if (overflow) {
                PyObject* r = PyObject_Str(o);
                if (!r) throw py::error_already_set();
                Py_ssize_t n = 0;
                const char* s = PyUnicode_AsUTF8AndSize(r, &n);
                out.append(s, static_cast<size_t>(n));
                Py_DECREF(r);
            } else {
                char buf[32];
                int n = std::snprintf(buf, sizeof buf, "%lld", v);
                out.append(buf, static_cast<size_t>(n));
            }
        } else if (PyFloat_Check(o)) {
            double d = PyFloat_AS_DOUBLE(o);
            if (!std::isfinite(d)) throw py::value_error("dumps: out of range float values are not JSON compliant");
            char* s = PyOS_double_to_string(d, 'r', 0, Py_DTSF_ADD_DOT_0, nullptr);
            if (!s) throw py::error_already_set();
            out.append(s);
            PyMem_Free(s);
        } else if (PyDict_Check(o)) {
            out.push_back('{');
            PyObject *k, *v;
            Py_ssize_t pos = 0;
            bool first = true;
            while (PyDict_Next(o, &pos, &k, &v)) {
                if (!first) out.push_back(',');
                first = false;
                if (PyUnicode_Check(k)) {
                    str(k);
                } else {
                    PyObject* ks = PyObject_Str(k);  // json.dumps coerces int/float/bool keys to strings
                    if (!ks) throw py::error_already_set();
                    str(ks);
                    Py_DECREF(ks);
                }
                out.push_back(':');
                value(v, depth + 1);
            }
            out.push_back('}');
        } else if (PyList_Check(o) || PyTuple_Check(o)) {
            out.push_back('[');
            PyObject* seq = o;
            Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
            PyObject** items = PySequence_Fast_ITEMS(seq);
            for (Py_ssize_t i = 0; i < n; ++i) {
                if (i) out.push_back(',');
                value(items[i], depth + 1);
            }
            out.push_back(']');
        } else {
            throw py::type_error(std::string("dumps: object of type ") + Py_TYPE(o)->tp_name +
                                 " is not JSON serializable");
        }
    }

  private:
    void str(PyObject* o) {
        Py_ssize_t n = 0;
        const char* s = PyUnicode_AsUTF8AndSize(o, &n);
        if (!s) throw py::error_already_set();
        out.push_back('"');
        const char* run = s;
        const char* end = s + n;
        for (const char* p = s; p < end; ++p) {
            unsigned char c = static_cast<unsigned char>(*p);
            if (c >= 0x20 && c != '"' && c != '\\') continue;
            out.append(run, static_cast<size_t>(p - run));
            run = p + 1;
            switch (c) {
                case '"': out.append("\\\"", 2); break;
                case '\\': out.append("\\\\", 2); break;
                case '\n': out.append("\\n", 2); break;
                case '\r': out.append("\\r", 2); break;
                case '\t': out.append("\\t", 2); break;
                case '\b': out.append("\\b", 2); break;
                case '\f': out.append("\\f", 2); break;
                default: {
                    char buf[8];
                    std::snprintf(buf, sizeof buf, "\\u%04x", c);
                    out.append(buf, 6);
                }
            }
        }
        out.append(run, static_cast<size_t>(end - run));
        out.push_back('"');
    }
};

py::bytes dumps(py::handle obj) {
    JsonWriter w;
    w.out.reserve(1024);
    w.value(obj.ptr(), 0);
    return py::bytes(w.out.data(), w.out.size());
}

// scan_object(body) -> (namespace, name, resourceVersion, uid) of a JSON object's metadata | None
py::object scan_object(py::bytes body) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(body.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view ns, name, rv, uid;
    Scanner sc(buf, static_cast<size_t>(len));
    sc.uid = &uid;
    if (!sc.scan_object(ns, name, rv)) return py::none();
    return py::make_tuple(py::str(ns.data(), ns.size()), py::str(name.data(), name.size()),
                          py::str(rv.data(), rv.size()), py::str(uid.data(), uid.size()));
}

// members_equal(a, b, keys) -> True iff every top-level member named in `keys` has byte-identical raw
// JSON in both objects (or is absent from both).  False when either is not a JSON object this scanner
// reads (e.g. escaped keys): the caller then decodes.  A slim writer compares its request body with the
// write response this way to see whether the server rewrote the payload (defaulting, pruning, webhooks).
bool members_equal(py::bytes a, py::bytes b, py::sequence key_seq) {
    std::vector<std::string> keys;
    for (auto k : key_seq) keys.push_back(k.cast<std::string>());
    char* pa = nullptr;
    char* pb = nullptr;
    Py_ssize_t na = 0, nb = 0;
    if (PyBytes_AsStringAndSize(a.ptr(), &pa, &na) != 0 || PyBytes_AsStringAndSize(b.ptr(), &pb, &nb) != 0)
        throw py::error_already_set();
    std::vector<std::string_view> ma, mb;
    Scanner sa(pa, static_cast<size_t>(na)), sb(pb, static_cast<size_t>(nb));
    if (!sa.members(keys, ma) || !sb.members(keys, mb)) return false;
    for (size_t i = 0; i < keys.size(); ++i) {
        if ((ma[i].data() == nullptr) != (mb[i].data() == nullptr)) return false;
        if (ma[i].data() != nullptr && ma[i] != mb[i]) return false;
    }
    return true;
}


// ----------------------------------------------------------------------------- JSON -> Python
// A direct JSON decoder into CPython objects (dict/list/str/int/float/bool/None, key order kept), and
// `template_event_slim`, which decodes a template watch line into the coordinator's slim form: metadata
// (without managedFields) and status as Python values, the spec reduced to the references the
// coordinator reads plus a digest of its raw bytes.  A malformed line returns None (callers fall back
// to json.loads, which raises the proper error).
// An interned str for a constant key, made once per call site: PyDict_GetItemString / SetItemString would build
// and hash a new str on every call (a dozen per template line).
#define PY_CONST_KEY(lit) ([]() -> PyObject* { static PyObject* k_ = PyUnicode_InternFromString(lit); return k_; }())

class PyJson {
  public:
    PyJson(const char* p, size_t n) : p_(p), e_(p + n) {}

    // template_event_slim with a cache: `items` (borrowed; the informer store's dict keyed (namespace, name))
    // lets an unchanged status, or unchanged references, be taken from the cached version instead of decoded
    PyObject* items_ = nullptr;
    std::string default_ns_;

    // New reference, or nullptr: parse error (no Python exception set) or allocation failure (set).
    PyObject* value(int depth = 0) {
        ws();
        if (p_ >= e_ || depth > 512) return nullptr;
        switch (*p_) {
            case '{': return object(depth);
            case '[': return array(depth);
            case '"': return string();
            case 't': return literal("true", 4, Py_True);
            case 'f': return literal("false", 5, Py_False);
            case 'n': return literal("null", 4, Py_None);
            default: return number();
        }
    }
    bool at_end() {
        ws();
        return p_ == e_;
    }

    // {"type": "...", "object": {...}} with the object's spec slimmed → (type, object) | nullptr
    PyObject* template_event() {
        if (!expect('{')) return nullptr;
        PyObject* type = nullptr;
        PyObject* obj = nullptr;
        bool ok = true;
        if (!peek('}')) {
            for (;;) {
                std::string_view key;
                if (!raw_key(key)) { ok = false; break; }
                if (key == "type") {
                    Py_XDECREF(type);
                    type = value(1);
                    if (type == nullptr) { ok = false; break; }
                } else if (key == "object") {
                    Py_XDECREF(obj);
                    obj = slim_template();
                    if (obj == nullptr) { ok = false; break; }
                } else if (!skip_value()) {
                    ok = false;
                    break;
                }
                if (peek(',')) { ++p_; continue; }
                break;
            }
        }
        if (ok) ok = expect('}') && at_end() && type != nullptr && obj != nullptr;
        if (!ok) {
            Py_XDECREF(type);
            Py_XDECREF(obj);
            return nullptr;
        }
        PyObject* t = PyTuple_Pack(2, type, obj);
        Py_DECREF(type);
        Py_DECREF(obj);
        return t;
    }

  private:
    const char* p_;
    const char* e_;
    std::string tmp_;
    PyObject* prev_ = nullptr;  // borrowed: the cached version of the object being decoded, if any

    // After the metadata: find the cached version of this object (items_[(namespace, name)]).
    void find_prev(PyObject* md) {
        prev_ = nullptr;
        if (items_ == nullptr || md == nullptr || !PyDict_Check(md)) return;
        PyObject* name = PyDict_GetItem(md, PY_CONST_KEY("name"));
        PyObject* ns = PyDict_GetItem(md, PY_CONST_KEY("namespace"));
        if (name == nullptr) return;
        PyObject* nso = nullptr;
        if (ns == nullptr || (PyUnicode_Check(ns) && PyUnicode_GET_LENGTH(ns) == 0)) {
            nso = PyUnicode_FromStringAndSize(default_ns_.data(), static_cast<Py_ssize_t>(default_ns_.size()));
            if (nso == nullptr) {
                PyErr_Clear();
                return;
            }
            ns = nso;
        }
        PyObject* key = PyTuple_Pack(2, ns, name);
        Py_XDECREF(nso);
        if (key == nullptr) {
            PyErr_Clear();
            return;
        }
        PyObject* cur = PyDict_GetItemWithError(items_, key);
        Py_DECREF(key);
        if (cur == nullptr) {
            PyErr_Clear();
            return;
        }
        if (PyDict_Check(cur)) prev_ = cur;
    }
    // The value at p_ when its text hashes to `want` (the cached version's digest of it): `reuse` (new
    // reference) and *fp set, p_ past the value.  Otherwise p_ stays and nullptr is returned (*fp set when the
    // value could be skipped).
    PyObject* reuse_if_same(PyObject* want, PyObject* reuse, uint64_t* fp) {
        ws();
        const char* s0 = p_;
        if (!skip_value()) {
            p_ = s0;
            return nullptr;
        }
        Hasher h;
        h.bytes(s0, static_cast<size_t>(p_ - s0));
        *fp = h.digest();
        if (want != nullptr && reuse != nullptr && PyLong_Check(want) &&
            PyLong_AsUnsignedLongLong(want) == *fp && !PyErr_Occurred()) {
            Py_INCREF(reuse);
            return reuse;
        }
        PyErr_Clear();
        p_ = s0;
        return nullptr;
    }

    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    bool peek(char c) {
        ws();
        return p_ < e_ && *p_ == c;
    }
    bool expect(char c) {
        ws();
        if (p_ >= e_ || *p_ != c) return false;
        ++p_;
        return true;
    }
    PyObject* literal(const char* lit, size_t n, PyObject* v) {
        if (static_cast<size_t>(e_ - p_) < n || std::memcmp(p_, lit, n) != 0) return nullptr;
        p_ += n;
        Py_INCREF(v);
        return v;
    }
    static void put_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) {
            out.push_back(static_cast<char>(cp));
        } else if (cp < 0x800) {
            out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {  // lone surrogates too: "surrogatepass" decodes them back, as json.loads keeps them
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
    bool hex4(uint32_t& v) {
        if (e_ - p_ < 4) return false;
        v = 0;
        for (int i = 0; i < 4; ++i) {
            char c = p_[i];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= static_cast<uint32_t>(c - '0');
            else if (c >= 'a' && c <= 'f') v |= static_cast<uint32_t>(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= static_cast<uint32_t>(c - 'A' + 10);
            else return false;
        }
        p_ += 4;
        return true;
    }
    // The string at p_ (after ws) as UTF-8 bytes: a view into the input when it has no escapes, else tmp_.
    bool raw_string(std::string_view& out) {
        ws();
        if (p_ >= e_ || *p_ != '"') return false;
        const char* s = ++p_;
        p_ = ncc::find_quote_or_ctl(p_, e_);
        if (p_ >= e_ || static_cast<unsigned char>(*p_) < 0x20) return false;
        if (*p_ == '"') {
            out = std::string_view(s, static_cast<size_t>(p_ - s));
            ++p_;
            return true;
        }
        tmp_.assign(s, static_cast<size_t>(p_ - s));
        while (p_ < e_) {
            char c = *p_;
            if (c == '"') {
                ++p_;
                out = tmp_;
                return true;
            }
            if (static_cast<unsigned char>(c) < 0x20) return false;
            if (c != '\\') {
                tmp_.push_back(c);
                ++p_;
                continue;
            }
            if (++p_ >= e_) return false;
            char esc = *p_++;
            switch (esc) {
                case '"': tmp_.push_back('"'); break;
                case '\\': tmp_.push_back('\\'); break;
                case '/': tmp_.push_back('/'); break;
                case 'b': tmp_.push_back('\b'); break;
                case 'f': tmp_.push_back('\f'); break;
                case 'n': tmp_.push_back('\n'); break;
                case 'r': tmp_.push_back('\r'); break;
                case 't': tmp_.push_back('\t'); break;
                case 'u': {
                    uint32_t cp;
                    if (!hex4(cp)) return false;
                    if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                        const char* save = p_;
                        p_ += 2;
                        uint32_t lo;
                        if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) {
                            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        } else {
                            p_ = save;
                        }
                    }
                    put_utf8(tmp_, cp);
                    break;
                }
                default: return false;
            }
        }
        return false;
    }
    // ASCII (almost every Kubernetes string) is copied straight into a compact str; the rest is decoded.
    static PyObject* make_str(std::string_view v) {
        const unsigned char* b = reinterpret_cast<const unsigned char*>(v.data());
        size_t i = 0;
        while (i < v.size() && b[i] < 0x80) ++i;
        if (i < v.size()) return PyUnicode_DecodeUTF8(v.data(), static_cast<Py_ssize_t>(v.size()), "surrogatepass");
        PyObject* o = PyUnicode_New(static_cast<Py_ssize_t>(v.size()), 127);
        if (o != nullptr && !v.empty()) std::memcpy(PyUnicode_1BYTE_DATA(o), v.data(), v.size());
        return o;
    }
    PyObject* string() {
        std::string_view v;
        if (!raw_string(v)) return nullptr;
        return make_str(v);
    }
    bool raw_key(std::string_view& key) { return raw_string(key) && expect(':'); }
    // Object keys repeat across every object of a kind: a small direct-mapped cache of interned key strings
    // (GIL-protected; entries live for the process) saves building and hashing them again.
    struct KeySlot {
        std::string text;
        PyObject* obj = nullptr;
    };
    static KeySlot* key_cache() {
        static KeySlot slots[1024];
        return slots;
    }
    PyObject* key_object(std::string_view key) {
        if (key.size() > 48) return make_str(key);
        uint64_t h = 1469598103934665603ULL;
        for (unsigned char c : key) h = (h ^ c) * 1099511628211ULL;
        KeySlot& slot = key_cache()[h & 1023];
        if (slot.obj != nullptr && slot.text == key) {
            Py_INCREF(slot.obj);
            return slot.obj;
        }
        PyObject* k = make_str(key);
        if (k == nullptr) return nullptr;
        PyUnicode_InternInPlace(&k);
        Py_XDECREF(slot.obj);
        slot.text.assign(key.data(), key.size());
        slot.obj = k;
        Py_INCREF(k);
        return k;
    }
    PyObject* number() {
        const char* s = p_;
        if (p_ < e_ && *p_ == '-') ++p_;
        if (p_ >= e_ || *p_ < '0' || *p_ > '9') return nullptr;
        if (*p_ == '0') {
            ++p_;
        } else {
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        bool is_float = false;
        if (p_ < e_ && *p_ == '.') {
            is_float = true;
            ++p_;
            if (p_ >= e_ || *p_ < '0' || *p_ > '9') return nullptr;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
            is_float = true;
            ++p_;
            if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
            if (p_ >= e_ || *p_ < '0' || *p_ > '9') return nullptr;
            while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        std::string num(s, static_cast<size_t>(p_ - s));
        if (is_float) return PyFloat_FromDouble(std::strtod(num.c_str(), nullptr));
        if (num.size() <= 18) return PyLong_FromLongLong(std::strtoll(num.c_str(), nullptr, 10));
        return PyLong_FromString(num.c_str(), nullptr, 10);
    }
    PyObject* array(int depth) {
        ++p_;  // '['
        PyObject* list = PyList_New(0);
        if (list == nullptr) return nullptr;
        if (peek(']')) {
            ++p_;
            return list;
        }
        for (;;) {
            PyObject* v = value(depth + 1);
            if (v == nullptr || PyList_Append(list, v) != 0) {
                Py_XDECREF(v);
                Py_DECREF(list);
                return nullptr;
            }
            Py_DECREF(v);
            if (peek(',')) { ++p_; continue; }
            if (expect(']')) return list;
            Py_DECREF(list);
            return nullptr;
        }
    }
    // `skip` (may be empty): a member name left out (metadata.managedFields)
    PyObject* object(int depth, std::string_view skip = std::string_view()) {
        ++p_;  // '{'
        PyObject* d = PyDict_New();
        if (d == nullptr) return nullptr;
        if (peek('}')) {
            ++p_;
            return d;
        }
        for (;;) {
            std::string_view key;
            if (!raw_key(key)) break;
            if (!skip.empty() && key == skip) {
                if (!skip_value()) break;
            } else {
                PyObject* k = key_object(key);
                if (k == nullptr) break;
                PyObject* v = value(depth + 1);
                if (v == nullptr || PyDict_SetItem(d, k, v) != 0) {
                    Py_DECREF(k);
                    Py_XDECREF(v);
                    break;
                }
                Py_DECREF(k);
                Py_DECREF(v);
            }
            if (peek(',')) { ++p_; continue; }
            if (expect('}')) return d;
            break;
        }
        Py_DECREF(d);
        return nullptr;
    }
    bool skip_value() {
        ws();
        if (p_ >= e_) return false;
        char c = *p_;
        if (c == '"') {
            std::string_view v;
            return raw_string(v);
        }
        if (c == '{' || c == '[') {  // a skipped member (managedFields) is not validated
            const char* q = ncc::skip_container_text(p_, e_);
            if (q == nullptr) return false;
            p_ = q;
            return true;
        }
        const char* s = p_;
        while (p_ < e_ && *p_ != ',' && *p_ != '}' && *p_ != ']' && *p_ != ' ' && *p_ != '\n' && *p_ != '\t' &&
               *p_ != '\r')
            ++p_;
        return p_ > s;
    }
    // {"name": "..."} → a new {"name": str} dict (other members dropped), or None for null
    PyObject* name_ref() {
        ws();
        if (p_ < e_ && *p_ == 'n') return literal("null", 4, Py_None);
        if (!expect('{')) return nullptr;
        PyObject* d = PyDict_New();
        if (d == nullptr) return nullptr;
        if (peek('}')) {
            ++p_;
            return d;
        }
        for (;;) {
            std::string_view key;
            if (!raw_key(key)) break;
            if (key == "name") {
                PyObject* v = value(8);
                if (v == nullptr || PyDict_SetItem(d, PY_CONST_KEY("name"), v) != 0) {
                    Py_XDECREF(v);
                    break;
                }
                Py_DECREF(v);
            } else if (!skip_value()) {
                break;
            }
            if (peek(',')) { ++p_; continue; }
            if (expect('}')) return d;
            break;
        }
        Py_DECREF(d);
        return nullptr;
    }
    // mappedEnvironmentVariables: [{"secretRef": {"name"}, "configMapRef": {"name"}, ...}, ...] keeping the refs
    PyObject* mapped_env() {
        ws();
        if (p_ < e_ && *p_ == 'n') return literal("null", 4, Py_None);
        if (!expect('[')) return nullptr;
        PyObject* list = PyList_New(0);
        if (list == nullptr) return nullptr;
        if (peek(']')) {
            ++p_;
            return list;
        }
        for (;;) {
            ws();
            PyObject* item = nullptr;
            if (p_ < e_ && *p_ == '{') {
                ++p_;
                item = PyDict_New();
                if (item == nullptr) break;
                bool ok = true;
                if (peek('}')) {
                    ++p_;
                } else {
                    for (;;) {
                        std::string_view key;
                        if (!raw_key(key)) { ok = false; break; }
                        if (key == "secretRef" || key == "configMapRef") {
                            PyObject* r = name_ref();
                            if (r == nullptr) { ok = false; break; }
                            int rc = r == Py_None ? 0 : PyDict_SetItem(item, key == "secretRef" ? PY_CONST_KEY("secretRef") : PY_CONST_KEY("configMapRef"), r);
                            Py_DECREF(r);
                            if (rc != 0) { ok = false; break; }
                        } else if (!skip_value()) {
                            ok = false;
                            break;
                        }
                        if (peek(',')) { ++p_; continue; }
                        ok = expect('}');
                        break;
                    }
                }
                if (!ok) {
                    Py_DECREF(item);
                    break;
                }
            } else {
                if (!skip_value()) break;
                item = PyDict_New();  // null / non-object entries carry no reference
                if (item == nullptr) break;
            }
            int rc = PyList_Append(list, item);
            Py_DECREF(item);
            if (rc != 0) break;
            if (peek(',')) { ++p_; continue; }
            if (expect(']')) return list;
            break;
        }
        Py_DECREF(list);
        return nullptr;
    }
    // spec → {"runtimeEnvironment": {"mappedEnvironmentVariables": [...]}, "_fp": digest of the raw spec}
    PyObject* slim_spec() {
        ws();
        const char* s = p_;
        if (p_ >= e_ || *p_ != '{') {
            if (!skip_value()) return nullptr;
            Py_INCREF(Py_None);
            return Py_None;
        }
        ++p_;
        PyObject* env = nullptr;
        uint64_t env_fp = 0;
        bool ok = true;
        if (!peek('}')) {
            for (;;) {
                std::string_view key;
                if (!raw_key(key)) { ok = false; break; }
                if (key == "runtimeEnvironment" && peek('{')) {
                    ++p_;
                    if (!peek('}')) {
                        for (;;) {
                            std::string_view k2;
                            if (!raw_key(k2)) { ok = false; break; }
                            if (k2 == "mappedEnvironmentVariables") {
                                Py_XDECREF(env);
                                env = nullptr;
                                if (prev_ != nullptr) {  // unchanged references: the cached version's list
                                    PyObject* ps = PyDict_GetItem(prev_, PY_CONST_KEY("spec"));
                                    PyObject* prt = ps != nullptr && PyDict_Check(ps)
                                                        ? PyDict_GetItem(ps, PY_CONST_KEY("runtimeEnvironment")) : nullptr;
                                    PyObject* penv = prt != nullptr && PyDict_Check(prt)
                                                         ? PyDict_GetItem(prt, PY_CONST_KEY("mappedEnvironmentVariables"))
                                                         : nullptr;
                                    if (penv != nullptr)
                                        env = reuse_if_same(PyDict_GetItem(ps, PY_CONST_KEY("_rfp")), penv, &env_fp);
                                }
                                if (env == nullptr) {
                                    ws();
                                    const char* e0 = p_;
                                    env = mapped_env();
                                    if (env == nullptr) { ok = false; break; }
                                    Hasher he;
                                    he.bytes(e0, static_cast<size_t>(p_ - e0));
                                    env_fp = he.digest();
                                }
                            } else if (!skip_value()) {
                                ok = false;
                                break;
                            }
                            if (peek(',')) { ++p_; continue; }
                            break;
                        }
                    }
                    if (!ok || !expect('}')) { ok = false; break; }
                } else if (!skip_value()) {
                    ok = false;
                    break;
                }
                if (peek(',')) { ++p_; continue; }
                break;
            }
        }
        if (ok) ok = expect('}');
        if (!ok) {
            Py_XDECREF(env);
            return nullptr;
        }
        Hasher hs;
        hs.bytes(s, static_cast<size_t>(p_ - s));
        PyObject* spec = PyDict_New();
        PyObject* fp = PyLong_FromUnsignedLongLong(hs.digest());
        bool built = spec != nullptr && fp != nullptr;
        if (built && env != nullptr && env != Py_None) {
            PyObject* rt = PyDict_New();
            built = rt != nullptr && PyDict_SetItem(rt, PY_CONST_KEY("mappedEnvironmentVariables"), env) == 0 &&
                    PyDict_SetItem(spec, PY_CONST_KEY("runtimeEnvironment"), rt) == 0;
            Py_XDECREF(rt);
        }
        if (built) built = PyDict_SetItem(spec, PY_CONST_KEY("_fp"), fp) == 0;
        if (built) {  // a digest of the references' text: the coordinator compares it instead of the list
            PyObject* rfp = PyLong_FromUnsignedLongLong(env_fp);
            built = rfp != nullptr && PyDict_SetItem(spec, PY_CONST_KEY("_rfp"), rfp) == 0;
            Py_XDECREF(rfp);
        }
        Py_XDECREF(env);
        Py_XDECREF(fp);
        if (!built) {
            Py_XDECREF(spec);
            return nullptr;
        }
        return spec;
    }
    PyObject* slim_template() {
        if (!expect('{')) return nullptr;
        PyObject* d = PyDict_New();
        if (d == nullptr) return nullptr;
        if (peek('}')) {
            ++p_;
            return d;
        }
        for (;;) {
            std::string_view key;
            if (!raw_key(key)) break;
            PyObject* v;
            if (key == "spec") {
                v = slim_spec();
            } else if (key == "metadata" && peek('{')) {
                v = object(1, "managedFields");
                find_prev(v);
            } else if (key == "status") {
                // and a digest of the status text under "__ncc_sfp__": an unchanged status compares as one int,
                // and is taken from the cached version instead of decoded again
                uint64_t fp = 0;
                v = nullptr;
                if (prev_ != nullptr) {
                    PyObject* pst = PyDict_GetItem(prev_, PY_CONST_KEY("status"));
                    if (pst != nullptr) v = reuse_if_same(PyDict_GetItem(prev_, PY_CONST_KEY("__ncc_sfp__")), pst, &fp);
                }
                if (v == nullptr) {
                    ws();
                    const char* s0 = p_;
                    v = value(1);
                    if (v != nullptr) {
                        Hasher hs;
                        hs.bytes(s0, static_cast<size_t>(p_ - s0));
                        fp = hs.digest();
                    }
                }
                if (v != nullptr) {
                    PyObject* sfp = PyLong_FromUnsignedLongLong(fp);
                    if (sfp == nullptr || PyDict_SetItem(d, PY_CONST_KEY("__ncc_sfp__"), sfp) != 0) {
                        Py_XDECREF(sfp);
                        Py_DECREF(v);
                        break;
                    }
                    Py_DECREF(sfp);
                }
            } else {
                v = value(1);
            }
            PyObject* k = v == nullptr ? nullptr : key_object(key);
            if (k == nullptr || PyDict_SetItem(d, k, v) != 0) {
                Py_XDECREF(k);
                Py_XDECREF(v);
                break;
            }
            Py_DECREF(k);
            Py_DECREF(v);
            if (peek(',')) { ++p_; continue; }
            if (expect('}')) return d;
            break;
        }
        Py_DECREF(d);
        return nullptr;
    }
};

static std::string_view bytes_view(const py::bytes& b) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(b.ptr(), &buf, &len) != 0) throw py::error_already_set();
    return std::string_view(buf, static_cast<size_t>(len));
}

// loads(bytes) -> value | None (malformed: the caller falls back to json.loads for the error)
py::object loads(py::bytes data) {
    std::string_view v = bytes_view(data);
    PyJson pj(v.data(), v.size());
    PyObject* o = pj.value();
    if (o != nullptr && !pj.at_end()) {
        Py_DECREF(o);
        o = nullptr;
    }
    if (o == nullptr) {
        // invalid UTF-8 inside a string is malformed input too: None, and the caller's stdlib fallback
        // reports it
        if (PyErr_Occurred() && !PyErr_ExceptionMatches(PyExc_UnicodeDecodeError)) throw py::error_already_set();
        PyErr_Clear();
        return py::none();
    }
    return py::reinterpret_steal<py::object>(o);
}

// template_index_same(old, new) -> bool: the coordinator's template indices read the same in both versions —
// ncc/controller/controller.py `_reference_guard(old) == _reference_guard(new)` (namespace, and the references
// digest `spec._rfp` of a slim template or else the mapped environment) in one call instead of two tuples.
// Anything but dicts where the guard reads dicts raises TypeError (the caller then compares the guards).
bool template_index_same(py::handle old, py::handle nw) {
    auto get = [](PyObject* d, PyObject* k) -> PyObject* {  // borrowed, Py_None when absent
        PyObject* v = PyDict_GetItemWithError(d, k);
        if (v == nullptr && PyErr_Occurred()) throw py::error_already_set();
        return v != nullptr ? v : Py_None;
    };
    auto sub = [&](PyObject* d, PyObject* k) -> PyObject* {  // `d.get(k) or {}`: nullptr for an empty one
        PyObject* v = get(d, k);
        int t = PyObject_IsTrue(v);
        if (t < 0) throw py::error_already_set();
        if (t == 0) return nullptr;
        if (!PyDict_Check(v)) throw py::type_error("template_index_same: not a mapping");
        return v;
    };
    auto refs = [&](PyObject* t) -> PyObject* {
        PyObject* spec = sub(t, PY_CONST_KEY("spec"));
        if (spec == nullptr) return Py_None;
        PyObject* r = get(spec, PY_CONST_KEY("_rfp"));
        if (r != Py_None) return r;
        PyObject* env = sub(spec, PY_CONST_KEY("runtimeEnvironment"));
        return env != nullptr ? get(env, PY_CONST_KEY("mappedEnvironmentVariables")) : Py_None;
    };
    auto eq = [](PyObject* a, PyObject* b) {
        int r = PyObject_RichCompareBool(a, b, Py_EQ);
        if (r < 0) throw py::error_already_set();
        return r == 1;
    };
    if (!PyDict_Check(old.ptr()) || !PyDict_Check(nw.ptr())) throw py::type_error("template_index_same: not a dict");
    PyObject* om = sub(old.ptr(), PY_CONST_KEY("metadata"));
    PyObject* nm = sub(nw.ptr(), PY_CONST_KEY("metadata"));
    PyObject* ons = om != nullptr ? get(om, PY_CONST_KEY("namespace")) : Py_None;
    PyObject* nns = nm != nullptr ? get(nm, PY_CONST_KEY("namespace")) : Py_None;
    return eq(ons, nns) && eq(refs(old.ptr()), refs(nw.ptr()));
}

// template_event_slim(line) -> (type, slim object) | None
py::object template_event_slim(py::bytes line, py::object items, const std::string& default_ns) {
    std::string_view v = bytes_view(line);
    PyJson pj(v.data(), v.size());
    if (!items.is_none()) {
        if (!PyDict_Check(items.ptr())) throw py::type_error("template_event_slim: items must be a dict");
        pj.items_ = items.ptr();
        pj.default_ns_ = default_ns;
    }
    PyObject* o = pj.template_event();
    if (o == nullptr) {
        if (PyErr_Occurred()) throw py::error_already_set();
        return py::none();
    }
    return py::reinterpret_steal<py::object>(o);
}
