// native/ext/scan.hpp — watch-line scanners, crc32 key partitions, the metadata-only owner filter and the relay's index loop.
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// ----------------------------------------------------------------------------- watch-event scanner
// scan_event(line) -> (type, namespace, name, resourceVersion) | None
//
// Structural scan of one watch-stream line {"type":..., "object":{..., "metadata":{...}}} that reads
// only the four strings the informer needs to recognise the echo of its own write, skipping every
// other value by bracket matching.  No Python objects are built for the (large) spec/data payloads;
// a full json.loads happens only for events that are not our own echoes.  Any input it does not
// fully understand (escaped keys or values, malformed JSON) returns None and the caller falls back.
class Scanner {
  public:
    Scanner(const char* p, size_t n) : p_(p), e_(p + n) {}

    // owners != nullptr → also collect metadata.ownerReferences[*].name and .uid (escapes → failure)
    std::vector<std::string_view>* owners = nullptr;
    std::vector<std::string_view>* owner_uids = nullptr;
    std::string_view* uid = nullptr;  // non-null → also read metadata.uid

    // top-level object {"apiVersion":..., "metadata":{...}, ...} (a write response)
    bool scan_object(std::string_view& ns, std::string_view& name, std::string_view& rv) {
        return object_meta(ns, name, rv);
    }

    // raw JSON of the top-level members named in `keys` (out[i].data() == nullptr: absent)
    bool members(const std::vector<std::string>& keys, std::vector<std::string_view>& out) {
        out.assign(keys.size(), std::string_view());
        if (!expect('{')) return false;
        if (peek('}')) { ++p_; return true; }
        for (;;) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            ws();
            const char* s = p_;
            if (!skip_value()) return false;
            for (size_t i = 0; i < keys.size(); ++i)
                if (key == keys[i]) out[i] = std::string_view(s, static_cast<size_t>(p_ - s));
            if (peek(',')) { ++p_; continue; }
            return expect('}');
        }
    }

    bool scan(std::string_view& type, std::string_view& ns, std::string_view& name, std::string_view& rv) {
        if (!expect('{')) return false;
        bool have_type = false, have_obj = false;
        if (peek('}')) return false;
        for (;;) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            if (key == "type") {
                if (!str(type)) return false;
                have_type = true;
            } else if (key == "object") {
                if (!object_meta(ns, name, rv)) return false;
                have_obj = true;
            } else if (!skip_value()) {
                return false;
            }
            if (have_type && have_obj) return true;
            if (peek(',')) { ++p_; continue; }
            return false;
        }
    }

  private:
    const char* p_;
    const char* e_;

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
    // a string without escapes (anything escaped makes the caller fall back to json.loads)
    bool str(std::string_view& out) {
        ws();
        if (p_ >= e_ || *p_ != '"') return false;
        const char* s = ++p_;
        p_ = ncc::find_quote(p_, e_);
        if (p_ >= e_ || *p_ == '\\') return false;
        out = std::string_view(s, static_cast<size_t>(p_ - s));
        ++p_;
        return true;
    }
    bool skip_string() {
        if (p_ >= e_ || *p_ != '"') return false;
        const char* q = ncc::skip_string_text(p_, e_);
        if (q == nullptr) return false;
        p_ = q;
        return true;
    }
    bool skip_value() {
        ws();
        if (p_ >= e_) return false;
        char c = *p_;
        if (c == '"') return skip_string();
        if (c == '{' || c == '[') {  // 64 bytes per step (native/common/byte_scan.hpp)
            const char* q = ncc::skip_container_text(p_, e_);
            if (q == nullptr) return false;
            p_ = q;
            return true;
        }
        while (p_ < e_ && *p_ != ',' && *p_ != '}' && *p_ != ']' && *p_ != ' ' && *p_ != '\n' &&
               *p_ != '\t' && *p_ != '\r')
            ++p_;
        return true;
    }
    bool object_meta(std::string_view& ns, std::string_view& name, std::string_view& rv) {
        if (!expect('{')) return false;
        bool found = false;
        if (peek('}')) { ++p_; return false; }
        for (;;) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            if (key == "metadata") {
                if (!meta(ns, name, rv)) return false;
                found = true;
            } else if (!skip_value()) {
                return false;
            }
            if (peek(',')) { ++p_; continue; }
            if (!expect('}')) return false;
            return found;
        }
    }
    // [{"apiVersion":..., "kind":..., "name": "...", "uid": ...}, ...] → owners->push_back(name)
    bool owner_refs() {
        ws();
        if (p_ < e_ && *p_ == 'n') return skip_value();  // null
        if (!expect('[')) return false;
        if (peek(']')) { ++p_; return true; }
        for (;;) {
            if (!expect('{')) return false;
            std::string_view oname, ouid;
            if (!peek('}')) {
                for (;;) {
                    std::string_view key;
                    if (!str(key) || !expect(':')) return false;
                    if (key == "name") {
                        if (!str(oname)) return false;
                    } else if (key == "uid") {
                        if (!str(ouid)) return false;
                    } else if (!skip_value()) {
                        return false;
                    }
                    if (peek(',')) { ++p_; continue; }
                    break;
                }
            }
            if (!expect('}')) return false;
            owners->push_back(oname);
            owner_uids->push_back(ouid);
            if (peek(',')) { ++p_; continue; }
            return expect(']');
        }
    }
    bool meta(std::string_view& ns, std::string_view& name, std::string_view& rv) {
        if (!expect('{')) return false;
        bool have_name = false, have_rv = false;
        if (peek('}')) { ++p_; return false; }
        for (;;) {
            std::string_view key;
            if (!str(key) || !expect(':')) return false;
            if (key == "name") {
                if (!str(name)) return false;
                have_name = true;
            } else if (key == "namespace") {
                if (!str(ns)) return false;
            } else if (key == "resourceVersion") {
                if (!str(rv)) return false;
                have_rv = true;
            } else if (uid != nullptr && key == "uid") {
                if (!str(*uid)) return false;
            } else if (owners != nullptr && key == "ownerReferences") {
                if (!owner_refs()) return false;
            } else if (!skip_value()) {
                return false;
            }
            if (peek(',')) { ++p_; continue; }
            if (!expect('}')) return false;
            return have_name && have_rv;
        }
    }
};

py::object scan_event(py::bytes line) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(line.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view type, ns, name, rv;
    Scanner sc(buf, static_cast<size_t>(len));
    if (!sc.scan(type, ns, name, rv)) return py::none();
    return py::make_tuple(py::str(type.data(), type.size()), py::str(ns.data(), ns.size()),
                          py::str(name.data(), name.size()), py::str(rv.data(), rv.size()));
}

// scan_event_owners(line) -> (type, namespace, name, resourceVersion, (owner names...), (owner uids...)) | None
py::object scan_event_owners(py::bytes line) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(line.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view type, ns, name, rv;
    std::vector<std::string_view> owners, uids;
    Scanner sc(buf, static_cast<size_t>(len));
    sc.owners = &owners;
    sc.owner_uids = &uids;
    if (!sc.scan(type, ns, name, rv)) return py::none();
    py::tuple o(owners.size()), u(uids.size());
    for (size_t i = 0; i < owners.size(); ++i) o[i] = py::str(owners[i].data(), owners[i].size());
    for (size_t i = 0; i < uids.size(); ++i) u[i] = py::str(uids[i].data(), uids[i].size());
    return py::make_tuple(py::str(type.data(), type.size()), py::str(ns.data(), ns.size()),
                          py::str(name.data(), name.size()), py::str(rv.data(), rv.size()), o, u);
}

// ----------------------------------------------------------------------------- partitions
// crc32 (IEEE, reflected; identical to zlib.crc32) of "<ns>/<name>": the executors' key → partition map
// (ncc.controller.executor.key_part), computed here so foreign-partition watch lines are dropped without
// building Python strings.
static uint32_t kCrcTable[256];
static bool crc_table_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        kCrcTable[i] = c;
    }
    return true;
}
static const bool kCrcReady = crc_table_init();

static uint32_t crc_update(uint32_t c, std::string_view s) {
    for (unsigned char ch : s) c = kCrcTable[(c ^ ch) & 0xFFu] ^ (c >> 8);
    return c;
}

static uint32_t key_crc(std::string_view ns, std::string_view name) {
    uint32_t c = crc_update(0xFFFFFFFFu, ns);
    c = crc_update(c, std::string_view("/", 1));
    return crc_update(c, name) ^ 0xFFFFFFFFu;
}

// scan_event_part(line, parts, default_ns) -> (type, namespace, name, resourceVersion, (owner names...),
//     (owner uids...), key_partition, owner_partition_mask) | None
// key_partition = crc32("ns/name") % parts; bit p of owner_partition_mask is set when some owner
// template "ns/<owner>" falls in partition p (parts <= 63).  An empty namespace uses `default_ns`.
py::object scan_event_part(py::bytes line, int parts, const std::string& default_ns) {
    if (parts < 1 || parts > 63) throw py::value_error("scan_event_part: parts must be in 1..63");
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(line.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view type, ns, name, rv;
    std::vector<std::string_view> owners, uids;
    Scanner sc(buf, static_cast<size_t>(len));
    sc.owners = &owners;
    sc.owner_uids = &uids;
    if (!sc.scan(type, ns, name, rv)) return py::none();
    std::string_view kns = ns.empty() ? std::string_view(default_ns) : ns;
    const uint32_t up = static_cast<uint32_t>(parts);
    long long kp = static_cast<long long>(key_crc(kns, name) % up);
    unsigned long long mask = 0;
    py::tuple o(owners.size()), u(uids.size());
    for (size_t i = 0; i < owners.size(); ++i) {
        mask |= 1ull << (key_crc(kns, owners[i]) % up);
        o[i] = py::str(owners[i].data(), owners[i].size());
    }
    for (size_t i = 0; i < uids.size(); ++i) u[i] = py::str(uids[i].data(), uids[i].size());
    return py::make_tuple(py::str(type.data(), type.size()), py::str(ns.data(), ns.size()),
                          py::str(name.data(), name.size()), py::str(rv.data(), rv.size()), o, u, kp, mask);
}

// relay_scan(line, parts, default_ns) -> (type_code, namespace, name, key_partition, owner_partition_mask,
//     n_owners) | None.  The coordinator's watch relay (ncc/controller/relay.py) routes every controller-side
// watch line to the executors whose key partitions need it with this one call: type_code 0 ADDED,
// 1 MODIFIED, 2 DELETED, 3 anything else (BOOKMARK, ERROR); `namespace` is already defaulted.
py::object relay_scan(py::bytes line, int parts, const std::string& default_ns) {
    if (parts < 1 || parts > 63) throw py::value_error("relay_scan: parts must be in 1..63");
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(line.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view type, ns, name, rv;
    std::vector<std::string_view> owners, uids;
    Scanner sc(buf, static_cast<size_t>(len));
    sc.owners = &owners;
    sc.owner_uids = &uids;
    if (!sc.scan(type, ns, name, rv)) return py::none();
    int code = type == "ADDED" ? 0 : type == "MODIFIED" ? 1 : type == "DELETED" ? 2 : 3;
    std::string_view kns = ns.empty() ? std::string_view(default_ns) : ns;
    const uint32_t up = static_cast<uint32_t>(parts);
    long long kp = static_cast<long long>(key_crc(kns, name) % up);
    unsigned long long mask = 0;
    for (const auto& o : owners) mask |= 1ull << (key_crc(kns, o) % up);
    return py::make_tuple(code, py::str(kns.data(), kns.size()), py::str(name.data(), name.size()), kp, mask,
                          static_cast<long long>(owners.size()));
}

// Does a Python str equal these UTF-8 bytes?
static bool str_eq(PyObject* o, std::string_view v) {
    if (o == nullptr || !PyUnicode_Check(o)) return v.empty() && o == nullptr;
    Py_ssize_t n = 0;
    const char* u = PyUnicode_AsUTF8AndSize(o, &n);
    if (u == nullptr) {
        PyErr_Clear();
        return false;
    }
    return static_cast<size_t>(n) == v.size() && std::memcmp(u, v.data(), v.size()) == 0;
}

// owner_filter(lines, items, assumed, default_ns) -> (kept lines, dropped, rv of the last line if dropped)
// The metadata-only informer's filter over a whole batch (ncc/cache/informer.py `_consume`): a MODIFIED
// line of an object cached in `items` (the store's dict, keyed (namespace, name)) whose ownerReferences
// names and uids equal the cached ones carries nothing such a store keeps, and is dropped.  Every other line
// — other event types, unknown or overlaid (`assumed`) keys, unreadable lines — is kept for the Python path.
py::tuple owner_filter(py::list lines, py::dict items, py::dict assumed, const std::string& default_ns) {
    py::list keep;
    long long dropped = 0;
    std::string_view last_rv;
    bool last_dropped = false;
    const Py_ssize_t n = PyList_GET_SIZE(lines.ptr());
    std::vector<std::string_view> owners, uids;
    static PyObject* k_meta = PyUnicode_InternFromString("metadata");
    static PyObject* k_refs = PyUnicode_InternFromString("ownerReferences");
    static PyObject* k_name = PyUnicode_InternFromString("name");
    static PyObject* k_uid = PyUnicode_InternFromString("uid");
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* line = PyList_GET_ITEM(lines.ptr(), i);
        last_dropped = false;
        char* buf = nullptr;
        Py_ssize_t len = 0;
        bool drop = false;
        std::string_view type, ns, name, rv;
        if (PyBytes_Check(line) && PyBytes_AsStringAndSize(line, &buf, &len) == 0) {
            owners.clear();
            uids.clear();
            Scanner sc(buf, static_cast<size_t>(len));
            sc.owners = &owners;
            sc.owner_uids = &uids;
            PyObject* kn = nullptr;
            PyObject* nm = nullptr;
            if (sc.scan(type, ns, name, rv) && type == "MODIFIED") {
                std::string_view kns = ns.empty() ? std::string_view(default_ns) : ns;
                kn = PyUnicode_DecodeUTF8(kns.data(), static_cast<Py_ssize_t>(kns.size()), nullptr);
                nm = kn == nullptr ? nullptr : PyUnicode_DecodeUTF8(name.data(), static_cast<Py_ssize_t>(name.size()), nullptr);
                if (nm == nullptr) {  // not UTF-8: kept, the Python path decides
                    Py_XDECREF(kn);
                    PyErr_Clear();
                }
            }
            if (nm != nullptr) {
                py::tuple key = py::make_tuple(py::reinterpret_steal<py::object>(kn), py::reinterpret_steal<py::object>(nm));
                PyObject* cur = PyDict_GetItemWithError(items.ptr(), key.ptr());
                if (cur == nullptr && PyErr_Occurred()) throw py::error_already_set();
                int overlaid = PyDict_Contains(assumed.ptr(), key.ptr());
                if (overlaid < 0) throw py::error_already_set();
                if (cur != nullptr && !overlaid && PyDict_Check(cur)) {
                    PyObject* m = PyDict_GetItem(cur, k_meta);
                    PyObject* refs = m != nullptr && PyDict_Check(m) ? PyDict_GetItem(m, k_refs) : nullptr;
                    if (refs == nullptr || refs == Py_None) {
                        drop = owners.empty();
                    } else if (PyList_Check(refs) && static_cast<size_t>(PyList_GET_SIZE(refs)) == owners.size()) {
                        drop = true;
                        for (size_t j = 0; j < owners.size() && drop; ++j) {
                            PyObject* r = PyList_GET_ITEM(refs, static_cast<Py_ssize_t>(j));
                            if (!PyDict_Check(r)) {
                                drop = false;
                                break;
                            }
                            PyObject* rn = PyDict_GetItem(r, k_name);
                            PyObject* ru = PyDict_GetItem(r, k_uid);
                            drop = (rn == nullptr ? owners[j].empty() : str_eq(rn, owners[j])) &&
                                   (ru == nullptr ? uids[j].empty() : str_eq(ru, uids[j]));
                        }
                    }
                }
            }
        } else {
            PyErr_Clear();
        }
        if (drop) {
            ++dropped;
            last_rv = rv;
            last_dropped = true;
        } else if (PyList_Append(keep.ptr(), line) != 0) {
            throw py::error_already_set();
        }
    }
    py::object rv_o = last_dropped ? py::object(py::str(last_rv.data(), last_rv.size())) : py::object(py::none());
    return py::make_tuple(keep, dropped, rv_o);
}

// OwnerFilter()(lines, items, assumed, default_ns): owner_filter's result, with a memo per informer so a dropped
// line builds no Python object.  The memo maps "namespace\0name" to the store's key tuple, the cached object it
// last compared against (a strong reference: identity is the test, so the address cannot be reused) and that
// object's owners in a canonical byte form (length-prefixed name, uid per reference).  A line is then one scan,
// one C++ lookup, one dict lookup of the memoised key to see that the store still holds the same object, and a
// byte compare of the owners.  An entry whose object was replaced is refreshed from the new one; the memo is
// dropped whole when it outgrows the store by 4096 keys (deleted keys), as the Python filter's signatures are.
class OwnerFilter {
  public:
    OwnerFilter() = default;
    OwnerFilter(const OwnerFilter&) = delete;
    OwnerFilter& operator=(const OwnerFilter&) = delete;
    ~OwnerFilter() { clear(); }  // the Python object's deallocation: the GIL is held

    void clear() {
        for (auto& kv : memo_) {
            Py_XDECREF(kv.second.key);
            Py_XDECREF(kv.second.obj);
        }
        memo_.clear();
    }
    size_t size() const { return memo_.size(); }

    py::tuple call(py::list lines, py::dict items, py::dict assumed, const std::string& default_ns) {
        py::list keep;
        long long dropped = 0;
        std::string_view last_rv;
        bool last_dropped = false;
        const Py_ssize_t n = PyList_GET_SIZE(lines.ptr());
        PyObject* itd = items.ptr();
        const bool any_assumed = PyDict_GET_SIZE(assumed.ptr()) > 0;
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject* line = PyList_GET_ITEM(lines.ptr(), i);
            last_dropped = false;
            char* buf = nullptr;
            Py_ssize_t len = 0;
            bool drop = false;
            std::string_view type, ns, name, rv;
            if (PyBytes_Check(line) && PyBytes_AsStringAndSize(line, &buf, &len) == 0) {
                owners_.clear();
                uids_.clear();
                Scanner sc(buf, static_cast<size_t>(len));
                sc.owners = &owners_;
                sc.owner_uids = &uids_;
                if (sc.scan(type, ns, name, rv) && type == "MODIFIED")
                    drop = judge(ns.empty() ? std::string_view(default_ns) : ns, name, itd, assumed.ptr(), any_assumed);
            } else {
                PyErr_Clear();
            }
            if (drop) {
                ++dropped;
                last_rv = rv;
                last_dropped = true;
            } else if (PyList_Append(keep.ptr(), line) != 0) {
                throw py::error_already_set();
            }
        }
        py::object rv_o = last_dropped ? py::object(py::str(last_rv.data(), last_rv.size())) : py::object(py::none());
        return py::make_tuple(keep, dropped, rv_o);
    }

  private:
    struct Entry {
        PyObject* key = nullptr;  // the store's (namespace, name) tuple
        PyObject* obj = nullptr;  // the cached object `owners` was read from
        std::string owners;       // canonical owners of `obj`
        bool comparable = false;  // false: some reference is not {name: str, uid: str}; never dropped
    };
    std::unordered_map<std::string, Entry> memo_;
    std::string kbuf_, line_owners_;
    std::vector<std::string_view> owners_, uids_;

    static void put(std::string& out, std::string_view v) {
        uint32_t l = static_cast<uint32_t>(v.size());
        out.append(reinterpret_cast<const char*>(&l), sizeof l);
        out.append(v.data(), v.size());
    }
    // the cached object's owners in canonical form; false when they cannot compare equal to a scanned line
    static bool cached_owners(PyObject* cur, std::string& out) {
        static PyObject* k_meta = PyUnicode_InternFromString("metadata");
        static PyObject* k_refs = PyUnicode_InternFromString("ownerReferences");
        static PyObject* k_name = PyUnicode_InternFromString("name");
        static PyObject* k_uid = PyUnicode_InternFromString("uid");
        out.clear();
        if (!PyDict_Check(cur)) return false;
        PyObject* m = PyDict_GetItem(cur, k_meta);
        PyObject* refs = m != nullptr && PyDict_Check(m) ? PyDict_GetItem(m, k_refs) : nullptr;
        if (refs == nullptr || refs == Py_None) return true;
        if (!PyList_Check(refs)) return false;
        for (Py_ssize_t j = 0; j < PyList_GET_SIZE(refs); ++j) {
            PyObject* r = PyList_GET_ITEM(refs, j);
            if (!PyDict_Check(r)) return false;
            for (PyObject* k : {k_name, k_uid}) {
                PyObject* v = PyDict_GetItem(r, k);
                if (v == nullptr) {
                    put(out, std::string_view());
                    continue;
                }
                if (!PyUnicode_Check(v)) return false;
                Py_ssize_t vn = 0;
                const char* u = PyUnicode_AsUTF8AndSize(v, &vn);
                if (u == nullptr) {
                    PyErr_Clear();
                    return false;
                }
                put(out, std::string_view(u, static_cast<size_t>(vn)));
            }
        }
        return true;
    }
    bool judge(std::string_view kns, std::string_view name, PyObject* items, PyObject* assumed, bool any_assumed) {
        kbuf_.assign(kns.data(), kns.size());
        kbuf_ += '\0';
        kbuf_.append(name.data(), name.size());
        auto it = memo_.find(kbuf_);
        if (it == memo_.end()) {
            PyObject* kn = PyUnicode_DecodeUTF8(kns.data(), static_cast<Py_ssize_t>(kns.size()), nullptr);
            PyObject* nm = kn == nullptr ? nullptr : PyUnicode_DecodeUTF8(name.data(), static_cast<Py_ssize_t>(name.size()), nullptr);
            if (nm == nullptr) {  // not UTF-8: kept, the Python path decides
                Py_XDECREF(kn);
                PyErr_Clear();
                return false;
            }
            PyObject* key = PyTuple_Pack(2, kn, nm);
            Py_DECREF(kn);
            Py_DECREF(nm);
            if (key == nullptr) throw py::error_already_set();
            PyObject* cur = PyDict_GetItemWithError(items, key);
            if (cur == nullptr) {
                Py_DECREF(key);
                if (PyErr_Occurred()) throw py::error_already_set();
                return false;  // not cached: kept, and not memoised (the store may never hold it)
            }
            if (memo_.size() > static_cast<size_t>(PyDict_GET_SIZE(items)) + 4096) clear();
            it = memo_.emplace(kbuf_, Entry{}).first;
            it->second.key = key;  // the reference PyTuple_Pack gave
        }
        Entry& e = it->second;
        if (any_assumed) {
            int overlaid = PyDict_Contains(assumed, e.key);
            if (overlaid < 0) throw py::error_already_set();
            if (overlaid) return false;
        }
        PyObject* cur = PyDict_GetItemWithError(items, e.key);
        if (cur == nullptr) {
            if (PyErr_Occurred()) throw py::error_already_set();
            return false;
        }
        if (cur != e.obj) {
            Py_INCREF(cur);
            Py_XDECREF(e.obj);
            e.obj = cur;
            e.comparable = cached_owners(cur, e.owners);
        }
        if (!e.comparable) return false;
        line_owners_.clear();
        for (size_t j = 0; j < owners_.size(); ++j) {
            put(line_owners_, owners_[j]);
            put(line_owners_, uids_[j]);
        }
        return line_owners_ == e.owners;
    }
};

// relay_index(lines, raw, default_ns) -> the lines to forward.  The one-partition relay's whole loop in one
// call: each ADDED/MODIFIED line is stored in `raw` under (namespace, name), a DELETED one removes its key,
// and every object event is forwarded; BOOKMARK/ERROR and unreadable lines are dropped (the coordinator's
// informer handles those).  Same result as relay_scan per line (ncc/controller/relay.py `on_lines`).
py::list relay_index(py::list lines, py::dict raw, const std::string& default_ns) {
    py::list keep;
    PyObject* rd = raw.ptr();
    const Py_ssize_t n = PyList_GET_SIZE(lines.ptr());
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* line = PyList_GET_ITEM(lines.ptr(), i);
        char* buf = nullptr;
        Py_ssize_t len = 0;
        if (PyBytes_AsStringAndSize(line, &buf, &len) != 0) throw py::error_already_set();
        std::string_view type, ns, name, rv;
        Scanner sc(buf, static_cast<size_t>(len));
        if (!sc.scan(type, ns, name, rv)) continue;
        int code = type == "ADDED" ? 0 : type == "MODIFIED" ? 1 : type == "DELETED" ? 2 : 3;
        if (code == 3) continue;
        std::string_view kns = ns.empty() ? std::string_view(default_ns) : ns;
        PyObject* kn = PyUnicode_DecodeUTF8(kns.data(), static_cast<Py_ssize_t>(kns.size()), nullptr);
        PyObject* nm = kn == nullptr ? nullptr : PyUnicode_DecodeUTF8(name.data(), static_cast<Py_ssize_t>(name.size()), nullptr);
        if (nm == nullptr) {  // not UTF-8: forwarded for the executor to judge, not indexed
            Py_XDECREF(kn);
            PyErr_Clear();
            if (PyList_Append(keep.ptr(), line) != 0) throw py::error_already_set();
            continue;
        }
        py::tuple key = py::make_tuple(py::reinterpret_steal<py::object>(kn), py::reinterpret_steal<py::object>(nm));
        if (code == 2) {
            if (PyDict_DelItem(rd, key.ptr()) != 0) {
                if (!PyErr_ExceptionMatches(PyExc_KeyError)) throw py::error_already_set();
                PyErr_Clear();
            }
        } else if (PyDict_SetItem(rd, key.ptr(), line) != 0) {
            throw py::error_already_set();
        }
        if (PyList_Append(keep.ptr(), line) != 0) throw py::error_already_set();
    }
    return keep;
}

// RelayIndex()(lines, raw, default_ns): relay_index with a memo of the (namespace, name) key tuples, so a line
// of a key seen before builds no Python object: one scan, one C++ lookup, one dict store.  The memo forgets a
// key on its DELETED line, and is dropped whole when it outgrows `raw` by 4096 keys.
class RelayIndex {
  public:
    RelayIndex() = default;
    RelayIndex(const RelayIndex&) = delete;
    RelayIndex& operator=(const RelayIndex&) = delete;
    ~RelayIndex() { clear(); }

    void clear() {
        for (auto& kv : memo_) Py_XDECREF(kv.second);
        memo_.clear();
    }
    size_t size() const { return memo_.size(); }

    py::list call(py::list lines, py::dict raw, const std::string& default_ns) {
        py::list keep;
        PyObject* rd = raw.ptr();
        const Py_ssize_t n = PyList_GET_SIZE(lines.ptr());
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject* line = PyList_GET_ITEM(lines.ptr(), i);
            char* buf = nullptr;
            Py_ssize_t len = 0;
            if (PyBytes_AsStringAndSize(line, &buf, &len) != 0) throw py::error_already_set();
            std::string_view type, ns, name, rv;
            Scanner sc(buf, static_cast<size_t>(len));
            if (!sc.scan(type, ns, name, rv)) continue;
            int code = type == "ADDED" ? 0 : type == "MODIFIED" ? 1 : type == "DELETED" ? 2 : 3;
            if (code == 3) continue;
            std::string_view kns = ns.empty() ? std::string_view(default_ns) : ns;
            kbuf_.assign(kns.data(), kns.size());
            kbuf_ += '\0';
            kbuf_.append(name.data(), name.size());
            PyObject* key = nullptr;
            auto it = memo_.find(kbuf_);
            if (it != memo_.end()) {
                key = it->second;
            } else {
                PyObject* kn = PyUnicode_DecodeUTF8(kns.data(), static_cast<Py_ssize_t>(kns.size()), nullptr);
                PyObject* nm = kn == nullptr ? nullptr : PyUnicode_DecodeUTF8(name.data(), static_cast<Py_ssize_t>(name.size()), nullptr);
                if (nm == nullptr) {  // not UTF-8: forwarded for the executor to judge, not indexed
                    Py_XDECREF(kn);
                    PyErr_Clear();
                    if (PyList_Append(keep.ptr(), line) != 0) throw py::error_already_set();
                    continue;
                }
                key = PyTuple_Pack(2, kn, nm);
                Py_DECREF(kn);
                Py_DECREF(nm);
                if (key == nullptr) throw py::error_already_set();
                if (code != 2) {
                    if (memo_.size() > static_cast<size_t>(PyDict_GET_SIZE(rd)) + 4096) clear();
                    it = memo_.emplace(kbuf_, key).first;  // the memo owns the reference PyTuple_Pack gave
                }
            }
            if (code == 2) {
                int rc = PyDict_DelItem(rd, key);
                if (it != memo_.end()) {
                    memo_.erase(it);
                }
                Py_DECREF(key);  // the memo's reference, or the one PyTuple_Pack gave
                if (rc != 0) {
                    if (!PyErr_ExceptionMatches(PyExc_KeyError)) throw py::error_already_set();
                    PyErr_Clear();
                }
            } else if (PyDict_SetItem(rd, key, line) != 0) {
                throw py::error_already_set();
            }
            if (PyList_Append(keep.ptr(), line) != 0) throw py::error_already_set();
        }
        return keep;
    }

  private:
    std::unordered_map<std::string, PyObject*> memo_;  // "namespace\0name" -> (namespace, name), a strong reference
    std::string kbuf_;
};

py::int_ key_partition(const std::string& ns, const std::string& name, int parts) {
    if (parts < 1) throw py::value_error("key_partition: parts must be >= 1");
    return py::int_(key_crc(ns, name) % static_cast<uint32_t>(parts));
}
