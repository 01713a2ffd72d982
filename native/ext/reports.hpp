// native/ext/reports.hpp — the coordinator's fold of shard-executor reports (msgpack frames).
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// ----------------------------------------------------------------------------- executor reports
// The coordinator folds every shard executor's per-pass reports into "which shards have reported on which
// version of each object" (ncc/controller/reports.py is the Python twin and the specification).  At 8
// shards that is 8 reports per template and wave; decoding them into dicts and folding them in Python was
// a third of the coordinator's CPU.  ReportTable.feed takes a raw IPC frame (ncc/controller/ipc.py: one
// msgpack message, or an array of them), folds the reports natively and hands back only what Python acts
// on: the keys whose report set became complete, the keys whose pass wrote, the failing shards, and every
// other message decoded.

class MpReader {
  public:
    MpReader(const char* p, size_t n) : p_(reinterpret_cast<const uint8_t*>(p)), e_(p_ + n) {}
    bool at_end() const { return p_ == e_; }

    [[noreturn]] static void fail() { throw py::value_error("msgpack: malformed frame"); }
    void need(size_t n) const {
        if (static_cast<size_t>(e_ - p_) < n) fail();
    }
    uint8_t peek() const {
        need(1);
        return *p_;
    }
    uint64_t be(int n) {
        need(static_cast<size_t>(n));
        uint64_t v = 0;
        for (int k = 0; k < n; ++k) v = (v << 8) | p_[k];
        p_ += n;
        return v;
    }
    // container headers: false (nothing consumed) when the next value is not of that kind
    // (a container cannot hold more elements than there are bytes left: one byte each at least, so a
    // corrupt length fails here instead of sizing a huge list)
    bool map_len(size_t& n) {
        uint8_t c = peek();
        if ((c & 0xf0) == 0x80) { ++p_; n = c & 0x0f; }
        else if (c == 0xde) { ++p_; n = be(2); }
        else if (c == 0xdf) { ++p_; n = be(4); }
        else return false;
        if (n > static_cast<size_t>(e_ - p_) / 2) fail();
        return true;
    }
    bool arr_len(size_t& n) {
        uint8_t c = peek();
        if ((c & 0xf0) == 0x90) { ++p_; n = c & 0x0f; }
        else if (c == 0xdc) { ++p_; n = be(2); }
        else if (c == 0xdd) { ++p_; n = be(4); }
        else return false;
        if (n > static_cast<size_t>(e_ - p_)) fail();
        return true;
    }
    bool str(std::string_view& out) {  // str or bin
        uint8_t c = peek();
        size_t n;
        if ((c & 0xe0) == 0xa0) { ++p_; n = c & 0x1f; }
        else if (c == 0xd9 || c == 0xc4) { ++p_; n = be(1); }
        else if (c == 0xda || c == 0xc5) { ++p_; n = be(2); }
        else if (c == 0xdb || c == 0xc6) { ++p_; n = be(4); }
        else return false;
        need(n);
        out = std::string_view(reinterpret_cast<const char*>(p_), n);
        p_ += n;
        return true;
    }
    bool integer(int64_t& v) {
        uint8_t c = peek();
        if (c <= 0x7f) { ++p_; v = c; return true; }
        if (c >= 0xe0) { ++p_; v = static_cast<int8_t>(c); return true; }
        switch (c) {
            case 0xcc: ++p_; v = static_cast<int64_t>(be(1)); return true;
            case 0xcd: ++p_; v = static_cast<int64_t>(be(2)); return true;
            case 0xce: ++p_; v = static_cast<int64_t>(be(4)); return true;
            case 0xcf: ++p_; v = static_cast<int64_t>(be(8)); return true;
            case 0xd0: ++p_; v = static_cast<int8_t>(be(1)); return true;
            case 0xd1: ++p_; v = static_cast<int16_t>(be(2)); return true;
            case 0xd2: ++p_; v = static_cast<int32_t>(be(4)); return true;
            case 0xd3: ++p_; v = static_cast<int64_t>(be(8)); return true;
            default: return false;
        }
    }
    bool nil() {
        if (peek() != 0xc0) return false;
        ++p_;
        return true;
    }
    // Python truthiness of the next value, consuming it (nil/false/0/""/empty containers are false)
    bool truthy() {
        uint8_t c = peek();
        if (c == 0xc0 || c == 0xc2) { ++p_; return false; }
        if (c == 0xc3) { ++p_; return true; }
        int64_t i;
        if (integer(i)) return i != 0;
        std::string_view s;
        if (str(s)) return !s.empty();
        size_t n;
        const uint8_t* at = p_;
        if (map_len(n) || arr_len(n)) {
            p_ = at;
            skip();
            return n != 0;
        }
        skip();  // floats
        return true;
    }
    void skip(int depth = 0) {
        if (depth > 64) fail();
        size_t n;
        std::string_view s;
        int64_t i;
        if (map_len(n)) {
            for (size_t k = 0; k < 2 * n; ++k) skip(depth + 1);
        } else if (arr_len(n)) {
            for (size_t k = 0; k < n; ++k) skip(depth + 1);
        } else if (str(s) || integer(i) || nil()) {
        } else {
            uint8_t c = peek();
            if (c == 0xc2 || c == 0xc3) { ++p_; }
            else if (c == 0xca) { ++p_; be(4); }
            else if (c == 0xcb) { ++p_; be(8); }
            else fail();
        }
    }
    // generic decode into a new reference (msgpack -> Python, as msgpack.unpackb(raw=False) does)
    PyObject* value(int depth = 0) {
        if (depth > 64) fail();
        size_t n;
        std::string_view s;
        int64_t i;
        uint8_t c = peek();
        if (map_len(n)) {
            PyObject* d = PyDict_New();
            if (d == nullptr) throw py::error_already_set();
            for (size_t k = 0; k < n; ++k) {
                PyObject* kk = nullptr;
                PyObject* vv = nullptr;
                try {
                    kk = value(depth + 1);
                    vv = value(depth + 1);
                } catch (...) {
                    Py_XDECREF(kk);
                    Py_DECREF(d);
                    throw;
                }
                int rc = PyDict_SetItem(d, kk, vv);
                Py_DECREF(kk);
                Py_DECREF(vv);
                if (rc != 0) { Py_DECREF(d); throw py::error_already_set(); }
            }
            return d;
        }
        if (arr_len(n)) {
            PyObject* l = PyList_New(static_cast<Py_ssize_t>(n));
            if (l == nullptr) throw py::error_already_set();
            for (size_t k = 0; k < n; ++k) {
                try {
                    PyList_SET_ITEM(l, static_cast<Py_ssize_t>(k), value(depth + 1));
                } catch (...) {
                    for (size_t j = k; j < n; ++j) { Py_INCREF(Py_None); PyList_SET_ITEM(l, static_cast<Py_ssize_t>(j), Py_None); }
                    Py_DECREF(l);
                    throw;
                }
            }
            return l;
        }
        if ((c & 0xe0) == 0xa0 || c == 0xd9 || c == 0xda || c == 0xdb) {
            str(s);
            PyObject* o = PyUnicode_DecodeUTF8(s.data(), static_cast<Py_ssize_t>(s.size()), "strict");
            if (o == nullptr) throw py::error_already_set();
            return o;
        }
        if (c == 0xc4 || c == 0xc5 || c == 0xc6) {
            str(s);
            return PyBytes_FromStringAndSize(s.data(), static_cast<Py_ssize_t>(s.size()));
        }
        if (c == 0xcf) {  // uint64: may not fit int64
            ++p_;
            return PyLong_FromUnsignedLongLong(be(8));
        }
        if (integer(i)) return PyLong_FromLongLong(i);
        if (nil()) Py_RETURN_NONE;
        if (c == 0xc2) { ++p_; Py_RETURN_FALSE; }
        if (c == 0xc3) { ++p_; Py_RETURN_TRUE; }
        if (c == 0xca) {
            ++p_;
            uint32_t u = static_cast<uint32_t>(be(4));
            float f;
            std::memcpy(&f, &u, 4);
            return PyFloat_FromDouble(f);
        }
        if (c == 0xcb) {
            ++p_;
            uint64_t u = be(8);
            double d;
            std::memcpy(&d, &u, 8);
            return PyFloat_FromDouble(d);
        }
        fail();
    }
    const uint8_t* pos() const { return p_; }
    void seek(const uint8_t* q) { p_ = q; }

  private:
    const uint8_t* p_;
    const uint8_t* e_;
};

class ReportTable {
  public:
    struct Slot {
        std::string shard;
        std::string uid;
        int64_t gen = 0;
        // the reported failure as its raw msgpack value (a typed failure map, ncc/controller/failures.py, or
        // a free-form string); empty: success (nil, or an empty string, which is falsy in the Python twin too)
        std::string err;
    };

    void set_shards(const std::vector<std::string>& shards) { shards_ = shards; }
    // This coordinator owns the keys of partition `part` of `parts`; reports on other keys are not folded but
    // kept, raw, for take_forwards() (the parent coordinator relays them to the partition's process).
    void set_partition(int part, int parts) {
        if (parts < 1 || part < 0 || part >= parts) throw py::value_error("set_partition: 0 <= part < parts");
        part_ = part;
        parts_ = parts;
    }
    // {partition: [raw msgpack report message, ...]} collected since the last call
    py::dict take_forwards() {
        py::dict out;
        for (auto& kv : forwards_) {
            py::list l;
            for (auto& m : kv.second) l.append(py::bytes(m));
            out[py::int_(kv.first)] = l;
        }
        forwards_.clear();
        return out;
    }
    std::vector<std::string> shards() const { return shards_; }
    size_t size() const { return state_.size(); }
    void pop(const std::string& key) { state_.erase(key); }
    void drop_shards(const std::vector<std::string>& names) {
        for (auto& kv : state_) {
            auto& v = kv.second;
            v.erase(std::remove_if(v.begin(), v.end(), [&](const Slot& s) {
                        return std::find(names.begin(), names.end(), s.shard) != names.end();
                    }), v.end());
        }
    }

    // feed(frame body, batch) -> (complete keys, wrote keys, failing shards, other messages, reports, pending)
    struct Folded {
        py::list complete, wrote, errors, others;
        int64_t reports = 0, pending = 0;
    };

    py::tuple feed(py::bytes body, bool batch) {
        std::string_view v = bytes_view(body);
        Folded f;
        fold_frame(v.data(), v.size(), batch, f);
        return py::make_tuple(f.complete, f.wrote, f.errors, f.others, f.reports, f.pending);
    }

    // feed_stream(buffer, start) -> (complete, wrote, errors, others, reports, pending, end): every complete
    // frame (4-byte big-endian length, high bit = batch, then the msgpack body) in buffer[start:], folded;
    // `end` is the offset of the first byte not consumed (a partial frame's header or body).
    py::tuple feed_stream(py::buffer buf, size_t start) {
        py::buffer_info info = buf.request();
        if (info.ndim != 1 || info.itemsize != 1) throw py::value_error("feed_stream: a byte buffer is required");
        const char* p = static_cast<const char*>(info.ptr);
        size_t len = static_cast<size_t>(info.size);
        if (start > len) throw py::value_error("feed_stream: start past the end");
        Folded f;
        size_t pos = start;
        while (len - pos >= 4) {
            const auto* h = reinterpret_cast<const uint8_t*>(p + pos);
            uint32_t n = (uint32_t(h[0]) << 24) | (uint32_t(h[1]) << 16) | (uint32_t(h[2]) << 8) | uint32_t(h[3]);
            bool batch = (n & 0x80000000u) != 0;
            n &= 0x7fffffffu;
            if (n > kMaxFrame) throw py::value_error("frame too large: " + std::to_string(n));
            if (len - pos - 4 < n) break;
            fold_frame(p + pos + 4, n, batch, f);
            pos += 4 + n;
        }
        return py::make_tuple(f.complete, f.wrote, f.errors, f.others, f.reports, f.pending, pos);
    }

    // readiness(key, uid, generation) -> None while some shard has not reported on this version, else
    // {shard: error | None} in shard order
    py::object readiness(const std::string& key, const std::string& uid, int64_t gen) const {
        auto it = state_.find(key);
        if (it == state_.end()) return py::none();
        py::dict out;
        for (const auto& s : shards_) {
            const Slot* e = find(it->second, s);
            if (e == nullptr || e->uid != uid || e->gen < gen) return py::none();
            if (e->err.empty()) {
                out[py::str(s)] = py::none();
            } else {
                MpReader er(e->err.data(), e->err.size());
                out[py::str(s)] = py::reinterpret_steal<py::object>(er.value());
            }
        }
        return std::move(out);
    }

    // ready_ok(key, uid, generation) -> None while some shard has not reported on this version, else
    // whether every shard succeeded (readiness() without building the dict)
    py::object ready_ok(const std::string& key, const std::string& uid, int64_t gen) const {
        auto it = state_.find(key);
        if (it == state_.end()) return py::none();
        bool ok = true;
        for (const auto& s : shards_) {
            const Slot* e = find(it->second, s);
            if (e == nullptr || e->uid != uid || e->gen < gen) return py::none();
            ok = ok && e->err.empty();
        }
        return py::bool_(ok);
    }

    // template_update(old, new, adopted, generation_filter, same_references) -> None | False | key
    // The coordinator's on_update handler for a template (ncc/controller/controller.py `_on_crd_update`, the
    // specification, with the adoption cache on) without running Python per event: None — nothing to do (an
    // informer resync or a status-only change); False — an early pass skipped (some shard has not reported on
    // the adopted version yet; its last report enqueues it); else the work-queue key to enqueue.  A new version
    // with the same references stays adopted.  `same_references` (ncc/api/refs.py) is called only when the
    // slim form's references digest cannot decide.  Anything of an unexpected type raises TypeError, and the
    // caller runs the Python handler instead.
    py::object template_update(py::dict old, py::dict nw, py::dict adopted, bool generation_filter,
                               py::object same_references) const {
        static PyObject* k_metadata = PyUnicode_InternFromString("metadata");
        static PyObject* k_rv = PyUnicode_InternFromString("resourceVersion");
        static PyObject* k_uid = PyUnicode_InternFromString("uid");
        static PyObject* k_gen = PyUnicode_InternFromString("generation");
        static PyObject* k_ns = PyUnicode_InternFromString("namespace");
        static PyObject* k_name = PyUnicode_InternFromString("name");
        static PyObject* k_labels = PyUnicode_InternFromString("labels");
        static PyObject* k_ann = PyUnicode_InternFromString("annotations");
        static PyObject* k_spec = PyUnicode_InternFromString("spec");
        static PyObject* k_rfp = PyUnicode_InternFromString("_rfp");
        static PyObject* k_status = PyUnicode_InternFromString("status");
        static PyObject* k_conditions = PyUnicode_InternFromString("conditions");
        auto get = [](PyObject* d, PyObject* k) -> PyObject* {  // borrowed; Py_None when absent
            PyObject* v = PyDict_GetItemWithError(d, k);
            if (v == nullptr && PyErr_Occurred()) throw py::error_already_set();
            return v != nullptr ? v : Py_None;
        };
        auto truthy = [](PyObject* v) {
            int t = PyObject_IsTrue(v);
            if (t < 0) throw py::error_already_set();
            return t == 1;
        };
        auto eq = [](PyObject* a, PyObject* b) {
            int r = PyObject_RichCompareBool(a, b, Py_EQ);
            if (r < 0) throw py::error_already_set();
            return r == 1;
        };
        // `x.get("metadata") or {}`: a dict, or None for an empty/absent one
        auto sub = [&](PyObject* d, PyObject* k) -> PyObject* {
            PyObject* v = get(d, k);
            if (!truthy(v)) return nullptr;
            if (!PyDict_Check(v)) throw py::type_error("template_update: not a mapping");
            return v;
        };
        auto str_of = [](PyObject* v, std::string& out) {  // `v or ""` of a string field
            if (v == Py_None) return;
            if (!PyUnicode_Check(v)) throw py::type_error("template_update: not a string");
            Py_ssize_t n = 0;
            const char* c = PyUnicode_AsUTF8AndSize(v, &n);
            if (c == nullptr) throw py::error_already_set();
            out.assign(c, static_cast<size_t>(n));
        };
        PyObject* om = sub(old.ptr(), k_metadata);
        PyObject* nm = sub(nw.ptr(), k_metadata);
        PyObject* nrv = nm != nullptr ? get(nm, k_rv) : Py_None;
        PyObject* orv = om != nullptr ? get(om, k_rv) : Py_None;
        std::string ns, name, key = "template/";
        if (nm != nullptr) {
            str_of(get(nm, k_ns), ns);
            PyObject* nv = get(nm, k_name);
            if (nv == Py_None && PyDict_Contains(nm, k_name) == 1)
                throw py::type_error("template_update: name is None");  // f"{None}" in the Python handler
            str_of(nv, name);
        }
        key.append(ns).append(1, '/').append(name);
        py::str pkey(key);
        // a new version with the same references stays adopted
        if (eq(get(adopted.ptr(), pkey.ptr()), orv) &&
            eq(om != nullptr ? get(om, k_uid) : Py_None, nm != nullptr ? get(nm, k_uid) : Py_None)) {
            bool same = false;
            PyObject* sa = get(old.ptr(), k_spec);
            PyObject* sb = get(nw.ptr(), k_spec);
            if (PyDict_Check(sa) && PyDict_Check(sb) && truthy(sa) && truthy(sb)) {
                PyObject* ra = get(sa, k_rfp);
                same = ra != Py_None && eq(ra, get(sb, k_rfp));
            }
            if (!same) same = same_references(old, nw).cast<bool>();
            if (same && PyDict_SetItem(adopted.ptr(), pkey.ptr(), nrv) < 0) throw py::error_already_set();
        }
        if (generation_filter) {
            if (eq(orv, nrv)) return py::none();  // informer resync: nothing changed
            PyObject* gen = om != nullptr ? get(om, k_gen) : Py_None;
            PyObject* none_ = Py_None;
            if (gen != Py_None && eq(gen, nm != nullptr ? get(nm, k_gen) : none_) &&
                eq(om != nullptr ? get(om, k_labels) : none_, nm != nullptr ? get(nm, k_labels) : none_) &&
                eq(om != nullptr ? get(om, k_ann) : none_, nm != nullptr ? get(nm, k_ann) : none_) &&
                eq(get(old.ptr(), k_spec), get(nw.ptr(), k_spec)))
                return py::none();  // status-only change (typically our own status write)
        }
        // an initialised, adopted version that not every shard has reported on: its last report enqueues it
        PyObject* st = sub(nw.ptr(), k_status);
        if (st != nullptr && truthy(get(st, k_conditions)) && eq(get(adopted.ptr(), pkey.ptr()), nrv)) {
            std::string uid;
            int64_t g = 0;
            if (nm != nullptr) {
                PyObject* u = get(nm, k_uid);
                if (truthy(u)) str_of(u, uid);
                PyObject* gv = get(nm, k_gen);
                if (truthy(gv)) {
                    if (!PyLong_Check(gv)) throw py::type_error("template_update: generation is not an int");
                    g = PyLong_AsLongLong(gv);
                    if (g == -1 && PyErr_Occurred()) throw py::error_already_set();
                }
            }
            if (ready(key, uid, g) < 0) return py::bool_(false);
        }
        return std::move(pkey);
    }

    // finish_batch(keys, items, assumed, adopted, memos, shards, queue, pending_event, event_on_noop)
    //     -> (rest, verify, events, done, superseded)
    // The coordinator's inline finish (ncc/controller/reconcile.py `finish_inline_many`, the specification) over
    // a batch of template keys whose report sets completed, read straight off the Python state it uses:
    // `items`/`assumed` the template store's dict and mutation overlay, `adopted` key -> adopted resourceVersion,
    // `memos` key -> (status digest, references digest, shard list) of the last verified status, `queue` the
    // work queue core (busy keys need a pass), `pending_event` the keys owing a Synced Event.  Per key: `rest`
    // (a queued pass is needed), `verify` (the Python path decides: an overlaid object, a non-slim template, no
    // memo for this status), `events` (finished, the template whose Synced Event is due), `done` finished
    // without an Event, or `superseded` (a newer version reached the cache: its own last report brings it back).
    py::tuple finish_batch(py::iterable keys, py::dict items, py::dict assumed, py::dict adopted, py::dict memos,
                           py::object shards, py::object queue, py::set pending_event, bool event_on_noop) const {
        static PyObject* k_status = PyUnicode_InternFromString("status");
        static PyObject* k_conditions = PyUnicode_InternFromString("conditions");
        static PyObject* k_metadata = PyUnicode_InternFromString("metadata");
        static PyObject* k_rv = PyUnicode_InternFromString("resourceVersion");
        static PyObject* k_uid = PyUnicode_InternFromString("uid");
        static PyObject* k_gen = PyUnicode_InternFromString("generation");
        static PyObject* k_sfp = PyUnicode_InternFromString("__ncc_sfp__");
        static PyObject* k_spec = PyUnicode_InternFromString("spec");
        static PyObject* k_rfp = PyUnicode_InternFromString("_rfp");
        RateLimitingQueue* nq = nullptr;
        if (py::isinstance<RateLimitingQueue>(queue)) nq = &queue.cast<RateLimitingQueue&>();
        py::list rest, verify, events;
        long long done = 0, superseded = 0;
        std::string k;
        const bool overlay = PyDict_GET_SIZE(assumed.ptr()) > 0;
        for (py::handle kh : keys) {
            PyObject* key = kh.ptr();
            Py_ssize_t klen = 0;
            const char* kc = PyUnicode_Check(key) ? PyUnicode_AsUTF8AndSize(key, &klen) : nullptr;
            if (kc == nullptr) {
                PyErr_Clear();
                verify.append(kh);
                continue;
            }
            k.assign(kc, static_cast<size_t>(klen));
            size_t a = k.find('/'), b = a == std::string::npos ? a : k.find('/', a + 1);
            bool is_busy = nq != nullptr ? nq->busy(k) : queue.attr("busy")(kh).cast<bool>();
            if (b == std::string::npos || k.compare(0, a, "template") != 0 || is_busy) {
                rest.append(kh);
                continue;
            }
            py::tuple ik = py::make_tuple(py::str(kc + a + 1, b - a - 1), py::str(kc + b + 1, k.size() - b - 1));
            if (overlay && PyDict_Contains(assumed.ptr(), ik.ptr()) == 1) {
                verify.append(kh);
                continue;
            }
            PyObject* t = PyDict_GetItem(items.ptr(), ik.ptr());
            if (t == nullptr || !PyDict_Check(t)) {
                rest.append(kh);
                continue;
            }
            PyObject* st = PyDict_GetItem(t, k_status);
            PyObject* conds = st != nullptr && PyDict_Check(st) ? PyDict_GetItem(st, k_conditions) : nullptr;
            PyObject* m = PyDict_GetItem(t, k_metadata);
            if (m == nullptr || !PyDict_Check(m)) m = nullptr;
            int conds_true = conds == nullptr ? 0 : PyObject_IsTrue(conds);
            if (conds_true < 0) throw py::error_already_set();
            PyObject* rv = m != nullptr ? PyDict_GetItem(m, k_rv) : nullptr;
            PyObject* ad = PyDict_GetItem(adopted.ptr(), key);
            int ne = PyObject_RichCompareBool(ad != nullptr ? ad : Py_None, rv != nullptr ? rv : Py_None, Py_NE);
            if (ne < 0) throw py::error_already_set();
            if (!conds_true || ne) {
                rest.append(kh);
                continue;
            }
            PyObject* uid = m != nullptr ? PyDict_GetItem(m, k_uid) : nullptr;
            PyObject* gen = m != nullptr ? PyDict_GetItem(m, k_gen) : nullptr;
            std::string uid_s;
            if (uid != nullptr && uid != Py_None) {
                Py_ssize_t ul = 0;
                const char* uc = PyUnicode_Check(uid) ? PyUnicode_AsUTF8AndSize(uid, &ul) : nullptr;
                if (uc == nullptr) {
                    PyErr_Clear();
                    verify.append(kh);
                    continue;
                }
                uid_s.assign(uc, static_cast<size_t>(ul));
            }
            int64_t g = 0;
            if (gen != nullptr && gen != Py_None) {
                if (!PyLong_Check(gen)) {
                    verify.append(kh);
                    continue;
                }
                g = PyLong_AsLongLong(gen);
                if (g == -1 && PyErr_Occurred()) {
                    PyErr_Clear();
                    verify.append(kh);
                    continue;
                }
            }
            int ok = ready(k, uid_s, g);
            if (ok < 0) {
                ++superseded;
                continue;
            }
            if (ok == 0) {
                rest.append(kh);
                continue;
            }
            PyObject* sfp = PyDict_GetItem(t, k_sfp);
            PyObject* spec = PyDict_GetItem(t, k_spec);
            PyObject* rfp = spec != nullptr && PyDict_Check(spec) ? PyDict_GetItem(spec, k_rfp) : nullptr;
            PyObject* memo = PyDict_GetItem(memos.ptr(), key);
            bool hit = sfp != nullptr && rfp != nullptr && memo != nullptr && PyTuple_Check(memo) &&
                       PyTuple_GET_SIZE(memo) == 3 && PyTuple_GET_ITEM(memo, 2) == shards.ptr();
            if (hit) {
                int e0 = PyObject_RichCompareBool(PyTuple_GET_ITEM(memo, 0), sfp, Py_EQ);
                int e1 = e0 == 1 ? PyObject_RichCompareBool(PyTuple_GET_ITEM(memo, 1), rfp, Py_EQ) : 0;
                if (e0 < 0 || e1 < 0) throw py::error_already_set();
                hit = e0 == 1 && e1 == 1;
            }
            if (!hit) {
                verify.append(kh);
                continue;
            }
            int pend = PySet_Contains(pending_event.ptr(), key);
            if (pend < 0) throw py::error_already_set();
            if (pend || event_on_noop) {
                if (pend && PySet_Discard(pending_event.ptr(), key) < 0) throw py::error_already_set();
                events.append(py::handle(t));
            } else {
                ++done;
            }
        }
        return py::make_tuple(rest, verify, events, done, superseded);
    }

  private:
    static constexpr uint32_t kMaxFrame = 64u * 1024 * 1024;  // ipc.MAX_FRAME

    // ready_ok without Python objects: -1 some shard has not reported on this version, 0 a failure, 1 all ok
    int ready(const std::string& key, const std::string& uid, int64_t gen) const {
        auto it = state_.find(key);
        if (it == state_.end()) return -1;
        bool ok = true;
        for (const auto& s : shards_) {
            const Slot* e = find(it->second, s);
            if (e == nullptr || e->uid != uid || e->gen < gen) return -1;
            ok = ok && e->err.empty();
        }
        return ok ? 1 : 0;
    }

    void fold_frame(const char* p, size_t len, bool batch, Folded& f) {
        MpReader r(p, len);
        size_t n = 1;
        if (batch && !r.arr_len(n)) MpReader::fail();
        for (size_t k = 0; k < n; ++k) {
            const uint8_t* at = r.pos();
            int rc = report(r, f.complete, f.wrote, f.errors);
            if (rc < 0) {  // not a report: decode it for Python
                r.seek(at);
                f.others.append(py::reinterpret_steal<py::object>(r.value()));
                continue;
            }
            if (rc == 2) continue;  // forwarded
            ++f.reports;
            if (rc == 0) ++f.pending;
        }
        if (!r.at_end()) MpReader::fail();
    }

    static const Slot* find(const std::vector<Slot>& v, std::string_view shard) {
        for (const auto& s : v)
            if (s.shard == shard) return &s;
        return nullptr;
    }

    // One message at the reader.  -1: not a report (nothing folded; the caller rewinds), 0: folded, some
    // shard still to report on this version, 1: folded and complete.
    int report(MpReader& r, py::list& complete, py::list& wrote, py::list& errors) {
        const uint8_t* msg = r.pos();
        size_t n;
        if (!r.map_len(n)) return -1;
        const uint8_t* body = r.pos();
        // first pass: is it {"t": "report", ...}?  (key order is the sender's)
        bool is_report = false;
        for (size_t k = 0; k < n; ++k) {
            std::string_view key, val;
            if (!r.str(key)) return -1;
            if (key == "t") {
                if (!r.str(val)) return -1;
                is_report = val == "report";
                break;
            }
            r.skip();
        }
        if (!is_report) return -1;
        r.seek(body);
        std::string_view rkey, uid;
        int64_t gen = 0;
        bool w = false, have_k = false;
        const uint8_t* results = nullptr;
        for (size_t k = 0; k < n; ++k) {
            std::string_view key;
            if (!r.str(key)) MpReader::fail();
            if (key == "k") {
                if (!r.str(rkey)) MpReader::fail();
                have_k = true;
            } else if (key == "u") {
                if (!r.str(uid)) MpReader::fail();
            } else if (key == "g") {
                if (!r.integer(gen) && !r.nil()) MpReader::fail();
            } else if (key == "w") {
                w = r.truthy();
            } else if (key == "r") {
                results = r.pos();
                r.skip();
            } else {
                r.skip();
            }
        }
        if (!have_k || results == nullptr) MpReader::fail();
        const uint8_t* end = r.pos();
        if (parts_ > 1) {  // ipc key "kind/ns/name": its partition is crc32("ns/name") % C (executor.key_part)
            size_t slash = rkey.find('/');
            std::string_view nsname = slash == std::string_view::npos ? std::string_view() : rkey.substr(slash + 1);
            int p = static_cast<int>((crc_update(0xFFFFFFFFu, nsname) ^ 0xFFFFFFFFu) % static_cast<uint32_t>(parts_));
            if (p != part_) {  // another coordinator partition's key: hand its raw bytes on, unfolded
                forwards_[p].emplace_back(reinterpret_cast<const char*>(msg), static_cast<size_t>(end - msg));
                return 2;
            }
        }
        std::string skey(rkey);
        auto& slots = state_[skey];
        r.seek(results);
        size_t m;
        if (!r.map_len(m)) MpReader::fail();
        bool changed = false;
        for (size_t k = 0; k < m; ++k) {
            std::string_view shard, err, text;
            if (!r.str(shard)) MpReader::fail();
            const uint8_t* v = r.pos();
            if (!r.nil()) {
                bool is_str = r.str(text);
                if (!is_str) r.skip();  // a typed failure map (or any other value): kept raw
                if (!is_str || !text.empty())  // an empty string is a success
                    err = std::string_view(reinterpret_cast<const char*>(v), static_cast<size_t>(r.pos() - v));
            }
            Slot* s = const_cast<Slot*>(find(slots, shard));
            if (s == nullptr) {
                slots.push_back(Slot{std::string(shard), {}, 0, {}});
                s = &slots.back();
                changed = true;
            } else if (!changed && (s->uid != uid || s->gen != gen || s->err != err)) {
                changed = true;
            }
            s->uid.assign(uid.data(), uid.size());
            s->gen = gen;
            s->err.assign(err.data(), err.size());
            if (!err.empty()) errors.append(py::str(shard.data(), shard.size()));
        }
        r.seek(end);
        py::str pkey(skey);
        if (w) wrote.append(pkey);
        for (const auto& sh : shards_) {
            const Slot* e = find(slots, sh);
            if (e == nullptr || e->uid != uid || e->gen < gen) return 0;
        }
        if (changed || w) complete.append(pkey);  // a repeat of a complete set changes nothing
        return 1;
    }

    std::vector<std::string> shards_;
    std::unordered_map<std::string, std::vector<Slot>> state_;
    int part_ = 0, parts_ = 1;
    std::map<int, std::vector<std::string>> forwards_;
};
