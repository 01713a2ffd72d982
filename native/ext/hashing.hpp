// native/ext/hashing.hpp — structural fingerprints of JSON-shaped Python values (O(1) drift checks).
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

constexpr uint64_t kC1 = 0x87c37b91114253d5ULL;
constexpr uint64_t kC2 = 0x4cf5ad432745937fULL;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

inline uint64_t fmix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// Streaming murmur3-style 64-bit hasher (word-at-a-time; not adversarially secure — it only has
// to tell controller-desired content from shard-observed content).
struct Hasher {
    uint64_t h = 0x9e3779b97f4a7c15ULL;
    uint64_t n = 0;

    inline void word(uint64_t k) {
        k *= kC1;
        k = rotl(k, 31);
        k *= kC2;
        h ^= k;
        h = rotl(h, 27) * 5 + 0x52dce729;
        n += 8;
    }
    inline void tag(char t, uint64_t len) { word((static_cast<uint64_t>(static_cast<unsigned char>(t)) << 56) ^ len); }
    void bytes(const char* p, size_t len) {
        size_t i = 0;
        for (; i + 8 <= len; i += 8) {
            uint64_t k;
            std::memcpy(&k, p + i, 8);
            word(k);
        }
        uint64_t tail = 0;
        size_t rem = len - i;
        if (rem) {
            std::memcpy(&tail, p + i, rem);
            word(tail ^ (static_cast<uint64_t>(rem) << 59));
        }
    }
    uint64_t digest() const { return fmix(h ^ n); }
};

struct KV {
    const char* k;
    Py_ssize_t klen;
    PyObject* v;
};

void hash_obj(Hasher& hs, PyObject* o, int depth);

void hash_str(Hasher& hs, PyObject* o) {
    Py_ssize_t len = 0;
    const char* s = PyUnicode_AsUTF8AndSize(o, &len);
    if (!s) throw py::error_already_set();
    hs.tag('s', static_cast<uint64_t>(len));
    hs.bytes(s, static_cast<size_t>(len));
}

void hash_obj(Hasher& hs, PyObject* o, int depth) {
    if (depth > 512) throw py::value_error("fingerprint: nesting too deep");
    if (o == Py_None) {
        hs.tag('n', 0);
    } else if (o == Py_True) {
        hs.tag('t', 1);
    } else if (o == Py_False) {
        hs.tag('f', 0);
    } else if (PyUnicode_Check(o)) {
        hash_str(hs, o);
    } else if (PyLong_Check(o)) {
        int overflow = 0;
        long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
        if (overflow) {
            PyObject* r = PyObject_Str(o);
            if (!r) throw py::error_already_set();
            hs.tag('I', 0);
            hash_str(hs, r);
            Py_DECREF(r);
        } else {
            hs.tag('i', 8);
            hs.word(static_cast<uint64_t>(v));
        }
    } else if (PyFloat_Check(o)) {
        double d = PyFloat_AS_DOUBLE(o);
        if (d == 0.0) d = 0.0;  // fold -0.0
        uint64_t bits;
        std::memcpy(&bits, &d, 8);
        hs.tag('r', 8);
        hs.word(bits);
    } else if (PyDict_Check(o)) {
        Py_ssize_t n = PyDict_Size(o);
        hs.tag('d', static_cast<uint64_t>(n));
        std::vector<KV> items;
        items.reserve(static_cast<size_t>(n));
        PyObject *k, *v;
        Py_ssize_t pos = 0;
        while (PyDict_Next(o, &pos, &k, &v)) {
            if (!PyUnicode_Check(k)) throw py::type_error("fingerprint: dict keys must be str");
            Py_ssize_t klen = 0;
            const char* ks = PyUnicode_AsUTF8AndSize(k, &klen);
            if (!ks) throw py::error_already_set();
            items.push_back({ks, klen, v});
        }
        std::sort(items.begin(), items.end(), [](const KV& a, const KV& b) {
            int c = std::memcmp(a.k, b.k, static_cast<size_t>(std::min(a.klen, b.klen)));
            return c != 0 ? c < 0 : a.klen < b.klen;
        });
        for (const auto& it : items) {
            hs.tag('k', static_cast<uint64_t>(it.klen));
            hs.bytes(it.k, static_cast<size_t>(it.klen));
            hash_obj(hs, it.v, depth + 1);
        }
    } else if (PyList_Check(o) || PyTuple_Check(o)) {
        PyObject* seq = o;
        Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
        PyObject** items = PySequence_Fast_ITEMS(seq);
        hs.tag('l', static_cast<uint64_t>(n));
        for (Py_ssize_t i = 0; i < n; ++i) hash_obj(hs, items[i], depth + 1);
    } else if (PyBytes_Check(o)) {
        hs.tag('b', static_cast<uint64_t>(PyBytes_GET_SIZE(o)));
        hs.bytes(PyBytes_AS_STRING(o), static_cast<size_t>(PyBytes_GET_SIZE(o)));
    } else {
        PyObject* r = PyObject_Repr(o);
        if (!r) throw py::error_already_set();
        hs.tag('o', 0);
        hash_str(hs, r);
        Py_DECREF(r);
    }
}

uint64_t fingerprint(py::handle obj) {
    Hasher hs;
    hash_obj(hs, obj.ptr(), 0);
    return hs.digest();
}

py::list fingerprint_many(py::sequence objs) {
    py::list out;
    for (auto o : objs) out.append(py::int_(fingerprint(o)));
    return out;
}
