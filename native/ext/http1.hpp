// native/ext/http1.hpp — HTTP/1.1 response heads and chunked watch bodies (the clients' transport).
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// ----------------------------------------------------------------------------- HTTP/1.1 response heads
static std::string_view trim(std::string_view v) {
    while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t' || v.back() == '\r')) v.remove_suffix(1);
    return v;
}

static bool ieq(std::string_view a, std::string_view b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
        char x = a[i], y = b[i];
        if (x >= 'A' && x <= 'Z') x = static_cast<char>(x - 'A' + 'a');
        if (x != y) return false;
    }
    return true;
}

static bool icontains(std::string_view hay, std::string_view needle) {
    if (needle.size() > hay.size()) return false;
    for (size_t i = 0; i + needle.size() <= hay.size(); ++i)
        if (ieq(hay.substr(i, needle.size()), needle)) return true;
    return false;
}

// parse_response_head(head) -> (status, content_length | -1, chunked, connection_close, retry_after | None)
// `head` is everything before the blank line.  Only the headers the client acts on are extracted.
py::object parse_response_head(py::bytes head) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(head.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view h(buf, static_cast<size_t>(len));
    size_t eol = h.find("\r\n");
    std::string_view first = h.substr(0, eol);
    size_t sp = first.find(' ');
    if (sp == std::string_view::npos || first.substr(0, 5) != "HTTP/") throw py::value_error("bad status line");
    long status = 0;
    size_t i = sp + 1;
    int digits = 0;
    for (; i < first.size() && first[i] >= '0' && first[i] <= '9'; ++i, ++digits) status = status * 10 + (first[i] - '0');
    if (digits != 3) throw py::value_error("bad status code");
    long long clen = -1;
    bool chunked = false, close = false;
    py::object retry = py::none();
    size_t pos = eol == std::string_view::npos ? h.size() : eol + 2;
    while (pos < h.size()) {
        size_t e = h.find("\r\n", pos);
        std::string_view line = h.substr(pos, e == std::string_view::npos ? std::string_view::npos : e - pos);
        pos = e == std::string_view::npos ? h.size() : e + 2;
        size_t c = line.find(':');
        if (c == std::string_view::npos) continue;
        std::string_view k = trim(line.substr(0, c)), v = trim(line.substr(c + 1));
        if (ieq(k, "content-length")) {
            long long n = 0;
            if (v.empty()) throw py::value_error("bad content-length");
            for (char ch : v) {
                if (ch < '0' || ch > '9') throw py::value_error("bad content-length");
                n = n * 10 + (ch - '0');
                if (n > (1LL << 40)) throw py::value_error("content-length too large");
            }
            clen = n;
        } else if (ieq(k, "transfer-encoding")) {
            chunked = chunked || icontains(v, "chunked");
        } else if (ieq(k, "connection")) {
            close = ieq(v, "close");
        } else if (ieq(k, "retry-after")) {
            retry = py::str(v.data(), v.size());
        }
    }
    return py::make_tuple(status, clen, chunked, close, retry);
}

// chunk_lines(buf, state, linebuf) -> (lines, state, consumed, done, linebuf)
// Walks the chunked-transfer body bytes in `buf` (a bytearray; the caller deletes the `consumed` prefix) and
// returns the complete non-empty newline-terminated lines they carry, a chunk's data taken as it arrives,
// not once the whole chunk is in.  `state`: -1 a chunk-size line is next, -2 trailer lines after the last
// chunk, -3 the CRLF after a chunk's data, n > 0 data bytes left in the current chunk.  `linebuf` holds the
// start of an unfinished line between calls; `done` once the blank line ending the trailers was read.
// Same lines as ncc/kube/transport.py's Python path (`_parse_chunks` + `_feed_stream`).
py::object chunk_lines(py::object buf_o, long long state, py::object linebuf_o) {
    PyObject* b = buf_o.ptr();
    PyObject* lb = linebuf_o.ptr();
    if (!PyByteArray_Check(b) || !PyByteArray_Check(lb)) throw py::type_error("chunk_lines: bytearray expected");
    const char* p = PyByteArray_AS_STRING(b);
    const size_t n = static_cast<size_t>(PyByteArray_GET_SIZE(b));
    std::string cur(PyByteArray_AS_STRING(lb), static_cast<size_t>(PyByteArray_GET_SIZE(lb)));
    PyObject* lines = PyList_New(0);
    if (lines == nullptr) throw py::error_already_set();
    py::object lines_o = py::reinterpret_steal<py::object>(lines);
    auto push = [&](const char* d, size_t len) {
        PyObject* line = PyBytes_FromStringAndSize(d, static_cast<Py_ssize_t>(len));
        if (line == nullptr || PyList_Append(lines, line) != 0) {
            Py_XDECREF(line);
            throw py::error_already_set();
        }
        Py_DECREF(line);
    };
    auto data = [&](const char* d, size_t len) {
        size_t s0 = 0;
        while (s0 < len) {
            const char* nl = static_cast<const char*>(std::memchr(d + s0, '\n', len - s0));
            if (nl == nullptr) {
                cur.append(d + s0, len - s0);
                return;
            }
            size_t e = static_cast<size_t>(nl - d);
            if (cur.empty()) {
                if (e > s0) push(d + s0, e - s0);
            } else {
                cur.append(d + s0, e - s0);
                push(cur.data(), cur.size());
                cur.clear();
            }
            s0 = e + 1;
        }
    };
    auto crlf = [&](size_t from) -> size_t {
        for (size_t i = from; i + 1 < n; ++i) {
            const char* q = static_cast<const char*>(std::memchr(p + i, '\r', n - 1 - i));
            if (q == nullptr) return std::string::npos;
            i = static_cast<size_t>(q - p);
            if (p[i + 1] == '\n') return i;
        }
        return std::string::npos;
    };
    size_t pos = 0;
    bool done = false;
    while (pos < n && !done) {
        if (state == -1) {
            size_t e = crlf(pos);
            if (e == std::string::npos) break;
            std::string_view line(p + pos, e - pos);
            size_t semi = line.find(';');
            std::string_view hex = trim(line.substr(0, semi));
            if (hex.empty()) throw py::value_error("bad chunk size line");
            long long size = 0;
            for (char ch : hex) {
                int v = ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10
                      : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10 : -1;
                if (v < 0) throw py::value_error("bad chunk size line");
                size = size * 16 + v;
                if (size > (1LL << 40)) throw py::value_error("chunk too large");
            }
            pos = e + 2;
            state = size > 0 ? size : -2;
        } else if (state == -2) {
            size_t e = crlf(pos);
            if (e == std::string::npos) break;
            done = e == pos;
            pos = e + 2;
        } else if (state == -3) {
            if (n - pos < 2) break;
            if (p[pos] != '\r' || p[pos + 1] != '\n') throw py::value_error("chunk data not followed by CRLF");
            pos += 2;
            state = -1;
        } else if (state > 0) {
            size_t take = std::min(static_cast<size_t>(state), n - pos);
            data(p + pos, take);
            pos += take;
            state -= static_cast<long long>(take);
            if (state == 0) state = -3;
        } else {
            throw py::value_error("bad chunk state");
        }
    }
    PyObject* rest = PyByteArray_FromStringAndSize(cur.data(), static_cast<Py_ssize_t>(cur.size()));
    if (rest == nullptr) throw py::error_already_set();
    return py::make_tuple(lines_o, state, pos, done, py::reinterpret_steal<py::object>(rest));
}
