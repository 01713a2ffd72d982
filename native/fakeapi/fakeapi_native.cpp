// ncc.fakeapi._native — the fake kube-apiserver's native pieces (test and benchmark substrate, not product).
//
// The fake apiserver (ncc/fakeapi/) stands in for envtest/kind in tests and benchmarks; its
// per-request hot spots are here: the HTTP/1.1 request-head parser of its HTTP server (ncc/fakeapi/httpserver.py)
// and the HTTP/2 server side of ncc/fakeapi/h2.py — frame parser with HPACK decoding, and the response encoder.
// Until round 5 they lived in the controller's own extension (ncc/_native); they were split out so that the
// product ships and loads no server code.  HPACK itself (native/common/hpack.hpp) is shared
// with the clients: the encoder/decoder pair both sides of a connection run.
#include "../common/hpack.hpp"

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <Python.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
#include <vector>

#define NCC_FAKEAPI_NATIVE_ABI 1

namespace py = pybind11;

namespace {

std::string_view trim(std::string_view v) {
    while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t' || v.back() == '\r')) v.remove_suffix(1);
    return v;
}

// parse_request_head(head) -> (method, target, {lower-cased header name: value}) of an HTTP/1.1 request
// head (everything before the blank line); the fake apiserver's HTTP server.
py::object parse_request_head(py::bytes head) {
    char* buf = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(head.ptr(), &buf, &len) != 0) throw py::error_already_set();
    std::string_view h(buf, static_cast<size_t>(len));
    size_t eol = h.find("\r\n");
    std::string_view first = h.substr(0, eol);
    size_t s1 = first.find(' ');
    size_t s2 = s1 == std::string_view::npos ? s1 : first.find(' ', s1 + 1);
    if (s1 == std::string_view::npos || s2 == std::string_view::npos || s1 == 0 || s2 == s1 + 1)
        throw py::value_error("bad request line");
    std::string_view method = first.substr(0, s1), target = first.substr(s1 + 1, s2 - s1 - 1);
    py::dict headers;
    std::string key;
    size_t pos = eol == std::string_view::npos ? h.size() : eol + 2;
    while (pos < h.size()) {
        size_t e = h.find("\r\n", pos);
        std::string_view line = h.substr(pos, e == std::string_view::npos ? std::string_view::npos : e - pos);
        pos = e == std::string_view::npos ? h.size() : e + 2;
        size_t c = line.find(':');
        if (c == std::string_view::npos) continue;
        std::string_view k = trim(line.substr(0, c)), v = trim(line.substr(c + 1));
        key.assign(k.data(), k.size());
        for (auto& ch : key)
            if (ch >= 'A' && ch <= 'Z') ch = static_cast<char>(ch - 'A' + 'a');
        // latin-1 like the pure-Python server: every byte maps to one code point
        PyObject* ks = PyUnicode_DecodeLatin1(key.data(), static_cast<Py_ssize_t>(key.size()), nullptr);
        PyObject* vs = PyUnicode_DecodeLatin1(v.data(), static_cast<Py_ssize_t>(v.size()), nullptr);
        if (ks == nullptr || vs == nullptr) {
            Py_XDECREF(ks);
            Py_XDECREF(vs);
            throw py::error_already_set();
        }
        int rc = PyDict_SetItem(headers.ptr(), ks, vs);
        Py_DECREF(ks);
        Py_DECREF(vs);
        if (rc != 0) throw py::error_already_set();
    }
    PyObject* ms = PyUnicode_DecodeLatin1(method.data(), static_cast<Py_ssize_t>(method.size()), nullptr);
    PyObject* ts = PyUnicode_DecodeLatin1(target.data(), static_cast<Py_ssize_t>(target.size()), nullptr);
    if (ms == nullptr || ts == nullptr) {
        Py_XDECREF(ms);
        Py_XDECREF(ts);
        throw py::error_already_set();
    }
    return py::make_tuple(py::reinterpret_steal<py::object>(ms), py::reinterpret_steal<py::object>(ts), headers);
}


// HPACK for the fake apiserver's HTTP/2 server (ncc/fakeapi/h2.py): the decoder keeps the connection's dynamic
// table; the encoder is stateless (native/common/hpack.hpp)
class HpackDecoder {
public:
    explicit HpackDecoder(size_t max_table) : d_(max_table) {}
    py::list decode(const py::bytes& block) {
        std::string_view b = block;
        std::vector<ncc::hpack::Decoder::Header> hs;
        try {
            d_.decode(reinterpret_cast<const uint8_t*>(b.data()), b.size(), hs);
        } catch (const ncc::hpack::Error& e) {
            throw py::value_error(std::string("HPACK: ") + e.what());
        }
        py::list out;
        for (auto& h : hs) out.append(py::make_tuple(py::str(h.first), py::str(h.second)));
        return out;
    }
    void set_limit(size_t n) { d_.set_limit(n); }
    size_t table_size() const { return d_.table_size(); }
    size_t table_entries() const { return d_.table_entries(); }

private:
    ncc::hpack::Decoder d_;
};

// The fake apiserver's HTTP/2 framing (ncc/fakeapi/h2.py `H2Connection`): the frame parser, stream assembly and
// HPACK decoding of a connection, and the response encoder — the per-request work of its HTTP/2 path in C++, as
// the HTTP/1.1 path has its head parser here (parse_request_head).  Python keeps the policy: flow control of
// responses, the stream limit, GOAWAY, dispatch.
class H2ServerParser {
public:
    explicit H2ServerParser(bool credit_data, int64_t conn_credit_at = int64_t{1} << 29)
        : credit_(credit_data), conn_credit_at_(conn_credit_at) {}

    // Feed received bytes; returns the events they complete, in order:
    //   ("req", sid, method, path, {lower-cased name: value}, body)  a request whose END_STREAM arrived
    //   ("settings", [(id, value), ...])                              a SETTINGS frame to apply and ack
    //   ("window", sid, increment)   ("rst", sid, code)   ("ping", payload)   ("goaway", last, code)
    //   ("credit", sid, n)            DATA consumed (with credit_data, a small advertised window: per frame and
    //                                 stream; always, for the connection (sid 0), once half its 1 GiB is used)
    //   ("error", code, message)      a connection error: send GOAWAY and close
    py::list feed(const py::bytes& data) {
        std::string_view d = data;
        buf_.append(d.data(), d.size());
        py::list out;
        try {
            parse(out);
        } catch (const ncc::hpack::Error& e) {
            out.append(py::make_tuple("error", 9, std::string("HPACK: ") + e.what()));
            buf_.clear();
            pos_ = 0;
        } catch (const std::runtime_error& e) {
            out.append(py::make_tuple("error", 1, std::string(e.what())));
            buf_.clear();
            pos_ = 0;
        }
        if (pos_ > 0 && (pos_ == buf_.size() || pos_ > 65536)) {
            buf_.erase(0, pos_);
            pos_ = 0;
        }
        return out;
    }
    size_t open_streams() const { return streams_.size(); }

private:
    struct Stream {
        std::string method, path, authority;
        std::vector<std::pair<std::string, std::string>> headers;
        std::string body;
        bool have_headers = false, ended = false;
        bool malformed = false;  // RFC 9113 §8.2-8.3: misordered or missing pseudo-headers, uppercase names
    };
    std::string buf_;
    size_t pos_ = 0;
    bool preface_ = false, credit_;
    int64_t conn_unacked_ = 0;  // DATA bytes read since the last connection-level credit
    int64_t conn_credit_at_;
    uint32_t last_stream_ = 0, cont_id_ = 0;
    bool cont_end_ = false;
    std::string cont_block_;
    ncc::hpack::Decoder dec_{4096};
    std::unordered_map<uint32_t, Stream> streams_;

    static uint32_t u32(const char* p) {
        const auto* u = reinterpret_cast<const unsigned char*>(p);
        return (uint32_t{u[0]} << 24) | (uint32_t{u[1]} << 16) | (uint32_t{u[2]} << 8) | u[3];
    }
    static std::string_view strip(uint8_t flags, std::string_view p, bool headers) {
        size_t pad = 0;
        if (flags & 0x8) {
            if (p.empty()) throw std::runtime_error("padded frame without a pad length");
            pad = static_cast<uint8_t>(p[0]);
            p.remove_prefix(1);
        }
        if (headers && (flags & 0x20)) {
            if (p.size() < 5) throw std::runtime_error("short PRIORITY fields");
            p.remove_prefix(5);
        }
        if (pad > p.size()) throw std::runtime_error("padding longer than the frame");
        p.remove_suffix(pad);
        return p;
    }
    void emit_request(py::list& out, uint32_t sid, Stream& st) {
        if (st.malformed) {  // as Go's server: the stream is reset with PROTOCOL_ERROR, the connection lives on
            out.append(py::make_tuple("malformed", sid));
            streams_.erase(sid);
            return;
        }
        py::dict h;
        for (auto& kv : st.headers) h[py::str(kv.first)] = py::str(kv.second);
        if (!h.contains("host") && !st.authority.empty()) h["host"] = py::str(st.authority);
        out.append(py::make_tuple("req", sid, py::str(st.method.empty() ? "GET" : st.method),
                                  py::str(st.path.empty() ? "/" : st.path), h, py::bytes(st.body)));
        streams_.erase(sid);
    }
    void headers_done(py::list& out, uint32_t sid) {
        std::vector<ncc::hpack::Decoder::Header> hs;
        dec_.decode(reinterpret_cast<const uint8_t*>(cont_block_.data()), cont_block_.size(), hs);
        auto it = streams_.find(sid);
        if (it == streams_.end()) {  // a new stream (a HEADERS block on an open one is trailers)
            if (sid <= last_stream_ && sid != 0) throw std::runtime_error("stream id reused");
            last_stream_ = sid;
            it = streams_.emplace(sid, Stream{}).first;
        }
        Stream& st = it->second;
        if (!st.have_headers) {
            st.have_headers = true;
            bool regular = false, scheme = false;
            for (auto& h : hs) {
                if (!h.first.empty() && h.first[0] == ':') {
                    if (regular) st.malformed = true;
                    scheme = scheme || h.first == ":scheme";
                } else {
                    regular = true;
                    // field names are lowercase in HTTP/2 (RFC 9113 §8.2.1)
                    for (char c : h.first)
                        if (c >= 'A' && c <= 'Z') st.malformed = true;
                }
                if (h.first == ":method")
                    st.method = std::move(h.second);
                else if (h.first == ":path")
                    st.path = std::move(h.second);
                else if (h.first == ":authority")
                    st.authority = std::move(h.second);
                else if (!h.first.empty() && h.first[0] != ':' && h.first != "connection" && h.first != "keep-alive" &&
                         h.first != "transfer-encoding" && h.first != "upgrade" && h.first != "proxy-connection")
                    st.headers.emplace_back(std::move(h.first), std::move(h.second));
            }
            // :method, :scheme and :path are required (RFC 9113 §8.3.1), as Go's server checks
            if (st.method.empty() || st.path.empty() || !scheme) st.malformed = true;
        }
        if (cont_end_) emit_request(out, sid, st);
    }
    void parse(py::list& out) {
        static const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
        if (!preface_) {
            if (buf_.size() - pos_ < 24) return;
            if (buf_.compare(pos_, 24, kPreface, 24) != 0) throw std::runtime_error("bad connection preface");
            pos_ += 24;
            preface_ = true;
        }
        while (buf_.size() - pos_ >= 9) {
            const char* p = buf_.data() + pos_;
            uint32_t len = (uint32_t{static_cast<uint8_t>(p[0])} << 16) | (uint32_t{static_cast<uint8_t>(p[1])} << 8) |
                           static_cast<uint8_t>(p[2]);
            if (len > (1u << 14)) throw std::runtime_error("frame larger than SETTINGS_MAX_FRAME_SIZE");
            if (buf_.size() - pos_ < 9 + len) return;
            uint8_t type = static_cast<uint8_t>(p[3]), flags = static_cast<uint8_t>(p[4]);
            uint32_t sid = u32(p + 5) & 0x7fffffffu;
            std::string_view pl(p + 9, len);
            pos_ += 9 + len;
            if (cont_id_ != 0 && (type != 9 || sid != cont_id_)) throw std::runtime_error("expected CONTINUATION");
            switch (type) {
                case 0: {  // DATA
                    if (credit_ && len > 0) out.append(py::make_tuple("credit", sid, len));
                    // the connection window the server opened to 1 GiB is given back as it is used: without this
                    // a client stops sending request bodies after 1 GiB of them (a soak of ~300 bench waves)
                    conn_unacked_ += len;
                    if (conn_unacked_ >= conn_credit_at_) {
                        out.append(py::make_tuple("credit", 0, conn_unacked_));
                        conn_unacked_ = 0;
                    }
                    std::string_view d = strip(flags, pl, false);
                    auto it = streams_.find(sid);
                    if (it == streams_.end() || it->second.ended) {
                        out.append(py::make_tuple("rst_closed", sid));
                        break;
                    }
                    it->second.body.append(d.data(), d.size());
                    if (flags & 0x1) emit_request(out, sid, it->second);
                    break;
                }
                case 1: {  // HEADERS
                    if (sid == 0 || sid % 2 == 0) throw std::runtime_error("HEADERS on an even stream");
                    std::string_view b = strip(flags, pl, true);
                    cont_block_.assign(b.data(), b.size());
                    cont_end_ = (flags & 0x1) != 0;
                    if (flags & 0x4)
                        headers_done(out, sid);
                    else
                        cont_id_ = sid;
                    break;
                }
                case 9: {  // CONTINUATION
                    if (cont_id_ == 0) throw std::runtime_error("CONTINUATION without HEADERS");
                    cont_block_.append(pl.data(), pl.size());
                    if (flags & 0x4) {
                        uint32_t id = cont_id_;
                        cont_id_ = 0;
                        headers_done(out, id);
                    }
                    break;
                }
                case 4: {  // SETTINGS
                    if (flags & 0x1) break;
                    py::list kv;
                    for (size_t k = 0; k + 6 <= pl.size(); k += 6)
                        kv.append(py::make_tuple((static_cast<uint8_t>(pl[k]) << 8) | static_cast<uint8_t>(pl[k + 1]),
                                                 u32(pl.data() + k + 2)));
                    out.append(py::make_tuple("settings", kv));
                    break;
                }
                case 8:  // WINDOW_UPDATE
                    out.append(py::make_tuple("window", sid, pl.size() >= 4 ? (u32(pl.data()) & 0x7fffffffu) : 0u));
                    break;
                case 3:  // RST_STREAM
                    streams_.erase(sid);
                    out.append(py::make_tuple("rst", sid, pl.size() >= 4 ? u32(pl.data()) : 0u));
                    break;
                case 6:  // PING
                    if (!(flags & 0x1)) out.append(py::make_tuple("ping", py::bytes(pl.data(), pl.size())));
                    break;
                case 7:  // GOAWAY
                    out.append(py::make_tuple("goaway", pl.size() >= 4 ? (u32(pl.data()) & 0x7fffffffu) : 0u,
                                              pl.size() >= 8 ? u32(pl.data() + 4) : 0u));
                    break;
                case 5:
                    throw std::runtime_error("PUSH_PROMISE from a client");
                default:  // PRIORITY, unknown types
                    break;
            }
        }
    }
};

// HEADERS (+ CONTINUATION) and DATA frames of a whole response on stream `sid`, the last frame ending the stream;
// `extra`: further header fields.  The caller has checked the flow-control windows.
py::bytes h2_response(uint32_t sid, int status, const std::string& content_type, const py::bytes& body,
                      const std::vector<std::pair<std::string, std::string>>& extra, size_t max_frame) {
    std::string_view b = body;
    std::string block;
    ncc::hpack::encode_field(block, ":status", std::to_string(status));
    ncc::hpack::encode_literal(block, "content-type", content_type);
    ncc::hpack::encode_literal(block, "content-length", std::to_string(b.size()));
    for (const auto& kv : extra) ncc::hpack::encode_field(block, kv.first, kv.second);
    std::string out;
    out.reserve(block.size() + b.size() + 32);
    auto frame = [&out](uint8_t type, uint8_t flags, uint32_t id, const char* p, size_t n) {
        out.push_back(static_cast<char>(n >> 16));
        out.push_back(static_cast<char>(n >> 8));
        out.push_back(static_cast<char>(n));
        out.push_back(static_cast<char>(type));
        out.push_back(static_cast<char>(flags));
        out.push_back(static_cast<char>((id >> 24) & 0x7f));
        out.push_back(static_cast<char>(id >> 16));
        out.push_back(static_cast<char>(id >> 8));
        out.push_back(static_cast<char>(id));
        out.append(p, n);
    };
    max_frame = std::max<size_t>(max_frame, 1);
    size_t n = std::min(block.size(), max_frame);
    bool more = n < block.size();
    frame(1, static_cast<uint8_t>((b.empty() ? 0x1 : 0) | (more ? 0 : 0x4)), sid, block.data(), n);
    for (size_t off = n; off < block.size(); off += n) {
        n = std::min(block.size() - off, max_frame);
        frame(9, off + n < block.size() ? 0 : 0x4, sid, block.data() + off, n);
    }
    for (size_t off = 0; off < b.size(); off += n) {
        n = std::min(b.size() - off, max_frame);
        frame(0, off + n == b.size() ? 0x1 : 0, sid, b.data() + off, n);
    }
    return py::bytes(out);
}


py::bytes hpack_encode(const std::vector<std::pair<std::string, std::string>>& fields, bool huffman) {
    std::string out;
    for (const auto& f : fields) ncc::hpack::encode_field(out, f.first, f.second, huffman);
    return py::bytes(out);
}
}  // namespace

PYBIND11_MODULE(_native, m) {
    m.doc() = "the fake kube-apiserver's native pieces (ncc/fakeapi): HTTP/1.1 request heads, HTTP/2 server framing";
    m.attr("ABI_VERSION") = NCC_FAKEAPI_NATIVE_ABI;
    m.def("parse_request_head", &parse_request_head, py::arg("head"),
          "(method, target, {lower-cased name: value}) of an HTTP/1.1 request head");
    m.def("hpack_encode", &hpack_encode, py::arg("fields"), py::arg("huffman") = false,
          "a header block of static-table fields and literals without indexing");
    py::class_<HpackDecoder>(m, "HpackDecoder")
        .def(py::init<size_t>(), py::arg("max_table") = 4096)
        .def("decode", &HpackDecoder::decode, py::arg("block"),
             "one complete header block -> [(name, value)]; ValueError on a malformed block")
        .def("set_limit", &HpackDecoder::set_limit)
        .def("table_size", &HpackDecoder::table_size)
        .def("table_entries", &HpackDecoder::table_entries);
    py::class_<H2ServerParser>(m, "H2ServerParser")
        .def(py::init<bool, int64_t>(), py::arg("credit_data") = false, py::arg("conn_credit_at") = int64_t{1} << 29)
        .def("feed", &H2ServerParser::feed, py::arg("data"))
        .def("open_streams", &H2ServerParser::open_streams);
    m.def("h2_response", &h2_response, py::arg("sid"), py::arg("status"), py::arg("content_type"), py::arg("body"),
          py::arg("extra"), py::arg("max_frame"), "the HEADERS and DATA frames of a whole HTTP/2 response");
}
