// native/ext/h2client.hpp — HTTP/2 framing and HPACK for the Python clients (ncc/kube/h2client.py).
// Part of the `ncc._native` extension: included, in order, inside native/ncc_native.cpp's anonymous
// namespace (it uses what the headers before it define); not a standalone header.
#pragma once

// The Python clients' HTTP/2 framing (ncc/kube/h2client.py `H2Conn`, the coordinator's connection to the
// controller cluster and the Python executor's to its shards): the frame parser, HPACK decoding of response heads,
// body assembly, the line splitting of watch bodies, and the replies the connection owes by itself (SETTINGS and
// PING acks, WINDOW_UPDATE for consumed DATA).  Python keeps the policy: streams, send windows, limits, GOAWAY.
class H2ClientParser {
public:
    static constexpr uint32_t kMaxFrame = 1u << 20;       // what the client advertises (SETTINGS_MAX_FRAME_SIZE)
    static constexpr int64_t kStreamWindow = 1 << 24;      // SETTINGS_INITIAL_WINDOW_SIZE from the client
    static constexpr int64_t kConnWindow = int64_t{1} << 30;  // the connection window after the opening update

    // The client's connection preface, SETTINGS and the connection-window update.
    static py::bytes preface() {
        std::string out("PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n", 24);
        std::string s;
        auto setting = [&s](uint16_t id, uint32_t v) {
            s.push_back(static_cast<char>(id >> 8));
            s.push_back(static_cast<char>(id));
            put32(s, v);
        };
        setting(0x2, 0);  // ENABLE_PUSH
        setting(0x4, static_cast<uint32_t>(kStreamWindow));
        setting(0x5, kMaxFrame);
        frame(out, 4, 0, 0, s);
        std::string w;
        put32(w, static_cast<uint32_t>(kConnWindow - 65535));
        frame(out, 8, 0, 0, w);
        return py::bytes(out);
    }

    // DATA of stream `sid` comes back as complete lines ("lines" events) instead of one body.
    void watch(uint32_t sid) { streams_[sid].watch = true; }
    // A stream the client reset: its remaining frames are dropped.  (Other streams are known from their response
    // HEADERS on; the set of reset ones is pruned of its oldest half past 1024: the server stopped those long ago.)
    void forget(uint32_t sid) {
        streams_.erase(sid);
        dead_.insert(sid);
        if (dead_.size() > 1024) dead_.erase(dead_.begin(), std::next(dead_.begin(), 512));
    }
    size_t open_streams() const { return streams_.size(); }

    // Feed received bytes -> (events, bytes to send).  Events, in order:
    //   ("resp", sid, status, retry_after | None, body)  a whole response (END_STREAM seen)
    //   ("head", sid, status, retry_after | None)        a watch stream's response head
    //   ("lines", sid, [line, ...], data_bytes, ended)   a watch stream's complete lines (and its end)
    //   ("settings", [(id, value), ...])  ("window", sid, n)  ("rst", sid, code)  ("goaway", last, code, debug)
    //   ("error", code, message)   a connection error (send GOAWAY, close)
    //   ("noh2",)                   the first frame was not SETTINGS: the server does not speak HTTP/2
    // Sent bytes: SETTINGS / PING acks and WINDOW_UPDATEs for the connection and for unwatched streams (a watch's
    // stream window is credited by Python as its consumer takes the lines).
    py::tuple feed(const py::bytes& data) {
        std::string_view d = data;
        buf_.append(d.data(), d.size());
        py::list ev;
        out_.clear();
        try {
            parse(ev);
        } catch (const ncc::hpack::Error& e) {
            ev.append(py::make_tuple("error", 9, std::string("HPACK: ") + e.what()));
            buf_.clear();
            pos_ = 0;
        } catch (const std::runtime_error& e) {
            ev.append(py::make_tuple("error", 1, std::string(e.what())));
            buf_.clear();
            pos_ = 0;
        }
        if (pos_ > 0 && (pos_ == buf_.size() || pos_ > 65536)) {
            buf_.erase(0, pos_);
            pos_ = 0;
        }
        if (conn_unacked_ >= (1 << 24)) {
            std::string w;
            put32(w, static_cast<uint32_t>(conn_unacked_));
            frame(out_, 8, 0, 0, w);
            conn_unacked_ = 0;
        }
        return py::make_tuple(ev, py::bytes(out_));
    }

private:
    struct Stream {
        std::string body, pending;  // unary: the body; watch: the partial line
        int status = 0;
        py::object retry = py::none();
        int64_t unacked = 0;
        bool watch = false, have_head = false;
    };
    std::string buf_, out_;
    size_t pos_ = 0;
    bool first_ = true;
    uint32_t cont_id_ = 0;
    bool cont_end_ = false;
    std::string cont_block_;
    int64_t conn_unacked_ = 0;
    ncc::hpack::Decoder dec_{4096};
    std::unordered_map<uint32_t, Stream> streams_;
    std::set<uint32_t> dead_;

    static uint32_t u32(const char* p) {
        const auto* u = reinterpret_cast<const unsigned char*>(p);
        return (uint32_t{u[0]} << 24) | (uint32_t{u[1]} << 16) | (uint32_t{u[2]} << 8) | u[3];
    }
    static void put32(std::string& s, uint32_t v) {
        s.push_back(static_cast<char>(v >> 24));
        s.push_back(static_cast<char>(v >> 16));
        s.push_back(static_cast<char>(v >> 8));
        s.push_back(static_cast<char>(v));
    }
    static void frame(std::string& out, uint8_t type, uint8_t flags, uint32_t id, std::string_view p) {
        size_t n = p.size();
        out.push_back(static_cast<char>(n >> 16));
        out.push_back(static_cast<char>(n >> 8));
        out.push_back(static_cast<char>(n));
        out.push_back(static_cast<char>(type));
        out.push_back(static_cast<char>(flags));
        put32(out, id & 0x7fffffffu);
        out.append(p.data(), n);
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
    void finish(py::list& ev, uint32_t sid, Stream& st) {
        if (st.watch) {
            py::list lines;
            size_t a = st.pending.find_first_not_of(" \t\r\n");
            if (a != std::string::npos) lines.append(py::bytes(st.pending));
            ev.append(py::make_tuple("lines", sid, lines, 0, true));
        } else {
            ev.append(py::make_tuple("resp", sid, st.status, st.retry, py::bytes(st.body)));
        }
        streams_.erase(sid);
    }
    void headers_done(py::list& ev, uint32_t sid) {
        std::vector<ncc::hpack::Decoder::Header> hs;
        dec_.decode(reinterpret_cast<const uint8_t*>(cont_block_.data()), cont_block_.size(), hs);
        auto it = streams_.find(sid);
        if (it == streams_.end()) {
            if (sid % 2 == 0 || dead_.count(sid)) return;  // a stream the client gave up on (the block fed the table)
            it = streams_.emplace(sid, Stream{}).first;
        }
        Stream& st = it->second;
        if (!st.have_head) {
            int status = 0;
            for (auto& h : hs) {
                if (h.first == ":status") {
                    status = std::atoi(h.second.c_str());
                } else if (h.first == "retry-after") {
                    st.retry = py::str(h.second);
                }
            }
            if (status == 0) throw std::runtime_error("response without :status");
            if (status >= 200) {  // 1xx heads are informational: the real one follows
                st.status = status;
                st.have_head = true;
                if (st.watch) ev.append(py::make_tuple("head", sid, status, st.retry));
            }
        }  // else trailers: nothing in them is used
        if (cont_end_) finish(ev, sid, st);
    }
    void on_data(py::list& ev, uint32_t sid, uint8_t flags, std::string_view pl, uint32_t len) {
        conn_unacked_ += len;
        std::string_view d = strip(flags, pl, false);
        auto it = streams_.find(sid);
        if (it == streams_.end()) return;  // reset by us: already counted against the connection, dropped
        Stream& st = it->second;
        if (!st.have_head) throw std::runtime_error("DATA before the response head");
        if (st.watch) {
            py::list lines;
            std::string& p = st.pending;
            size_t start = 0, nl;
            while ((nl = d.find('\n', start)) != std::string_view::npos) {
                if (p.empty()) {
                    if (nl > start) lines.append(py::bytes(d.data() + start, nl - start));
                } else {
                    p.append(d.data() + start, nl - start);
                    lines.append(py::bytes(p));
                    p.clear();
                }
                start = nl + 1;
            }
            p.append(d.data() + start, d.size() - start);
            if (py::len(lines) > 0 || len > 0)
                ev.append(py::make_tuple("lines", sid, lines, len, false));
        } else {
            st.body.append(d.data(), d.size());
            st.unacked += len;
            if (st.unacked >= kStreamWindow / 2 && !(flags & 0x1)) {
                std::string w;
                put32(w, static_cast<uint32_t>(st.unacked));
                frame(out_, 8, 0, sid, w);
                st.unacked = 0;
            }
        }
        if (flags & 0x1) finish(ev, sid, st);
    }
    void parse(py::list& ev) {
        while (buf_.size() - pos_ >= 9) {
            const char* p = buf_.data() + pos_;
            uint32_t len = (uint32_t{static_cast<uint8_t>(p[0])} << 16) | (uint32_t{static_cast<uint8_t>(p[1])} << 8) |
                           static_cast<uint8_t>(p[2]);
            uint8_t type = static_cast<uint8_t>(p[3]), flags = static_cast<uint8_t>(p[4]);
            if (first_) {  // a server speaking HTTP/2 opens with SETTINGS (not an ack)
                if (type != 4 || (flags & 0x1) || len % 6 != 0 || len > 6 * 64) {
                    ev.append(py::make_tuple("noh2"));
                    buf_.clear();
                    pos_ = 0;
                    return;
                }
                first_ = false;
            }
            if (len > kMaxFrame) throw std::runtime_error("frame larger than SETTINGS_MAX_FRAME_SIZE");
            if (buf_.size() - pos_ < 9 + len) return;
            uint32_t sid = u32(p + 5) & 0x7fffffffu;
            std::string_view pl(p + 9, len);
            pos_ += 9 + len;
            if (cont_id_ != 0 && (type != 9 || sid != cont_id_)) throw std::runtime_error("expected CONTINUATION");
            switch (type) {
                case 0:
                    on_data(ev, sid, flags, pl, len);
                    break;
                case 1: {  // HEADERS
                    if (sid == 0) throw std::runtime_error("HEADERS on stream 0");
                    std::string_view b = strip(flags, pl, true);
                    cont_block_.assign(b.data(), b.size());
                    cont_end_ = (flags & 0x1) != 0;
                    if (flags & 0x4)
                        headers_done(ev, sid);
                    else
                        cont_id_ = sid;
                    break;
                }
                case 9:  // CONTINUATION
                    if (cont_id_ == 0) throw std::runtime_error("CONTINUATION without HEADERS");
                    cont_block_.append(pl.data(), pl.size());
                    if (flags & 0x4) {
                        uint32_t id = cont_id_;
                        cont_id_ = 0;
                        headers_done(ev, id);
                    }
                    break;
                case 4: {  // SETTINGS
                    if (flags & 0x1) break;
                    if (len % 6 != 0) throw std::runtime_error("SETTINGS length not a multiple of 6");
                    py::list kv;
                    for (size_t k = 0; k + 6 <= pl.size(); k += 6) {
                        uint32_t id = (static_cast<uint8_t>(pl[k]) << 8) | static_cast<uint8_t>(pl[k + 1]);
                        uint32_t v = u32(pl.data() + k + 2);
                        // SETTINGS_HEADER_TABLE_SIZE (0x1) bounds the table of *our* encoder, which keeps none;
                        // the server's encoder stays bound by the size we advertise (the 4096 default), so our
                        // decoder keeps it (RFC 9113 §6.5.2, RFC 7541 §4.2) whatever the server sends here
                        kv.append(py::make_tuple(id, v));
                    }
                    frame(out_, 4, 0x1, 0, {});
                    ev.append(py::make_tuple("settings", kv));
                    break;
                }
                case 8:  // WINDOW_UPDATE
                    ev.append(py::make_tuple("window", sid, pl.size() >= 4 ? (u32(pl.data()) & 0x7fffffffu) : 0u));
                    break;
                case 3:  // RST_STREAM (also of a stream whose response had not begun: Python knows it)
                    streams_.erase(sid);
                    ev.append(py::make_tuple("rst", sid, pl.size() >= 4 ? u32(pl.data()) : 0u));
                    break;
                case 6:  // PING
                    if (!(flags & 0x1)) frame(out_, 6, 0x1, 0, pl);
                    break;
                case 7:  // GOAWAY
                    ev.append(py::make_tuple("goaway", pl.size() >= 4 ? (u32(pl.data()) & 0x7fffffffu) : 0u,
                                             pl.size() >= 8 ? u32(pl.data() + 4) : 0u,
                                             py::bytes(pl.size() > 8 ? pl.substr(8) : std::string_view())));
                    break;
                case 5:
                    throw std::runtime_error("PUSH_PROMISE with push disabled");
                default:  // PRIORITY, unknown types
                    break;
            }
        }
    }
};

// A request's HEADERS (+ CONTINUATION) and, when `body` is not empty, its DATA frames on stream `sid`.  `fixed` is
// the caller's pre-encoded block of the fields every request repeats (:scheme, :authority, user-agent, accept,
// content-type, authorization); `content_length` < 0 sends none; `end` ends the stream on the last frame (false:
// the body follows as DATA frames the caller sends when the flow-control windows allow).
py::bytes h2_request(uint32_t sid, const std::string& method, const std::string& path, const py::bytes& fixed,
                     int64_t content_length, const py::bytes& body, bool end, size_t max_frame) {
    std::string_view f = fixed, b = body;
    std::string block;
    block.reserve(f.size() + path.size() + 16);
    ncc::hpack::encode_field(block, ":method", method);
    ncc::hpack::encode_literal_indexed_name(block, 4, path);  // :path
    block.append(f.data(), f.size());
    if (content_length >= 0) ncc::hpack::encode_literal_indexed_name(block, 28, std::to_string(content_length));
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
    frame(1, static_cast<uint8_t>((b.empty() && end ? 0x1 : 0) | (more ? 0 : 0x4)), sid, block.data(), n);
    for (size_t off = n; off < block.size(); off += n) {
        n = std::min(block.size() - off, max_frame);
        frame(9, off + n < block.size() ? 0 : 0x4, sid, block.data() + off, n);
    }
    for (size_t off = 0; off < b.size(); off += n) {
        n = std::min(b.size() - off, max_frame);
        frame(0, off + n == b.size() && end ? 0x1 : 0, sid, b.data() + off, n);
    }
    return py::bytes(out);
}

py::bytes hpack_encode(const std::vector<std::pair<std::string, std::string>>& fields, bool huffman) {
    std::string out;
    for (const auto& f : fields) ncc::hpack::encode_field(out, f.first, f.second, huffman);
    return py::bytes(out);
}

py::bytes hpack_huffman_decode(const py::bytes& data) {
    std::string_view b = data;
    std::string out;
    try {
        ncc::hpack::huffman_decode(reinterpret_cast<const uint8_t*>(b.data()), b.size(), out);
    } catch (const ncc::hpack::Error& e) {
        throw py::value_error(std::string("HPACK: ") + e.what());
    }
    return py::bytes(out);
}
