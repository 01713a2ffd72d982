// HTTP/2 (RFC 9113) framing and per-connection state for the shard client (http.hpp `Client`, which drives it:
// `exchange_h2`, `h2_read`, `h2_frame`).  kube-apiservers speak HTTP/2 — client-go negotiates it by ALPN on
// every TLS connection and multiplexes a clientset's requests over it (/root/reference/main.go:52-68) — so
// with `client-http2` the executor writes to a shard over a few connections carrying many concurrent
// streams, instead of up to `client-pool-size` HTTP/1.1 keep-alive connections each carrying one request:
// one TLS handshake per connection instead of one per concurrent request, and no head-of-line blocking.
//
// What is implemented (client side): the connection preface, SETTINGS both ways (ENABLE_PUSH 0, a 16 MiB stream
// window and a 1 GiB connection window from us; the server's MAX_CONCURRENT_STREAMS, INITIAL_WINDOW_SIZE and
// MAX_FRAME_SIZE obeyed), HEADERS/CONTINUATION with HPACK (native/common/hpack.hpp), DATA within the server's
// connection and stream windows (a request body waits for WINDOW_UPDATE), WINDOW_UPDATE for what we consume,
// PING acks, RST_STREAM (REFUSED_STREAM: re-sent), GOAWAY (streams past the last one the server will serve are
// re-sent on another connection; the connection takes no new ones and closes when its streams are done),
// per-stream deadlines (RST_STREAM CANCEL).  Watches are streams too (`Client::stream`), as client-go's: a
// shard's four watches and its writes share its HTTP/2 connection.
//
// Error codes: a GOAWAY with an error code (ENHANCE_YOUR_CALM, PROTOCOL_ERROR, ...) makes
// the re-sends of the streams it refused back off (`Client::h2_backoff_until_`) instead of going out at once;
// HTTP_1_1_REQUIRED in RST_STREAM or GOAWAY downgrades the shard to HTTP/1.1, as an ALPN refusal does, with a
// Warning; a WINDOW_UPDATE of 0 or one that overflows a window past 2^31-1 is an error (RFC 9113 §6.9, a
// stream error on a stream, a connection error on the connection); and a connection error is announced with
// GOAWAY before the connection closes (§5.4.1).
#pragma once

#include <algorithm>
#include <cstdint>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>

#include "../common/hpack.hpp"

namespace ncc {
namespace h2 {

inline constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
inline constexpr size_t kPrefaceLen = 24;

enum FrameType : uint8_t {
    DATA = 0, HEADERS = 1, PRIORITY = 2, RST_STREAM = 3, SETTINGS = 4, PUSH_PROMISE = 5, PING = 6, GOAWAY = 7,
    WINDOW_UPDATE = 8, CONTINUATION = 9
};
enum Flag : uint8_t { END_STREAM = 0x1, ACK = 0x1, END_HEADERS = 0x4, PADDED = 0x8, PRIORITY_FLAG = 0x20 };
enum Setting : uint16_t {
    HEADER_TABLE_SIZE = 1, ENABLE_PUSH = 2, MAX_CONCURRENT_STREAMS = 3, INITIAL_WINDOW_SIZE = 4, MAX_FRAME_SIZE = 5
};
enum ErrorCode : uint32_t {
    NO_ERROR = 0, PROTOCOL_ERROR = 1, FLOW_CONTROL_ERROR = 3, FRAME_SIZE_ERROR = 6, REFUSED_STREAM = 7, CANCEL = 8,
    COMPRESSION_ERROR = 9, ENHANCE_YOUR_CALM = 0xb, HTTP_1_1_REQUIRED = 0xd
};
inline constexpr int64_t kMaxWindow = 0x7fffffff;  // a flow-control window never exceeds 2^31-1 (RFC 9113 §6.9.1)
// re-sends of a request the server did not take (REFUSED_STREAM, ENHANCE_YOUR_CALM, past a GOAWAY, no HTTP/2), as
// ncc/kube/h2client.py MAX_UNPROCESSED_RETRIES: with the refusal backoff (50 ms doubling to 5 s) about a minute
inline constexpr int kMaxResends = 16;

// A connection error (RFC 9113 §5.4.1): the client sends GOAWAY with `code` and closes the connection.
struct ConnectionError : std::runtime_error {
    uint32_t code;
    ConnectionError(uint32_t c, const std::string& what) : std::runtime_error(what), code(c) {}
};

// GOAWAY (last stream id 0: the server opens no streams here) with `code` and a short debug text.
inline std::string goaway_frame(uint32_t code, std::string_view debug);

inline constexpr int64_t kStreamWindow = 1 << 24;  // what we let the server send per stream before an update
inline constexpr int64_t kConnWindow = 1 << 30;
inline constexpr uint32_t kOurMaxFrame = 1 << 20;  // the largest frame we accept (SETTINGS_MAX_FRAME_SIZE)

inline uint32_t get32(const char* p) {
    const auto* u = reinterpret_cast<const unsigned char*>(p);
    return (uint32_t{u[0]} << 24) | (uint32_t{u[1]} << 16) | (uint32_t{u[2]} << 8) | u[3];
}
inline void put32(std::string& out, uint32_t v) {
    out.push_back(static_cast<char>(v >> 24));
    out.push_back(static_cast<char>(v >> 16));
    out.push_back(static_cast<char>(v >> 8));
    out.push_back(static_cast<char>(v));
}
inline void put_frame_header(std::string& out, size_t len, uint8_t type, uint8_t flags, uint32_t stream) {
    out.push_back(static_cast<char>(len >> 16));
    out.push_back(static_cast<char>(len >> 8));
    out.push_back(static_cast<char>(len));
    out.push_back(static_cast<char>(type));
    out.push_back(static_cast<char>(flags));
    put32(out, stream & 0x7fffffffu);
}
inline void put_frame(std::string& out, uint8_t type, uint8_t flags, uint32_t stream, const char* p, size_t n) {
    put_frame_header(out, n, type, flags, stream);
    out.append(p, n);
}
inline std::string goaway_frame(uint32_t code, std::string_view debug) {
    std::string p, out;
    put32(p, 0);
    put32(p, code);
    p.append(debug.substr(0, 200));
    put_frame(out, GOAWAY, 0, 0, p.data(), p.size());
    return out;
}

// One request/response exchange: owned by the requesting coroutine (exchange_h2), referenced by the session
// while it is open.
struct Stream {
    uint32_t id = 0;
    Response r;
    const std::string* body = nullptr;  // request body (the caller's; alive until the stream completes)
    size_t body_off = 0;
    bool body_pending = false;  // DATA left to send (waiting for send window)
    int64_t send_window = 0;
    int64_t recv_unacked = 0;   // DATA received since our last stream WINDOW_UPDATE
    double deadline = 0;
    bool got_headers = false, done = false, ok = false, timed_out = false;
    bool retryable = false;  // refused before the server processed it (REFUSED_STREAM, past a GOAWAY, no h2)
    std::string err;
    std::coroutine_handle<> h;
    // a watch: DATA goes to `on_data` as it arrives (once the status is a 2xx) and each DATA frame moves the
    // deadline `idle` seconds on — a silent watch is cancelled as an HTTP/1.1 one's connection is aborted
    std::function<void(std::string_view)> on_data;
    double idle = 0;
    std::exception_ptr failure;  // what `on_data` threw (an in-stream 410, say): the stream is cancelled, and the
                                 // watcher rethrows it — never out of the connection's reader
};

// One HTTP/2 connection.  Everything the client writes goes through `out`, flushed once per loop iteration
// (requests issued together share a send); the reader coroutine parses frames as they arrive.
struct Session {
    Conn c;
    bool connected = false, broken = false, goaway = false;
    bool got_settings = false;  // the server's first frame (must be SETTINGS: else it does not speak HTTP/2)
    bool flush_posted = false, writing = false, reading = false;
    uint32_t next_id = 1;
    uint32_t goaway_last = 0;
    std::unordered_map<uint32_t, Stream*> streams;
    std::deque<Stream*> blocked;  // streams with DATA waiting for send window
    std::string out;
    int64_t conn_send_window = 65535;
    int64_t peer_initial_window = 65535;
    uint32_t peer_max_frame = 16384;
    uint32_t peer_max_streams = 100;  // until the server's SETTINGS say otherwise
    // lowered for good, to 7/8 of the streams in flight, each time the server refuses one (REFUSED_STREAM,
    // ENHANCE_YOUR_CALM): a server whose own count of open streams lags ours (nghttp2 under Node frees a stream
    // some time after its END_STREAM went out) refuses streams opened at or near its limit
    uint32_t stream_cap = 0xffffffffu;
    int64_t conn_recv_unacked = 0;
    hpack::Decoder dec{4096};
    double last_read = 0;  // when bytes last arrived (liveness: Client::sweep PINGs a connection silent too long)
    double ping_sent = 0;  // an unanswered PING's send time, 0 = none
    uint32_t cont_id = 0;  // the stream whose header block continues in CONTINUATION frames
    bool cont_end_stream = false;
    std::string cont_block;

    Session() {
        out.append(kPreface, kPrefaceLen);
        std::string s;
        auto setting = [&s](uint16_t id, uint32_t v) {
            s.push_back(static_cast<char>(id >> 8));
            s.push_back(static_cast<char>(id));
            put32(s, v);
        };
        setting(ENABLE_PUSH, 0);
        setting(INITIAL_WINDOW_SIZE, static_cast<uint32_t>(kStreamWindow));
        setting(MAX_FRAME_SIZE, kOurMaxFrame);
        put_frame(out, SETTINGS, 0, 0, s.data(), s.size());
        std::string wu;
        put32(wu, static_cast<uint32_t>(kConnWindow - 65535));
        put_frame(out, WINDOW_UPDATE, 0, 0, wu.data(), wu.size());
    }
    bool usable() const { return !broken && !goaway && next_id < 0x7ffffff0u; }
    // Until the server's SETTINGS arrive its MAX_CONCURRENT_STREAMS is unknown: one stream goes out with the
    // preface, the rest wait for the SETTINGS (one round trip, once per connection).  Opening up to a guessed
    // 100 instead had nghttp2 (50 streams) reset the excess with ENHANCE_YOUR_CALM on a TLS connection, where
    // the handshake leaves time to queue many (tests/test_http2_interop.py).
    bool has_room() const {
        return usable() && streams.size() < (got_settings ? std::min(peer_max_streams, stream_cap) : 1u);
    }

    void rst(uint32_t id, uint32_t code) {
        std::string p;
        put32(p, code);
        put_frame(out, RST_STREAM, 0, id, p.data(), p.size());
    }
    void ping(double now) {
        ping_sent = now;
        put_frame(out, PING, 0, 0, "ncc-live", 8);
    }
    void window_update(uint32_t id, int64_t n) {
        std::string p;
        put32(p, static_cast<uint32_t>(n));
        put_frame(out, WINDOW_UPDATE, 0, id, p.data(), p.size());
    }
    // Queue as much of a stream's body as the windows allow; true when all of it (and END_STREAM) is queued.
    bool send_body(Stream* s) {
        const std::string& b = *s->body;
        while (s->body_off < b.size()) {
            int64_t room = std::min<int64_t>({s->send_window, conn_send_window, static_cast<int64_t>(peer_max_frame)});
            if (room <= 0) return false;
            size_t n = std::min(b.size() - s->body_off, static_cast<size_t>(room));
            bool last = s->body_off + n == b.size();
            put_frame(out, DATA, last ? END_STREAM : 0, s->id, b.data() + s->body_off, n);
            s->body_off += n;
            s->send_window -= static_cast<int64_t>(n);
            conn_send_window -= static_cast<int64_t>(n);
        }
        return true;
    }
};
using SessionPtr = std::shared_ptr<Session>;

}  // namespace h2
}  // namespace ncc
