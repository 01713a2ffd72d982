// ncc-h2probe — a test tool, never shipped: the C++ executor's HTTP client (native/executor/http.hpp, the same
// header the executor compiles) driven from stdin, so tests can run it against scripted HTTP/2 servers and
// independent implementations (tests/test_http2_errors.py, tests/test_http2_interop.py).
//
//   ncc-h2probe URL HTTP2 [--ca FILE] [--insecure] [--timeout S] [--pool N] [--h2-cap N]
//
// HTTP2 is client-http2's mode (0 off, 1 ALPN on TLS, 2 prior knowledge).  Each stdin line is one step:
//   METHOD PATH [BODY]   a request (issued at once: the steps of a group run concurrently)
//   WATCH PATH           a watch stream, read until it ends (or 5 s of silence); reports the lines read
//   WAIT                 wait for every request of the group so far
//   SLEEP MS
// Output: one JSON line per request as it completes ({"i", "status", "bytes", "ms"} or {"i", "error", "ms"}),
// then {"stats": {...}, "notices": [...]} — the client's HTTP/2 counters and what it would log as Warnings.
#ifdef NCC_COVERAGE
extern "C" void __gcov_dump(void);
#endif
#include <csignal>
#include <cstdio>
#include <iostream>

#include "../executor/http.hpp"

namespace {

using namespace ncc;

struct Step {
    std::string verb, path, body;
};

struct Probe {
    Client* cl = nullptr;
    double t0 = 0;
    int pending = 0;

    static std::string ms(double t) { return std::to_string(static_cast<long long>(t * 1000.0)); }

    Task<void> run_one(int i, Step s) {
        std::string line = "{\"i\":" + std::to_string(i);
        try {
            if (s.verb == "WATCH") {
                size_t n = 0;
                co_await cl->stream(s.path, [&n](std::vector<std::string>& lines) { n += lines.size(); }, 5.0);
                line += ",\"lines\":" + std::to_string(n);
            } else {
                const std::string* body = s.body.empty() ? nullptr : &s.body;
                Response r = co_await cl->request(s.verb, s.path, body);
                line += ",\"status\":" + std::to_string(r.status) + ",\"bytes\":" + std::to_string(r.body.size());
            }
        } catch (const std::exception& e) {
            line += ",\"error\":";
            write_string(line, e.what());
        }
        line += ",\"ms\":" + ms(now_s() - t0) + "}";
        std::printf("%s\n", line.c_str());
        std::fflush(stdout);
        --pending;
    }

    Task<void> main(std::vector<Step> steps) {
        int i = 0;
        for (auto& s : steps) {
            if (s.verb == "WAIT") {
                while (pending > 0) co_await loop().sleep(0.002);
            } else if (s.verb == "SLEEP") {
                co_await loop().sleep(std::atof(s.path.c_str()) / 1000.0);
            } else {
                ++pending;
                spawn(run_one(i++, s), "probe request");
            }
        }
        while (pending > 0) co_await loop().sleep(0.002);
        std::printf("{\"stats\":{\"http2\":%d,\"h2_streams\":%lld,\"h2_refused\":%lld,\"h2_goaways\":%lld,"
                    "\"h2_goaway_errors\":%lld,\"h2_calm\":%lld,\"h2_downgraded\":%d,\"h2_dead\":%lld,\"connections\":%d,\"requests\":%lld,"
                    "\"request_errors\":%lld,\"max_inflight\":%d,\"cap\":%d},\"notices\":[",
                    cl->http2() ? 1 : 0, cl->h2_streams, cl->h2_refused, cl->h2_goaways, cl->h2_goaway_errors,
                    cl->h2_calm, cl->h2_downgraded ? 1 : 0, cl->h2_dead, cl->connections(), cl->requests, cl->request_errors,
                    cl->flow.max_inflight, cl->cap());
        std::printf("%s]}\n", notices.c_str());
        std::fflush(stdout);
        loop().stop();
    }
    std::string notices;
};

}  // namespace

int main(int argc, char** argv) {
    using namespace ncc;
    if (argc < 3) {
        std::fprintf(stderr, "usage: ncc-h2probe URL HTTP2 [--ca FILE] [--insecure] [--timeout S] [--pool N] [--h2-cap N]\n");
        return 2;
    }
    Credentials creds;
    creds.server = argv[1];
    int http2 = std::atoi(argv[2]);
    double timeout = 10;
    int pool = 4;
    int h2_cap = 0;
    for (int k = 3; k < argc; ++k) {
        std::string a = argv[k];
        if (a == "--ca" && k + 1 < argc) {
            std::ifstream f(argv[++k]);
            std::stringstream ss;
            ss << f.rdbuf();
            creds.ca_pem = ss.str();
        } else if (a == "--insecure") {
            creds.insecure = true;
        } else if (a == "--timeout" && k + 1 < argc) {
            timeout = std::atof(argv[++k]);
        } else if (a == "--pool" && k + 1 < argc) {
            pool = std::atoi(argv[++k]);
        } else if (a == "--h2-cap" && k + 1 < argc) {
            h2_cap = std::atoi(argv[++k]);
        }
    }
    std::vector<Step> steps;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        Step s;
        size_t a = line.find(' ');
        s.verb = line.substr(0, a);
        if (a != std::string::npos) {
            size_t b = line.find(' ', a + 1);
            s.path = line.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
            if (b != std::string::npos) s.body = line.substr(b + 1);
        }
        steps.push_back(std::move(s));
    }
    ::signal(SIGPIPE, SIG_IGN);
    Loop lp;
    g_loop = &lp;
    FlowLimits fl;
    fl.adaptive = false;
    fl.h2_cap = h2_cap;
    Client cl(creds, pool, timeout, fl, 1, http2);
    Probe p;
    p.cl = &cl;
    p.t0 = now_s();
    cl.on_notice = [&p](const std::string& m) {
        if (!p.notices.empty()) p.notices += ',';
        write_string(p.notices, m);
    };
    spawn(p.main(std::move(steps)), "probe");
    lp.run();
    std::fflush(stdout);
#ifdef NCC_COVERAGE
    __gcov_dump();  // coverage builds (scripts/cpp_coverage.py): the counters, before skipping the exit handlers
#endif
    std::_Exit(0);  // skip destructors of still-suspended coroutines
}
