// ncc-executor: the native shard executor (native mode's data plane).
//
// One process per shard group and key partition, spawned and supervised by the coordinator
// (ncc/controller/executor.py) exactly like the Python executor (`python -m ncc.executor`) it
// replaces, and speaking the same socketpair protocol (ncc/controller/ipc.py, msgpack frames):
//
//   coordinator -> executor   {"t":"cfg","c":<json>}   shards (resolved credentials) + options
//                             {"t":"s"|"w","k":kind,"l":[raw watch line...]}  watch relay
//                                (ncc/controller/relay.py): the controller cluster's objects; a listing
//                                ("s") may come in chunks, all but the last with "more": true
//                             {"t":"go"}   warm standby acquired the Lease: start the workers
//                             {"t":"resync","p":p,"n":C}   pass again over the keys of coordinator partition p
//                             {"t":"cred","s":shard,"token":...}   refreshed exec credential
//   executor -> coordinator   {"t":"synced","i":n}, {"t":"ready","i":n}, {"t":"status",...} (every 5 s)
//                             {"t":"report","k":key,"u":uid,"g":generation,"r":{shard:error|nil},"w":wrote}
//                             {"t":"need","k":kind,"n":"ns/name"}   a referenced dependent not yet relayed
//
// Reconcile semantics are those of the Python executor role (ncc/controller/reconcile.py,
// `_executor_sync_template`/`_sync_template_to_shard`/`_sync_dependent`, native options), which in
// turn follow the reference's templateSyncHandler / syncSecretsToShard / syncConfigMapsToShard /
// workgroupSyncHandler (controller.go:504-626, 697-845) with native-mode scheduling:
//   * every shard concurrently, failures isolated per shard and reported;
//   * the template first (its shard UID is needed for the dependents' ownerRefs), then all of its
//     Secrets/ConfigMaps concurrently; one PUT per dependent (data + ownerRef together);
//   * rogue shard objects (no ownerRefs) refused; Secret.type changes re-create the shard copy;
//     ConfigMap.binaryData synced; 409 races resolved by re-reading the live object;
//   * queued, retried deletes of templates/workgroups that left the controller cluster; an orphan
//     sweep by the configuration-owner label; shard-side drift repaired from the shard watches.
// The shard caches hold the *server's* answer to every write (never the request body), and a
// per-object memo of "the version our last write produced and the spec/data it was meant to carry"
// keeps a server that rewrites what we send (CRD defaulting, pruning, mutating webhooks) from
// triggering a write loop.
#include <fcntl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <ucontext.h>
#include <pthread.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#if defined(__x86_64__)
#include <x86intrin.h>
#endif
#include <csignal>
#include <functional>
#include <optional>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <unordered_map>
#include <unordered_set>

#ifdef NCC_GPROF
extern "C" void _mcleanup(void);
#endif
#ifdef NCC_COVERAGE
extern "C" void __gcov_dump(void);
#endif

#ifndef NCC_SYSTEM_MALLOC
#include "alloc.hpp"
#endif
#include "http.hpp"
#include "json.hpp"
#include "loop.hpp"
#include "msgpack.hpp"
#include "strmap.hpp"

namespace ncc {

// ------------------------------------------------------------------------------------ constants
constexpr const char* kApiVersion = "science.sneaksanddata.com/v1";
constexpr const char* kTemplateKind = "NexusAlgorithmTemplate";
constexpr const char* kWorkgroupKind = "NexusAlgorithmWorkgroup";
constexpr const char* kFieldManagerQuery = "?fieldManager=nexus-configuration-controller";
// server-side apply (`server-side-apply: true`): the controller is the sole manager of what it applies
constexpr const char* kApplyQuery = "?fieldManager=nexus-configuration-controller&force=true";
constexpr const char* kApplyType = "application/apply-patch+yaml";
constexpr const char* kLabelApp = "science.sneaksanddata.com/controller-app";
constexpr const char* kLabelOwner = "science.sneaksanddata.com/configuration-owner";
constexpr const char* kAgent = "nexus-configuration-controller";

enum Kind { TEMPLATES = 0, WORKGROUPS = 1, SECRETS = 2, CONFIGMAPS = 3 };
constexpr const char* kPlural[] = {"nexusalgorithmtemplates", "nexusalgorithmworkgroups", "secrets", "configmaps"};

// a collection's path, then optionally "/<name>" and a query: built in one reserved string
inline std::string api_path(int k, const std::string& ns, const std::string* name = nullptr,
                            std::string_view query = {}) {
    std::string p;
    p.reserve(64 + ns.size() + (name ? name->size() : 0) + query.size());
    p += k < 2 ? "/apis/science.sneaksanddata.com/v1/namespaces/" : "/api/v1/namespaces/";
    p += ns;
    p += '/';
    p += kPlural[k];
    if (name != nullptr) {
        p += '/';
        p += *name;
    }
    p += query;
    return p;
}
inline std::string base_path(int k, const std::string& ns) { return api_path(k, ns); }
inline std::string item_path(int k, const std::string& ns, const std::string& name) { return api_path(k, ns, &name); }

// crc32 (zlib) of "ns/name": the key -> partition map shared with ncc.controller.executor.key_part
static uint32_t g_crc[256];
static void crc_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        g_crc[i] = c;
    }
}
static uint32_t crc32(std::string_view s) {
    uint32_t c = 0xFFFFFFFFu;
    for (unsigned char ch : s) c = g_crc[(c ^ ch) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

struct Options {
    int index = 0;
    int part = 0, parts = 1;
    std::string ns = "nexus";
    std::string alias = "controller-cluster";
    int workers = 256;
    int pool_size = 256;
    int pipeline_depth = 1;  // requests per connection (HTTP/1.1 pipelining); in flight ≤ pool_size × depth
    int http2 = 1;  // client-http2: 0 off, 1 auto (ALPN h2 on TLS, as client-go), 2 on (prior knowledge on cleartext)
    FlowLimits flow;  // client-side flow control per shard (http.hpp): AIMD limit, client-qps bucket
    double request_timeout = 30;
    double coalesce = 0.002;
    double base_delay = 0.03, max_delay = 5.0;
    double qps = 50, burst = 300;
    double shard_sync_timeout = 10;
    double full_resync = 600;
    bool sync_binary_data = true;
    bool sync_secret_type = true;
    bool orphan_sweep = true;
    bool propagate_workgroup_deletes = true;
    bool server_side_apply = false;  // shard writes as one apply PATCH (create-or-update) instead of POST/PUT
    bool sync_dependent_metadata = false;  // shard Secrets/ConfigMaps carry the source's labels/annotations
    int log_level = 30;  // Python logging levels
    bool gated = false;
};
static Options g_opt;

static void log_at(int level, const char* fmt, ...) {
    if (level < g_opt.log_level) return;
    char msg[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    std::string m;
    write_string(m, msg);
    const char* lv = level >= 40 ? "ERROR" : level >= 30 ? "WARNING" : level >= 20 ? "INFO" : "DEBUG";
    std::fprintf(stderr, "{\"level\":\"%s\",\"logger\":\"ncc.executor.native\",\"executor\":%d,\"message\":%s}\n", lv,
                 g_opt.index, m.c_str());
    std::fflush(stderr);
}
#define LOG_ERROR(...) log_at(40, __VA_ARGS__)
#define LOG_WARN(...) log_at(30, __VA_ARGS__)
#define LOG_INFO(...) log_at(20, __VA_ARGS__)
#define LOG_DEBUG(...) log_at(10, __VA_ARGS__)

// NCC_CPU_REPORT: CPU cycles per phase of the data plane (rdtsc; reported as shares of the process's CPU)
// relay_decode is the part of relay_in spent reading the lines (the rest: stores, indexes, enqueues)
enum Phase { PH_RELAY, PH_SHARD_LINE, PH_RESPONSE, PH_BODY, PH_CHANNEL_IN, PH_RELAY_DECODE, PH_N };
static const char* kPhaseName[PH_N] = {"relay_in", "shard_watch", "write_response", "write_body", "channel_read",
                                       "relay_decode"};
static unsigned long long g_phase[PH_N] = {};
static bool g_phases_on = false;
// phase timer ticks: the TSC on x86_64, the steady clock's nanoseconds elsewhere (aarch64 builds)
static inline unsigned long long ticks() {
#if defined(__x86_64__)
    return __rdtsc();
#else
    return static_cast<unsigned long long>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count());
#endif
}
static long long g_scan_hits = 0, g_scan_misses = 0;  // write responses read without / with a DOM
static long long g_sent_hits = 0;  // response payloads recognised as the text we sent (not fingerprinted)
struct PhaseTimer {
    int ph;
    unsigned long long t0;
    explicit PhaseTimer(int p) : ph(p), t0(g_phases_on ? ticks() : 0) {}
    ~PhaseTimer() {
        if (g_phases_on) g_phase[ph] += ticks() - t0;
    }
};


// A reconcile failure with the Python exception class name the reports carry.
struct NamedError : std::runtime_error {
    std::string kind;
    NamedError(std::string k, const std::string& m) : std::runtime_error(m), kind(std::move(k)) {}
};

// A failed step tagged with the shard object it concerns (a dependent's failure inside a template pass).
struct ObjectError : std::runtime_error {
    std::string cls, kind, name;
    int code;
    ObjectError(std::string c, std::string k, std::string n, int h, const std::string& m)
        : std::runtime_error(m), cls(std::move(c)), kind(std::move(k)), name(std::move(n)), code(h) {}
};

// The typed failure a report carries per shard (ncc/controller/failures.py): class, object kind and name,
// HTTP code, message.
struct Failure {
    std::string cls, kind, name, msg;
    int code = 0;
};

static Failure failure_of(const std::exception_ptr& ep, const std::string& kind, const std::string& name) {
    Failure f{"", kind, name, "", 0};
    try {
        std::rethrow_exception(ep);
    } catch (const ObjectError& e) {
        f = Failure{e.cls, e.kind, e.name, e.what(), e.code};
    } catch (const ApiError& e) {
        f.cls = e.kind();
        f.code = e.code;
        f.msg = e.what();
    } catch (const NamedError& e) {
        f.cls = e.kind;
        f.msg = e.what();
        if (e.kind == "ShardNotReadyError") f.kind.clear(), f.name.clear();
    } catch (const TransportError& e) {
        f.cls = "TransportError";
        f.msg = e.what();
    } catch (const std::exception& e) {
        f.cls = "Error";
        f.msg = e.what();
    } catch (...) {
        f.cls = "Error";
        f.msg = "unknown";
    }
    if (f.msg.size() > 500) f.msg.resize(500);
    return f;
}

static std::string describe(const std::exception_ptr& ep) {
    try {
        std::rethrow_exception(ep);
    } catch (const ObjectError& e) {
        return e.kind + " \"" + e.name + "\": " + e.cls + ": " + e.what();
    } catch (const ApiError& e) {
        return std::string(e.kind()) + ": " + e.what();
    } catch (const NamedError& e) {
        return e.kind + ": " + e.what();
    } catch (const TransportError& e) {
        return std::string("TransportError: ") + e.what();
    } catch (const std::exception& e) {
        return std::string("Error: ") + e.what();
    } catch (...) {
        return "Error: unknown";
    }
}

// ------------------------------------------------------------------------------------ objects
static const Value* meta_of(const Value& o) { return o.get("metadata"); }
static std::string mget(const Value& o, std::string_view k) {
    const Value* m = meta_of(o);
    return m ? std::string(m->sget(k)) : std::string();
}
static long long rv_num(std::string_view rv) {
    if (rv.empty()) return -1;
    long long v = 0;
    for (char c : rv) {
        if (c < '0' || c > '9') return -1;
        v = v * 10 + (c - '0');
    }
    return v;
}
static std::vector<std::string> template_owner_names(const Value& o) {
    std::vector<std::string> out;
    const Value* m = meta_of(o);
    const Value* refs = m ? m->get("ownerReferences") : nullptr;
    if (refs && refs->is_arr())
        for (const auto& r : refs->a)
            if (r.sget("kind") == kTemplateKind) out.emplace_back(r.sget("name"));
    return out;
}
// GetSecretNames() / GetConfigMapNames(): spec.runtimeEnvironment.mappedEnvironmentVariables[*]
// (`spec`: the template's spec, or a view of it holding at least runtimeEnvironment)
static void dependent_names(const Value* spec, std::vector<std::string>& secrets, std::vector<std::string>& cms) {
    const Value* rte = spec ? spec->get("runtimeEnvironment") : nullptr;
    const Value* mev = rte ? rte->get("mappedEnvironmentVariables") : nullptr;
    if (!mev || !mev->is_arr()) return;
    for (const auto& ef : mev->a) {
        if (!ef.is_obj()) continue;
        const Value* s = ef.get("secretRef");
        if (s && !s->is_null()) secrets.emplace_back(s->sget("name"));
        const Value* c = ef.get("configMapRef");
        if (c && !c->is_null()) cms.emplace_back(c->sget("name"));
    }
}

// dependent_names of spec.runtimeEnvironment's raw text; false when the scan cannot read it in place (the
// caller parses)
static bool dependent_names_rte(std::string_view rte, std::vector<std::string>& secrets, std::vector<std::string>& cms) {
    auto is_obj = [](std::string_view v) { return !v.empty() && v[0] == '{'; };
    auto ref = [&](std::string_view r, std::vector<std::string>& out) {
        if (r == "null") return true;
        std::string_view name;
        if (is_obj(r) && !RawCursor(r).members([&](std::string_view k, std::string_view v) {
                if (k == "name" && !v.empty() && v[0] == '"') return RawCursor(v).str(name);
                return true;
            }))
            return false;
        out.emplace_back(name);
        return true;
    };
    if (!is_obj(rte)) return true;
    return RawCursor(rte).members([&](std::string_view k, std::string_view mev) {
        if (k != "mappedEnvironmentVariables" || mev.empty() || mev[0] != '[') return true;
        return RawCursor(mev).elements([&](std::string_view ef) {
            if (!is_obj(ef)) return true;
            return RawCursor(ef).members([&](std::string_view fk, std::string_view fv) {
                if (fk == "secretRef") return ref(fv, secrets);
                if (fk == "configMapRef") return ref(fv, cms);
                return true;
            });
        });
    });
}

// Payload members: kept as raw JSON text (fingerprinted, re-sent verbatim), never decoded into a DOM.
static const std::string_view kPayloadKeys[2][3] = {{"spec", "status", ""}, {"data", "binaryData", "stringData"}};
static const std::string_view* payload_keys(int kind) { return kPayloadKeys[kind < 2 ? 0 : 1]; }
static size_t payload_count(int kind) { return kind < 2 ? 2 : 3; }
static bool raw_null(std::string_view raw) { return raw.empty() || raw == "null"; }

// Controller-side object as relayed by the coordinator (immutable once stored).  The payload the shard
// copy gets (templates/workgroups: spec; Secrets/ConfigMaps: data, binaryData) is kept as its raw JSON.
struct CtlObj {
    std::string spec_raw, data_raw, bin_raw;
    std::string labels_raw, ann_raw;  // dependents with sync_dependent_metadata: metadata.labels/annotations
    std::string ns, name, uid, rv;
    long long generation = 0;
    bool has_generation = false;
    uint64_t fp_spec = 0, fp_data = 0, fp_bin = 0, fp_labels = 0, fp_ann = 0;
    std::string type;  // Secret.type ("" = Opaque)
    std::vector<std::string> secrets, configmaps;  // templates
    std::vector<std::string> owners;               // NexusAlgorithmTemplate owner names (dependents)
    double recv_at = 0;                            // when this version reached the executor (now_s)
};
using CtlPtr = std::shared_ptr<const CtlObj>;

// `obj`: the object without its payload members; `raw`: their text (payload_keys order, empty = absent)
static CtlPtr make_ctl(int kind, const Value& obj, const std::string_view* raw) {
    auto c = std::make_shared<CtlObj>();
    c->recv_at = now_s();
    const Value* m = meta_of(obj);
    if (m) {
        c->ns = std::string(m->sget("namespace"));
        c->name = std::string(m->sget("name"));
        c->uid = std::string(m->sget("uid"));
        c->rv = std::string(m->sget("resourceVersion"));
        const Value* g = m->get("generation");
        if (g && g->t == Value::NUM) {
            c->generation = std::atoll(g->s.c_str());
            c->has_generation = true;
        }
        c->fp_labels = fp_opt(m->get("labels"));
        c->fp_ann = fp_opt(m->get("annotations"));
        if (kind >= 2 && g_opt.sync_dependent_metadata) {
            if (const Value* l = m->get("labels")) c->labels_raw = dumps(*l);
            if (const Value* a = m->get("annotations")) c->ann_raw = dumps(*a);
        }
    }
    if (c->ns.empty()) c->ns = g_opt.ns;
    if (kind < 2) {
        c->spec_raw.assign(raw[0]);
        c->fp_spec = raw[0].empty() ? fingerprint(Value()) : fingerprint_text(raw[0]);
        if (kind == TEMPLATES && !raw_null(raw[0])) {
            static const std::string_view rte[1] = {"runtimeEnvironment"};
            Value view = Parser(raw[0].data(), raw[0].size()).parse_only(rte, 1);
            dependent_names(&view, c->secrets, c->configmaps);
        }
    } else {
        c->data_raw.assign(raw[0]);
        c->bin_raw.assign(raw[1]);
        c->fp_data = fp_opt_text(raw[0]);
        c->fp_bin = fp_opt_text(raw[1]);
        c->type = std::string(obj.sget("type"));
        c->owners = template_owner_names(obj);
    }
    return c;
}

// A relayed watch line straight into a CtlObj without a DOM of its metadata (make_ctl's result for the same
// line); nullptr when the scan meets anything it does not read in place (an escaped string...): the caller
// parses the line instead.  `type` gets the event type.
static CtlPtr ctl_scan(int kind, std::string_view line, std::string& type) {
    PhaseTimer pt(PH_RELAY_DECODE);
    auto c = std::make_shared<CtlObj>();
    c->recv_at = now_s();
    const std::string_view* keys = payload_keys(kind);
    size_t nk = payload_count(kind);
    std::string_view raw[3];
    bool have_obj = false;
    auto meta = [&](std::string_view mk, RawCursor& x) {
        std::string_view mv;
        if (!x.value(mv)) return false;
        std::string_view t;
        if (mk == "name" || mk == "namespace" || mk == "uid" || mk == "resourceVersion") {
            if (!RawCursor(mv).str(t)) return mv == "null";
            (mk == "name" ? c->name : mk == "namespace" ? c->ns : mk == "uid" ? c->uid : c->rv).assign(t);
            return true;
        }
        if (mk == "generation") {
            if (mv.empty() || !(mv[0] == '-' || (mv[0] >= '0' && mv[0] <= '9'))) return mv == "null";
            c->generation = std::atoll(std::string(mv).c_str());
            c->has_generation = true;
            return true;
        }
        if (mk == "labels") {
            c->fp_labels = fp_opt_text(mv);
            if (kind >= 2 && g_opt.sync_dependent_metadata) c->labels_raw.assign(mv);
            return true;
        }
        if (mk == "annotations") {
            c->fp_ann = fp_opt_text(mv);
            if (kind >= 2 && g_opt.sync_dependent_metadata) c->ann_raw.assign(mv);
            return true;
        }
        if (mk == "ownerReferences" && kind >= 2) {
            if (mv == "null") return true;
            return RawCursor(mv).elements([&](std::string_view ref) {
                std::string_view rk, rn;
                bool ok = RawCursor(ref).members([&](std::string_view fk, std::string_view fv) {
                    if (fk == "kind") return RawCursor(fv).str(rk);
                    if (fk == "name") return RawCursor(fv).str(rn);
                    return true;
                });
                if (ok && rk == kTemplateKind) c->owners.emplace_back(rn);
                return ok;
            });
        }
        return true;
    };
    uint64_t fps[3] = {0, 0, 0};
    std::string_view rte;  // templates: spec.runtimeEnvironment
    auto object = [&](std::string_view k, RawCursor& x) {
        if (k == "metadata") return x.walk(meta);
        for (size_t i = 0; i < nk; ++i)
            if (k == keys[i]) {  // fingerprinted as it is skipped: one pass over the payload
                x.ws();
                const char* s = x.p;
                if (kind == TEMPLATES && i == 0 && x.at('{')) {
                    // the spec member by member (fingerprint's object formula), keeping runtimeEnvironment's span
                    uint64_t acc = 0, count = 0;
                    bool spec_ok = x.walk([&](std::string_view sk, RawCursor& y) {
                        y.ws();
                        const char* vs = y.p;
                        const char* end = nullptr;
                        uint64_t vf = Parser(vs, static_cast<size_t>(y.e - vs)).fingerprint_prefix(&end);
                        if (sk == "runtimeEnvironment") rte = std::string_view(vs, static_cast<size_t>(end - vs));
                        acc += Parser::fp_member(Parser::hash_key(sk), vf);
                        ++count;
                        y.p = end;
                        return true;
                    });
                    if (!spec_ok) return false;
                    fps[0] = Parser::fp_object(acc, count);
                    raw[0] = std::string_view(s, static_cast<size_t>(x.p - s));
                    return true;
                }
                const char* end = nullptr;
                fps[i] = Parser(s, static_cast<size_t>(x.e - s)).fingerprint_prefix(&end);
                raw[i] = std::string_view(s, static_cast<size_t>(end - s));
                x.p = end;
                return true;
            }
        std::string_view v;
        if (!x.value(v)) return false;
        if (k == "type" && kind >= 2) {
            std::string_view t;
            if (!RawCursor(v).str(t)) return v == "null";
            c->type.assign(t);
        }
        return true;
    };
    static const uint64_t kNoMap = fp_opt(nullptr);
    c->fp_labels = c->fp_ann = kNoMap;
    auto event = [&](std::string_view k, RawCursor& x) {
        if (k == "object") {
            have_obj = true;
            return x.walk(object);
        }
        std::string_view v;
        if (!x.value(v)) return false;
        if (k == "type") {
            std::string_view t;
            if (!RawCursor(v).str(t)) return false;
            type.assign(t);
        }
        return true;
    };
    bool ok = false;
    try {
        ok = RawCursor(line).walk(event);
    } catch (const JsonError&) {
        return nullptr;  // a malformed payload: the parser path reports it
    }
    if (!ok || !have_obj) return nullptr;
    if (kind == TEMPLATES && !raw_null(raw[0]) && raw[0][0] != '{') return nullptr;  // the parser's error path
    if (c->ns.empty()) c->ns = g_opt.ns;
    if (kind < 2) {
        c->spec_raw.assign(raw[0]);
        c->fp_spec = raw[0].empty() ? fingerprint(Value()) : fps[0];
        if (kind == TEMPLATES && !raw_null(raw[0])) {
            if (!dependent_names_rte(rte, c->secrets, c->configmaps)) return nullptr;
        }
    } else {
        static const uint64_t kNullFp = fingerprint(Value());
        c->data_raw.assign(raw[0]);
        c->bin_raw.assign(raw[1]);
        c->fp_data = raw_is_empty(raw[0]) ? kNullFp : fps[0];
        c->fp_bin = raw_is_empty(raw[1]) ? kNullFp : fps[1];
    }
    return c;
}

// Slim shard-side object: everything but the payloads, plus their fingerprints.
struct ShardObj {
    std::string rest;  // JSON text of the object without spec/status/data/binaryData/stringData (re-sent on PUT)
    std::string ns, name, uid;
    long long rv = -1;
    uint64_t fp_spec = 0, fp_data = 0, fp_bin = 0;
    std::string type;
    bool has_owner_refs = false;
    std::vector<std::pair<std::string, std::string>> template_owners;  // (name, uid) of template owners
    std::vector<std::string> other_owner_names;  // owners of other kinds (template owners are not repeated here)
    // the owner labels this controller puts on its copies (app = kAgent, owner = the alias), as two flags: every
    // cached object carried both strings before, 128 bytes of 240 000 objects at BASELINE config 4
    bool app_label_ours = false, owner_label_ours = false;
    // sync_dependent_metadata: metadata.labels / annotations, parsed from `rest` on first use (meta_in_sync)
    mutable std::unique_ptr<std::pair<Value, Value>> meta_maps;
};
using ShardPtr = std::shared_ptr<const ShardObj>;

// `raw` (optional): the payload members' text when `obj` was parsed without them (parse_split)
static ShardPtr make_shard_obj(int kind, Value obj, const std::string_view* raw = nullptr) {
    auto s = std::make_shared<ShardObj>();
    // managedFields (server-side apply's field ownership, hundreds of bytes per object on a real apiserver)
    // is not kept: an update without it leaves the server's as they are (metadata.managedFields unset = keep)
    if (Value* mm = obj.get("metadata"); mm != nullptr && mm->is_obj()) mm->erase("managedFields");
    const Value* m = meta_of(obj);
    if (m) {
        s->ns = std::string(m->sget("namespace"));
        s->name = std::string(m->sget("name"));
        s->uid = std::string(m->sget("uid"));
        s->rv = rv_num(m->sget("resourceVersion"));
        const Value* refs = m->get("ownerReferences");
        if (refs && refs->is_arr() && !refs->a.empty()) {
            s->has_owner_refs = true;
            for (const auto& r : refs->a) {
                if (r.sget("kind") == kTemplateKind) s->template_owners.emplace_back(r.sget("name"), r.sget("uid"));
                else s->other_owner_names.emplace_back(r.sget("name"));
            }
        }
        const Value* labels = m->get("labels");
        if (labels) {
            s->app_label_ours = labels->sget(kLabelApp) == std::string_view(kAgent);
            s->owner_label_ours = labels->sget(kLabelOwner) == std::string_view(g_opt.alias);
        }
    }
    if (s->ns.empty()) s->ns = g_opt.ns;
    if (raw != nullptr) {  // payloads never decoded
        if (kind < 2) {
            s->fp_spec = raw[0].empty() ? fingerprint(Value()) : fingerprint_text(raw[0]);
        } else {
            s->fp_data = fp_opt_text(raw[0]);
            s->fp_bin = fp_opt_text(raw[1]);
            s->type = std::string(obj.sget("type"));
        }
    } else if (kind < 2) {
        const Value* spec = obj.get("spec");
        s->fp_spec = spec ? fingerprint(*spec) : fingerprint(Value());
        obj.erase("spec");
        obj.erase("status");
    } else {
        s->fp_data = fp_opt(obj.get("data"));
        s->fp_bin = fp_opt(obj.get("binaryData"));
        s->type = std::string(obj.sget("type"));
        obj.erase("data");
        obj.erase("binaryData");
        obj.erase("stringData");
    }
    s->rest = dumps(obj);
    s->rest.shrink_to_fit();  // cached for the object's lifetime: no growth slack (240 000 of them at config 4)
    return s;
}

// metadata fields of a shard object from its raw text (no DOM); false: anything unexpected (an escaped
// string, a non-string where a string belongs) — the caller parses the object instead
// `managed` (optional): set when the metadata has a managedFields member
static bool scan_meta(ShardObj& s, std::string_view meta, bool* managed = nullptr) {
    RawCursor c(meta);
    return c.members([&](std::string_view k, std::string_view v) {
        RawCursor vc(v);
        std::string_view t;
        if (k == "managedFields") {
            if (managed != nullptr) *managed = true;
            return true;
        }
        if (k == "name" || k == "namespace" || k == "uid" || k == "resourceVersion") {
            if (!vc.str(t)) return v == "null";
            if (k == "name") s.name.assign(t);
            else if (k == "namespace") s.ns.assign(t);
            else if (k == "uid") s.uid.assign(t);
            else s.rv = rv_num(t);
            return true;
        }
        if (k == "labels") {
            if (v == "null") return true;
            return vc.members([&](std::string_view lk, std::string_view lv) {
                RawCursor x(lv);
                std::string_view val;
                if (lk == kLabelApp || lk == kLabelOwner) {
                    if (!x.str(val)) return false;
                    if (lk == kLabelApp) s.app_label_ours = val == std::string_view(kAgent);
                    else s.owner_label_ours = val == std::string_view(g_opt.alias);
                }
                return true;
            });
        }
        if (k == "ownerReferences") {
            if (v == "null") return true;
            return vc.elements([&](std::string_view ref) {
                std::string_view rk, rn, ru;
                RawCursor rc(ref);
                bool ok = rc.members([&](std::string_view fk, std::string_view fv) {
                    RawCursor f(fv);
                    if (fk == "kind") return f.str(rk);
                    if (fk == "name") return f.str(rn);
                    if (fk == "uid") return f.str(ru);
                    return true;
                });
                if (!ok) return false;
                s.has_owner_refs = true;
                if (rk == kTemplateKind) s.template_owners.emplace_back(std::string(rn), std::string(ru));
                else s.other_owner_names.emplace_back(rn);
                return true;
            });
        }
        return true;
    });
}

// Payload texts a write sent (spec, or data and binaryData), each with its fingerprint as the controller side
// computed it (raw_is_empty-normalised).  A response payload with the same text has the same fingerprint, so
// the answer to a write is checked with a memcmp instead of fingerprinted again — the apiserver returns the
// payload as sent unless something rewrote it (both sides are compact JSON with the keys in the same order).
struct SentPayload {
    std::string_view raw[2];
    uint64_t fp[2] = {0, 0};
};

// A write response straight into the slim form without a DOM: the non-payload members are copied as text
// (the next PUT's body), the metadata fields read in place, the payloads fingerprinted from their text.
static ShardPtr shard_obj_scan(int kind, std::string_view body, const SentPayload* sent = nullptr) {
    auto s = std::make_shared<ShardObj>();
    const std::string_view* keys = payload_keys(kind);
    size_t nk = payload_count(kind);
    std::string_view raw[3];
    uint64_t fps[3] = {0, 0, 0};
    std::string& rest = s->rest;
    rest.reserve(body.size());
    rest.push_back('{');
    bool first = true;
    bool ok = false;
    auto member = [&](std::string_view k, RawCursor& x) {
        for (size_t i = 0; i < nk; ++i)
            if (k == keys[i]) {  // fingerprinted as it is skipped
                x.ws();
                const char* b = x.p;
                if (sent != nullptr && i < 2) {
                    // a complete object's text as a prefix here is this member's whole value
                    std::string_view h = sent->raw[i];
                    if (h.size() > 1 && h.front() == '{' && static_cast<size_t>(x.e - b) >= h.size() &&
                        std::memcmp(b, h.data(), h.size()) == 0) {
                        fps[i] = sent->fp[i];
                        raw[i] = std::string_view(b, h.size());
                        x.p = b + h.size();
                        ++g_sent_hits;
                        return true;
                    }
                }
                const char* end = nullptr;
                fps[i] = Parser(b, static_cast<size_t>(x.e - b)).fingerprint_prefix(&end);
                raw[i] = std::string_view(b, static_cast<size_t>(end - b));
                x.p = end;
                return true;
            }
        std::string_view v;
        if (!x.value(v)) return false;
        if (!first) rest.push_back(',');
        first = false;
        rest.push_back('"');
        rest.append(k);
        rest.append("\":");
        bool managed = false;
        if (k == "metadata" && !scan_meta(*s, v, &managed)) return false;
        if (managed) {
            // kept without managedFields (see make_shard_obj): the other members copied as text
            rest.push_back('{');
            bool mfirst = true;
            bool mok = RawCursor(v).members([&](std::string_view mk, std::string_view mv) {
                if (mk == "managedFields") return true;
                if (!mfirst) rest.push_back(',');
                mfirst = false;
                rest.push_back('"');
                rest.append(mk);
                rest.append("\":");
                rest.append(mv);
                return true;
            });
            if (!mok) return false;
            rest.push_back('}');
            return true;
        }
        rest.append(v);
        if (k == "metadata") return true;
        if (k == "type" && kind >= 2) {  // Secret.type
            std::string_view t;
            if (!RawCursor(v).str(t)) return v == "null";
            s->type.assign(t);
        }
        return true;
    };
    try {
        ok = RawCursor(body).walk(member);
    } catch (const JsonError&) {
        return nullptr;  // a malformed payload: the parser path reports it
    }
    if (!ok) return nullptr;
    rest.push_back('}');
    rest.shrink_to_fit();  // reserved for the whole body, payloads included: cached, it keeps only its own text
    if (s->ns.empty()) s->ns = g_opt.ns;
    static const uint64_t kNullFp = fingerprint(Value());
    if (kind < 2) {
        s->fp_spec = raw[0].empty() ? kNullFp : fps[0];
    } else {
        s->fp_data = raw_is_empty(raw[0]) ? kNullFp : fps[0];
        s->fp_bin = raw_is_empty(raw[1]) ? kNullFp : fps[1];
    }
    return s;
}

// A write/GET response body straight into the slim form, payloads fingerprinted from their text.
static ShardPtr shard_obj_from_body(int kind, std::string_view body, const SentPayload* sent = nullptr) {
    PhaseTimer pt(PH_RESPONSE);
    if (ShardPtr fast = shard_obj_scan(kind, body, sent)) {
        ++g_scan_hits;
        return fast;
    }
    ++g_scan_misses;
    std::string_view raw[3];
    Value rest = Parser(body.data(), body.size()).parse_split(payload_keys(kind), payload_count(kind), raw);
    return make_shard_obj(kind, std::move(rest), raw);
}

static bool is_ours(const ShardObj& s) { return s.owner_label_ours && s.app_label_ours; }

static std::string key_of(const std::string& ns, const std::string& name) { return ns + "/" + name; }
// The same key in a scratch buffer, for a lookup or an erase that completes before the next call (never stored,
// never held across a co_await): the hot path's finds cost no allocation.
static const std::string& key_tmp(const std::string& ns, std::string_view name) {
    static std::string buf;
    buf.assign(ns);
    buf += '/';
    buf.append(name.data(), name.size());
    return buf;
}
static bool in_partition(const std::string& ns, std::string_view name) {
    return g_opt.parts <= 1 || static_cast<int>(crc32(key_tmp(ns, name)) % g_opt.parts) == g_opt.part;
}

// ------------------------------------------------------------------------------------ channel
static double g_flush_interval = 0.001;  // NCC_REPORT_FLUSH_MS overrides (0: every loop iteration)

class Channel {
public:
    explicit Channel(int fd) : fd_(fd) {
        int fl = fcntl(fd_, F_GETFL);
        fcntl(fd_, F_SETFL, fl | O_NONBLOCK);
        loop().add_fd(fd_);
        spawn(writer(), "channel writer");
    }
    // Queue one message (an encoded msgpack map).  Frames are coalesced per loop iteration, and under load
    // to at most one per `g_flush_interval`: a busy executor reports after every pass, and at 8 shards the
    // coordinator's cost is per frame (a wake-up and a read), not per report.  The first message after a
    // quiet interval still goes out on the next loop iteration.
    void send(std::string msg) {
        pending_.push_back(std::move(msg));
        if (!flush_scheduled_) {
            flush_scheduled_ = true;
            double due = last_flush_ + g_flush_interval;
            if (g_flush_interval <= 0 || now_s() >= due)
                loop().call_soon([this] { flush(); });
            else
                loop().call_at(due, [this] { flush(); });
        }
    }
    bool closed() const { return closed_; }

    // Next batch of messages; empty on EOF.
    Task<std::vector<mp::Obj>> recv() {
        while (true) {
            if (in_.size() - pos_ >= 4) {
                const unsigned char* p = reinterpret_cast<const unsigned char*>(in_.data() + pos_);
                uint32_t n = (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
                bool batch = (n & 0x80000000u) != 0;
                n &= 0x7FFFFFFFu;
                if (in_.size() - pos_ >= 4 + n) {
                    PhaseTimer pt(PH_CHANNEL_IN);
                    mp::Obj o = mp::decode(std::string_view(in_).substr(pos_ + 4, n));  // straight from the buffer
                    pos_ += 4 + n;
                    if (pos_ > (1 << 20)) {
                        in_.erase(0, pos_);
                        pos_ = 0;
                    }
                    std::vector<mp::Obj> out;
                    if (batch && o.t == mp::Obj::ARR)
                        out = std::move(o.a);
                    else
                        out.push_back(std::move(o));
                    co_return out;
                }
            }
            char* buf = read_scratch();
            ssize_t r = ::recv(fd_, buf, kReadScratch, 0);
            if (r > 0) {
                in_.append(buf, static_cast<size_t>(r));
                continue;
            }
            if (r == 0) {
                closed_ = true;
                co_return std::vector<mp::Obj>{};
            }
            if (errno == EAGAIN || errno == EWOULDBLOCK) {
                co_await loop().readable(fd_);
                continue;
            }
            if (errno == EINTR) continue;
            closed_ = true;
            co_return std::vector<mp::Obj>{};
        }
    }

    // Write out everything queued (bounded wait) — used before exiting.
    Task<void> drain(double timeout) {
        flush();
        if (!out_.empty() && !closed_) co_await drained_.wait_for(timeout);
    }

private:
    int fd_;
    bool closed_ = false;
    bool flush_scheduled_ = false;
    double last_flush_ = 0;
    std::vector<std::string> pending_;
    std::string in_;
    size_t pos_ = 0;
    std::string out_;
    Event has_out_;
    Event drained_;  // set while nothing is waiting to be written (or the channel is closed)

    void flush() {
        flush_scheduled_ = false;
        last_flush_ = now_s();
        if (pending_.empty()) return;
        // frame = 4-byte length (top bit: a batch) + one message, or a msgpack array header + the messages,
        // written straight into the output buffer
        bool batch = pending_.size() > 1;
        mp::Encoder e;
        if (batch) e.array(pending_.size());
        size_t size = e.out.size();
        for (const auto& m : pending_) size += m.size();
        uint32_t n = static_cast<uint32_t>(size) | (batch ? 0x80000000u : 0u);
        char hdr[4] = {static_cast<char>(n >> 24), static_cast<char>(n >> 16), static_cast<char>(n >> 8),
                       static_cast<char>(n)};
        // (grow only: GCC 11's reserve() below the capacity reallocates to shrink)
        if (out_.capacity() < out_.size() + 4 + size) out_.reserve(out_.size() + 4 + size);
        out_.append(hdr, 4);
        out_ += e.out;
        for (const auto& m : pending_) out_ += m;
        pending_.clear();
        drained_.clear();
        has_out_.set();
    }

    Task<void> writer() {
        size_t off = 0;
        while (true) {
            if (off >= out_.size()) {
                out_.clear();
                off = 0;
                has_out_.clear();
                drained_.set();
                co_await has_out_.wait();
                continue;
            }
            ssize_t r = ::send(fd_, out_.data() + off, out_.size() - off, MSG_NOSIGNAL);
            if (r > 0) {
                off += static_cast<size_t>(r);
                if (off > (1 << 20)) {
                    out_.erase(0, off);
                    off = 0;
                }
                continue;
            }
            if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
                co_await loop().writable(fd_);
                continue;
            }
            if (r < 0 && errno == EINTR) continue;
            closed_ = true;
            out_.clear();
            drained_.set();
            co_return;
        }
    }
};
static Channel* g_chan = nullptr;

// {"t":"status","i":n,"s":{shard:{plural:[synced, watching, events, relists, last error]}},"q":queued,
// "r":passes,"w":writes,"e":errors} every NCC_STATUS_S (5) seconds: the coordinator's /debug/state shows
// each executor's view of its shards (is the watch up, what failed last).
static void send_status();
static Task<void> status_loop();

static void send_simple(const char* t) {
    mp::Encoder e;
    e.map(2);
    e.str("t");
    e.str(t);
    e.str("i");
    e.integer(g_opt.index);
    g_chan->send(std::move(e.out));
}

// ------------------------------------------------------------------------------------ work queue
// client-go's rate-limiting queue semantics (as ncc/workqueue + native/ncc_native.cpp RateLimitingQueue):
// dedup of queued keys, a key is never processed twice at once (re-added keys wait for `done`),
// delayed adds, per-key exponential failure backoff max'ed with a token bucket for AddRateLimited.
// client-go's workqueue (dirty / processing sets, delayed and rate-limited adds) over one table of per-key
// state: a key costs one node while it has work pending, the FIFO holds pointers to the nodes, and a pass's
// add / get / done are a lookup each — no set of key copies per state.  A node is dropped once its key is
// idle (not dirty, not processing, no delayed add or failure count pending, no timer holding it).
class WorkQueue {
    struct Item {
        bool dirty = false, processing = false;
        double wait_at = 0;  // a delayed add is due then (0: none)
        int timers = 0;      // delayed() coroutines still holding the node
        int failures = 0;
    };
    using Node = std::pair<const std::string, Item>;
    using Items = std::unordered_map<std::string, Item>;

public:
    void add(const std::string& key) {
        if (shutdown_) return;
        mark(node(key));
    }
    void add_after(const std::string& key, double delay) {
        if (shutdown_) return;
        if (delay <= 0) {
            add(key);
            return;
        }
        double at = now_s() + delay;
        Node& n = node(key);
        Item& i = n.second;
        if (i.wait_at > 0 && i.wait_at <= at) return;
        if (i.wait_at == 0) ++waiting_;
        i.wait_at = at;
        ++i.timers;
        spawn(delayed(&n, at), "delayed add");
    }
    void add_rate_limited(const std::string& key) {
        int f = node(key).second.failures++;
        double exp_delay = std::min(g_opt.base_delay * std::pow(2.0, f), g_opt.max_delay);
        double now = now_s();
        tokens_ = std::min(g_opt.burst, tokens_ + (now - last_) * g_opt.qps);
        last_ = now;
        tokens_ -= 1.0;
        double bucket = tokens_ < 0 ? -tokens_ / g_opt.qps : 0.0;
        add_after(key, std::max(exp_delay, bucket));
    }
    void forget(const std::string& key) {
        auto it = items_.find(key);
        if (it == items_.end()) return;
        it->second.failures = 0;
        drop_if_idle(it);
    }
    // (`key` may be the node's own key, as get() hands out: it is not used after the node is dropped)
    void done(const std::string& key) {
        auto it = items_.find(key);
        if (it == items_.end()) return;
        Item& i = it->second;
        if (i.processing) {
            i.processing = false;
            --processing_;
        }
        if (i.dirty) {
            queue_.push_back(&*it);
            wake();
            return;
        }
        drop_if_idle(it);
    }
    size_t length() const { return queue_.size(); }
    size_t load() const { return queue_.size() + processing_ + waiting_; }  // keys with work pending
    // a pass over `key` is pending (added while queued or processing): the next one will see the latest state
    bool dirty(const std::string& key) const {
        auto it = items_.find(key);
        return it != items_.end() && it->second.dirty && !shutdown_;
    }
    void shutdown() {
        shutdown_ = true;
        for (auto h : getters_) loop().post(h);
        getters_.clear();
    }

    struct GetAwait {
        WorkQueue* q;
        bool await_ready() { return !q->queue_.empty() || q->shutdown_; }
        void await_suspend(std::coroutine_handle<> h) { q->getters_.push_back(h); }
        void await_resume() {}
    };
    // Next key to process (nullptr after shutdown).  The key lives in the queue until done() on it.
    Task<const std::string*> get() {
        while (queue_.empty() && !shutdown_) co_await GetAwait{this};
        if (shutdown_) co_return nullptr;
        Node* n = queue_.front();
        queue_.pop_front();
        n->second.processing = true;
        ++processing_;
        n->second.dirty = false;
        co_return &n->first;
    }

private:
    Items items_;
    std::deque<Node*> queue_;  // dirty keys not being processed, in order (node pointers stay valid)
    size_t processing_ = 0, waiting_ = 0;
    std::deque<std::coroutine_handle<>> getters_;
    double tokens_ = 300, last_ = now_s();
    bool shutdown_ = false;

    Node& node(const std::string& key) { return *items_.try_emplace(key).first; }
    void mark(Node& n) {
        if (n.second.dirty) return;
        n.second.dirty = true;
        if (n.second.processing) return;
        queue_.push_back(&n);
        wake();
    }
    void drop_if_idle(Items::iterator it) {
        const Item& i = it->second;
        if (!i.dirty && !i.processing && i.wait_at == 0 && i.timers == 0 && i.failures == 0) items_.erase(it);
    }
    void wake() {
        if (!getters_.empty()) {
            loop().post(getters_.front());
            getters_.pop_front();
        }
    }
    Task<void> delayed(Node* n, double at) {
        co_await loop().sleep(std::max(0.0, at - now_s()));
        Item& i = n->second;
        --i.timers;
        if (i.wait_at == 0 || i.wait_at > at + 1e-9) {  // superseded by an earlier/later add
            drop_if_idle(items_.find(n->first));
            co_return;
        }
        i.wait_at = 0;
        --waiting_;
        if (shutdown_) co_return;
        mark(*n);
    }
};

// ------------------------------------------------------------------------------------ state
struct Shard;
struct Executor;
static Executor* g_ex = nullptr;

struct Informer {
    Shard* shard = nullptr;
    int kind = 0;
    StrMap<ShardPtr> store;
    bool synced = false;
    bool watching = false;   // a watch request is open (status reports)
    std::string last_error;  // the last list/watch failure, "" once a watch succeeds again
    Event synced_ev;
    std::string last_rv;
    long long events = 0, relists = 0, echoes = 0, foreign = 0;
};

struct Memo {  // the version our last write produced, and the fingerprints it was meant to carry
    long long rv = -1;
    uint64_t fp_a = 0, fp_b = 0;
};

struct Shard {
    std::string name;
    std::unique_ptr<Client> client;
    Informer inf[4];
    StrMap<Memo> memo[4];
    Event answering;  // set when a write or read was answered (< 500): reflectors in an outage backoff retry
    bool synced() const {
        for (const auto& i : inf)
            if (!i.synced) return false;
        return true;
    }
    ShardPtr get(int k, const std::string& key) const {
        auto it = inf[k].store.find(key);
        return it == inf[k].store.end() ? nullptr : it->second;
    }
    const ShardObj* find(int k, const std::string& key) const {
        auto it = inf[k].store.find(key);
        return it == inf[k].store.end() ? nullptr : it->second.get();
    }
};

static double kDependentHold = 5.0;  // NCC_DEPENDENT_HOLD overrides
static constexpr double kMaxReportSkip = 0.25;  // a key skips reports of superseded passes for at most this long


// NCC_TRACE_STAGES=<dir>: wall-clock times of every relayed controller object received ("r", kind) and of
// every key a worker dequeues ("q"), written to <dir>/executor-<index>.tsv on exit (bench.py --stages)
struct TraceRec {
    char what;
    int kind;
    std::string key;
    long long t_ns;
};
static std::vector<TraceRec>* g_trace = nullptr;
static long long wall_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
}
static void trace(char what, int kind, const std::string& key) {
    if (g_trace != nullptr) g_trace->push_back(TraceRec{what, kind, key, wall_ns()});
}
static void dump_trace() {
    const char* dir = std::getenv("NCC_TRACE_STAGES");
    if (g_trace == nullptr || dir == nullptr) return;
    ::mkdir(dir, 0755);
    std::string path = std::string(dir) + "/executor-" + std::to_string(g_opt.index) + "-" + std::to_string(getpid()) +
                       ".tsv";
    FILE* f = std::fopen(path.c_str(), "w");
    if (f == nullptr) return;
    for (const auto& r : *g_trace) std::fprintf(f, "%c\t%d\t%s\t%lld\n", r.what, r.kind, r.key.c_str(), r.t_ns);
    std::fclose(f);
}
// NCC_SAMPLE_PROFILE=<dir>: a sampling CPU profiler.  SIGPROF fires every `NCC_SAMPLE_US` (default 500) µs of
// the process's CPU time and records the interrupted instruction's address; on exit the process's
// executable mappings and the addresses go to <dir>/executor-<index>-<pid>.samples
// (scripts/executor_profile.py maps them to functions of the executable and its shared libraries, inlined
// ones included, with addr2line).  Unlike -pg it needs no rebuild and attributes time in coroutine frames and
// inlined code correctly; time in the kernel lands on the libc system-call wrapper that entered it.
// Each sample also keeps the word at the top of the stack: in a frameless leaf (memcpy, a system-call
// wrapper) that is the return address, i.e. the caller.
// Each sample: the interrupted pc, the word on top of the stack (a leaf's return address: who called a libc
// routine), and — in the frame-pointer build (native/build.py profile flavor, NCC_FRAME_POINTERS) — the return
// addresses of up to kWalk frames up the rbp chain, 0 past its end.  Without frame pointers rbp is an ordinary
// register, so the release build records no chain.
static constexpr size_t kMaxSamples = 1 << 18;
static constexpr size_t kWalk = 6;
static constexpr size_t kWords = 2 + kWalk;
static uintptr_t* g_samples = nullptr;
static volatile size_t g_nsamples = 0;
static uintptr_t g_stack_lo = 0, g_stack_hi = 0;  // the main thread's stack: the only memory the walk reads
#if defined(__x86_64__)
static void on_sigprof(int, siginfo_t*, void* ucv) {
    auto* uc = static_cast<ucontext_t*>(ucv);
    size_t n = g_nsamples;
    if (n < kMaxSamples) {
        uintptr_t* out = g_samples + kWords * n;
        out[0] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
        out[1] = *reinterpret_cast<const uintptr_t*>(uc->uc_mcontext.gregs[REG_RSP]);
        for (size_t k = 0; k < kWalk; ++k) out[2 + k] = 0;
#ifdef NCC_FRAME_POINTERS
        uintptr_t fp = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RBP]);
        for (size_t k = 0; k < kWalk; ++k) {
            if (fp < g_stack_lo || fp + 16 > g_stack_hi || (fp & 7) != 0) break;
            const uintptr_t* f = reinterpret_cast<const uintptr_t*>(fp);
            out[2 + k] = f[1];
            if (f[0] <= fp) break;  // the chain only goes up the stack
            fp = f[0];
        }
#endif
        g_nsamples = n + 1;
    }
}
#endif
static void start_sampling() {
    if (std::getenv("NCC_SAMPLE_PROFILE") == nullptr) return;
#if !defined(__x86_64__)
    LOG_WARN("NCC_SAMPLE_PROFILE: the sampling profiler reads x86_64 registers; not available on this build");
    return;
#else
    g_samples = new uintptr_t[kWords * kMaxSamples];
    pthread_attr_t attr;
    if (pthread_getattr_np(pthread_self(), &attr) == 0) {
        void* lo = nullptr;
        size_t size = 0;
        if (pthread_attr_getstack(&attr, &lo, &size) == 0) {
            g_stack_lo = reinterpret_cast<uintptr_t>(lo);
            g_stack_hi = g_stack_lo + size;
        }
        pthread_attr_destroy(&attr);
    }
    struct sigaction sa {};
    sa.sa_sigaction = on_sigprof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGPROF, &sa, nullptr);
    long us = 500;
    if (const char* v = std::getenv("NCC_SAMPLE_US")) us = std::max(50L, std::atol(v));
    struct itimerval it {};
    it.it_interval.tv_sec = us / 1000000;
    it.it_interval.tv_usec = us % 1000000;
    it.it_value = it.it_interval;
    setitimer(ITIMER_PROF, &it, nullptr);
#endif
}
static void dump_samples() {
    const char* dir = std::getenv("NCC_SAMPLE_PROFILE");
    if (g_samples == nullptr || dir == nullptr) return;
    struct itimerval off {};
    setitimer(ITIMER_PROF, &off, nullptr);
    ::mkdir(dir, 0755);
    std::string path = std::string(dir) + "/executor-" + std::to_string(g_opt.index) + "-" + std::to_string(getpid()) +
                       ".samples";
    FILE* f = std::fopen(path.c_str(), "w");
    if (f == nullptr) return;
    if (FILE* maps = std::fopen("/proc/self/maps", "r")) {  // "# map <start>-<end> <perms> <offset> ... <path>"
        char line[4096];
        while (std::fgets(line, sizeof line, maps) != nullptr)
            if (std::strstr(line, " r-xp ") != nullptr) std::fprintf(f, "# map %s", line);
        std::fclose(maps);
    }
    for (size_t i = 0; i < g_nsamples; ++i) {
        const uintptr_t* w = g_samples + kWords * i;
        std::fprintf(f, "%zx %zx", static_cast<size_t>(w[0]), static_cast<size_t>(w[1]));
        for (size_t k = 0; k < kWalk && w[2 + k] != 0; ++k) std::fprintf(f, " %zx", static_cast<size_t>(w[2 + k]));
        std::fputc('\n', f);
    }
    std::fclose(f);
}

// enqueues by cause (NCC_CPU_REPORT diagnostics): template/workgroup event, dependent event, shard-side
// template drift, shard-side dependent drift, failure retry, orphan sweep, full resync, delete
enum EnqCause { ENQ_OBJECT, ENQ_DEPENDENT, ENQ_SHARD_OBJECT, ENQ_SHARD_DEPENDENT, ENQ_RETRY, ENQ_SWEEP, ENQ_RESYNC,
                ENQ_DELETE, ENQ_N };
static long long g_enq[ENQ_N] = {};  // coalesce windows a dependent-triggered pass waits in a burst

struct PassState {
    bool wrote = false;
};

static void on_shard_event(Shard& sh, int kind, const ShardPtr& old, const ShardPtr& cur, bool deleted);
static void on_ctl_event(int kind, const CtlPtr& old, const CtlPtr& cur, bool deleted);

struct Executor {
    std::vector<std::unique_ptr<Shard>> shards;
    StrMap<CtlPtr> ctl[4];
    bool ctl_synced[4] = {false, false, false, false};
    Event ctl_synced_ev;
    StrMap<std::set<std::string>> refs[2];  // dep key -> template keys (secret, configmap)
    std::unordered_set<std::string> pending_deletes[2];              // templates, workgroups
    WorkQueue queue;
    Event gate;
    Event stop_ev;
    std::unordered_map<std::string, double> needed;  // dependent keys asked from the coordinator
    std::vector<CtlPtr> partial_snapshot[4];          // chunks of a listing still arriving (per kind)
    long long stats_reconciles = 0, stats_errors = 0, stats_writes = 0, stats_reports_skipped = 0;
    std::unordered_set<std::string> carry_wrote;  // keys whose unreported (superseded) pass wrote
    std::unordered_map<std::string, double> skipping_since;  // keys whose reports are being skipped: since when

    CtlPtr cget(int k, const std::string& key) const {
        auto it = ctl[k].find(key);
        return it == ctl[k].end() ? nullptr : it->second;
    }
    // the same without taking a reference (a check that completes before the cache changes)
    const CtlObj* cfind(int k, const std::string& key) const {
        auto it = ctl[k].find(key);
        return it == ctl[k].end() ? nullptr : it->second.get();
    }

    // Event-driven enqueue.  Inside a burst — a run of more than kBurstMin events, each less than one
    // coalesce window after the previous, while at least kBurstMin keys have work pending (back-to-back
    // small batches make a run but no load) — the key is parked for the window, so a template and its
    // Secret/ConfigMap changing together reconcile once.  An isolated change, or a small batch, goes straight
    // to the workers and pays no coalescing delay (an extra pass there costs nothing that matters).
    // A pass triggered by a dependent is parked `hold` windows: users roll a new configuration out
    // dependents first, and the template's own event (relayed over another watch stream, so often a
    // loop iteration later) pulls the pass in to one window — one pass instead of two.
    static constexpr int kBurstMin = 32;
    double last_event = -1e18;
    int run_len = 0;
    void enqueue(int kind, const std::string& ns, std::string_view name, double hold = 1.0) {
        if (!in_partition(ns, name)) return;
        static std::string key;  // the queue copies it only when the key has no pending work yet
        key.assign(kind == TEMPLATES ? "template/" : "workgroup/");
        key += ns;
        key += '/';
        key += name;
        double now = now_s();
        run_len = now - last_event < g_opt.coalesce ? run_len + 1 : 1;
        bool burst = run_len > kBurstMin && queue.load() >= static_cast<size_t>(kBurstMin);
        last_event = now;
        if (g_opt.coalesce > 0 && burst)
            queue.add_after(key, g_opt.coalesce * hold);
        else
            queue.add(key);
    }
};

// ------------------------------------------------------------------------------------ controller side
static void index_template(const CtlPtr& old, const CtlPtr& cur) {
    Executor& ex = *g_ex;
    const CtlObj* o = old.get();
    const CtlObj* c = cur.get();
    const CtlObj* any = c ? c : o;
    std::string tkey = key_of(any->ns, any->name);
    for (int i = 0; i < 2; ++i) {
        const std::vector<std::string>* ov = o ? (i == 0 ? &o->secrets : &o->configmaps) : nullptr;
        const std::vector<std::string>* nv = c ? (i == 0 ? &c->secrets : &c->configmaps) : nullptr;
        if (ov && nv && *ov == *nv) continue;
        if (ov)
            for (const auto& n : *ov) {
                auto it = ex.refs[i].find(key_tmp(any->ns, n));
                if (it != ex.refs[i].end()) {
                    it->second.erase(tkey);
                    if (it->second.empty()) ex.refs[i].erase(it);
                }
            }
        if (nv)
            for (const auto& n : *nv) ex.refs[i][key_of(any->ns, n)].insert(tkey);
    }
}

// Apply one relayed controller-side event.
static void ctl_apply(int kind, const std::string& type, CtlPtr cur) {
    Executor& ex = *g_ex;
    auto& store = ex.ctl[kind];
    auto it = store.find(key_tmp(cur->ns, cur->name));
    CtlPtr old = it == store.end() ? nullptr : it->second;
    if (type == "DELETED") {
        if (it != store.end()) store.erase(it);
        if (kind == TEMPLATES) index_template(old ? old : cur, nullptr);
        on_ctl_event(kind, old ? old : cur, nullptr, true);
        return;
    }
    if (it != store.end())
        it->second = cur;
    else
        it = store.emplace(key_of(cur->ns, cur->name), cur).first;
    const std::string& key = it->first;  // (a node's key stays put: index_template below touches only ex.refs)
    trace('r', kind, key);
    if (kind == TEMPLATES) index_template(old, cur);
    if (kind >= 2) ex.needed.erase(key);
    on_ctl_event(kind, old, cur, false);
}

static void ctl_snapshot(int kind, std::vector<CtlPtr> objs) {
    Executor& ex = *g_ex;
    auto& store = ex.ctl[kind];
    StrMap<CtlPtr> fresh;
    for (auto& c : objs) fresh[key_of(c->ns, c->name)] = c;
    bool was_synced = ex.ctl_synced[kind];
    std::vector<std::pair<CtlPtr, CtlPtr>> changes;  // (old, new); new null = deleted
    for (auto& kv : fresh) {
        auto it = store.find(kv.first);
        changes.emplace_back(it == store.end() ? nullptr : it->second, kv.second);
    }
    for (auto& kv : store)
        if (!fresh.count(kv.first)) changes.emplace_back(kv.second, nullptr);
    store = std::move(fresh);
    if (kind == TEMPLATES) {
        ex.refs[0].clear();
        ex.refs[1].clear();
        for (auto& kv : store) index_template(nullptr, kv.second);
    }
    ex.ctl_synced[kind] = true;
    for (auto& ch : changes) {
        if (ch.second)
            on_ctl_event(kind, ch.first, ch.second, false);
        else if (was_synced)
            on_ctl_event(kind, ch.first, nullptr, true);
    }
    if (ex.ctl_synced[0] && ex.ctl_synced[1] && ex.ctl_synced[2] && ex.ctl_synced[3]) ex.ctl_synced_ev.set();
}

// templates referencing the dependent, then template owners that no longer reference it
// (handleObject's ownerRef walk, controller.go:206-223; native: reverse index first)
// The hold of a pass a dependent's event triggers: `kDependentHold` windows wait for the template's own event
// (users roll dependents out first), unless that event already came (the template changed within the
// hold): then the dependent is the follower and waits one window like any event in a burst.
static double dependent_hold(const std::string& tkey) {
    const CtlObj* t = g_ex->cfind(TEMPLATES, tkey);
    return t != nullptr && now_s() - t->recv_at < g_opt.coalesce * kDependentHold ? 1.0 : kDependentHold;
}

static void on_dependent(int kind, const CtlObj& obj) {
    Executor& ex = *g_ex;
    auto& idx = ex.refs[kind == SECRETS ? 0 : 1];
    auto it = idx.find(key_tmp(obj.ns, obj.name));
    if (it != idx.end()) {
        for (const auto& tkey : it->second) {
            std::string_view tname = std::string_view(tkey).substr(tkey.find('/') + 1);
            ++g_enq[ENQ_DEPENDENT];
            ex.enqueue(TEMPLATES, obj.ns, tname, dependent_hold(tkey));
        }
    }
    for (const auto& owner : obj.owners) {
        if (it != idx.end() && it->second.count(key_tmp(obj.ns, owner)) > 0) continue;  // enqueued above
        std::string tkey = key_of(obj.ns, owner);
        if (!ex.cget(TEMPLATES, tkey)) return;  // stops at the first orphaned owner
        ++g_enq[ENQ_DEPENDENT];
        ex.enqueue(TEMPLATES, obj.ns, owner, dependent_hold(tkey));
    }
}

static void on_ctl_event(int kind, const CtlPtr& old, const CtlPtr& cur, bool deleted) {
    Executor& ex = *g_ex;
    if (kind == TEMPLATES || kind == WORKGROUPS) {
        const CtlObj& o = deleted ? *old : *cur;
        if (deleted) {
            if (kind == TEMPLATES || g_opt.propagate_workgroup_deletes) {
                if (in_partition(o.ns, o.name)) ex.pending_deletes[kind].insert(key_of(o.ns, o.name));
                ++g_enq[ENQ_DELETE];
                ex.enqueue(kind, o.ns, o.name);
            }
            return;
        }
        if (old) {  // generation filter: skip resyncs and status-only changes (our coordinator's writes)
            if (old->rv == cur->rv) return;
            if (old->has_generation && old->generation == cur->generation && old->fp_labels == cur->fp_labels &&
                old->fp_ann == cur->fp_ann && old->fp_spec == cur->fp_spec)
                return;
        }
        ++g_enq[ENQ_OBJECT];
        ex.enqueue(kind, o.ns, o.name);
        return;
    }
    if (deleted || !old) {
        on_dependent(kind, deleted ? *old : *cur);
        return;
    }
    if (old->rv == cur->rv) return;
    if (old->fp_data == cur->fp_data && old->fp_bin == cur->fp_bin && old->type == cur->type &&
        old->owners == cur->owners &&
        (!g_opt.sync_dependent_metadata || (old->fp_labels == cur->fp_labels && old->fp_ann == cur->fp_ann)))
        return;  // e.g. the coordinator's adoption write: ownerRef UIDs changed, payload did not
    on_dependent(kind, *cur);
}

// ------------------------------------------------------------------------------------ shard side
static bool spec_in_sync(const Shard& sh, int kind, const ShardObj& so, uint64_t desired) {
    if (so.fp_spec == desired) return true;
    auto it = sh.memo[kind].find(key_tmp(so.ns, so.name));
    // the server rewrote what we sent (defaulting / pruning / a mutating webhook): the version our own
    // write produced counts as in sync, or every pass would write again
    return it != sh.memo[kind].end() && it->second.rv == so.rv && it->second.fp_a == desired;
}
static bool data_in_sync(const Shard& sh, int kind, const ShardObj& so, const CtlObj& src) {
    bool with_bin = kind == CONFIGMAPS && g_opt.sync_binary_data;
    if (so.fp_data == src.fp_data && (!with_bin || so.fp_bin == src.fp_bin)) return true;
    auto it = sh.memo[kind].find(key_tmp(so.ns, so.name));
    return it != sh.memo[kind].end() && it->second.rv == so.rv && it->second.fp_a == src.fp_data &&
           (!with_bin || it->second.fp_b == src.fp_bin);
}

// sync_dependent_metadata (Shard.dependent_metadata): the labels and annotations a shard copy of `src`
// carries — the source's labels under the owner labels (they mark the copy as ours), its annotations without
// kubectl's last-applied record, and kSyncedMetadata naming the source's keys.  A copy is in sync when it
// carries all of them (keys others added on the shard are left alone); a key removed at the source changes
// kSyncedMetadata, and the next write drops the keys it named before and the source no longer has.
constexpr const char* kLastApplied = "kubectl.kubernetes.io/last-applied-configuration";
constexpr const char* kSyncedMetadata = "science.sneaksanddata.com/synced-metadata";
static Value owner_labels();
static std::pair<Value, Value> desired_metadata(const CtlObj& src) {
    Value labels = Value::object(), ann = Value::object();
    if (!raw_null(src.labels_raw)) {
        Value l = parse(src.labels_raw);
        if (l.is_obj()) labels = std::move(l);
    }
    std::vector<std::string> lkeys, akeys;
    Value owner = owner_labels();
    for (const auto& kv : labels.o)
        if (owner.get(kv.first) == nullptr) lkeys.push_back(kv.first);
    for (auto& kv : owner.o) labels.set(kv.first, std::move(kv.second));
    if (!raw_null(src.ann_raw)) {
        Value a = parse(src.ann_raw);
        if (a.is_obj()) {
            a.erase(kLastApplied);
            a.erase(kSyncedMetadata);
            ann = std::move(a);
        }
    }
    for (const auto& kv : ann.o) akeys.push_back(kv.first);
    std::sort(lkeys.begin(), lkeys.end());
    std::sort(akeys.begin(), akeys.end());
    std::string v = "labels=";
    for (size_t i = 0; i < lkeys.size(); ++i) v += (i ? "," : "") + lkeys[i];
    v += ";annotations=";
    for (size_t i = 0; i < akeys.size(); ++i) v += (i ? "," : "") + akeys[i];
    ann.set(kSyncedMetadata, Value::str(v));
    return {std::move(labels), std::move(ann)};
}
static bool carries(const Value* have, const Value& want) {
    for (const auto& kv : want.o) {
        const Value* h = have != nullptr && have->is_obj() ? have->get(kv.first) : nullptr;
        if (h == nullptr || fingerprint(*h) != fingerprint(kv.second)) return false;
    }
    return true;
}
static bool meta_in_sync(const ShardObj& so, const CtlObj& src) {
    if (!so.meta_maps) {
        auto maps = std::make_unique<std::pair<Value, Value>>();
        Value rest = parse(so.rest);
        if (Value* m = rest.get("metadata")) {
            if (Value* l = m->get("labels")) maps->first = std::move(*l);
            if (Value* a = m->get("annotations")) maps->second = std::move(*a);
        }
        so.meta_maps = std::move(maps);
    }
    auto [labels, ann] = desired_metadata(src);
    return carries(&so.meta_maps->first, labels) && carries(&so.meta_maps->second, ann);
}
// the keys a kSyncedMetadata value names for `what` ("labels" / "annotations")
static std::vector<std::string> synced_keys(const Value* ann, std::string_view what) {
    std::vector<std::string> out;
    const Value* v = ann != nullptr && ann->is_obj() ? ann->get(kSyncedMetadata) : nullptr;
    if (v == nullptr || !v->is_str()) return out;
    std::string_view s = v->s;
    while (!s.empty()) {
        size_t semi = s.find(';');
        std::string_view part(s.data(), semi == std::string_view::npos ? s.size() : semi);
        const void* eqp = part.empty() ? nullptr : std::memchr(part.data(), '=', part.size());
        size_t eq = eqp == nullptr ? std::string_view::npos : static_cast<size_t>(static_cast<const char*>(eqp) - part.data());
        if (eq != std::string_view::npos && part.substr(0, eq) == what) {
            std::string_view keys = part.substr(eq + 1);
            size_t start = 0;
            while (start < keys.size()) {
                size_t comma = keys.find(',', start);
                size_t end = comma == std::string_view::npos ? keys.size() : comma;
                if (end > start) out.emplace_back(keys.data() + start, end - start);
                start = end + 1;
            }
        }
        if (semi == std::string_view::npos) break;
        s.remove_prefix(semi + 1);
    }
    return out;
}
// metadata `m` of a copy about to be written: keys synced before and gone at the source dropped, the
// desired ones set, the rest kept (merge_synced_metadata)
static void set_metadata(Value& m, const CtlObj& src) {
    auto [labels, ann] = desired_metadata(src);
    const Value* have_ann = m.get("annotations");
    std::vector<std::string> prev_l = synced_keys(have_ann, "labels"), prev_a = synced_keys(have_ann, "annotations");
    auto merge = [&](const char* k, Value& want, const std::vector<std::string>& prev) {
        Value out = Value::object();
        if (const Value* have = m.get(k); have != nullptr && have->is_obj())
            for (const auto& kv : have->o)
                if (std::find(prev.begin(), prev.end(), kv.first) == prev.end()) out.set(kv.first, kv.second);
        for (auto& kv : want.o) out.set(kv.first, std::move(kv.second));
        m.set(k, std::move(out));
    };
    merge("labels", labels, prev_l);
    merge("annotations", ann, prev_a);
}

// A shard Secret/ConfigMap in sync, unless a referencing template whose shard copy exists lost its ownerRef on
// it (another writer replaced the list: two creating applies at once, a user's edit): that template's pass
// puts it back — or shard GC could delete the copy with the other owners.
static void repair_lost_owners(Shard& sh, int kind, const ShardObj& o) {
    Executor& ex = *g_ex;
    auto& idx = ex.refs[kind == SECRETS ? 0 : 1];
    auto it = idx.find(key_tmp(o.ns, o.name));
    if (it == idx.end()) return;
    for (const auto& tkey : it->second) {
        const ShardObj* st = sh.find(TEMPLATES, tkey);
        if (st == nullptr) continue;
        bool owned = false;
        for (const auto& p : o.template_owners)
            if (p.second == st->uid) owned = true;
        if (!owned) {
            ++g_enq[ENQ_SHARD_DEPENDENT];
            ex.enqueue(TEMPLATES, o.ns, tkey.substr(tkey.find('/') + 1));
        }
    }
}

static void on_shard_event(Shard& sh, int kind, const ShardPtr& old, const ShardPtr& cur, bool deleted) {
    Executor& ex = *g_ex;
    if (!deleted && !old) return;  // adds are not drift (the reference only repairs on update/delete)
    const ShardObj& o = deleted ? *old : *cur;
    if (kind == TEMPLATES || kind == WORKGROUPS) {
        const CtlObj* c = ex.cfind(kind, key_tmp(o.ns, o.name));
        if (c == nullptr) return;
        if (deleted || !spec_in_sync(sh, kind, o, c->fp_spec)) {
            ++g_enq[ENQ_SHARD_OBJECT];
            ex.enqueue(kind, o.ns, o.name);
        }
        return;
    }
    const CtlObj* src = ex.cfind(kind, key_tmp(o.ns, o.name));
    if (src == nullptr) return;
    if (!deleted && data_in_sync(sh, kind, o, *src) && (!g_opt.sync_dependent_metadata || meta_in_sync(o, *src))) {
        repair_lost_owners(sh, kind, o);
        return;
    }
    std::vector<std::string> owners;
    for (const auto& p : o.template_owners) owners.push_back(p.first);
    if (owners.empty()) owners = src->owners;
    for (const auto& n : owners)
        if (ex.cget(TEMPLATES, key_tmp(o.ns, n))) {
            ++g_enq[ENQ_SHARD_DEPENDENT];
            ex.enqueue(TEMPLATES, o.ns, n);
        }
}

// Keep a shard object in this executor's cache?  Templates/workgroups of our key partition; dependents
// without owners or with an owner template in our partition (others' are dropped, as in the Python
// executor's partition filters).
static bool wanted(int kind, const ShardObj& s) {
    if (g_opt.parts <= 1) return true;
    if (kind < 2) return in_partition(s.ns, s.name);
    if (s.template_owners.empty() && s.other_owner_names.empty()) return true;
    for (const auto& o : s.template_owners)
        if (in_partition(s.ns, o.first)) return true;
    for (const auto& n : s.other_owner_names)
        if (in_partition(s.ns, n)) return true;
    return false;
}

// Store a shard object version unless we already hold a newer one (our write's response and its watch
// echo arrive in either order).
static void shard_upsert(Shard& sh, int kind, const ShardPtr& so, bool dispatch) {
    Informer& inf = sh.inf[kind];
    auto it = inf.store.find(key_tmp(so->ns, so->name));
    ShardPtr old = it == inf.store.end() ? nullptr : it->second;
    if (old && so->rv >= 0 && old->rv >= so->rv) return;
    if (!wanted(kind, *so)) {
        if (old) inf.store.erase(it);
        return;
    }
    if (it != inf.store.end())
        it->second = so;
    else
        inf.store.emplace(key_of(so->ns, so->name), so);
    if (dispatch) on_shard_event(sh, kind, old, so, false);
}

static void shard_apply_line(Shard& sh, int kind, const std::string& line) {
    PhaseTimer pt(PH_SHARD_LINE);
    {  // nothing to decode: the echo of our own write (its response is already cached), or an object of
       // another executor's key partition (several executors share a shard's watch streams)
        std::string_view type, ns, name, rv;
        std::vector<std::string_view> owners;
        EventScanner sc(line);
        if (kind >= 2 && g_opt.parts > 1) sc.owners = &owners;
        if (sc.scan(type, ns, name, rv) && (type == "ADDED" || type == "MODIFIED" || type == "DELETED")) {
            Informer& inf = sh.inf[kind];
            std::string sns = ns.empty() ? g_opt.ns : std::string(ns);  // (short: no allocation)
            auto it = inf.store.find(key_tmp(sns, name));
            long long r = rv_num(rv);
            bool mine = true;
            if (g_opt.parts > 1) {
                if (kind < 2) {
                    mine = in_partition(sns, name);
                } else if (!owners.empty()) {
                    mine = false;
                    for (auto o : owners)
                        if (in_partition(sns, o)) mine = true;
                }
            }
            if (!mine) {
                ++inf.events;
                ++inf.foreign;
                inf.last_rv.assign(rv);
                if (it != inf.store.end()) {  // it left our partition (as shard_upsert does for !wanted)
                    inf.store.erase(it);
                    sh.memo[kind].erase(key_tmp(sns, name));
                }
                return;
            }
            if (type != "DELETED" && it != inf.store.end() && r >= 0 && it->second->rv >= r) {
                ++inf.events;
                ++inf.echoes;
                inf.last_rv.assign(rv);
                return;
            }
        }
    }
    std::string type;
    std::string_view raw[3];
    Value obj = Parser(line.data(), line.size()).parse_event_split(type, payload_keys(kind), payload_count(kind), raw);
    if (!obj.is_obj()) return;
    Informer& inf = sh.inf[kind];
    ++inf.events;
    if (type == "ERROR") {  // a Status object: no payload members were split off
        ApiError e = api_error(200, dumps(obj));
        throw e;
    }
    std::string rv = mget(obj, "resourceVersion");
    if (type == "BOOKMARK") {
        if (!rv.empty()) inf.last_rv = rv;
        return;
    }
    ShardPtr so = make_shard_obj(kind, std::move(obj), raw);
    if (!rv.empty()) inf.last_rv = rv;
    if (type == "DELETED") {
        std::string key = key_of(so->ns, so->name);
        auto it = inf.store.find(key);
        if (it == inf.store.end()) return;
        ShardPtr old = it->second;
        inf.store.erase(it);
        sh.memo[kind].erase(key);
        on_shard_event(sh, kind, old, nullptr, true);
        return;
    }
    shard_upsert(sh, kind, so, true);
}

static Task<void> shard_list(Shard& sh, int kind, std::string list_rv) {
    Informer& inf = sh.inf[kind];
    StrMap<ShardPtr> fresh;
    std::string token, rv;
    bool first = true;
    while (true) {
        std::string target = base_path(kind, g_opt.ns) + "?limit=500";
        if (first && !list_rv.empty()) target += "&resourceVersion=" + list_rv;
        if (!token.empty()) target += "&continue=" + token;
        first = false;
        Response r = co_await sh.client->request("GET", target, nullptr);
        if (r.status >= 300) throw api_error(r.status, r.body);
        Value lst = parse(r.body);
        Value* items = lst.get("items");
        if (items && items->is_arr())
            for (auto& it : items->a) {
                ShardPtr so = make_shard_obj(kind, std::move(it));
                if (!wanted(kind, *so)) continue;
                std::string key = key_of(so->ns, so->name);
                // the cached version when the listing has the same one: a relist of an unchanged shard holds one
                // copy of its objects, not two (the relist-storm peak, bench/suite.py config 4)
                auto old = inf.store.find(key);
                fresh[std::move(key)] = old != inf.store.end() && old->second->rv == so->rv ? old->second : so;
            }
        const Value* lm = lst.get("metadata");
        rv = lm ? std::string(lm->sget("resourceVersion")) : rv;
        token = lm ? std::string(lm->sget("continue")) : std::string();
        if (token.empty()) break;
    }
    bool was_synced = inf.synced;
    std::vector<std::pair<ShardPtr, ShardPtr>> changes;
    for (auto& kv : fresh) {
        auto it = inf.store.find(kv.first);
        if (it != inf.store.end()) changes.emplace_back(it->second, kv.second);
    }
    std::vector<ShardPtr> gone;
    for (auto& kv : inf.store)
        if (!fresh.count(kv.first)) {
            gone.push_back(kv.second);
            sh.memo[kind].erase(kv.first);
        }
    inf.store = std::move(fresh);
    inf.last_rv = rv;
    ++inf.relists;
    inf.synced = true;
    inf.synced_ev.set();
    for (auto& ch : changes) on_shard_event(sh, kind, ch.first, ch.second, false);
    if (was_synced)
        for (auto& g : gone) on_shard_event(sh, kind, g, nullptr, true);
}

static std::mt19937_64 g_rng(12345);
static double jitter() { return std::uniform_real_distribution<double>(0.0, 1.0)(g_rng); }

static Task<void> shard_watch(Shard& sh, int kind) {
    Informer& inf = sh.inf[kind];
    int timeout = 300 + static_cast<int>(jitter() * 300);
    std::string target = base_path(kind, g_opt.ns) + "?watch=1&resourceVersion=" + inf.last_rv +
                         "&timeoutSeconds=" + std::to_string(timeout) + "&allowWatchBookmarks=true";
    co_await sh.client->stream(
        target,
        [&sh, kind](std::vector<std::string>& lines) {
            for (const auto& l : lines) shard_apply_line(sh, kind, l);
        },
        timeout + 30.0);
}

// Reflector loop (list -> watch -> re-watch; 410 -> consistent relist; errors back off 0.8 s..30 s, as
// client-go's reflector).  After an outage (transport error or 5xx) the backoff can reach 30 s; when the
// workers' own requests to the shard are answered again (`Shard::answering`), the sleeping reflector
// retries at once — once per outage, so an endpoint that keeps failing while writes succeed (RBAC on watch,
// say) still backs off.
static Task<void> shard_informer(Shard* shp, int kind) {
    Shard& sh = *shp;
    double backoff = 0.8;
    bool need_list = true, woken = false;
    std::string list_rv = "0";
    while (!g_ex->stop_ev.is_set()) {
        bool gone = false, transport = false, failed = false, outage = false;
        std::string err;
        try {
            if (need_list) {
                co_await shard_list(sh, kind, list_rv);
                need_list = false;
            }
            sh.inf[kind].watching = true;
            sh.inf[kind].last_error.clear();
            co_await shard_watch(sh, kind);
            sh.inf[kind].watching = false;
            backoff = 0.8;
            woken = false;
        } catch (const ApiError& e) {
            if (e.code == 410) {
                gone = true;
            } else {
                failed = true;
                outage = e.code >= 500;
                err = describe(std::current_exception());
            }
        } catch (const TransportError& e) {
            failed = transport = outage = true;
            err = e.what();
        } catch (const std::exception& e) {
            failed = true;
            err = e.what();
        }
        if (gone) {
            need_list = true;
            list_rv = "";
            continue;
        }
        sh.inf[kind].watching = false;
        if (failed) {
            sh.inf[kind].last_error = err.substr(0, 300);
            LOG_DEBUG("shard %s %s: list/watch failed: %s; retry in %.2fs", sh.name.c_str(), kPlural[kind],
                      err.c_str(), backoff);
            double wait = backoff * (1 + jitter() * 0.2);
            if (outage && !woken) {
                sh.answering.clear();
                if (co_await sh.answering.wait_for(wait)) woken = true;  // the shard answers again
            } else {
                co_await loop().sleep(wait);
            }
            backoff = std::min(backoff * 2, 30.0);
            if (!transport) {
                need_list = true;
                list_rv = sh.inf[kind].last_rv.empty() ? "0" : sh.inf[kind].last_rv;
            }
        }
    }
}

// ------------------------------------------------------------------------------------ writes
// An answer below 500 means the shard's apiserver is serving: wake reflectors waiting out an outage backoff.
static void note_answer(Shard& sh, int status) {
    if (status > 0 && status < 500 && !sh.answering.is_set()) sh.answering.set();
}

static Value owner_labels() {
    Value l = Value::object();
    l.set(kLabelApp, Value::str(kAgent));
    l.set(kLabelOwner, Value::str(g_opt.alias));
    return l;
}
static Value owner_ref(const std::string& name, const std::string& uid) {
    Value r = Value::object();
    r.set("apiVersion", Value::str(kApiVersion));
    r.set("kind", Value::str(kTemplateKind));
    r.set("name", Value::str(name));
    r.set("uid", Value::str(uid));
    return r;
}

// One write; the server's answer goes into the cache (and the memo of what we meant to write).
// `data`: the request body (rendered with dumps_with: cached metadata + the raw controller-side payload)
static Task<ShardPtr> shard_write(Shard& sh, int kind, const char* method, const std::string& ns,
                                  const std::string& name, std::string data, PassState* pass, uint64_t want_a,
                                  uint64_t want_b, std::string_view sent_a = {}, std::string_view sent_b = {}) {
    pass->wrote = true;
    ++g_ex->stats_writes;
    std::string_view m(method);
    bool apply = m == "PATCH";  // the only PATCH this executor sends is a server-side apply
    std::string target = api_path(kind, ns, m == "POST" ? nullptr : &name, apply ? kApplyQuery : kFieldManagerQuery);
    Response r = co_await sh.client->request(method, target, &data, apply ? kApplyType : "application/json");
    note_answer(sh, r.status);
    if (r.status >= 300) throw api_error(r.status, r.body);
    SentPayload sent;  // (sent_a/sent_b: texts whose fingerprints are want_a/want_b, as computed controller-side)
    sent.raw[0] = sent_a;
    sent.raw[1] = sent_b;
    sent.fp[0] = want_a;
    sent.fp[1] = want_b;
    ShardPtr so = shard_obj_from_body(kind, r.body, &sent);
    // remember the intent only when the server stored something else (keeps the memo as small as the set
    // of rewritten objects)
    bool with_bin = kind == CONFIGMAPS && g_opt.sync_binary_data;
    bool rewritten = kind < 2 ? so->fp_spec != want_a : (so->fp_data != want_a || (with_bin && so->fp_bin != want_b));
    if (rewritten)
        sh.memo[kind][key_of(so->ns, so->name)] = Memo{so->rv, want_a, want_b};
    else
        sh.memo[kind].erase(key_tmp(so->ns, so->name));
    shard_upsert(sh, kind, so, false);
    co_return so;
}

static Task<ShardPtr> shard_get_live(Shard& sh, int kind, const std::string& ns, const std::string& name) {
    Response r = co_await sh.client->request("GET", item_path(kind, ns, name), nullptr);
    note_answer(sh, r.status);
    if (r.status >= 300) throw api_error(r.status, r.body);
    ShardPtr so = shard_obj_from_body(kind, r.body);
    shard_upsert(sh, kind, so, false);
    co_return so;
}

static Task<void> shard_delete(Shard& sh, int kind, const std::string& ns, const std::string& name) {
    Response r = co_await sh.client->request("DELETE", item_path(kind, ns, name), nullptr);
    note_answer(sh, r.status);
    if (r.status >= 300 && r.status != 404) throw api_error(r.status, r.body);
}

// create-or-update of a template/workgroup (native `_write`: AlreadyExists/Conflict -> re-read the live
// object; a Conflict on update is retried once from it)
static Value crd_head(int kind, const CtlObj& want) {
    Value head = Value::object();
    head.set("apiVersion", Value::str(kApiVersion));
    head.set("kind", Value::str(kind == TEMPLATES ? kTemplateKind : kWorkgroupKind));
    Value m = Value::object();
    m.set("name", Value::str(want.name));
    m.set("namespace", Value::str(want.ns));
    m.set("labels", owner_labels());
    head.set("metadata", std::move(m));
    return head;
}

static Task<ShardPtr> write_crd(Shard& sh, int kind, ShardPtr cur, const CtlObj& want, PassState* pass) {
    std::string_view spec = want.spec_raw.empty() ? std::string_view("null") : std::string_view(want.spec_raw);
    if (g_opt.server_side_apply) {
        // Shard.apply_template / apply_workgroup: one apply creates or updates; it carries no
        // resourceVersion, so there is no AlreadyExists/Conflict race to resolve
        std::string body;
        {
            PhaseTimer pt(PH_BODY);
            body = dumps_with(crd_head(kind, want), {{"spec", spec}});
        }
        co_return co_await shard_write(sh, kind, "PATCH", want.ns, want.name, std::move(body), pass, want.fp_spec, 0,
                                       want.spec_raw);
    }
    bool update = cur != nullptr;
    for (int attempt = 0; attempt < 2; ++attempt) {
        std::string body;
        if (update) {
            PhaseTimer pt(PH_BODY);
            body = splice_members(cur->rest, {{"spec", spec}});
        } else {
            PhaseTimer pt(PH_BODY);
            body = dumps_with(crd_head(kind, want), {{"spec", spec}});
        }
        bool race = false, exists = false;
        try {
            co_return co_await shard_write(sh, kind, update ? "PUT" : "POST", want.ns, want.name, std::move(body),
                                           pass, want.fp_spec, 0, want.spec_raw);
        } catch (const ApiError& e) {
            if (e.conflict() || e.already_exists()) {
                race = true;
                exists = e.already_exists();
            } else {
                throw;
            }
        }
        if (!race) break;
        ShardPtr live = co_await shard_get_live(sh, kind, want.ns, want.name);
        if (exists || attempt == 1) co_return live;
        cur = live;  // Conflict on update: once more from the live version
    }
    co_return cur;
}

static Task<void> sync_dependent_steps(Shard* shp, int kind, CtlPtr tpl, ShardPtr st, std::string dep,
                                       PassState* pass);

static Task<void> update_crd(Shard* shp, int kind, ShardPtr cur, CtlPtr want, PassState* pass) {
    co_await write_crd(*shp, kind, cur, *want, pass);
}

// syncSecretsToShard / syncConfigMapsToShard for one dependent: a failure is tagged with the dependent, so the
// coordinator can record the reference's Warning Events for it (controller.go:497,525-557,587-619)
static Task<void> sync_dependent(Shard* shp, int kind, CtlPtr tpl, ShardPtr st, std::string dep, PassState* pass) {
    std::exception_ptr err;
    try {
        co_await sync_dependent_steps(shp, kind, tpl, st, dep, pass);
    } catch (...) {
        err = std::current_exception();
    }
    if (err) {
        Failure f = failure_of(err, kind == SECRETS ? "Secret" : "ConfigMap", dep);
        throw ObjectError(f.cls, f.kind, f.name, f.code, f.msg);
    }
}

static Task<void> sync_dependent_steps(Shard* shp, int kind, CtlPtr tpl, ShardPtr st, std::string dep,
                                       PassState* pass) {
    Shard& sh = *shp;
    Executor& ex = *g_ex;
    CtlPtr src = ex.cget(kind, key_tmp(tpl->ns, dep));
    if (!src) throw NamedError("ReferenceMissing", std::string(kPlural[kind]) + " \"" + dep + "\" not found");
    const std::string& shard_ns = st->ns;
    bool is_secret = kind == SECRETS;
    bool with_bin = !is_secret && g_opt.sync_binary_data;
    ShardPtr so = sh.get(kind, key_tmp(shard_ns, dep));
    // `live`: with server-side apply, the shard copy whose template ownerRefs the applied configuration keeps
    // (every template's pass applies with the same field manager, and an apply drops the ownerRef entries its
    // manager applied before and omits now — applying only ours would take the other owners' refs off a
    // shared Secret/ConfigMap, and shard GC would delete it with this template)
    auto create_body = [&](const ShardObj* live = nullptr) {
        Value body = Value::object();
        body.set("apiVersion", Value::str("v1"));
        body.set("kind", Value::str(is_secret ? "Secret" : "ConfigMap"));
        Value m = Value::object();
        m.set("name", Value::str(dep));
        m.set("namespace", Value::str(shard_ns));
        m.set("labels", owner_labels());
        if (g_opt.sync_dependent_metadata) set_metadata(m, *src);
        Value refs = Value::array();
        if (live != nullptr) {
            for (const auto& o : live->template_owners)
                if (o.second != st->uid) refs.a.push_back(owner_ref(o.first, o.second));
            // a precondition: an apply over a stale view would drop refs applied since (409 instead)
            if (live->rv >= 0) m.set("resourceVersion", Value::str(std::to_string(live->rv)));
        }
        refs.a.push_back(owner_ref(st->name, st->uid));
        m.set("ownerReferences", std::move(refs));
        body.set("metadata", std::move(m));
        if (is_secret && !src->type.empty()) body.set("type", Value::str(src->type));
        std::string_view data = raw_null(src->data_raw) ? std::string_view() : std::string_view(src->data_raw);
        std::string_view bin = (!is_secret && with_bin && !raw_null(src->bin_raw)) ? std::string_view(src->bin_raw)
                                                                                    : std::string_view();
        return dumps_with(body, {{"data", data}, {"binaryData", bin}});
    };
    auto create = [&]() -> Task<ShardPtr> {
        bool exists = false;
        try {
            co_return co_await shard_write(sh, kind, "POST", shard_ns, dep, create_body(), pass, src->fp_data,
                                           src->fp_bin, src->data_raw, src->bin_raw);
        } catch (const ApiError& e) {
            if (!e.already_exists()) throw;
            exists = true;
        }
        (void)exists;
        co_return co_await shard_get_live(sh, kind, shard_ns, dep);
    };
    if (g_opt.server_side_apply) {
        // Shard.apply_dependent / reconcile.py `_sync_dependent`: every template's pass applies with the same
        // field manager, and an apply drops the ownerRef entries its manager applied before and omits now.  So
        // an apply over a known copy carries that copy's template ownerRefs and its resourceVersion (a
        // concurrent change -> 409 -> once more from the live copy).  A ref lost anyway (two passes creating
        // the same copy at once from empty caches) is repaired from the shard watch (on_shard_event).  A rogue
        // copy is refused; one in sync that already carries our ownerRef is skipped.
        for (int attempt = 0; attempt < 2; ++attempt) {
            if (so) {
                if (!so->has_owner_refs)
                    throw NamedError("RogueResourceError", "Resource \"" + dep +
                                                               "\" already exists and is not managed by any Machine "
                                                               "Learning Algorithm");
                bool ours = false;
                for (const auto& o : so->template_owners)
                    if (o.second == st->uid) ours = true;
                bool type_changed = is_secret && g_opt.sync_secret_type &&
                                    (src->type.empty() ? std::string("Opaque") : src->type) !=
                                        (so->type.empty() ? std::string("Opaque") : so->type);
                if (type_changed) {  // Secret.type is immutable: an apply cannot change it, so replace the copy
                    pass->wrote = true;
                    co_await shard_delete(sh, kind, shard_ns, dep);
                    sh.inf[kind].store.erase(key_tmp(shard_ns, dep));
                    so = nullptr;
                } else if (ours && data_in_sync(sh, kind, *so, *src) &&
                           (!g_opt.sync_dependent_metadata || meta_in_sync(*so, *src))) {
                    co_return;
                }
            }
            bool conflict = false;
            try {
                ShardPtr w = co_await shard_write(sh, kind, "PATCH", shard_ns, dep, create_body(so.get()), pass,
                                                  src->fp_data, src->fp_bin, src->data_raw, src->bin_raw);
                if (!so) repair_lost_owners(sh, kind, *w);  // applied without a view of the copy: refs may be gone
                co_return;
            } catch (const ApiError& e) {
                if (!e.conflict() || attempt == 1) throw;
                conflict = true;
            }
            if (conflict) so = co_await shard_get_live(sh, kind, shard_ns, dep);
        }
        co_return;
    }
    if (!so) so = co_await create();
    // isMissingOwnership (controller.go:482-502): no ownerRefs at all = a rogue object we refuse to touch
    if (!so->has_owner_refs)
        throw NamedError("RogueResourceError", "Resource \"" + dep +
                                                   "\" already exists and is not managed by any Machine "
                                                   "Learning Algorithm");
    bool missing_owner = true;
    for (const auto& o : so->template_owners)
        if (o.second == st->uid) missing_owner = false;
    if (is_secret && g_opt.sync_secret_type &&
        (src->type.empty() ? std::string("Opaque") : src->type) != (so->type.empty() ? std::string("Opaque") : so->type)) {
        // Secret.type is immutable: replace the shard copy (other owners re-add their refs on their passes)
        pass->wrote = true;
        co_await shard_delete(sh, kind, shard_ns, dep);
        sh.inf[kind].store.erase(key_tmp(shard_ns, dep));
        co_await create();
        co_return;
    }
    bool differs = !data_in_sync(sh, kind, *so, *src);
    bool meta_differs = g_opt.sync_dependent_metadata && !meta_in_sync(*so, *src);
    if (!differs && !missing_owner && !meta_differs) co_return;
    for (int attempt = 0; attempt < 2; ++attempt) {
        std::string_view data = raw_null(src->data_raw) ? std::string_view("{}") : std::string_view(src->data_raw);
        // binaryData: the source's when it has any; otherwise the member is dropped ("" = drop; without
        // binaryData sync the shard copy's own member is kept as it is)
        std::string_view bin;
        bool touch_bin = with_bin;
        if (with_bin && !raw_is_empty(src->bin_raw)) bin = src->bin_raw;
        std::string body;
        if (missing_owner || meta_differs) {
            PhaseTimer pt(PH_BODY);
            Value copy = parse(so->rest);
            Value* m = copy.get("metadata");
            if (m == nullptr) m = &copy.set("metadata", Value::object());
            if (missing_owner) {
                Value* refs = m->get("ownerReferences");
                if (refs == nullptr || !refs->is_arr()) refs = &m->set("ownerReferences", Value::array());
                refs->a.push_back(owner_ref(st->name, st->uid));
            }
            if (meta_differs) set_metadata(*m, *src);
            body = touch_bin ? dumps_with(copy, {{"data", data}, {"binaryData", bin}}) : dumps_with(copy, {{"data", data}});
        } else {
            PhaseTimer pt(PH_BODY);
            body = touch_bin ? splice_members(so->rest, {{"data", data}, {"binaryData", bin}})
                             : splice_members(so->rest, {{"data", data}});
        }
        bool conflict = false;
        try {
            co_await shard_write(sh, kind, "PUT", shard_ns, dep, std::move(body), pass, src->fp_data, src->fp_bin,
                                 src->data_raw, src->bin_raw);
            co_return;
        } catch (const ApiError& e) {
            if (!e.conflict() || attempt == 1) throw;
            conflict = true;
        }
        if (conflict) {
            so = co_await shard_get_live(sh, kind, shard_ns, dep);
            missing_owner = true;
            for (const auto& o : so->template_owners)
                if (o.second == st->uid) missing_owner = false;
            if (!so->has_owner_refs) throw NamedError("RogueResourceError", "Resource \"" + dep + "\" lost its owners");
            meta_differs = g_opt.sync_dependent_metadata && !meta_in_sync(*so, *src);
            if (data_in_sync(sh, kind, *so, *src) && !missing_owner && !meta_differs) co_return;
        }
    }
}

// The condition under which sync_dependent_steps ends without a write (either path), checked without
// starting it: a pass triggered by one changed dependent leaves the others alone at the cost of two lookups.
static bool dependent_in_sync(Shard& sh, int kind, const CtlObj& tpl, const ShardObj& st, const std::string& dep) {
    Executor& ex = *g_ex;
    const CtlObj* src = ex.cfind(kind, key_tmp(tpl.ns, dep));
    if (src == nullptr) return false;
    const ShardObj* so = sh.find(kind, key_tmp(st.ns, dep));
    if (so == nullptr || !so->has_owner_refs) return false;
    bool owned = false;
    for (const auto& o : so->template_owners)
        if (o.second == st.uid) owned = true;
    if (!owned) return false;
    if (kind == SECRETS && g_opt.sync_secret_type &&
        (src->type.empty() ? std::string_view("Opaque") : std::string_view(src->type)) !=
            (so->type.empty() ? std::string_view("Opaque") : std::string_view(so->type)))
        return false;
    return data_in_sync(sh, kind, *so, *src) && (!g_opt.sync_dependent_metadata || meta_in_sync(*so, *src));
}

static Task<void> sync_template_to_shard(Shard* shp, CtlPtr tpl, PassState* pass) {
    Shard& sh = *shp;
    if (!sh.synced()) throw NamedError("ShardNotReadyError", "shard " + sh.name + " caches not synced");
    ShardPtr st = sh.get(TEMPLATES, key_tmp(tpl->ns, tpl->name));
    std::vector<Task<void>> jobs;
    jobs.reserve(1 + tpl->secrets.size() + tpl->configmaps.size());
    if (!st) {
        st = co_await write_crd(sh, TEMPLATES, st, *tpl, pass);  // the dependents' ownerRefs need its UID
    } else if (!spec_in_sync(sh, TEMPLATES, *st, tpl->fp_spec)) {
        // an update keeps the shard template's UID: its dependents go out alongside it, not one round trip
        // later (the reference's loop is strictly sequential, controller.go:790-831)
        jobs.push_back(update_crd(shp, TEMPLATES, st, tpl, pass));
    }
    for (const auto& n : tpl->secrets)
        if (!dependent_in_sync(sh, SECRETS, *tpl, *st, n)) jobs.push_back(sync_dependent(shp, SECRETS, tpl, st, n, pass));
    for (const auto& n : tpl->configmaps)
        if (!dependent_in_sync(sh, CONFIGMAPS, *tpl, *st, n))
            jobs.push_back(sync_dependent(shp, CONFIGMAPS, tpl, st, n, pass));
    if (jobs.empty()) co_return;
    auto errs = co_await when_all(std::move(jobs));
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
}

static Task<void> sync_workgroup_to_shard(Shard* shp, CtlPtr wg, PassState* pass) {
    Shard& sh = *shp;
    if (!sh.synced()) throw NamedError("ShardNotReadyError", "shard " + sh.name + " caches not synced");
    ShardPtr sw = sh.get(WORKGROUPS, key_tmp(wg->ns, wg->name));
    if (!sw || !spec_in_sync(sh, WORKGROUPS, *sw, wg->fp_spec)) co_await write_crd(sh, WORKGROUPS, sw, *wg, pass);
}

static void report(const std::string& key, const CtlObj& obj,
                   const std::vector<std::pair<std::string, std::optional<Failure>>>& results, bool wrote) {
    mp::Encoder e;
    e.out.reserve(64 + key.size() + obj.uid.size() + 48 * results.size());
    e.map(6);
    e.str("t");
    e.str("report");
    e.str("k");
    e.str(key);
    e.str("u");
    e.str(obj.uid);
    e.str("g");
    e.integer(obj.generation);
    e.str("r");
    e.map(results.size());
    for (const auto& r : results) {
        e.str(r.first);
        if (!r.second) {
            e.nil();
            continue;
        }
        const Failure& f = *r.second;
        e.map(5);
        e.str("c");
        e.str(f.cls);
        e.str("k");
        e.str(f.kind);
        e.str("n");
        e.str(f.name);
        e.str("h");
        e.integer(f.code);
        e.str("m");
        e.str(f.msg);
    }
    e.str("w");
    e.boolean(wrote);
    g_chan->send(std::move(e.out));
}

static void ask_coordinator(int kind, const std::string& key) {
    Executor& ex = *g_ex;
    double now = now_s();
    auto it = ex.needed.find(key);
    if (it != ex.needed.end() && now - it->second < 1.0) return;
    ex.needed[key] = now;
    mp::Encoder e;
    e.map(3);
    e.str("t");
    e.str("need");
    e.str("k");
    e.integer(kind);
    e.str("n");
    e.str(key);
    g_chan->send(std::move(e.out));
}

static Task<void> propagate_delete(int kind, std::string ns, std::string name) {
    Executor& ex = *g_ex;
    std::string key = key_of(ns, name);
    bool explicit_ = ex.pending_deletes[kind].count(key) > 0;
    std::vector<Task<void>> jobs;
    for (auto& sp : ex.shards) {
        Shard& sh = *sp;
        ShardPtr so = sh.get(kind, key);
        if (!so) continue;
        if (!explicit_ && !is_ours(*so)) continue;
        if (!sh.synced()) throw NamedError("ShardNotReadyError", "shard " + sh.name + " caches not synced");
        jobs.push_back(shard_delete(sh, kind, ns, name));
    }
    auto errs = co_await when_all(std::move(jobs));
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    ex.pending_deletes[kind].erase(key);
}

// `qkey`: the work queue's key, "template/<ns>/<name>" or "workgroup/<ns>/<name>" (the queue keeps it until the
// pass is done)
static Task<void> sync_object(int kind, std::string ns, std::string name, const std::string& qkey) {
    Executor& ex = *g_ex;
    CtlPtr obj = ex.cget(kind, key_tmp(ns, name));
    if (!obj) {
        ex.skipping_since.erase(qkey);
        if (kind == TEMPLATES || g_opt.propagate_workgroup_deletes) co_await propagate_delete(kind, ns, name);
        co_return;
    }
    if (kind == TEMPLATES) {
        // the coordinator adopts; an executor only refuses to write while a reference is missing
        for (int k = SECRETS; k <= CONFIGMAPS; ++k)
            for (const auto& n : (k == SECRETS ? obj->secrets : obj->configmaps)) {
                std::string dk = key_of(ns, n);
                if (!ex.cget(k, dk)) {
                    ask_coordinator(k, dk);
                    throw ApiError(404, "NotFound", std::string(kPlural[k]) + " \"" + n + "\" not found");
                }
            }
    }
    PassState pass;
    std::vector<Task<void>> jobs;
    jobs.reserve(ex.shards.size());
    for (auto& sp : ex.shards)
        jobs.push_back(kind == TEMPLATES ? sync_template_to_shard(sp.get(), obj, &pass)
                                         : sync_workgroup_to_shard(sp.get(), obj, &pass));
    auto errs = co_await when_all(std::move(jobs));
    if (ex.queue.dirty(qkey)) {
        // a newer version (or a dependent) re-queued the key while this pass ran: the next pass reports on
        // the version it sees, carrying this pass's writes — a report on a version the coordinator may already
        // have moved past would only cost it a fold and a superseded finish.  Not for ever, though: under a
        // steady stream of events every pass would be superseded and the status never advance, so a key
        // reports at least every kMaxReportSkip seconds
        double now = now_s();
        auto [it, fresh] = ex.skipping_since.try_emplace(qkey, now);
        if (fresh || now - it->second < kMaxReportSkip) {
            if (pass.wrote) ex.carry_wrote.insert(qkey);
            ++ex.stats_reports_skipped;
            for (auto& e : errs)
                if (e) std::rethrow_exception(e);
            co_return;
        }
    }
    ex.skipping_since.erase(qkey);
    if (ex.carry_wrote.erase(qkey) > 0) pass.wrote = true;
    std::vector<std::pair<std::string, std::optional<Failure>>> results;
    bool failed = false;
    std::string first;
    const char* obj_kind = kind == TEMPLATES ? kTemplateKind : kWorkgroupKind;
    for (size_t i = 0; i < ex.shards.size(); ++i) {
        std::optional<Failure> f;
        if (errs[i]) {
            f = failure_of(errs[i], obj_kind, name);
            if (!failed) first = ex.shards[i]->name + ": " + describe(errs[i]);
            failed = true;
        }
        results.emplace_back(ex.shards[i]->name, std::move(f));
    }
    report(qkey, *obj, results, pass.wrote);
    if (failed) throw NamedError("ShardSyncError", first);
}

static Task<void> worker() {
    Executor& ex = *g_ex;
    while (true) {
        const std::string* kp = co_await ex.queue.get();
        if (kp == nullptr) co_return;
        const std::string& key = *kp;  // (the queue's own copy: valid until done() below)
        trace('q', 0, key);
        size_t a = key.find('/');
        size_t b = key.find('/', a + 1);
        std::string_view kind(key.data(), a);
        std::string ns = key.substr(a + 1, b - a - 1), name = key.substr(b + 1);
        ++ex.stats_reconciles;
        bool ok = true;
        std::string err;
        try {
            co_await sync_object(kind == "template" ? TEMPLATES : WORKGROUPS, ns, name, key);
        } catch (const std::exception&) {
            ok = false;
            err = describe(std::current_exception());
        }
        if (ok) {
            ex.queue.forget(key);
        } else {
            ++ex.stats_errors;
            LOG_INFO("Error syncing %s; re-queuing for later retry: %s", key.c_str(), err.c_str());
            ++g_enq[ENQ_RETRY];
            ex.queue.add_rate_limited(key);
        }
        ex.queue.done(key);
    }
}

static void sweep_orphans() {
    Executor& ex = *g_ex;
    for (auto& sp : ex.shards) {
        for (int kind : {TEMPLATES, WORKGROUPS}) {
            if (kind == WORKGROUPS && !g_opt.propagate_workgroup_deletes) continue;
            for (auto& kv : sp->inf[kind].store)
                if (is_ours(*kv.second) && !ex.cget(kind, kv.first)) {
                    ++g_enq[ENQ_SWEEP];
                    ex.enqueue(kind, kv.second->ns, kv.second->name);
                }
        }
    }
}

static void enqueue_all() {
    Executor& ex = *g_ex;
    for (int kind : {TEMPLATES, WORKGROUPS})
        for (auto& kv : ex.ctl[kind]) {
            ++g_enq[ENQ_RESYNC];
            ex.enqueue(kind, kv.second->ns, kv.second->name);
        }
}

static Task<void> full_resync_loop() {
    while (!g_ex->stop_ev.is_set()) {
        co_await loop().sleep(g_opt.full_resync);
        enqueue_all();
        if (g_opt.orphan_sweep) sweep_orphans();
    }
}

static Task<void> wait_shard_synced(Shard* sh, double timeout) {
    double end = now_s() + timeout;
    for (auto& inf : sh->inf) {
        double left = end - now_s();
        if (left <= 0 || !(co_await inf.synced_ev.wait_for(left))) {
            LOG_WARN("shard %s did not sync within %.1fs; continuing without it for now", sh->name.c_str(), timeout);
            co_return;
        }
    }
}

// ------------------------------------------------------------------------------------ config / main
static Credentials creds_of(const Value& s) {
    Credentials c;
    c.server = std::string(s.sget("server"));
    c.ca_pem = std::string(s.sget("ca_pem"));
    const Value* ins = s.get("insecure");
    c.insecure = ins && ins->t == Value::BOOL && ins->b;
    c.tls_server_name = std::string(s.sget("tls_server_name"));
    c.cert_pem = std::string(s.sget("cert_pem"));
    c.key_pem = std::string(s.sget("key_pem"));
    c.token = std::string(s.sget("token"));
    c.token_file = std::string(s.sget("token_file"));
    c.username = std::string(s.sget("username"));
    c.password = std::string(s.sget("password"));
    c.proxy = std::string(s.sget("proxy"));
    c.proxy_connect = std::string(s.sget("proxy_connect"));
    c.proxy_user = std::string(s.sget("proxy_user"));
    c.proxy_pass = std::string(s.sget("proxy_pass"));
    return c;
}

static double num(const Value& o, const char* k, double d) {
    const Value* v = o.get(k);
    if (v && v->t == Value::NUM) return std::atof(v->s.c_str());
    if (v && v->t == Value::BOOL) return v->b ? 1.0 : 0.0;
    return d;
}

static void configure(const Value& c) {
    Options& o = g_opt;
    o.ns = std::string(c.sget("namespace"));
    o.alias = std::string(c.sget("alias"));
    o.workers = static_cast<int>(num(c, "workers", o.workers));
    o.pool_size = static_cast<int>(num(c, "pool_size", o.pool_size));
    o.flow.h2_cap = static_cast<int>(num(c, "h2_inflight", 0));
    if (const char* ps = std::getenv("NCC_POOL_SIZE")) {  // experiments: the cap over either protocol
        o.pool_size = std::max(1, std::atoi(ps));
        o.flow.h2_cap = 0;
    }
    if (const char* v = std::getenv("NCC_H2_INFLIGHT")) o.flow.h2_cap = std::atoi(v);  // experiments
    o.pipeline_depth = std::max(1, static_cast<int>(num(c, "pipeline_depth", o.pipeline_depth)));
    if (const char* v = std::getenv("NCC_PIPELINE_DEPTH")) o.pipeline_depth = std::max(1, std::atoi(v));  // experiments
    o.http2 = static_cast<int>(num(c, "http2", o.http2));
    if (const char* v = std::getenv("NCC_HTTP2")) o.http2 = std::atoi(v);  // experiments
    o.flow.qps = num(c, "client_qps", 0);
    o.flow.burst = num(c, "client_burst", 10);
    o.flow.adaptive = num(c, "adaptive_concurrency", 1) != 0;
    o.flow.initial = num(c, "initial_concurrency", o.flow.initial);
    o.flow.latency_s = num(c, "overload_latency", o.flow.latency_s);
    if (const char* v = std::getenv("NCC_AIMD")) o.flow.adaptive = std::atoi(v) != 0;  // experiments
    if (const char* v = std::getenv("NCC_LOOP_COALESCE_US"))  // experiments: software interrupt coalescing
        loop().set_coalesce(std::max(0L, std::atol(v)) * 1000L, 32);
    o.request_timeout = num(c, "request_timeout", o.request_timeout);
    o.coalesce = num(c, "coalesce_window", o.coalesce);
    o.base_delay = num(c, "failure_base_delay", o.base_delay);
    o.max_delay = num(c, "failure_max_delay", o.max_delay);
    o.qps = num(c, "rate_limit_qps", o.qps);
    o.burst = num(c, "rate_limit_burst", o.burst);
    o.shard_sync_timeout = num(c, "shard_sync_timeout", o.shard_sync_timeout);
    o.full_resync = num(c, "full_resync_period", o.full_resync);
    o.sync_binary_data = num(c, "sync_binary_data", 1) != 0;
    o.sync_secret_type = num(c, "sync_secret_type", 1) != 0;
    o.orphan_sweep = num(c, "orphan_sweep", 1) != 0;
    o.propagate_workgroup_deletes = num(c, "propagate_workgroup_deletes", 1) != 0;
    o.server_side_apply = num(c, "server_side_apply", 0) != 0;
    o.sync_dependent_metadata = num(c, "sync_dependent_metadata", 0) != 0;
    o.log_level = static_cast<int>(num(c, "log_level", o.log_level));
    if (o.full_resync <= 0) o.full_resync = 1e9;
    Executor& ex = *g_ex;
    const Value* shards = c.get("shards");
    if (shards && shards->is_arr())
        for (const auto& s : shards->a) {
            auto sh = std::make_unique<Shard>();
            sh->name = std::string(s.sget("name"));
            sh->client = std::make_unique<Client>(creds_of(s), o.pool_size, o.request_timeout, o.flow,
                                                  o.pipeline_depth, o.http2);
            sh->client->on_notice = [name = sh->name](const std::string& m) {
                LOG_WARN("shard %s: %s", name.c_str(), m.c_str());
            };
            for (int k = 0; k < 4; ++k) {
                sh->inf[k].shard = sh.get();
                sh->inf[k].kind = k;
            }
            ex.shards.push_back(std::move(sh));
        }
}

static void handle_message(const mp::Obj& m) {
    PhaseTimer pt(PH_RELAY);
    Executor& ex = *g_ex;
    std::string_view t = m.sget("t");
    if (t == "w" || t == "s") {
        int kind = static_cast<int>(m.iget("k"));
        const mp::Obj* lines = m.get("l");
        if (kind < 0 || kind > 3 || lines == nullptr || lines->t != mp::Obj::ARR) return;
        std::string type;
        std::string_view raw[3];
        if (t == "s") {
            // a large listing arrives in chunks: every one but the last carries "more" (relay.py)
            std::vector<CtlPtr>& objs = ex.partial_snapshot[kind];
            objs.reserve(objs.size() + lines->a.size());
            auto& cached = ex.ctl[kind];
            for (const auto& l : lines->a) {
                if (CtlPtr fast = ctl_scan(kind, l.s, type)) {
                    if (type == "ADDED" || type == "MODIFIED") {
                        // the cached version when the snapshot has the same one (a coordinator relist): one copy
                        auto old = cached.find(key_tmp(fast->ns, fast->name));
                        objs.push_back(old != cached.end() && old->second->rv == fast->rv ? old->second : std::move(fast));
                    }
                    continue;
                }
                try {
                    Value o = Parser(l.s.data(), l.s.size()).parse_event_split(type, payload_keys(kind),
                                                                                payload_count(kind), raw);
                    if (o.is_obj() && (type == "ADDED" || type == "MODIFIED")) objs.push_back(make_ctl(kind, o, raw));
                } catch (const std::exception& e) {  // one bad line costs that object, not the rest of the batch
                    LOG_ERROR("unreadable relayed line (kind %d): %s", kind, e.what());
                }
            }
            const mp::Obj* more = m.get("more");
            if (more != nullptr && more->t == mp::Obj::BOOL && more->b) return;
            ctl_snapshot(kind, std::move(objs));
            objs = std::vector<CtlPtr>();
        } else {
            for (const auto& l : lines->a) {
                if (CtlPtr fast = ctl_scan(kind, l.s, type)) {
                    if (type == "ADDED" || type == "MODIFIED" || type == "DELETED") ctl_apply(kind, type, fast);
                    continue;
                }
                CtlPtr parsed;
                try {
                    Value o = Parser(l.s.data(), l.s.size()).parse_event_split(type, payload_keys(kind),
                                                                                payload_count(kind), raw);
                    if (o.is_obj() && (type == "ADDED" || type == "MODIFIED" || type == "DELETED"))
                        parsed = make_ctl(kind, o, raw);
                } catch (const std::exception& e) {  // one bad line costs that object, not the rest of the batch
                    LOG_ERROR("unreadable relayed line (kind %d): %s", kind, e.what());
                }
                if (parsed) ctl_apply(kind, type, parsed);
            }
        }
    } else if (t == "go") {
        ex.gate.set();
    } else if (t == "resync") {
        // a coordinator partition (re)started and has no report state: pass over its keys again so every
        // shard reports on them (in-sync keys cost no write)
        long long part = m.iget("p"), parts = m.iget("n", 1);
        if (parts < 1 || part < 0 || part >= parts) return;
        for (int kind : {TEMPLATES, WORKGROUPS})
            for (auto& kv : ex.ctl[kind])
                if (static_cast<long long>(crc32(key_of(kv.second->ns, kv.second->name)) % parts) == part) {
                    ++g_enq[ENQ_RESYNC];
                    ex.enqueue(kind, kv.second->ns, kv.second->name);
                }
    } else if (t == "cred") {
        std::string_view shard = m.sget("s");
        for (auto& sp : ex.shards)
            if (sp->name == shard) sp->client->set_token(std::string(m.sget("token")));
    }
}

static Task<void> reader(Event* configured) {
    Executor& ex = *g_ex;
    while (true) {
        std::vector<mp::Obj> batch = co_await g_chan->recv();
        if (batch.empty() && g_chan->closed()) break;
        for (const auto& m : batch) {
            if (m.sget("t") == "cfg") {
                if (!configured->is_set()) {
                    configure(parse(m.sget("c")));
                    configured->set();
                }
                continue;
            }
            try {
                handle_message(m);
            } catch (const std::exception& e) {
                LOG_ERROR("bad message from the coordinator: %s", e.what());
            }
        }
    }
    ex.stop_ev.set();  // the coordinator closing its end (or dying) ends this executor
}

static Task<void> run_main() {
    Executor& ex = *g_ex;
    static Event configured;
    spawn(reader(&configured), "channel reader");
    co_await configured.wait();
    for (auto& sp : ex.shards)
        for (int k = 0; k < 4; ++k) spawn(shard_informer(sp.get(), k), "shard informer");
    spawn(status_loop(), "status");
    co_await ex.ctl_synced_ev.wait();
    std::vector<Task<void>> waits;
    for (auto& sp : ex.shards) waits.push_back(wait_shard_synced(sp.get(), g_opt.shard_sync_timeout));
    co_await when_all(std::move(waits));
    send_simple("synced");
    if (g_opt.gated) co_await ex.gate.wait();
    for (int i = 0; i < g_opt.workers; ++i) spawn(worker(), "worker");
    if (g_opt.orphan_sweep) sweep_orphans();
    spawn(full_resync_loop(), "full resync");
    send_simple("ready");
    LOG_INFO("native executor %d ready: %zu shard(s), partition %d/%d, %d workers", g_opt.index, ex.shards.size(),
             g_opt.part, g_opt.parts, g_opt.workers);
}

static void send_status() {
    Executor& ex = *g_ex;
    mp::Encoder e;
    e.map(7);
    e.str("t");
    e.str("status");
    e.str("i");
    e.integer(g_opt.index);
    e.str("s");
    e.map(ex.shards.size());
    for (const auto& sp : ex.shards) {
        e.str(sp->name);
        e.map(5);
        for (int k = 0; k < 4; ++k) {
            const Informer& inf = sp->inf[k];
            e.str(kPlural[k]);
            e.array(5);
            e.boolean(inf.synced);
            e.boolean(inf.watching);
            e.integer(inf.events);
            e.integer(inf.relists);
            e.str(inf.last_error);
        }
        // client-side flow control: [limit, in flight, most in flight, 429s, overload signals, cuts, gated, qps wait ms,
        // connections, write batches, requests, slow starts left on rising latency, increases held back, the
        // executor loop's wake-ups and coalesced wake-ups (process-wide), and HTTP/2: in use (0/1), streams
        // opened, streams re-sent after REFUSED_STREAM, GOAWAYs received, connections dropped for an unanswered PING,
        // GOAWAYs with an error code, downgraded to HTTP/1.1 by HTTP_1_1_REQUIRED (0/1), streams reset with
        // ENHANCE_YOUR_CALM, the in-flight cap]
        const Client& cl = *sp->client;
        e.str("flow");
        e.array(24);
        e.integer(static_cast<long long>(cl.limit()));
        e.integer(cl.inflight());
        e.integer(cl.flow.max_inflight);
        e.integer(cl.flow.rejected);
        e.integer(cl.flow.overloads);
        e.integer(cl.flow.cuts);
        e.integer(cl.flow.gated);
        e.integer(static_cast<long long>(cl.flow.qps_wait_s * 1000));
        e.integer(cl.connections());
        e.integer(cl.sends);
        e.integer(cl.requests);
        e.integer(cl.flow.hystart);
        e.integer(cl.flow.held);
        e.integer(static_cast<long long>(loop().wakeups()));
        e.integer(static_cast<long long>(loop().coalesced()));
        e.integer(cl.http2() ? 1 : 0);
        e.integer(cl.h2_streams);
        e.integer(cl.h2_refused);
        e.integer(cl.h2_goaways);
        e.integer(cl.h2_dead);
        e.integer(cl.h2_goaway_errors);
        e.integer(cl.h2_downgraded ? 1 : 0);
        e.integer(cl.h2_calm);
        e.integer(cl.cap());
    }
    e.str("q");
    e.integer(static_cast<long long>(ex.queue.load()));
    e.str("r");
    e.integer(ex.stats_reconciles);
    e.str("w");
    e.integer(ex.stats_writes);
    e.str("e");
    e.integer(ex.stats_errors);
    g_chan->send(std::move(e.out));
}

static Task<void> status_loop() {
    Executor& ex = *g_ex;
    double period = 5.0;
    if (const char* v = std::getenv("NCC_STATUS_S")) period = std::max(0.05, std::atof(v));
    while (!ex.stop_ev.is_set()) {
        send_status();
        co_await ex.stop_ev.wait_for(period);
    }
}

// The coordinator closing the channel (or dying), or a signal, ends the executor — at any point, including
// while it still waits for a shard's caches.
static Task<void> shutdown_watch() {
    Executor& ex = *g_ex;
    co_await ex.stop_ev.wait();
    long long echoes = 0, shard_events = 0, foreign = 0;
    for (auto& sp : ex.shards)
        for (int k = 0; k < 4; ++k) {
            echoes += sp->inf[k].echoes;
            shard_events += sp->inf[k].events;
            foreign += sp->inf[k].foreign;
        }
    if (std::getenv("NCC_CPU_REPORT"))
        LOG_WARN("executor stats shard_events=%lld echoes_skipped=%lld other_partition_skipped=%lld loop_wakeups=%llu "
                 "coalesced=%llu",
                 shard_events, echoes, foreign, static_cast<unsigned long long>(loop().wakeups()),
                 static_cast<unsigned long long>(loop().coalesced()));
    if (g_phases_on) {
        // ticks -> seconds: calibrate the TSC against the steady clock
        unsigned long long c0 = ticks();
        double w0 = now_s();
        while (now_s() - w0 < 0.02) {
        }
        double hz = static_cast<double>(ticks() - c0) / (now_s() - w0);
        struct rusage ru;
        getrusage(RUSAGE_SELF, &ru);
        double user = ru.ru_utime.tv_sec + ru.ru_utime.tv_usec / 1e6, sys = ru.ru_stime.tv_sec + ru.ru_stime.tv_usec / 1e6;
        std::string parts;
        for (int i = 0; i < PH_N; ++i) {
            char b[96];
            std::snprintf(b, sizeof b, " %s=%.3fs", kPhaseName[i], static_cast<double>(g_phase[i]) / hz);
            parts += b;
        }
        LOG_WARN("executor cpu user=%.3fs sys=%.3fs phases:%s response_scan=%lld/%lld", user, sys, parts.c_str(),
                 g_scan_hits, g_scan_hits + g_scan_misses);
        LOG_WARN("executor response payloads matched as sent: %lld", g_sent_hits);
    }
    if (std::getenv("NCC_CPU_REPORT"))
        LOG_WARN("executor stats reconciles=%lld writes=%lld errors=%lld reports_skipped=%lld enqueues: object=%lld "
                 "dependent=%lld shard_object=%lld shard_dependent=%lld retry=%lld sweep=%lld resync=%lld delete=%lld",
                 ex.stats_reconciles, ex.stats_writes, ex.stats_errors, ex.stats_reports_skipped, g_enq[ENQ_OBJECT],
                 g_enq[ENQ_DEPENDENT],
                 g_enq[ENQ_SHARD_OBJECT], g_enq[ENQ_SHARD_DEPENDENT], g_enq[ENQ_RETRY], g_enq[ENQ_SWEEP],
                 g_enq[ENQ_RESYNC], g_enq[ENQ_DELETE]);
    ex.queue.shutdown();
    dump_trace();
    co_await g_chan->drain(2.0);
    loop().stop();
}

static int g_sigpipe[2] = {-1, -1};
static void on_signal(int) {
    char c = 1;
    (void)!write(g_sigpipe[1], &c, 1);
}
static Task<void> signal_watch() {
    while (true) {
        char c;
        ssize_t r = ::read(g_sigpipe[0], &c, 1);
        if (r > 0) break;
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            co_await loop().readable(g_sigpipe[0]);
            continue;
        }
        if (r < 0 && errno == EINTR) continue;
        co_return;
    }
    g_ex->stop_ev.set();
}

}  // namespace ncc

int main(int argc, char** argv) {
    using namespace ncc;
    int fd = -1;
    for (int i = 1; i + 1 < argc; ++i) {
        std::string a = argv[i];
        if (a == "--fd") fd = std::atoi(argv[++i]);
        else if (a == "--index") g_opt.index = std::atoi(argv[++i]);
        else if (a == "--part") {
            std::string p = argv[++i];
            size_t sl = p.find('/');
            g_opt.part = std::atoi(p.substr(0, sl).c_str());
            g_opt.parts = sl == std::string::npos ? 1 : std::atoi(p.c_str() + sl + 1);
        }
    }
    if (argc > 1 && std::string(argv[1]) == "--version") {
        std::puts("ncc-executor 1");
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--json-selftest") {
        // one JSON text per stdin line -> "<fingerprint of the DOM> <streaming fingerprint> <split render>"
        // (tests/test_native_executor_json.py compares them and the render against the input)
        std::string line;
        char buf[1 << 16];
        while (std::fgets(buf, sizeof buf, stdin) != nullptr) {
            line.assign(buf);
            while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
            try {
                Value v = parse(line);
                uint64_t a = fingerprint(v), b = fingerprint_text(line);
                std::string render = "-";
                if (v.is_obj()) {
                    static const std::string_view keys[2] = {"spec", "data"};
                    std::string_view raw[2];
                    Value rest = Parser(line.data(), line.size()).parse_split(keys, 2, raw);
                    render = dumps_with(rest, {{"spec", raw[0]}, {"data", raw[1]}});
                }
                std::printf("%llu %llu %s\n", static_cast<unsigned long long>(a), static_cast<unsigned long long>(b),
                            render.c_str());
            } catch (const std::exception& e) {
                std::printf("error %s\n", e.what());
            }
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--msgpack-selftest") {
        // one hex-encoded msgpack value per stdin line -> "<decoded value as JSON>\t<hex of its re-encoding>"
        // (maps as [[key, value], ...], bin as {"bin": "<hex>"}; "-" when the value holds a type the
        // executor never sends: float, bin), or "error" (tests/test_native_executor_json.py)
        static char buf[1 << 20];
        std::function<void(std::string&, const mp::Obj&)> render = [&](std::string& out, const mp::Obj& o) {
            char num[64];
            switch (o.t) {
                case mp::Obj::NIL: out += "null"; break;
                case mp::Obj::BOOL: out += o.b ? "true" : "false"; break;
                case mp::Obj::INT: out += std::to_string(o.i); break;
                case mp::Obj::FLOAT: std::snprintf(num, sizeof num, "%.17g", o.d); out += num; break;
                case mp::Obj::STR: write_string(out, o.s); break;
                case mp::Obj::BIN: {
                    out += "{\"bin\":\"";
                    for (unsigned char ch : o.s) {
                        std::snprintf(num, sizeof num, "%02x", ch);
                        out += num;
                    }
                    out += "\"}";
                    break;
                }
                case mp::Obj::ARR:
                    out += '[';
                    for (size_t k = 0; k < o.a.size(); ++k) {
                        if (k) out += ',';
                        render(out, o.a[k]);
                    }
                    out += ']';
                    break;
                case mp::Obj::MAP:
                    out += '[';
                    for (size_t k = 0; k < o.m.size(); ++k) {
                        if (k) out += ',';
                        out += '[';
                        render(out, o.m[k].first);
                        out += ',';
                        render(out, o.m[k].second);
                        out += ']';
                    }
                    out += ']';
                    break;
            }
        };
        std::function<bool(mp::Encoder&, const mp::Obj&)> encode = [&](mp::Encoder& en, const mp::Obj& o) {
            switch (o.t) {
                case mp::Obj::NIL: en.nil(); return true;
                case mp::Obj::BOOL: en.boolean(o.b); return true;
                case mp::Obj::INT: en.integer(o.i); return true;
                case mp::Obj::STR: en.str(o.s); return true;
                case mp::Obj::ARR:
                    en.array(o.a.size());
                    for (const auto& x : o.a)
                        if (!encode(en, x)) return false;
                    return true;
                case mp::Obj::MAP:
                    en.map(o.m.size());
                    for (const auto& kv : o.m)
                        if (!encode(en, kv.first) || !encode(en, kv.second)) return false;
                    return true;
                default: return false;
            }
        };
        while (std::fgets(buf, sizeof buf, stdin) != nullptr) {
            std::string hex(buf), body;
            while (!hex.empty() && (hex.back() == '\n' || hex.back() == '\r')) hex.pop_back();
            for (size_t k = 0; k + 1 < hex.size(); k += 2) body.push_back(static_cast<char>(std::stoi(hex.substr(k, 2), nullptr, 16)));
            try {
                mp::Obj o = mp::decode(body);
                std::string out;
                render(out, o);
                mp::Encoder en;
                std::string re = "-";
                if (encode(en, o)) {
                    re.clear();
                    for (unsigned char ch : en.out) {
                        char h[3];
                        std::snprintf(h, sizeof h, "%02x", ch);
                        re += h;
                    }
                }
                std::printf("%s\t%s\n", out.c_str(), re.c_str());
            } catch (const std::exception&) {
                std::printf("error\n");
            }
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--skip-selftest") {
        // one JSON container per stdin line (trailing text allowed) -> the byte offset just past it, or -1
        static char buf[1 << 20];
        while (std::fgets(buf, sizeof buf, stdin) != nullptr) {
            std::string_view line(buf);
            while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.remove_suffix(1);
            const char* end = skip_container_text(line.data(), line.data() + line.size());
            std::printf("%lld\n", end ? static_cast<long long>(end - line.data()) : -1LL);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--calibrate") {
        // fixed work for telling box speed from code speed (bench.py's "host" block): the relayed-line scan
        // of a synthetic ~1 KB template line, a streaming fingerprint and a body render, and a crc32 loop;
        // best of 7 rounds, ns per operation
        crc_init();
        std::string spec = "{\"container\":{\"image\":\"algo\",\"registry\":\"registry.example.com\",\"versionTag\":\"v1\","
                           "\"serviceAccountName\":\"sa\"},\"computeResources\":{\"cpuLimit\":\"1000m\",\"memoryLimit\":\"2000Mi\","
                           "\"customResources\":{\"amd.com/gpu\":\"1\"}},\"command\":\"python\",\"args\":[\"main.py\",\"--x\",\"1\"],"
                           "\"runtimeEnvironment\":{\"environmentVariables\":[{\"name\":\"A\",\"value\":\"0123456789abcdef\"}],"
                           "\"mappedEnvironmentVariables\":[{\"secretRef\":{\"name\":\"algo-secret\"}},"
                           "{\"configMapRef\":{\"name\":\"algo-config\"}}],\"annotations\":{\"a\":\"b\"},"
                           "\"deadlineSeconds\":120,\"maximumRetries\":3},\"errorHandlingBehaviour\":{\"transientExitCodes\":[1,2],"
                           "\"fatalExitCodes\":[3]},\"workgroupRef\":{\"name\":\"wg\",\"group\":\"science.sneaksanddata.com\","
                           "\"kind\":\"NexusAlgorithmWorkgroup\"}}";
        std::string line = "{\"type\":\"MODIFIED\",\"object\":{\"apiVersion\":\"science.sneaksanddata.com/v1\","
                           "\"kind\":\"NexusAlgorithmTemplate\",\"metadata\":{\"name\":\"algo-00001\",\"namespace\":\"nexus\","
                           "\"uid\":\"0b7c7a54-1f1e-4c7e-9d1a-5f6c2b9e8a01\",\"resourceVersion\":\"123456\",\"generation\":7,"
                           "\"creationTimestamp\":\"2025-01-01T00:00:00Z\"},\"spec\":" + spec + ",\"status\":{\"conditions\":[]}}}";
        size_t sink = 0;
        auto best = [&](int n, const std::function<void()>& fn) {
            double b = 1e30;
            for (int rep = 0; rep < 7; ++rep) {
                double t0 = now_s();
                for (int i = 0; i < n; ++i) fn();
                b = std::min(b, now_s() - t0);
            }
            return b / n * 1e9;
        };
        double scan = best(20000, [&] {
            std::string type;
            CtlPtr c = ctl_scan(TEMPLATES, line, type);
            sink += c ? c->spec_raw.size() : 0;
        });
        double fp = best(20000, [&] { sink += fingerprint_text(spec) & 1; });
        Value head = Value::object();
        head.set("apiVersion", Value::str(kApiVersion));
        double render = best(20000, [&] { sink += dumps_with(head, {{"spec", spec}}).size(); });
        std::string kb(1024, 'x');
        double crc = best(20000, [&] { sink += crc32(kb) & 1; });
        std::printf("{\"ctl_scan_ns\": %.0f, \"fingerprint_ns\": %.0f, \"render_ns\": %.0f, \"crc32_kb_ns\": %.0f, "
                    "\"line_bytes\": %zu, \"sink\": %zu}\n", scan, fp, render, crc, line.size(), sink);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--decode-bench") {
        // relayed watch lines (one per stdin line, kind argv[2]): ns per line of the scan and of the parser path
        int kind = argc > 2 ? std::atoi(argv[2]) : TEMPLATES;
        std::vector<std::string> lines;
        static char buf[1 << 20];
        while (std::fgets(buf, sizeof buf, stdin) != nullptr) {
            std::string line(buf);
            while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
            lines.push_back(std::move(line));
        }
        if (lines.empty()) return 1;
        size_t sink = 0;
        auto run = [&](bool scan) {
            double best = 1e30;
            for (int rep = 0; rep < 5; ++rep) {
                double t0 = now_s();
                for (const auto& l : lines) {
                    std::string type;
                    CtlPtr c;
                    if (scan) {
                        c = ctl_scan(kind, l, type);
                    } else {
                        std::string_view raw[3];
                        Value o = Parser(l.data(), l.size()).parse_event_split(type, payload_keys(kind),
                                                                              payload_count(kind), raw);
                        c = make_ctl(kind, o, raw);
                    }
                    sink += c ? c->name.size() : 0;
                }
                best = std::min(best, now_s() - t0);
            }
            return best / static_cast<double>(lines.size()) * 1e9;
        };
        double dom = run(false), scan = run(true);
        std::printf("{\"lines\": %zu, \"parser_ns\": %.0f, \"scan_ns\": %.0f, \"sink\": %zu}\n", lines.size(), dom,
                    scan, sink);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "--shardobj-selftest") {
        // one JSON object per stdin line -> per kind (template, secret): whether the DOM-free scan took it, and
        // the slim fields + rest text from the scan and from the DOM path (tests/test_native_executor_json.py)
        auto fields = [](const ShardPtr& o) {
            if (!o) return std::string("-");
            std::string f = o->ns + "|" + o->name + "|" + o->uid + "|" + std::to_string(o->rv) + "|" +
                            std::to_string(o->fp_spec) + "|" + std::to_string(o->fp_data) + "|" +
                            std::to_string(o->fp_bin) + "|" + o->type + "|" + (o->has_owner_refs ? "1" : "0") + "|" +
                            std::string(o->app_label_ours ? "app" : "-") + "|" +
                            std::string(o->owner_label_ours ? "owner" : "-") + "|";
            for (const auto& t : o->template_owners) f += t.first + "/" + t.second + ",";
            f += "|";
            for (const auto& n : o->other_owner_names) f += n + ",";
            return f;
        };
        std::string line;
        std::vector<char> buf(1 << 20);
        while (std::fgets(buf.data(), static_cast<int>(buf.size()), stdin) != nullptr) {
            line.assign(buf.data());
            while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
            for (int kind : {TEMPLATES, SECRETS}) {
                if (line.rfind("{\"type\"", 0) == 0) {  // a watch event: the relayed-line scan vs make_ctl
                    std::string t1, t2;
                    CtlPtr fast, slow;
                    try {
                        fast = ctl_scan(kind, line, t1);
                    } catch (const std::exception&) {
                        std::printf("-1\t0\t-\t-\n");
                        continue;
                    }
                    try {
                        std::string_view raw[3];
                        Value o = Parser(line.data(), line.size()).parse_event_split(t2, payload_keys(kind),
                                                                                    payload_count(kind), raw);
                        if (o.is_obj()) slow = make_ctl(kind, o, raw);
                    } catch (const std::exception&) {
                    }
                    auto cf = [](const CtlPtr& o, const std::string& t) {
                        if (!o) return std::string("-");
                        std::string f = t + "|" + o->ns + "|" + o->name + "|" + o->uid + "|" + o->rv + "|" +
                                        std::to_string(o->generation) + (o->has_generation ? "g" : "") + "|" +
                                        std::to_string(o->fp_spec) + "|" + std::to_string(o->fp_data) + "|" +
                                        std::to_string(o->fp_bin) + "|" + std::to_string(o->fp_labels) + "|" +
                                        std::to_string(o->fp_ann) + "|" + o->type + "|" + o->spec_raw + "|" +
                                        o->data_raw + "|" + o->bin_raw + "|";
                        for (const auto& n : o->secrets) f += n + ",";
                        f += "|";
                        for (const auto& n : o->configmaps) f += n + ",";
                        f += "|";
                        for (const auto& n : o->owners) f += n + ",";
                        return f;
                    };
                    std::string a = cf(fast, t1), b = cf(slow, t2);
                    std::printf("%d\t%d\t-\t-\n", fast ? 1 : 0, a == b ? 1 : 0);
                    continue;
                }
                ShardPtr fast = shard_obj_scan(kind, line);
                ShardPtr slow;
                try {
                    std::string_view raw[3];
                    Value rest = Parser(line.data(), line.size()).parse_split(payload_keys(kind), payload_count(kind), raw);
                    slow = make_shard_obj(kind, std::move(rest), raw);
                } catch (const std::exception&) {
                }
                std::string a = fields(fast), b = fields(slow);
                std::printf("%d\t%d\t%s\t%s\n", fast ? 1 : 0, a == b ? 1 : 0, fast ? fast->rest.c_str() : "-",
                            slow ? slow->rest.c_str() : "-");
            }
        }
        return 0;
    }
    if (fd < 0) {
        std::fprintf(stderr, "usage: ncc-executor --fd N --index I --part p/k\n");
        return 2;
    }
    crc_init();
    {  // soft RLIMIT_NOFILE up to the hard limit (256 connections per shard plus watch streams), as Go does
        struct rlimit rl;
        if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur < rl.rlim_max) {
            rl.rlim_cur = rl.rlim_max == RLIM_INFINITY ? (1u << 20) : std::min<rlim_t>(rl.rlim_max, 1u << 20);
            setrlimit(RLIMIT_NOFILE, &rl);
        }
    }
    if (const char* h = std::getenv("NCC_DEPENDENT_HOLD")) kDependentHold = std::max(1.0, std::atof(h));
    if (const char* f = std::getenv("NCC_REPORT_FLUSH_MS")) g_flush_interval = std::max(0.0, std::atof(f) / 1000.0);
    g_phases_on = std::getenv("NCC_CPU_REPORT") != nullptr;
    start_sampling();
    if (std::getenv("NCC_TRACE_STAGES") != nullptr) {
        g_trace = new std::vector<TraceRec>();
        g_trace->reserve(1 << 20);
    }
    const char* gated = std::getenv("NCC_GATED");
    g_opt.gated = gated != nullptr && std::string(gated) == "1";
    ::signal(SIGPIPE, SIG_IGN);
    Loop lp;
    g_loop = &lp;
    Executor ex;
    g_ex = &ex;
    if (pipe2(g_sigpipe, O_NONBLOCK | O_CLOEXEC) == 0) {
        lp.add_fd(g_sigpipe[0]);
        ::signal(SIGTERM, on_signal);
        ::signal(SIGINT, on_signal);
        spawn(signal_watch(), "signals");
    }
    Channel chan(fd);
    g_chan = &chan;
    spawn(shutdown_watch(), "shutdown");
    spawn(run_main(), "main");
    try {
        lp.run();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ncc-executor: fatal: %s\n", e.what());
        return 1;
    }
    dump_samples();
    std::fflush(stderr);
#ifdef NCC_GPROF
    _mcleanup();  // profiling builds (-pg): write gmon.out before skipping the exit handlers
#endif
#ifdef NCC_COVERAGE
    __gcov_dump();  // coverage builds: write the .gcda counters before skipping the exit handlers
#endif
    std::_Exit(0);  // skip destructors of still-suspended coroutines
}
