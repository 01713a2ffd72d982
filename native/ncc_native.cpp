// ncc._native — C++ runtime primitives for the Nexus configuration controller.
//
// The reference controller gets its hot runtime pieces from compiled client-go:
// the rate-limited exclusive-key work queue (k8s.io/client-go/util/workqueue, used at
// controller.go:257-260,280) and reflect.DeepEqual for drift checks (controller.go:539,600,725,795).
// This module provides MI355X-host-native equivalents for the asyncio control plane:
//
//  * RateLimitingQueue — dedup (dirty set) + per-key exclusivity (processing set) + delayed
//    re-adds (min-heap, earliest ready time wins) + MaxOf(ItemExponentialFailure(base, max),
//    Bucket(qps, burst)) rate limiting.  Time is passed in explicitly (seconds, monotonic) so
//    the Python reference implementation (ncc/workqueue/core.py) can be driven in lock-step by
//    property tests.  All methods take an internal mutex, so shard-executor threads may share it.
//  * fingerprint(obj) — 64-bit structural digest of a JSON-shaped Python value (dict keys sorted,
//    type-tagged scalars) computed by walking the CPython objects directly, ~10x cheaper than
//    canonical json.dumps + hashing; used for O(1) drift detection on slim shard caches.
//  * fingerprint_many(list) — batch form (one call per informer relist page).
//  * scan_event(bytes) — reads type/namespace/name/resourceVersion out of a raw watch-event line
//    without materialising the object, so informers can recognise echoes of their own writes.
//  * scan_event_owners(bytes) — the same plus ownerReferences names/uids, so a key-partitioned
//    executor can drop dependents owned only by another partition's templates without decoding them.
//  * scan_event_part(bytes, parts, ns) — the same plus the crc32 key partition of the object and the
//    bitmask of its owners' partitions, so the partition test itself builds no Python strings.
//  * parse_response_head(bytes) — HTTP/1.1 response heads for the client transport.
//  * H2ClientParser / h2_request / hpack_encode — HTTP/2 framing and HPACK for the Python clients.
//
// The code is split by concern into native/ext/*.hpp (hashing, workqueue, scan, http1, pyjson, reports,
// h2client, sampler), included in that order below; this file holds the bindings.
//
// The fake apiserver's native pieces (its HTTP/1.1 request-head parser, HTTP/2 server parser and response
// encoder) are not here: they are test substrate, built into ncc/fakeapi/_native from native/fakeapi/
//  — the product extension carries no server code.
//  * owner_filter(lines, items, assumed, ns) — the metadata-only informer's owner filter over a batch;
//    OwnerFilter — the same with a memo per informer (no Python object built for a dropped line).
//  * relay_index(lines, raw, ns) — the one-partition watch relay's index-and-forward loop; RelayIndex — the
//    same with a memo of the key tuples.
//  * chunk_lines(bytearray, state, bytearray) — a chunked watch body cut into its event lines in one call.
//  * scan_object(bytes) — namespace/name/resourceVersion/uid of a write response, so a slim-cache
//    writer can publish its write without decoding the echoed object.
//  * dumps(obj) — compact JSON encoder for request bodies and the fake apiserver's responses.
//  * members_equal(a, b, keys) — byte equality of named top-level members of two JSON objects, so a
//    slim-cache writer sees whether the server rewrote its payload without decoding the response.
//  * loads(bytes) — JSON decoder straight into CPython objects.
//  * template_event_slim(line) — a template watch line decoded into the coordinator's slim form
//    (metadata without managedFields, status, and a spec reduced to its references + raw digest).
//  * ReportTable — the coordinator's fold of shard-executor reports, fed raw IPC frames.

#include "common/byte_scan.hpp"
#include "common/hpack.hpp"

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <Python.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

#define NCC_NATIVE_ABI 33

namespace {
#include "ext/hashing.hpp"
#include "ext/workqueue.hpp"
#include "ext/scan.hpp"
#include "ext/http1.hpp"
#include "ext/pyjson.hpp"
#include "ext/reports.hpp"
#include "ext/h2client.hpp"
#include "ext/sampler.hpp"
}  // namespace

PYBIND11_MODULE(_native, m) {
    m.doc() = "ncc native runtime: rate-limited work queue + structural fingerprints";
    m.attr("ABI_VERSION") = NCC_NATIVE_ABI;
    m.def("fingerprint", &fingerprint, py::arg("obj"), "64-bit structural digest of a JSON-shaped value");
    m.def("fingerprint_many", &fingerprint_many, py::arg("objs"));
    m.def("scan_event", &scan_event, py::arg("line"),
          "(type, namespace, name, resourceVersion) of a watch-event line, or None");
    m.def("dumps", &dumps, py::arg("obj"), "compact JSON bytes of a JSON-shaped value (UTF-8, key order kept)");
    m.def("scan_object", &scan_object, py::arg("body"),
          "(namespace, name, resourceVersion, uid) from an object's metadata without decoding it, or None");
    m.def("scan_event_part", &scan_event_part, py::arg("line"), py::arg("parts"), py::arg("default_ns"),
          "scan_event_owners plus the key partition and the owner-partition bitmask (crc32 % parts)");
    m.def("parse_response_head", &parse_response_head, py::arg("head"),
          "(status, content_length|-1, chunked, connection_close, retry_after|None) of an HTTP/1.1 response head");
    m.def("chunk_lines", &chunk_lines, py::arg("buf"), py::arg("state"), py::arg("linebuf"),
          "complete event lines of a chunked watch body (see the comment at the definition)");
    m.def("relay_scan", &relay_scan, py::arg("line"), py::arg("parts"), py::arg("default_ns"),
          "(type_code, namespace, name, key_partition, owner_partition_mask, n_owners) of a watch line");
    m.def("owner_filter", &owner_filter, py::arg("lines"), py::arg("items"), py::arg("assumed"),
          py::arg("default_ns"), "the metadata-only informer's owner filter over a batch of watch lines");
    py::class_<OwnerFilter>(m, "OwnerFilter")
        .def(py::init<>())
        .def("__call__", &OwnerFilter::call, py::arg("lines"), py::arg("items"), py::arg("assumed"),
             py::arg("default_ns"), "owner_filter over a batch, memoising keys, cached objects and their owners")
        .def("clear", &OwnerFilter::clear)
        .def("__len__", &OwnerFilter::size);
    m.def("relay_index", &relay_index, py::arg("lines"), py::arg("raw"), py::arg("default_ns"),
          "the one-partition relay loop: index the lines in `raw`, return the object events to forward");
    py::class_<RelayIndex>(m, "RelayIndex")
        .def(py::init<>())
        .def("__call__", &RelayIndex::call, py::arg("lines"), py::arg("raw"), py::arg("default_ns"),
             "relay_index over a batch, memoising the key tuples")
        .def("clear", &RelayIndex::clear)
        .def("__len__", &RelayIndex::size);
    m.def("native_sample_start", &native_sample_start, py::arg("us"),
          "sample the interrupted instruction on every SIGPROF (NCC_NATIVE_SAMPLE; ncc/sampler.py)");
    m.def("native_sample_dump", &native_sample_dump, py::arg("path"), "write the samples; returns their count");
    m.def("key_partition", &key_partition, py::arg("namespace"), py::arg("name"), py::arg("parts"));
    m.def("members_equal", &members_equal, py::arg("a"), py::arg("b"), py::arg("keys"),
          "True iff the named top-level members of two JSON objects are byte-identical (or both absent)");
    m.def("loads", &loads, py::arg("data"), "JSON bytes -> Python value, or None when malformed");
    m.def("template_index_same", &template_index_same, py::arg("old"), py::arg("new"),
          "the template indices read the same in both versions (namespace and references)");
    m.def("template_event_slim", &template_event_slim, py::arg("line"), py::arg("items") = py::none(),
          py::arg("default_ns") = std::string(),
          "template watch line -> (type, object with metadata/status decoded and the spec slimmed) | None; "
          "with `items` (the store's dict) an unchanged status or reference list is taken from the cached version");
    m.def("scan_event_owners", &scan_event_owners, py::arg("line"),
          "scan_event plus the tuples of metadata.ownerReferences[*].name and [*].uid, or None");
    py::class_<H2ClientParser>(m, "H2ClientParser")
        .def(py::init<>())
        .def_static("preface", &H2ClientParser::preface)
        .def("watch", &H2ClientParser::watch, py::arg("sid"))
        .def("forget", &H2ClientParser::forget, py::arg("sid"))
        .def("feed", &H2ClientParser::feed, py::arg("data"))
        .def("open_streams", &H2ClientParser::open_streams);
    m.def("h2_request", &h2_request, py::arg("sid"), py::arg("method"), py::arg("path"), py::arg("fixed"),
          py::arg("content_length"), py::arg("body"), py::arg("end"), py::arg("max_frame"),
          "the HEADERS (and DATA) frames of an HTTP/2 request");
    m.def("hpack_encode", &hpack_encode, py::arg("fields"), py::arg("huffman") = false,
          "a header block of static-table fields and literals without indexing");
    m.def("hpack_huffman_encode", [](const py::bytes& s) { return py::bytes(ncc::hpack::huffman_encode(std::string_view(s))); },
          py::arg("data"));
    m.def("hpack_huffman_decode", &hpack_huffman_decode, py::arg("data"));
    py::class_<RateLimitingQueue>(m, "RateLimitingQueue")
        .def(py::init<double, double, double, int>(), py::arg("base_delay"), py::arg("max_delay"), py::arg("qps"),
             py::arg("burst"))
        .def("add", &RateLimitingQueue::add)
        .def("try_get", &RateLimitingQueue::try_get)
        .def("done", &RateLimitingQueue::done)
        .def("length", &RateLimitingQueue::length)
        .def("__len__", &RateLimitingQueue::length)
        .def("processing", &RateLimitingQueue::processing)
        .def("shutdown", &RateLimitingQueue::shutdown)
        .def("shutting_down", &RateLimitingQueue::shutting_down)
        .def("add_after", &RateLimitingQueue::add_after)
        .def("promote", &RateLimitingQueue::promote)
        .def("next_ready_in", &RateLimitingQueue::next_ready_in)
        .def("waiting", &RateLimitingQueue::waiting)
        .def("busy", &RateLimitingQueue::busy)
        .def("add_rate_limited", &RateLimitingQueue::add_rate_limited)
        .def("forget", &RateLimitingQueue::forget)
        .def("num_requeues", &RateLimitingQueue::num_requeues);
    py::class_<ReportTable>(m, "ReportTable")
        .def(py::init<>())
        .def("set_shards", &ReportTable::set_shards, py::arg("shards"))
        .def("shards", &ReportTable::shards)
        .def("feed", &ReportTable::feed, py::arg("body"), py::arg("batch"),
             "fold a raw executor IPC frame: (complete keys, wrote keys, failing shards, other messages, "
             "reports, pending)")
        .def("feed_stream", &ReportTable::feed_stream, py::arg("buffer"), py::arg("start"),
             "fold every complete frame of a byte stream from `start`: feed()'s tuple + the end offset")
        .def("readiness", &ReportTable::readiness, py::arg("key"), py::arg("uid"), py::arg("generation"))
        .def("ready_ok", &ReportTable::ready_ok, py::arg("key"), py::arg("uid"), py::arg("generation"))
        .def("template_update", &ReportTable::template_update, py::arg("old"), py::arg("new"), py::arg("adopted"),
             py::arg("generation_filter"), py::arg("same_references"))
        .def("finish_batch", &ReportTable::finish_batch, py::arg("keys"), py::arg("items"), py::arg("assumed"),
             py::arg("adopted"), py::arg("memos"), py::arg("shards"), py::arg("queue"), py::arg("pending_event"),
             py::arg("event_on_noop"))
        .def("pop", &ReportTable::pop, py::arg("key"))
        .def("set_partition", &ReportTable::set_partition, py::arg("part"), py::arg("parts"))
        .def("take_forwards", &ReportTable::take_forwards)
        .def("drop_shards", &ReportTable::drop_shards, py::arg("names"))
        .def("__len__", &ReportTable::size);
}
