"""Wire-level constants of the Nexus configuration-sync contract.

Every value here is part of the observable contract with the reference controller
(SneaksAndData/nexus-configuration-controller) and with the `nexus-core` CRD module it
consumes, so a cluster managed by the reference can be taken over by this framework
without any object being rewritten.

Citations (reference snapshot, /root/reference):
  * metric names            controller.go:50-56
  * agent / field manager   controller.go:58,83
  * event reasons/messages  controller.go:60-81
  * queue kinds             controller.go:93-96
  * owner labels            controller_test.go:183-188 (nexus-core shards.OwnerLabels)
  * group/version/plurals   .helm/templates/cluster-role-template-editor.yaml:25-36
"""
import functools

GROUP = "science.sneaksanddata.com"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"

TEMPLATE_KIND = "NexusAlgorithmTemplate"
WORKGROUP_KIND = "NexusAlgorithmWorkgroup"
TEMPLATE_PLURAL = "nexusalgorithmtemplates"
WORKGROUP_PLURAL = "nexusalgorithmworkgroups"

# controller.go:58 — also used as the Event source component and the field manager.
CONTROLLER_AGENT_NAME = "nexus-configuration-controller"
FIELD_MANAGER = CONTROLLER_AGENT_NAME

# statsd metric names, controller.go:50-56; namespace from main.go:44
METRIC_NAMESPACE = "nexus_configuration_controller"
RECONCILE_LATENCY_METRIC = "reconcile_latency"
WORKQUEUE_LENGTH_METRIC = "workqueue_length"
# native-mode operational metrics (not in the reference)
RECONCILE_ERRORS_METRIC = "reconcile_errors"          # count, tag kind
SHARD_SYNC_ERRORS_METRIC = "shard_sync_errors"        # count, tag shard (coordinator, from executor reports)
SHARDS_METRIC = "shards"                              # gauge: shards served
LEADER_METRIC = "leader"                              # gauge 1/0 when leader election is on
EXECUTOR_NATIVE_METRIC = "executor_native"            # gauge 1: the C++ shard executors run, 0: the Python ones
SHARD_FAILING_METRIC = "shard_failing_objects"        # gauge, tag shard: templates whose last sync there failed
# the C++ executors' shard clients (their status messages, native/executor/http.hpp), gauges tagged shard:
SHARD_CLIENT_METRICS = {"limit": "shard_client_inflight_limit",      # adaptive concurrency limit (AIMD)
                        "cap": "shard_client_inflight_cap",          # the most the limit may reach (pool; HTTP/2 cap)
                        "inflight": "shard_client_inflight",         # requests in flight
                        "rejected_429": "shard_client_throttled",    # 429s received (cumulative)
                        "connections": "shard_client_connections",   # open connections
                        "http2": "shard_client_http2",               # 1 when the shard is spoken to over HTTP/2
                        "h2_dead": "shard_client_dead_connections",  # connections dropped for an unanswered PING
                        "h2_goaway_errors": "shard_client_goaway_errors",  # GOAWAYs with an error code
                        "h2_downgraded": "shard_client_http2_downgraded"}  # 1: HTTP_1_1_REQUIRED moved it to HTTP/1.1

# Event reasons, controller.go:60-70
SUCCESS_SYNCED = "Synced"
ERR_RESOURCE_EXISTS = "ErrResourceExists"
ERR_RESOURCE_MISSING = "ErrResourceMissing"
ERR_RESOURCE_SYNC_ERROR = "ErrResourceSyncError"

# Event message formats, controller.go:72-81.  Go's %q is rendered by `go_quote`.
MESSAGE_RESOURCE_EXISTS = "Resource {0} already exists and is not managed by any Machine Learning Algorithm"
MESSAGE_RESOURCE_SYNCED = "Resource of type {0} synced successfully"
MESSAGE_RESOURCE_MISSING = "Resource {0} referenced by NexusAlgorithmTemplate {1} is missing in the controller cluster"
MESSAGE_RESOURCE_OPERATION_FAILED = (
    "Synchronization/update of a resource {0} referenced by NexusAlgorithmTemplate {1} failed with a fatal error {2}"
)

EVENT_TYPE_NORMAL = "Normal"
EVENT_TYPE_WARNING = "Warning"

# Queue element kinds, controller.go:93-96
KIND_TEMPLATE = "template"
KIND_WORKGROUP = "workgroup"

# Labels stamped on every object created in a shard (nexus-core shards.OwnerLabels).
LABEL_CONTROLLER_APP = f"{GROUP}/controller-app"
LABEL_CONFIGURATION_OWNER = f"{GROUP}/configuration-owner"

# Status condition (nexus-core v1.NewResourceReadyCondition).  The Reason string of the
# upstream helper is not visible from the reference; "ResourceReady" is a documented
# assumption and only matters for display.
CONDITION_READY = "Ready"
CONDITION_READY_REASON = "ResourceReady"
CONDITION_TRUE = "True"
CONDITION_FALSE = "False"


@functools.lru_cache(maxsize=65536)
def go_quote(s: str) -> str:
    """Render a string the way Go's fmt `%q` verb does for printable ASCII input (memoised: status and
    Event messages quote the same object names on every pass)."""
    out = ['"']
    for ch in s:
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\r":
            out.append("\\r")
        elif ord(ch) < 0x20 or ord(ch) == 0x7F:
            out.append("\\x%02x" % ord(ch))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def owner_labels(alias: str) -> dict:
    """Labels nexus-core stamps on shard objects it creates (controller_test.go:183-188)."""
    return {
        LABEL_CONTROLLER_APP: CONTROLLER_AGENT_NAME,
        LABEL_CONFIGURATION_OWNER: alias,
    }


# kubectl's client-side-apply record: never copied to shard dependents (`sync-dependent-metadata`)
LAST_APPLIED_ANNOTATION = "kubectl.kubernetes.io/last-applied-configuration"
# on a shard dependent with `sync-dependent-metadata`: which of its label/annotation keys came from the source,
# so a key removed at the source is removed from the copy, and keys others add to the copy are left alone
SYNCED_METADATA_ANNOTATION = "science.sneaksanddata.com/synced-metadata"


def synced_metadata_value(labels, annotations) -> str:
    return f"labels={','.join(sorted(labels))};annotations={','.join(sorted(annotations))}"


def parse_synced_metadata(value) -> tuple[set, set]:
    """(label keys, annotation keys) named by a SYNCED_METADATA_ANNOTATION value (empty sets if absent)."""
    out = {"labels": set(), "annotations": set()}
    for part in (value or "").split(";"):
        k, _, v = part.partition("=")
        if k in out and v:
            out[k] = set(v.split(","))
    return out["labels"], out["annotations"]


def merge_synced_metadata(have: dict, want: dict, previous: set) -> dict:
    """A copy's labels/annotations after a sync: keys we synced before and the source no longer has are
    dropped, the desired ones set, everything else (added on the shard by others) kept."""
    out = {k: v for k, v in (have or {}).items() if k not in previous}
    out.update(want)
    return out
