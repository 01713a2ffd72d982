"""Typed per-shard failures: what a shard pass reports, and the Events and status text derived from it.

The reference reconciles every shard in the controller process and records its Warning Events right where a
write fails (`/root/reference/controller.go:497` ErrResourceExists for a rogue shard dependent; `:525,533,546,557`
and the ConfigMap twin `:587-619` ErrResourceSyncError with `MessageResourceOperationFailed`, `:81`).  In the
native topology the shard writes happen in executor processes (Python `ncc.executor` or the C++
`ncc-executor`), which never write to the controller cluster.  So each executor puts a *typed* failure per
shard into its report (`{"t": "report", ..., "r": {shard: None | failure}}`), and the coordinator turns it
into the same Events and into the `Ready=False` status message.  The in-process path (role "all") records
its Events inline and uses the same status text, so all three implementations say the same thing.

A failure is a small dict (msgpack map on the wire), one letter per field:
  c  class: RogueResourceError, ReferenceMissing, ShardNotReadyError, TransportError, or the API error
     reason class (NotFound, Conflict, AlreadyExists, Forbidden, Invalid, ServiceUnavailable, ApiError...)
  k  kind of the object the failing step wrote: NexusAlgorithmTemplate, NexusAlgorithmWorkgroup, Secret,
     ConfigMap ("" when the step is not tied to one object, e.g. a shard whose caches have not synced)
  n  that object's name ("" likewise)
  h  HTTP status code of the failing request (0: no HTTP answer, or not an API error)
  m  the error text (what the reference formats with %s)
"""
from __future__ import annotations

from ..api import constants as C
from ..api.constants import go_quote as q
from ..kube import errors as E

MAX_MESSAGE = 500  # per failure, as the report strings were capped before
MAX_STATUS_DETAIL = 400  # the reason part of a Ready=False message

ROGUE = "RogueResourceError"
REFERENCE_MISSING = "ReferenceMissing"
DEPENDENT_KINDS = ("Secret", "ConfigMap")


def mark(e: BaseException, kind: str, name: str, cls: str | None = None) -> BaseException:
    """Tag an exception with the object whose step failed (and optionally its class); returns `e`."""
    try:
        e.ncc_object = (kind, name)
        if cls is not None:
            e.ncc_class = cls
    except AttributeError:  # pragma: no cover - exceptions with __slots__
        pass
    return e


def from_exception(e: BaseException, kind: str = "", name: str = "") -> dict:
    """The typed failure of an exception raised by a shard step (`kind`/`name`: default object)."""
    obj = getattr(e, "ncc_object", None)
    if obj is not None:
        kind, name = obj
    cls = getattr(e, "ncc_class", None)
    if cls is None:
        if isinstance(e, E.TransportError):
            cls = "TransportError"
        elif isinstance(e, E.ApiError):
            cls = type(e).__name__ if type(e) is not E.ApiError else "ApiError"
        else:
            cls = type(e).__name__
    code = int(getattr(e, "code", 0) or 0) if isinstance(e, E.ApiError) else 0
    msg = e.message if isinstance(e, E.ApiError) else str(e)
    return {"c": cls, "k": kind, "n": name, "h": code, "m": msg[:MAX_MESSAGE]}


def normalize(f) -> dict | None:
    """A reported per-shard result as a failure dict (None: success).  Free-form strings (older executors,
    tests) become class "Error"."""
    if not f:
        return None
    if isinstance(f, dict):
        return {"c": str(f.get("c") or "Error"), "k": str(f.get("k") or ""), "n": str(f.get("n") or ""),
                "h": int(f.get("h") or 0), "m": str(f.get("m") or "")}
    return {"c": "Error", "k": "", "n": "", "h": 0, "m": str(f)}


def summary(f: dict) -> str:
    """One line: `Secret "s0": RogueResourceError: Resource "s0" already exists ...`."""
    where = f"{f['k']} {q(f['n'])}: " if f.get("k") and f.get("n") else ""
    return f"{where}{f['c']}: {f['m']}"


def status_message(what: str, failures: dict) -> str:
    """`<what> failed to sync to shards: a, b (a: <first reason>)` — the failing shards in order, then the
    first one's reason, truncated, so an operator can tell a rogue Secret from a 403 or a 5xx."""
    names = sorted(failures)
    msg = f"{what} failed to sync to shards: {', '.join(names)}"
    first = normalize(failures[names[0]]) if names else None
    if first is not None:
        detail = f"{names[0]}: {summary(first)}"
        if len(detail) > MAX_STATUS_DETAIL:
            detail = detail[:MAX_STATUS_DETAIL - 3] + "..."
        msg += f" ({detail})"
    return msg


def events(f: dict, template_name: str, shard: str) -> list[tuple[str, str, str]]:
    """(type, reason, message) of the Warning Events the in-process reconcile records for this failure on a
    template (`_sync_dependent` / `is_missing_ownership` with native options):
      rogue shard dependent   ErrResourceExists naming kind and shard, then ErrResourceSyncError;
      other dependent failure ErrResourceSyncError with MessageResourceOperationFailed.
    A missing reference is reported by the coordinator's own adoption pass (ErrResourceMissing, from its
    cache, which is the authority); an executor that has not received the object yet is not an error to
    announce.  Template/workgroup write failures record no Event in the reference either (`:795-831`)."""
    kind, name = f.get("k", ""), f.get("n", "")
    if kind not in DEPENDENT_KINDS or not name or f["c"] in (REFERENCE_MISSING, "ShardNotReadyError"):
        return []
    out = []
    if f["c"] == ROGUE:
        out.append((C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_EXISTS,
                    f"{kind} {C.MESSAGE_RESOURCE_EXISTS.format(q(name))} (shard {q(shard)})"))
    out.append((C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_SYNC_ERROR,
                C.MESSAGE_RESOURCE_OPERATION_FAILED.format(q(name), q(template_name), f["m"])))
    return out


def signature(f: dict) -> tuple:
    """What makes two reports of a failure the same one (for Event de-duplication across retries)."""
    return f["c"], f["k"], f["n"], f["h"], f["m"]
