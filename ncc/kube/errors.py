"""Typed API errors mirroring k8s.io/apimachinery/pkg/api/errors.

Both the HTTP client and the in-memory fake raise these, so reconcile code can branch on
`NotFound` / `AlreadyExists` / `Conflict` exactly like `k8serrors.IsNotFound(err)` in the
reference (controller.go:509,518,705,769,805).
"""
from __future__ import annotations


class ApiError(Exception):
    code = 500
    reason = "InternalError"

    def __init__(self, message: str = "", *, code: int | None = None, reason: str | None = None,
                 details: dict | None = None, retry_after: float | None = None):
        super().__init__(message or self.reason)
        self.message = message or self.reason
        if code is not None:
            self.code = code
        if reason is not None:
            self.reason = reason
        self.details = details or {}
        self.retry_after = retry_after

    def status_object(self) -> dict:
        """Render as a metav1.Status (what an apiserver returns on failure)."""
        return {
            "kind": "Status",
            "apiVersion": "v1",
            "metadata": {},
            "status": "Failure",
            "message": self.message,
            "reason": self.reason,
            "details": self.details,
            "code": self.code,
        }

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.code} {self.reason}: {self.message})"


class BadRequest(ApiError):
    code, reason = 400, "BadRequest"


class Unauthorized(ApiError):
    code, reason = 401, "Unauthorized"


class Forbidden(ApiError):
    code, reason = 403, "Forbidden"


class NotFound(ApiError):
    code, reason = 404, "NotFound"


class MethodNotAllowed(ApiError):
    code, reason = 405, "MethodNotAllowed"


class AlreadyExists(ApiError):
    code, reason = 409, "AlreadyExists"


class Conflict(ApiError):
    code, reason = 409, "Conflict"


class Gone(ApiError):
    code, reason = 410, "Expired"


class Invalid(ApiError):
    code, reason = 422, "Invalid"


class TooManyRequests(ApiError):
    code, reason = 429, "TooManyRequests"


class InternalError(ApiError):
    code, reason = 500, "InternalError"


class ServiceUnavailable(ApiError):
    code, reason = 503, "ServiceUnavailable"


class Timeout(ApiError):
    code, reason = 504, "Timeout"


class TransportError(ApiError):
    """Connection refused / reset / TLS failure — no HTTP response at all."""
    code, reason = 0, "TransportError"


_BY_REASON = {c.reason: c for c in (BadRequest, Unauthorized, Forbidden, NotFound, MethodNotAllowed, AlreadyExists,
                                     Conflict, Gone, Invalid, TooManyRequests, InternalError, ServiceUnavailable,
                                     Timeout)}
_BY_CODE = {400: BadRequest, 401: Unauthorized, 403: Forbidden, 404: NotFound, 405: MethodNotAllowed,
            409: Conflict, 410: Gone, 422: Invalid, 429: TooManyRequests, 500: InternalError,
            503: ServiceUnavailable, 504: Timeout}


def from_status(code: int, status: dict | None, fallback_message: str = "") -> ApiError:
    """Build a typed error from an HTTP status code and an optional metav1.Status body."""
    status = status or {}
    reason = status.get("reason") or ""
    message = status.get("message") or fallback_message or f"HTTP {code}"
    cls = _BY_REASON.get(reason)
    if cls is None or (cls.code != code and code):
        cls = _BY_CODE.get(code, ApiError)
        if code == 409 and reason == "AlreadyExists":
            cls = AlreadyExists
    return cls(message, code=code or cls.code, reason=reason or cls.reason, details=status.get("details"))


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, NotFound)


def is_already_exists(e: BaseException) -> bool:
    return isinstance(e, AlreadyExists)


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, Conflict)


def is_gone(e: BaseException) -> bool:
    return isinstance(e, Gone) or (isinstance(e, ApiError) and e.code == 410)


def is_retriable(e: BaseException) -> bool:
    """Transient errors worth a quick client-side retry (throttling, 5xx, transport)."""
    if isinstance(e, (TooManyRequests, ServiceUnavailable, Timeout, TransportError, InternalError)):
        return True
    return isinstance(e, ApiError) and e.code >= 500
