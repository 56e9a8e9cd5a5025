"""Exception classes named after the TensorFlow error classes the reference raises.

The reference reports every failure on this path as a TF Status (OP_REQUIRES_OK with
errors::InvalidArgument / Aborted / ResourceExhausted / ... , e.g.
efls-train/cc/efl/math/fixed_point.cc:230-232, paillier.cc:497-499,550-552, communicator_ops.cc:86).
Callers written against the reference catch `tf.errors.<Name>Error`; the build raises the
same-named classes, carrying the same numeric code (error_codes.proto).
"""
from __future__ import annotations


class OpError(Exception):
    code = 2  # UNKNOWN

    def __init__(self, message: str = "", code: int | None = None):
        super().__init__(message)
        self.message = message
        if code is not None:
            self.code = code


class CancelledError(OpError):
    code = 1


class UnknownError(OpError):
    code = 2


class InvalidArgumentError(OpError, ValueError):
    code = 3


class DeadlineExceededError(OpError):
    code = 4


class NotFoundError(OpError):
    code = 5


class AlreadyExistsError(OpError):
    code = 6


class PermissionDeniedError(OpError):
    code = 7


class ResourceExhaustedError(OpError):
    code = 8


class FailedPreconditionError(OpError):
    code = 9


class AbortedError(OpError):
    code = 10


class OutOfRangeError(OpError):
    code = 11


class UnimplementedError(OpError):
    code = 12


class InternalError(OpError):
    code = 13


class UnavailableError(OpError):
    code = 14


class DataLossError(OpError):
    code = 15


_BY_CODE = {c.code: c for c in (CancelledError, UnknownError, InvalidArgumentError,
                                 DeadlineExceededError, NotFoundError, AlreadyExistsError,
                                 PermissionDeniedError, ResourceExhaustedError,
                                 FailedPreconditionError, AbortedError, OutOfRangeError,
                                 UnimplementedError, InternalError, UnavailableError,
                                 DataLossError)}


def from_code(code: int, message: str = "") -> OpError:
    """TF error code (positive, error_codes.proto) -> exception instance."""
    cls = _BY_CODE.get(abs(int(code)), UnknownError)
    return cls(message, abs(int(code)))
