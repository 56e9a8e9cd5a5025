"""Byte-level codec of the reference's cross-silo wire format (no protoc needed).

efls-train/protos/trainer_service.proto:13-22
    message MessageRequest  { string name = 1; uint64 step = 2; tensorflow.TensorProto tensor = 3; }
    message MessageResponse { tensorflow.error.Code code = 1; string msg = 2; }
third_party/tensorflow/tensorflow/core/framework/tensor.proto:15-64, tensor_shape.proto
    TensorProto { DataType dtype = 1; TensorShapeProto tensor_shape = 2; int32 version_number = 3;
                  bytes tensor_content = 4; repeated float float_val = 5 [packed]; ... }
    TensorShapeProto { repeated Dim dim = 2; bool unknown_rank = 3; }  Dim { int64 size = 1; string name = 2; }

The sender side writes what TF's Tensor::AsProtoTensorContent writes (communication_client.cc:41-42:
AsProtoField is overwritten, tensor_content wins): dtype, shape, raw little-endian bytes in
tensor_content (DT_STRING: varint32 lengths then bytes). The receiver accepts tensor_content or
the typed repeated *_val fields (TF's Tensor::FromProto semantics, last value repeated).
Large payloads are never re-encoded: the request is assembled from memoryview parts and the
received content is returned as a zero-copy memoryview.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT16, DT_INT8, DT_STRING = 1, 2, 3, 4, 5, 6, 7
DT_INT64, DT_BOOL = 9, 10
NP_OF_DT = {DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32, DT_UINT8: np.uint8,
            DT_INT16: np.int16, DT_INT8: np.int8, DT_INT64: np.int64, DT_BOOL: np.bool_}
DT_OF_NP = {np.dtype(v): k for k, v in NP_OF_DT.items()}

_VARINT, _I64, _LEN, _I32 = 0, 1, 2, 5


def varint(n: int) -> bytes:
    if n < 0:
        n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(buf, pos: int):
    result, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b < 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def key(field: int, wt: int) -> bytes:
    return varint((field << 3) | wt)


def _len_field(field: int, payload_len: int) -> bytes:
    return key(field, _LEN) + varint(payload_len)


def iter_fields(buf, start: int = 0, end: int | None = None):
    """Yield (field, wire_type, value, start, end) over a protobuf message; LEN values are
    (start, end) offsets so payloads are never copied."""
    pos = start
    end = len(buf) if end is None else end
    while pos < end:
        k, pos = read_varint(buf, pos)
        field, wt = k >> 3, k & 7
        if wt == _VARINT:
            v, pos = read_varint(buf, pos)
            yield field, wt, v, None, None
        elif wt == _I64:
            yield field, wt, bytes(buf[pos:pos + 8]), None, None
            pos += 8
        elif wt == _I32:
            yield field, wt, bytes(buf[pos:pos + 4]), None, None
            pos += 4
        elif wt == _LEN:
            n, pos = read_varint(buf, pos)
            yield field, wt, None, pos, pos + n
            pos += n
        else:
            raise ValueError(f"unsupported wire type {wt}")


# ----------------------------------------------------------------------------- TensorProto

def shape_proto(shape) -> bytes:
    out = bytearray()
    for d in shape:
        dim = key(1, _VARINT) + varint(int(d)) if int(d) != 0 else b""
        out += _len_field(2, len(dim)) + dim
    return bytes(out)


def _nbytes(piece) -> int:
    """Size of a payload piece: a bytes-like, or a contiguous uint8 torch tensor (e.g. text that
    still lives in device memory)."""
    if hasattr(piece, "is_cuda") and hasattr(piece, "numel"):
        return int(piece.numel())
    return memoryview(piece).nbytes


def tensor_proto_parts(dtype: int, shape, content) -> list:
    """Parts of a serialized TensorProto (content = bytes-like, or a tuple/list of bytes-likes /
    uint8 torch tensors that together form tensor_content; not copied)."""
    sp = shape_proto(shape)
    parts = [key(1, _VARINT) + varint(dtype), _len_field(2, len(sp)) + sp]
    pieces = list(content) if isinstance(content, (tuple, list)) else [content]
    n = sum(_nbytes(c) for c in pieces)
    if n:
        parts.append(_len_field(4, n))
        parts.extend(pieces)
    return parts


_bytes_new = ctypes.pythonapi.PyBytes_FromStringAndSize
_bytes_new.restype = ctypes.py_object
_bytes_new.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_bytes_addr = ctypes.pythonapi.PyBytes_AsString
_bytes_addr.restype = ctypes.c_void_p
_bytes_addr.argtypes = [ctypes.py_object]


def _assemble(parts, total: int) -> bytes:
    """One new `bytes` of `total` bytes filled with the parts in order — created uninitialised
    through the C API (PyBytes_FromStringAndSize(NULL, n), then written before anything else sees
    it, the documented way to build a bytes object in place), so each payload is copied exactly once
    into the message gRPC takes: host pieces by memcpy, device pieces (torch uint8 tensors) by one
    device-to-host copy straight into the message instead of into a host buffer that a join then
    copies again."""
    if total < 2:   # the interpreter shares its 0- and 1-byte objects: never write into those
        return b"".join(bytes(p) if not hasattr(p, "is_cuda") else p.cpu().numpy().tobytes() for p in parts)
    out = _bytes_new(None, total)
    view = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(_bytes_addr(out)))
    pos = 0
    for p in parts:
        if hasattr(p, "is_cuda"):
            n = int(p.numel())
            if n:
                from efl import staging
                staging.to_host_into(view[pos:pos + n], p)
        else:
            mv = memoryview(p).cast("B")
            n = mv.nbytes
            if n:
                view[pos:pos + n] = np.frombuffer(mv, np.uint8)
        pos += n
    if pos != total:
        raise ValueError("message parts do not add up to the message size")
    return out


def message_request(name: str, step: int, dtype: int, shape, content) -> bytes:
    """Serialized MessageRequest{name, step, tensor}: the payload copied once, into the message."""
    tparts = tensor_proto_parts(dtype, shape, content)
    tlen = sum(_nbytes(p) for p in tparts)
    nb = name.encode()
    head = [_len_field(1, len(nb)) + nb]
    if step:
        head.append(key(2, _VARINT) + varint(step))
    head.append(_len_field(3, tlen))
    parts = head + tparts
    return _assemble(parts, sum(_nbytes(p) for p in parts))


class TensorMsg:
    __slots__ = ("dtype", "shape", "content", "typed")

    def __init__(self, dtype, shape, content, typed):
        self.dtype, self.shape, self.content, self.typed = dtype, shape, content, typed

    def numel(self) -> int:
        return int(np.prod(self.shape, dtype=np.int64)) if self.shape else 1

    def to_numpy(self) -> np.ndarray:
        """Zero-copy view for tensor_content; typed *_val fields are expanded like TF FromProto."""
        if self.dtype == DT_STRING:
            raise TypeError("DT_STRING payload: use efl.HexTensor.from_tensor_content")
        npdt = np.dtype(NP_OF_DT[self.dtype])
        n = self.numel()
        if self.content is not None and len(self.content):
            if len(self.content) != n * npdt.itemsize:
                raise ValueError("tensor_content size does not match shape")
            return np.frombuffer(self.content, dtype=npdt).reshape(self.shape)
        vals = self.typed
        out = np.zeros(n, npdt)
        if vals:
            k = min(len(vals), n)
            out[:k] = vals[:k]
            out[k:] = vals[-1] if n > k else out[k:]
        return out.reshape(self.shape)


def _packed(buf, s, e, wt_scalar, fmt=None):
    if fmt:
        return list(struct.unpack(f"<{(e - s) // struct.calcsize(fmt)}{fmt}", bytes(buf[s:e])))
    vals, pos = [], s
    while pos < e:
        v, pos = read_varint(buf, pos)
        vals.append(v)
    return vals


def parse_tensor_proto(buf, s: int, e: int) -> TensorMsg:
    dtype, shape, content, typed = 0, [], None, []
    mv = memoryview(buf)
    for f, wt, v, a, b in iter_fields(buf, s, e):
        if f == 1 and wt == _VARINT:
            dtype = v
        elif f == 2 and wt == _LEN:
            for f2, wt2, _v2, a2, b2 in iter_fields(buf, a, b):
                if f2 == 2 and wt2 == _LEN:
                    size = 0
                    for f3, wt3, v3, _a3, _b3 in iter_fields(buf, a2, b2):
                        if f3 == 1 and wt3 == _VARINT:
                            size = _signed64(v3)
                    shape.append(size)
        elif f == 4 and wt == _LEN:
            content = mv[a:b]
        elif f == 5:
            typed += _packed(buf, a, b, None, "f") if wt == _LEN else list(struct.unpack("<f", v))
        elif f == 6:
            typed += _packed(buf, a, b, None, "d") if wt == _LEN else list(struct.unpack("<d", v))
        elif f in (7, 10, 11):
            typed += [_signed64(x) for x in _packed(buf, a, b, None)] if wt == _LEN else [_signed64(v)]
        elif f == 8 and wt == _LEN:
            typed.append(bytes(mv[a:b]))
    return TensorMsg(dtype, tuple(shape), content, typed)


def parse_message_request(buf):
    """-> (name, step, TensorMsg)."""
    name, step, tensor = "", 0, None
    for f, wt, v, a, b in iter_fields(buf):
        if f == 1 and wt == _LEN:
            name = bytes(buf[a:b]).decode()
        elif f == 2 and wt == _VARINT:
            step = v
        elif f == 3 and wt == _LEN:
            tensor = parse_tensor_proto(buf, a, b)
    if tensor is None:
        tensor = TensorMsg(0, (), None, [])
    return name, step, tensor


def message_response(code: int = 0, msg: str = "") -> bytes:
    out = b""
    if code:
        out += key(1, _VARINT) + varint(code)
    if msg:
        mb = msg.encode()
        out += _len_field(2, len(mb)) + mb
    return out


def parse_message_response(buf):
    code, msg = 0, ""
    for f, wt, v, a, b in iter_fields(buf):
        if f == 1 and wt == _VARINT:
            code = v
        elif f == 2 and wt == _LEN:
            msg = bytes(buf[a:b]).decode()
    return code, msg
