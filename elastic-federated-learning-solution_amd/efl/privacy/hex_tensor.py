"""HexTensor — the build's stand-in for the reference's DT_STRING tensors of hex integers.

In efls-train, Paillier ciphertexts and decrypted big plaintexts travel as `tf.string` tensors
whose elements are lowercase hex numbers written by `mpz_get_str(..., 16)`
(efls-train/cc/efl/math/gmp_utils.cc:146-150, paillier.cc:127,140). A HexTensor holds the same
strings packed back to back (one flat byte buffer + int64 offsets[n+1], a ragged array) with a
shape. It can live on the host (numpy) or in HBM (torch device tensors, as produced by the hex
kernels); each side is materialised on first use. It serialises to TensorProto.tensor_content
exactly like TF's string encoding (all varint32 lengths, then the bytes).
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from efl import staging


class HexTensor:
    __slots__ = ("_buf", "_offs", "shape", "_dev")

    def __init__(self, buf: np.ndarray | None, offs: np.ndarray | None, shape, device_parts=None):
        self._buf = None if buf is None else np.ascontiguousarray(buf, np.uint8)
        self._offs = None if offs is None else np.ascontiguousarray(offs, np.int64)
        self.shape = tuple(int(s) for s in shape)
        self._dev = device_parts          # (device, chars uint8 tensor, offsets int64 tensor)
        n = self._offs.size - 1 if self._offs is not None else int(device_parts[2].numel()) - 1
        if int(np.prod(self.shape, dtype=np.int64)) != n:
            raise ValueError("HexTensor: shape does not match the number of strings")

    # -- construction ---------------------------------------------------------------------
    @classmethod
    def from_strings(cls, strings, shape=None):
        if isinstance(strings, HexTensor):
            return strings
        arr = np.asarray(strings, dtype=object)
        shape = arr.shape if shape is None else tuple(shape)
        items = [s.encode() if isinstance(s, str) else bytes(s) for s in arr.reshape(-1)]
        offs = np.zeros(len(items) + 1, np.int64)
        if items:
            offs[1:] = np.cumsum([len(b) for b in items])
        buf = np.frombuffer(b"".join(items), np.uint8) if offs[-1] else np.zeros(0, np.uint8)
        return cls(buf, offs, shape)

    @classmethod
    def from_ints(cls, values, shape=None):
        """Python ints -> lowercase hex as mpz_get_str(…, 16) writes them ('-' sign, no prefix)."""
        vals = list(values)
        strs = [("-" + format(-v, "x")) if v < 0 else format(v, "x") for v in vals]
        return cls.from_strings(np.array(strs, dtype=object).reshape(shape if shape is not None else (len(strs),)))

    @classmethod
    def from_device(cls, chars: torch.Tensor, offs: torch.Tensor, shape):
        return cls(None, None, shape, (chars.device, chars, offs))

    # -- storage --------------------------------------------------------------------------
    @property
    def buf(self) -> np.ndarray:
        if self._buf is None:
            _, chars, offs = self._dev
            total = int(offs[-1].item()) if offs.numel() else 0
            self._buf = chars[:total].cpu().numpy() if total else np.zeros(0, np.uint8)
        return self._buf

    @property
    def offs(self) -> np.ndarray:
        if self._offs is None:
            self._offs = self._dev[2].cpu().numpy()
        return self._offs

    def numel(self) -> int:
        return (self._offs.size if self._offs is not None else int(self._dev[2].numel())) - 1

    def device_buffers(self, device):
        """(chars uint8, offsets int64) on `device` (copied once, cached). A host buffer (e.g. a
        read-only view of received message bytes) goes through the pinned staging buffer."""
        if self._dev is None or self._dev[0] != device:
            host = self.buf if self.buf.size else np.zeros(1, np.uint8)
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", UserWarning)   # torch cannot mark the view read-only
                chars = staging.to_device(host, device)
                offs = staging.to_device(self.offs, device)
            self._dev = (device, chars, offs)
        return self._dev[1], self._dev[2]

    # -- access ---------------------------------------------------------------------------
    def strings(self):
        b = self.buf.tobytes()
        o = self.offs
        return [b[o[i]:o[i + 1]].decode() for i in range(self.numel())]

    def to_ints(self):
        return [int(s, 16) for s in self.strings()]

    def numpy(self) -> np.ndarray:
        """object ndarray of bytes, the way a TF string tensor reads back in Python."""
        b = self.buf.tobytes()
        o = self.offs
        out = np.empty(self.numel(), dtype=object)
        for i in range(self.numel()):
            out[i] = b[o[i]:o[i + 1]]
        return out.reshape(self.shape)

    def reshape(self, shape):
        shape = tuple(int(s) for s in shape)
        if -1 in shape:
            known = int(np.prod([s for s in shape if s != -1], dtype=np.int64)) or 1
            shape = tuple(self.numel() // known if s == -1 else s for s in shape)
        return HexTensor(self._buf, self._offs, shape, self._dev)

    def transpose(self):
        if len(self.shape) != 2:
            raise ValueError("transpose needs rank 2")
        r, c = self.shape
        idx = np.arange(r * c).reshape(r, c).T.reshape(-1)
        return self.take(idx, (c, r))

    def take(self, idx, shape):
        idx = np.asarray(idx, np.int64).reshape(-1)
        offs0, buf0 = self.offs, self.buf
        lens = offs0[1:] - offs0[:-1]
        nl = lens[idx]
        offs = np.zeros(idx.size + 1, np.int64)
        offs[1:] = np.cumsum(nl)
        starts = offs0[idx]
        if offs[-1]:
            gather = np.repeat(starts - offs[:-1], nl) + np.arange(offs[-1])
            buf = buf0[gather]
        else:
            buf = np.zeros(0, np.uint8)
        return HexTensor(buf, offs, shape)

    # -- TF DT_STRING tensor_content codec (EncodeStringList: varint32 lengths, then bytes) ----
    # Vectorised over the strings (numpy): a ciphertext tensor of the paillier_mnist layer holds
    # 100k strings, and a per-string Python loop cost ~100 ms per message each way.
    def tensor_content_parts(self):
        """(varint32 length header, string bytes) as uint8 arrays: the two halves of
        tensor_content, for a serialiser that joins them without another copy."""
        return _varint32_encode(self.offs[1:] - self.offs[:-1]), self.buf

    def wire_parts(self):
        """tensor_content_parts for the sender: when the text still lives only in device memory
        (made by the hex kernels) the second part is that device uint8 tensor, which the message
        assembly copies straight into the outgoing request (efl.framework.wire._assemble) — the
        text is never staged in a host buffer of its own."""
        if self._buf is None and self._dev is not None:
            _, chars, _ = self._dev
            total = int(self.offs[-1]) if self.numel() else 0
            return _varint32_encode(self.offs[1:] - self.offs[:-1]), chars[:total]
        return self.tensor_content_parts()

    def to_tensor_content(self) -> bytes:
        return b"".join(self.tensor_content_parts())

    @classmethod
    def from_tensor_content(cls, content, shape):
        """Parse tensor_content (bytes or any buffer). The strings stay a view of `content`."""
        n = int(np.prod(shape, dtype=np.int64))
        raw = np.frombuffer(content, np.uint8)
        lens, pos = _varint32_decode(raw, n)
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        if pos + int(offs[-1]) > raw.size:
            raise ValueError("DT_STRING tensor_content is shorter than its lengths say")
        return cls(raw[pos:pos + int(offs[-1])], offs, shape)

    def __len__(self):
        return self.shape[0] if self.shape else 1

    def __repr__(self):
        s = self.strings()
        head = ", ".join(x[:16] + ("…" if len(x) > 16 else "") for x in s[:4])
        return f"HexTensor(shape={self.shape}, [{head}{', …' if len(s) > 4 else ''}])"

    def __eq__(self, other):
        return isinstance(other, HexTensor) and self.shape == other.shape and \
            np.array_equal(self.offs, other.offs) and np.array_equal(self.buf, other.buf)


def _varint32_encode(lens: np.ndarray) -> np.ndarray:
    """Protobuf varint32 of every length, back to back (uint8)."""
    v = np.asarray(lens, np.int64)
    if v.size and (int(v.min()) < 0 or int(v.max()) >= 1 << 32):
        raise ValueError("string length out of varint32 range")
    nb = np.ones(v.size, np.int64)
    for k in range(1, 5):
        nb += v >= (1 << (7 * k))
    starts = np.zeros(v.size, np.int64)
    if v.size > 1:
        np.cumsum(nb[:-1], out=starts[1:])
    out = np.empty(int(nb.sum()), np.uint8)
    for k in range(5):
        m = nb > k
        if not m.any():
            break
        byte = (v[m] >> (7 * k)) & 0x7F
        out[starts[m] + k] = (byte | ((nb[m] > k + 1).astype(np.int64) << 7)).astype(np.uint8)
    return out


def _varint32_decode(raw: np.ndarray, n: int):
    """The first n varint32s of raw -> (values int64[n], bytes they took)."""
    if n == 0:
        return np.zeros(0, np.int64), 0
    head = raw[:5 * n]
    ends = np.flatnonzero(head < 0x80)[:n]
    if ends.size < n:
        raise ValueError("DT_STRING tensor_content: truncated length header")
    starts = np.empty(n, np.int64)
    starts[0] = 0
    starts[1:] = ends[:-1] + 1
    width = ends - starts + 1
    if int(width.max()) > 5:
        raise ValueError("DT_STRING tensor_content: malformed varint32 length")
    vals = np.zeros(n, np.int64)
    for k in range(5):
        m = width > k
        if not m.any():
            break
        vals[m] |= (head[starts[m] + k].astype(np.int64) & 0x7F) << (7 * k)
    return vals, int(ends[-1]) + 1
