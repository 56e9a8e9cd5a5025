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

import numpy as np
import torch


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
        """(chars uint8, offsets int64) on `device` (copied once, cached)."""
        if self._dev is None or self._dev[0] != device:
            host = self.buf if self.buf.size else np.zeros(1, np.uint8)
            chars = torch.from_numpy(np.array(host, copy=True)).to(device)
            offs = torch.from_numpy(np.array(self.offs, copy=True)).to(device)
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
    def to_tensor_content(self) -> bytes:
        lens = (self.offs[1:] - self.offs[:-1]).tolist()
        out = bytearray()
        for n in lens:
            while n >= 0x80:
                out.append((n & 0x7F) | 0x80)
                n >>= 7
            out.append(n)
        out += self.buf.tobytes()
        return bytes(out)

    @classmethod
    def from_tensor_content(cls, content: bytes, shape):
        n = int(np.prod(shape, dtype=np.int64))
        lens = np.zeros(n, np.int64)
        pos = 0
        for i in range(n):
            v, s = 0, 0
            while True:
                c = content[pos]
                pos += 1
                v |= (c & 0x7F) << s
                if c < 0x80:
                    break
                s += 7
            lens[i] = v
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        buf = np.frombuffer(content, np.uint8, count=int(offs[-1]), offset=pos).copy()
        return cls(buf, offs, shape)

    def __len__(self):
        return self.shape[0] if self.shape else 1

    def __repr__(self):
        s = self.strings()
        head = ", ".join(x[:16] + ("…" if len(x) > 16 else "") for x in s[:4])
        return f"HexTensor(shape={self.shape}, [{head}{', …' if len(s) > 4 else ''}])"

    def __eq__(self, other):
        return isinstance(other, HexTensor) and self.shape == other.shape and \
            np.array_equal(self.offs, other.offs) and np.array_equal(self.buf, other.buf)
