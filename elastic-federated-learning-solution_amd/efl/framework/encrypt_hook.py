"""Pre-send / post-recv hook that applies the forward-encryption codec on the MI355X.

The reference's forward path (efls-train/python/efl/privacy/paillier_layer.py:64-67) encodes the
activation, encrypts the mantissa and sends two tensors, '<p>_[x]_mantissa' and '<p>_[x]_exponent';
the receiving side recv()s both (paillier_layer.py:121, 188). FixedPointHook packages the Stage-F
part of that pattern as a Communicator hook so existing send/recv callers need no change:

  send(name, float_tensor)  ->  ConvertToFixedPoint on GPU -> pinned host M, E ->
                                 send(name+'_mantissa', int64) + send(name+'_exponent', int64)
  recv(name, dtype=float)   ->  recv both -> FixedPointToFloatPoint on GPU -> tensor

Host tensors (the reference's case: its ops run on the CPU and the communicator ships host
buffers) go through efl.framework.host_pipeline.PinnedCodecPipeline: chunked H2D | codec | D2H on
three streams, so each leg runs at the rate of its slower PCIe direction; a pageable source (the
bytes gRPC hands over on receive) is staged through pinned chunk buffers inside the pipeline.
A device tensor is encoded where it is and copied out once; recv with return_device="cuda"
decodes on the device.

The codec functions are injectable (`encode=`, `decode=`) so CPU-only tests can run the same
plumbing with a CPU checker; by default they are the libefl_hip.so ops (no CPU fallback).
"""
from __future__ import annotations

import re
import time

import torch

from efl import exporter
from efl.framework.communicator import TensorHook

_FLOATS = (torch.float32, torch.float64)


class _PinnedPool:
    """Reusable page-locked host buffers for the D2H legs (keyed by dtype and size)."""

    def __init__(self):
        self._bufs = {}

    def get(self, like: torch.Tensor, slot: str) -> torch.Tensor:
        """A pinned buffer of like's dtype and shape (`like` may be a meta tensor)."""
        k = (slot, like.dtype, like.numel())
        b = self._bufs.get(k)
        if b is None:
            b = torch.empty(like.numel(), dtype=like.dtype, pin_memory=torch.cuda.is_available())
            self._bufs[k] = b
        return b.view(like.shape)


@exporter.export("privacy.FixedPointHook")
class FixedPointHook(TensorHook):
    readonly_recv = True   # post_recv reads the received payloads in place (False: private copies)

    def __init__(self, names=None, decrease_precision=False, return_device=None, encode=None,
                 decode=None, reuse_buffers=False, stats=None):
        """names: regex of logical tensor names to transform (default: every float tensor).
        return_device: where recv() returns the decoded tensor (default: host, like the
        reference's recv). reuse_buffers: keep pinned D2H buffers across sends (the caller must
        not send the same name again before the previous send completed). stats: a dict that
        receives per-stage wall times in seconds (adds device synchronisations; measurement only)."""
        self.stats = stats
        self._names = re.compile(names) if names else None
        self._dp = decrease_precision
        self._return_device = return_device
        # the pinned three-stream pipeline serves host tensors when the codec is the GPU one
        self._use_pipeline = encode is None and decode is None
        self._pipe = None
        if encode is None or decode is None:
            from efl.lib import ops
            encode = encode or ops.convert_to_fixed_point
            decode = decode or ops.fixed_point_to_float_point
        self._encode, self._decode = encode, decode
        self._pool = _PinnedPool() if reuse_buffers else None

    def _pipeline(self):
        if self._pipe is None:
            from efl.framework.host_pipeline import PinnedCodecPipeline
            self._pipe = PinnedCodecPipeline()
        return self._pipe

    def _match(self, name):
        return self._names is None or self._names.search(name) is not None

    def _to_host(self, t: torch.Tensor, slot: str) -> torch.Tensor:
        if not t.is_cuda:
            return t
        if self._pool is not None:
            h = self._pool.get(t, slot)
        else:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        return h

    def _pinned_like(self, shape, dtype, slot):
        """Output buffers of a pipeline leg: from the pool (reuse_buffers) or fresh pinned."""
        if self._pool is not None:
            return self._pool.get(torch.empty(shape, dtype=dtype, device="meta"), slot)
        return torch.empty(shape, dtype=dtype, pin_memory=True)

    def pre_send(self, name, tensor):
        if not isinstance(tensor, torch.Tensor) or tensor.dtype not in _FLOATS or not self._match(name):
            return None
        t = self._tick()
        if self._use_pipeline and not tensor.is_cuda:
            # host tensor: H2D | encode | D2H pipelined into pinned M, E (the gRPC payloads)
            out = (self._pinned_like(tensor.shape, torch.int64, name + "_m"),
                   self._pinned_like(tensor.shape, torch.int64, name + "_e"))
            M, E = self._pipeline().encode(tensor, decrease_precision=self._dp, out=out)
            self._tick("send_pipeline", t)
            return [(name + "_mantissa", M), (name + "_exponent", E)]
        if self.stats is not None and not tensor.is_cuda and torch.cuda.is_available():
            tensor = tensor.cuda(non_blocking=tensor.is_pinned())
            t = self._tick("send_h2d", t)
        M, E = self._encode(tensor, decrease_precision=self._dp)
        t = self._tick("send_encode", t)
        Mh, Eh = self._to_host(M, name + "_m"), self._to_host(E, name + "_e")
        if M.is_cuda:
            torch.cuda.current_stream(M.device).synchronize()
        self._tick("send_d2h", t)
        return [(name + "_mantissa", Mh), (name + "_exponent", Eh)]

    def _tick(self, stage=None, t0=None):
        if self.stats is None:
            return None
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        now = time.perf_counter()
        if stage is not None:
            self.stats[stage] = self.stats.get(stage, 0.0) + (now - t0)
        return now

    def post_recv(self, name, shape, dtype, raw_recv):
        from efl.lib import to_torch_dtype
        dt = to_torch_dtype(dtype)
        if dt not in _FLOATS or not self._match(name):
            return None
        t = self._tick()
        # the payloads are only read (copied to the GPU): views of the message bytes, no host copy
        M = raw_recv(name + "_mantissa", readonly=self.readonly_recv)
        E = raw_recv(name + "_exponent", readonly=self.readonly_recv)
        t = self._tick("recv_grpc", t)
        if self._use_pipeline and self._return_device is None and not M.is_cuda and not E.is_cuda:
            # host result (the reference's recv): staged H2D | decode | D2H into a pinned tensor
            y = self._pipeline().decode(M, E, dt, out=self._pinned_like(tuple(M.shape), dt, name + "_y"))
            self._tick("recv_pipeline", t)
            return y.reshape(tuple(int(s) for s in shape)) if shape is not None else y
        if torch.cuda.is_available():
            M = M.cuda() if not M.is_cuda else M
            E = E.cuda() if not E.is_cuda else E
        t = self._tick("recv_h2d", t)
        y = self._decode(M, E, dt)
        t = self._tick("recv_decode", t)
        if shape is not None:
            y = y.reshape(tuple(int(s) for s in shape))
        if self._return_device is not None:
            y = y.to(self._return_device)
        elif y.is_cuda:
            y = y.cpu()
        self._tick("recv_d2h", t)
        return y
