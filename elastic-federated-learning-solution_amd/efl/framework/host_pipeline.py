"""Host-resident legs of the forward-encryption path: pinned host -> GPU codec -> pinned host.

The reference's path starts and ends in host memory: the activation leaves the TF CPU op as a host
tensor and goes into the communicator's gRPC buffers (communication_client.cc:37-57, one TensorProto
copy per message, 1 GiB message cap communicator_ops.cc:437-440); the receiver parses the message
back into a host tensor (communicator_ops.cc:235-261). On the MI355X the codec runs in HBM, so each
leg is H2D -> kernel -> D2H over PCIe. `PinnedCodecPipeline` cuts a tensor into chunks and runs
the three stages of consecutive chunks concurrently on three HIP streams:

    copy-in stream   H2D of chunk i+1            (host -> device DMA)
    compute stream   encode / decode of chunk i  (libefl_hip.so)
    copy-out stream  D2H of chunk i-1            (device -> host DMA, the other PCIe direction)

with `nbuf` device slots per stream reused round-robin and events ordering every reuse, so the
leg runs at the rate of its slowest PCIe direction instead of the sum of the three. Host buffers
must be page-locked (`pin_memory()`) for the copies to be asynchronous DMA; a pageable source is
staged through pinned chunk buffers (one host memcpy per chunk, overlapped with the DMA of the
previous chunk).

Encrypt leg (fp32 in):  H2D 4 B/elem, D2H 16 B/elem (mantissa + exponent, int64 each).
Decrypt leg (fp32 out): H2D 16 B/elem, D2H 4 B/elem.
"""
from __future__ import annotations

import torch

from efl import errors
from efl import lib as _lib

DEFAULT_CHUNK_ELEMS = 1 << 22        # 16 MiB of fp32 in, 64 MiB of M+E out per chunk


class PinnedCodecPipeline:
    """Chunked, multi-buffered H2D -> codec -> D2H over three streams on one device."""

    def __init__(self, device=None, chunk_elems: int = DEFAULT_CHUNK_ELEMS, nbuf: int = 3):
        self.device = device if device is not None else _lib.require_gpu()
        if chunk_elems <= 0 or chunk_elems % 64:
            raise errors.InvalidArgumentError("chunk_elems must be a positive multiple of 64")
        self.chunk = int(chunk_elems)
        self.nbuf = max(2, int(nbuf))
        self.s_in = torch.cuda.Stream(self.device)
        self.s_run = torch.cuda.Stream(self.device)
        self.s_out = torch.cuda.Stream(self.device)
        self._slots = {}
        self._stage = {}

    # -- device / staging buffers, allocated once per (kind, dtype) -------------------------
    def _slot(self, kind: str, dtype: torch.dtype, b: int) -> torch.Tensor:
        key = (kind, dtype, b)
        t = self._slots.get(key)
        if t is None:
            t = torch.empty(self.chunk, dtype=dtype, device=self.device)
            self._slots[key] = t
        return t

    def _staging(self, kind: str, dtype: torch.dtype, b: int) -> torch.Tensor:
        key = (kind, dtype, b)
        t = self._stage.get(key)
        if t is None:
            t = torch.empty(self.chunk, dtype=dtype, pin_memory=True)
            self._stage[key] = t
        return t

    def _chunks(self, n: int):
        return [(s, min(n, s + self.chunk)) for s in range(0, n, self.chunk)]

    def _run(self, srcs, dsts, kernel, in_dtypes, out_dtypes):
        """srcs: host 1-D tensors (same numel); dsts: pinned host 1-D outputs. kernel(ins, outs,
        n, stream_handle) enqueues the codec on the compute stream.

        The pipeline's streams first wait for the caller's current stream: the device slots are
        allocated lazily on it, and the caching allocator may hand them a block just freed there
        while a kernel on that stream still reads it. The body runs without autograd: the cached
        slots and staging chunks must never join a caller's graph (an activation that requires grad
        reaches here through FixedPointHook.pre_send)."""
        cur = torch.cuda.current_stream(self.device)
        self.s_in.wait_stream(cur)
        self.s_run.wait_stream(cur)
        self.s_out.wait_stream(cur)
        with torch.no_grad():
            self._run_chunks(srcs, dsts, kernel, in_dtypes, out_dtypes)

    def _run_chunks(self, srcs, dsts, kernel, in_dtypes, out_dtypes):
        n = srcs[0].numel()
        ev_in = [torch.cuda.Event() for _ in range(self.nbuf)]
        ev_run = [torch.cuda.Event() for _ in range(self.nbuf)]
        ev_out = [torch.cuda.Event() for _ in range(self.nbuf)]
        used = [False] * self.nbuf
        pinned_src = all(s.is_pinned() for s in srcs)
        for i, (s, e) in enumerate(self._chunks(n)):
            b = i % self.nbuf
            m = e - s
            ins = [self._slot("in%d" % k, dt, b)[:m] for k, dt in enumerate(in_dtypes)]
            outs = [self._slot("out%d" % k, dt, b)[:m] for k, dt in enumerate(out_dtypes)]
            with torch.cuda.stream(self.s_in):
                if used[b]:
                    self.s_in.wait_event(ev_run[b])           # slot's inputs consumed
                for k, src in enumerate(srcs):
                    piece = src[s:e]
                    if not pinned_src:
                        if used[b]:
                            ev_in[b].synchronize()           # staging chunk's last H2D done
                        st = self._staging("in%d" % k, src.dtype, b)[:m]
                        st.copy_(piece)
                        piece = st
                    ins[k].copy_(piece, non_blocking=True)
                ev_in[b].record(self.s_in)
            self.s_run.wait_event(ev_in[b])
            if used[b]:
                self.s_run.wait_event(ev_out[b])              # slot's outputs drained
            kernel(ins, outs, m, self.s_run.cuda_stream)
            ev_run[b].record(self.s_run)
            with torch.cuda.stream(self.s_out):
                self.s_out.wait_event(ev_run[b])
                for k, dst in enumerate(dsts):
                    dst[s:e].copy_(outs[k], non_blocking=True)
                ev_out[b].record(self.s_out)
            used[b] = True
        self.s_out.synchronize()

    # -- the two legs ----------------------------------------------------------------------
    def encode(self, x: torch.Tensor, decrease_precision: bool = False, out=None):
        """ConvertToFixedPoint of a host tensor: returns pinned host (mantissa, exponent)."""
        if x.is_cuda:
            raise errors.InvalidArgumentError("PinnedCodecPipeline.encode takes a host tensor")
        code = _lib.dt_code(x.dtype)
        flat = x.detach().contiguous().reshape(-1)
        if out is None:
            out = (torch.empty(flat.numel(), dtype=torch.int64, pin_memory=True),
                   torch.empty(flat.numel(), dtype=torch.int64, pin_memory=True))
        M, E = (o.reshape(-1) for o in out)
        raw = _lib.raw()
        dp = int(bool(decrease_precision))

        def kern(ins, outs, m, sh):
            _lib.check(raw.efl_fxp_encode(ins[0].data_ptr(), code, outs[0].data_ptr(), outs[1].data_ptr(),
                                          m, dp, sh))
        self._run([flat], [M, E], kern, [x.dtype], [torch.int64, torch.int64])
        return M.view(x.shape), E.view(x.shape)

    def decode(self, mantissa: torch.Tensor, exponent: torch.Tensor, dtype=torch.float32,
               flush_denormal=None, out=None):
        """FixedPointToFloatPoint of host int64 tensors: returns a pinned host tensor."""
        if mantissa.is_cuda or exponent.is_cuda:
            raise errors.InvalidArgumentError("PinnedCodecPipeline.decode takes host tensors")
        if mantissa.numel() != exponent.numel():
            raise errors.InvalidArgumentError("mantissa and exponent should be the same size.")
        if mantissa.dtype != torch.int64 or exponent.dtype != torch.int64:
            raise errors.InvalidArgumentError("FixedPointToFloatPoint: mantissa and exponent must be int64")
        dtype = _lib.to_torch_dtype(dtype)
        code = _lib.dt_code(dtype)
        ftz = _lib.flush_denormal() if flush_denormal is None else bool(flush_denormal)
        Mf = mantissa.detach().contiguous().reshape(-1)
        Ef = exponent.detach().contiguous().reshape(-1)
        y = out if out is not None else torch.empty(Mf.numel(), dtype=dtype, pin_memory=True)
        yf = y.reshape(-1)
        raw = _lib.raw()

        def kern(ins, outs, m, sh):
            _lib.check(raw.efl_fxp_decode(ins[0].data_ptr(), ins[1].data_ptr(), outs[0].data_ptr(), code,
                                          m, m, 1 if ftz else 0, sh))
        self._run([Mf, Ef], [yf], kern, [torch.int64, torch.int64], [dtype])
        return yf.view(mantissa.shape)
