"""Host <-> HBM copies of large byte payloads through one grow-only pinned buffer per device.

A pageable copy of a received or outgoing message's hex text (51 MB for the paillier_mnist
activation's ciphertexts) lets the runtime pin or stage it page by page: 5-36 ms per copy on the
layer bench's boxes, with large spread. Here one DMA moves the bytes between HBM and the pinned
buffer, and torch's multi-threaded CPU copy moves them between the pinned buffer and the pageable
side. A lock serialises the buffer between threads; an event makes the next user wait until the
previous DMA has finished with it."""
from __future__ import annotations

import threading

import numpy as np
import torch

STAGE_MIN = 1 << 20          # smaller copies go straight through the runtime
_stage: dict = {}
_lock = threading.Lock()


def _buffer(dev: torch.device, n: int) -> torch.Tensor:
    buf, ev = _stage.get(dev, (None, None))
    if ev is not None:
        ev.synchronize()
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 2 * buf.numel() if buf is not None else n), dtype=torch.uint8, pin_memory=True)
        _stage[dev] = (buf, None)
    return buf


def _fence(dev: torch.device, buf: torch.Tensor):
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    _stage[dev] = (buf, ev)


def to_device(arr: np.ndarray, device) -> torch.Tensor:
    """A copy of the host array `arr` on `device` (same dtype and shape), enqueued on the device's
    current stream."""
    src = torch.from_numpy(arr)
    dev = torch.device(device)
    if arr.nbytes < STAGE_MIN or dev.type != "cuda":
        return src.to(dev, copy=True)
    flat = src.reshape(-1).view(torch.uint8)
    n = flat.numel()
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    with _lock:
        buf = _buffer(dev, n)
        buf[:n].copy_(flat)
        out.copy_(buf[:n], non_blocking=True)
        _fence(dev, buf)
    return out.view(src.dtype).reshape(src.shape)


def to_host_into(dst: np.ndarray, src: torch.Tensor) -> None:
    """Copy the device tensor `src` (uint8, as many bytes as `dst`) into the host array `dst`;
    returns when `dst` holds the bytes."""
    flat = src.reshape(-1).view(torch.uint8)
    n = flat.numel()
    out = torch.from_numpy(dst.reshape(-1).view(np.uint8))
    if n < STAGE_MIN or flat.device.type != "cuda":
        out.copy_(flat)
        return
    dev = flat.device
    with _lock:
        buf = _buffer(dev, n)
        buf[:n].copy_(flat, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        out.copy_(buf[:n])
        _stage[dev] = (buf, None)
