"""Loads libefl_hip.so (the MI355X kernels behind the C ABI in include/efl_hip.h) and exposes
the op functions under the names the reference's `fed_ops` has.

Reference: efls-train/python/efl/lib.py:24-28 loads libefl.so with `tf.load_op_library` and the
callers use `fed_ops.convert_to_fixed_point`, `fed_ops.fixed_point_to_float_point`, ...
(efls-train/python/efl/privacy/paillier.py:56-155). Here `efl.lib.ops` is that namespace, over
torch tensors instead of TF graph tensors.

There is no CPU fallback: the library must be present (ImportError otherwise) and every op needs a
ROCm device (a CPU input is staged through the GPU and the result copied back).
"""
from __future__ import annotations

import ctypes
import os
import threading
import types

import numpy as np
import torch

from efl import errors

_LIB_DIR = os.path.dirname(os.path.realpath(__file__))
# EFL_HIP_LIB: path of a tuning build of the same library (Makefile `variant`); default in-tree
LIB_PATH = os.environ.get("EFL_HIP_LIB") or os.path.join(_LIB_DIR, "libefl_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C elastic-federated-learning-solution_amd` "
        "(or __graft_entry__.build()). The efl ops have no CPU fallback.")

_lib = ctypes.CDLL(LIB_PATH)

_vp, _i64, _i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
_SIGS = {
    "efl_version": ([], ctypes.c_char_p),
    "efl_last_error": ([], ctypes.c_char_p),
    "efl_fxp_tune": ([_i32, _i32], _i32),
    "efl_fxp_encode": ([_vp, _i32, _vp, _vp, _i64, _i32, _vp], _i32),
    "efl_fxp_decode": ([_vp, _vp, _vp, _i32, _i64, _i64, _i32, _vp], _i32),
    "efl_fxp_decode_hex": ([_vp, _vp, _vp, _vp, _i32, _i64, _i32, _vp, _vp], _i32),
    "efl_fxp_encode_batched": ([_vp, _i32, _vp, _vp, _vp, _i64, _i64, _i32, _vp], _i32),
    "efl_fxp_decode_batched": ([_vp, _vp, _vp, _i32, _vp, _i64, _i64, _i32, _vp], _i32),
    "efl_ss_noise": ([_vp, _vp, _vp, _i64, _i32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float, _vp], _i32),
    "efl_ss_mask_cols": ([_vp, _vp, _vp, _vp, _i64, _i64, ctypes.c_uint64, ctypes.c_uint64, _vp], _i32),
    "efl_ss_mask_rows": ([_vp, _vp, _vp, _vp, _i64, _i64, ctypes.c_uint64, ctypes.c_uint64, _vp], _i32),
    "efl_dp_noise": ([_vp, _vp, _i64, _i32, ctypes.c_float, ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, _vp],
                     _i32),
}
for _name, (_args, _ret) in _SIGS.items():
    _f = getattr(_lib, _name)
    _f.argtypes = _args
    _f.restype = _ret

# TensorFlow DataType numbers (types.proto), as used by the C ABI and the wire format.
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT16, DT_INT8, DT_STRING, DT_INT64 = 1, 2, 3, 5, 6, 7, 9
_TORCH_TO_DT = {torch.float32: DT_FLOAT, torch.float64: DT_DOUBLE, torch.int32: DT_INT32,
                torch.int16: DT_INT16, torch.int8: DT_INT8, torch.int64: DT_INT64}
_DT_TO_TORCH = {v: k for k, v in _TORCH_TO_DT.items()}

# Decode's float32 rounding mode. The reference op's kernels run on TensorFlow threadpool threads,
# and TF 1.15 starts every threadpool thread with MXCSR FTZ|DAZ set (tensorflow/core/platform/
# threadpool.cc, EigenEnvironment::CreateThread: port::ScopedFlushDenormal; TF 1.15.5 is the
# reference's base image, docker/Dockerfile.efls-train:1). The implicit double -> float of
# fixed_point.cc:245 therefore flushes results below 2^-126 to signed zero: +-0.0 (encoded as
# (+-1, -127)) decodes to +-0.0, not 2^-127. That is the default here.
_flush_denormal = True


def raw():
    """The ctypes handle of libefl_hip.so."""
    return _lib


def version() -> str:
    return _lib.efl_version().decode()


def set_flush_denormal(enabled: bool) -> bool:
    """Decode float32 results below the normal range to signed zero, as the reference does inside
    TensorFlow's threadpool threads (MXCSR FTZ|DAZ). Default True; False reproduces the bare loop
    compiled outside TF (+0.0 -> 2^-127). Returns the previous setting."""
    global _flush_denormal
    old, _flush_denormal = _flush_denormal, bool(enabled)
    return old


def flush_denormal() -> bool:
    return _flush_denormal


def check(rc: int) -> None:
    if rc != 0:
        raise errors.from_code(-rc, _lib.efl_last_error().decode())


def to_torch_dtype(dtype) -> torch.dtype:
    """Accepts torch dtypes, numpy dtypes, TF-style names ('float32') and DataType numbers."""
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, int) and dtype in _DT_TO_TORCH:
        return _DT_TO_TORCH[dtype]
    name = getattr(dtype, "name", None) or str(dtype)
    name = name.replace("tf.", "").replace("torch.", "")
    table = {"float32": torch.float32, "float": torch.float32, "float64": torch.float64,
             "double": torch.float64, "int8": torch.int8, "int16": torch.int16,
             "int32": torch.int32, "int64": torch.int64}
    if name in table:
        return table[name]
    try:
        return to_torch_dtype(np.dtype(dtype).name)
    except TypeError:
        pass
    raise errors.InvalidArgumentError(f"unsupported dtype {dtype!r}")


def dt_code(dtype: torch.dtype) -> int:
    try:
        return _TORCH_TO_DT[dtype]
    except KeyError:
        raise errors.InvalidArgumentError(f"unsupported dtype {dtype}") from None


_device_checked = False


def require_gpu() -> torch.device:
    """The ROCm device the ops run on; raises if there is none (no CPU fallback)."""
    global _device_checked
    if not torch.cuda.is_available():
        raise RuntimeError("efl: no ROCm GPU visible; the forward-encryption ops run only on "
                           "MI355X (gfx950) through libefl_hip.so")
    if not _device_checked:
        arch = torch.cuda.get_device_properties(0).gcnArchName
        if not arch.startswith("gfx950"):
            raise RuntimeError(f"efl: libefl_hip.so is built for gfx950, device is {arch}")
        _device_checked = True
    return torch.device("cuda", torch.cuda.current_device())


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def as_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x))


def on_device(t: torch.Tensor):
    """Contiguous device view of `t` (staging host tensors through H2D), plus the device the
    result should be returned on."""
    home = t.device
    if t.is_cuda:
        return t.contiguous(), home
    dev = require_gpu()
    return t.contiguous().to(dev, non_blocking=t.is_pinned()), home


def back(t: torch.Tensor, home: torch.device) -> torch.Tensor:
    if t.device == home:
        return t
    return t.to(home)


# Host tensors from this many elements on take the pinned three-stream pipeline
# (efl.framework.host_pipeline: chunked H2D | codec | D2H, outputs in pinned memory) instead of one
# pageable H2D, the kernel and one pageable D2H back to back: the reference's ops are CPU ops, so a
# drop-in caller hands over host tensors. The pipeline of a GPU keeps its device
# chunk slots (about 250 MiB for fp32 encode + decode) and pinned staging chunks after first use.
HOST_PIPELINE_MIN_ELEMS = 1 << 22
_pipes: dict = {}
_pipes_lock = threading.Lock()


def _host_pipeline():
    """(pipeline, lock) of the current GPU; one caller at a time uses a pipeline's slots."""
    dev = require_gpu()
    with _pipes_lock:
        entry = _pipes.get(dev)
        if entry is None:
            from efl.framework.host_pipeline import PinnedCodecPipeline   # imports this module
            entry = _pipes[dev] = (PinnedCodecPipeline(dev), threading.Lock())
    return entry


# ----------------------------------------------------------------------------------------------
# ops (fed_ops names)
# ----------------------------------------------------------------------------------------------

def convert_to_fixed_point(t, decrease_precision=None):
    """REGISTER_OP("ConvertToFixedPoint") (efls-train/cc/efl/math/fixed_point.cc:24-40).
    Returns (mantissa int64, exponent int64) of t's shape, on t's device (pinned host memory for
    large host tensors, which go through the pipelined copies)."""
    t = as_tensor(t)
    code = dt_code(t.dtype)
    if not t.is_cuda and t.numel() >= HOST_PIPELINE_MIN_ELEMS:
        pipe, lock = _host_pipeline()
        with lock:
            return pipe.encode(t, decrease_precision=bool(decrease_precision))
    x, home = on_device(t)
    M = torch.empty(x.shape, dtype=torch.int64, device=x.device)
    E = torch.empty(x.shape, dtype=torch.int64, device=x.device)
    check(_lib.efl_fxp_encode(x.data_ptr(), code, M.data_ptr(), E.data_ptr(), x.numel(),
                              int(bool(decrease_precision)), stream_handle(x.device)))
    return back(M, home), back(E, home)


def _hex_list(m):
    """Flatten a string-tensor stand-in (numpy object/bytes array, nested list) to list[bytes]."""
    if isinstance(m, (bytes, str)):
        m = [m]
    arr = np.asarray(m, dtype=object).reshape(-1)
    return [s.encode() if isinstance(s, str) else bytes(s) for s in arr], np.shape(m)


def fixed_point_to_float_point(mantissa, exponent, dtype=torch.float32, flush_denormal=None):
    """REGISTER_OP("FixedPointToFloatPoint") (fixed_point.cc:201-214): y = mantissa * 2^exponent.
    `mantissa` is an int64 tensor, or (the reference's DT_STRING form) hex strings: a
    `efl.HexTensor`, numpy array / list of str|bytes. Output on exponent's device."""
    dtype = to_torch_dtype(dtype)
    if dtype not in (torch.float32, torch.float64):
        raise errors.InvalidArgumentError(f"FixedPointToFloatPoint: dtype must be float or double, got {dtype}")
    ftz = _flush_denormal if flush_denormal is None else bool(flush_denormal)
    flags = 1 if ftz else 0
    exponent = as_tensor(exponent)
    from efl.privacy.hex_tensor import HexTensor  # local import: avoids a cycle at import time
    if isinstance(mantissa, HexTensor) or not isinstance(mantissa, torch.Tensor) and \
            np.asarray(mantissa, dtype=object).dtype == object and _looks_textual(mantissa):
        hx = mantissa if isinstance(mantissa, HexTensor) else HexTensor.from_strings(mantissa)
        return _decode_hex(hx, exponent, dtype, flags)
    mantissa = as_tensor(mantissa)
    if mantissa.dtype != torch.int64 or exponent.dtype != torch.int64:
        raise errors.InvalidArgumentError("FixedPointToFloatPoint: mantissa and exponent must be int64")
    if not mantissa.is_cuda and not exponent.is_cuda and mantissa.numel() >= HOST_PIPELINE_MIN_ELEMS:
        if mantissa.numel() != exponent.numel():
            raise errors.InvalidArgumentError("mantissa and exponent should be the same size.")
        pipe, lock = _host_pipeline()
        with lock:
            return pipe.decode(mantissa, exponent, dtype, flush_denormal=ftz)
    m, home = on_device(mantissa)
    e, _ = on_device(exponent)
    if e.device != m.device:
        e = e.to(m.device)
    y = torch.empty(m.shape, dtype=dtype, device=m.device)
    check(_lib.efl_fxp_decode(m.data_ptr(), e.data_ptr(), y.data_ptr(), dt_code(dtype), m.numel(),
                              e.numel(), flags, stream_handle(m.device)))
    return back(y, home)


def _looks_textual(m) -> bool:
    a = np.asarray(m, dtype=object).reshape(-1)
    return a.size == 0 or isinstance(a[0], (str, bytes, bytearray))


def _decode_hex(hx, exponent, dtype, flags):
    if hx.numel() != exponent.numel():
        raise errors.InvalidArgumentError("mantissa and exponent should be the same size.")
    e, home = on_device(exponent)
    dev = e.device
    chars, offs = hx.device_buffers(dev)
    y = torch.empty(tuple(exponent.shape), dtype=dtype, device=dev)
    bad = torch.empty(1, dtype=torch.int64, device=dev)
    check(_lib.efl_fxp_decode_hex(chars.data_ptr(), offs.data_ptr(), e.data_ptr(), y.data_ptr(),
                                  dt_code(dtype), hx.numel(), flags, bad.data_ptr(),
                                  stream_handle(dev)))
    b = int(bad.item())
    if b >= 0:
        raise errors.InvalidArgumentError(
            f"FixedPointToFloatPoint: mantissa[{b}] = {hx.strings()[b]!r} is not a hex integer")
    return back(y, home)


def _carve(like, dtype, dev):
    """Outputs of a batched op as views of one buffer, in batch order and 16-byte aligned, so
    that adjacent inputs (slices of one table) make one run with them (coalesce_runs)."""
    q = max(1, 16 // torch.empty((), dtype=dtype).element_size())
    offs, total = [], 0
    for t in like:
        offs.append(total)
        total += -(-t.numel() // q) * q
    buf = torch.empty(total, dtype=dtype, device=dev)
    return [buf[o:o + t.numel()].view(t.shape) for o, t in zip(offs, like)]


def convert_to_fixed_point_batched(tensors, decrease_precision=None):
    """One launch for a list of device tensors of one dtype (BASELINE config 3, sparse-rec
    embedding slices). Returns ([mantissa], [exponent])."""
    if not tensors:
        return [], []
    dev = tensors[0].device
    if not dev.type == "cuda":
        raise errors.InvalidArgumentError("batched ops take device tensors")
    code = dt_code(tensors[0].dtype)
    xs = [t.contiguous() for t in tensors]
    if any(t.dtype != xs[0].dtype or t.device != dev for t in xs):
        raise errors.InvalidArgumentError("batched encode: tensors must share dtype and device")
    Ms = _carve(xs, torch.int64, dev)
    Es = _carve(xs, torch.int64, dev)
    tables = BatchTables(xs, Ms, Es)
    encode_batched_into(tables, code, decrease_precision, stream_handle(dev))
    return Ms, Es


RUN_CHUNK = 1 << 20     # elements per entry of a coalesced table (BatchTables)


def coalesce_runs(srcs, d0s, d1s, chunk=RUN_CHUNK):
    """[(src_ptr, d0_ptr, d1_ptr, n)] of the batch with adjacent entries merged: entry i + 1 joins
    entry i's run when each of its three buffers starts where entry i's ends (slices of one
    embedding table, outputs carved from one buffer, or neighbours the caching allocator placed
    back to back). The transform is element-wise, so a run is one tensor to the kernels. Runs
    longer than `chunk` elements are cut into `chunk`-element pieces so the batched grid (count x
    tiles of the longest entry) stays dense; empty entries are dropped."""
    runs = []
    for s, a, b in zip(srcs, d0s, d1s):
        n = s.numel()
        if n == 0:
            continue
        p = (s.data_ptr(), a.data_ptr(), b.data_ptr())
        es = (s.element_size(), a.element_size(), b.element_size())
        if runs:
            r = runs[-1]
            if all(p[i] == r[0][i] + r[1] * es[i] for i in range(3)):
                r[1] += n
                continue
        runs.append([p, n, es])
    out = []
    for p, n, es in runs:
        if n <= chunk:
            out.append((p[0], p[1], p[2], n))
            continue
        for off in range(0, n, chunk):
            out.append((p[0] + off * es[0], p[1] + off * es[1], p[2] + off * es[2], min(chunk, n - off)))
    return out


class BatchTables:
    """Device pointer/length tables for the batched ABI (built once, reusable across launches).

    coalesce: "single" (default) sends a batch whose slices form ONE run in all three streams
    (slices of one embedding table with outputs carved from one buffer, coalesce_runs) through the
    streaming kernels (efl_fxp_encode / efl_fxp_decode) and keeps one table entry per slice
    otherwise; True merges every run (cut into RUN_CHUNK pieces); False keeps one entry per slice.
    Measured on MI355X (tools/config3_coalesce_probe.py, profiles/r04/c3_coalesce.jsonl), config 3's
    4096 x 64 KiB slices: views of one table 0.753 of HBM per slice -> 0.837 as one run; the bench's
    4096 separate allocations (384 runs of ~11 slices) 0.820 per slice against 0.811 merged."""

    def __init__(self, srcs, d0s, d1s, coalesce="single"):
        dev = srcs[0].device
        if len(srcs) != len(d0s) or len(srcs) != len(d1s):
            raise errors.InvalidArgumentError("batched tables: as many entries in every stream")
        for i, (s, a, b) in enumerate(zip(srcs, d0s, d1s)):
            # the kernels read each entry as numel() contiguous elements from its data pointer
            if not (s.is_contiguous() and a.is_contiguous() and b.is_contiguous()):
                raise errors.InvalidArgumentError(f"batched tables: entry {i} is not contiguous")
            if a.numel() != s.numel() or b.numel() != s.numel():
                raise errors.InvalidArgumentError(f"batched tables: entry {i} has streams of different sizes")
        self.keep = (srcs, d0s, d1s)
        runs = None
        if coalesce:
            merged = coalesce_runs(srcs, d0s, d1s, chunk=1 << 62)
            if len(merged) == 1:
                runs = merged
            elif coalesce is True:
                runs = coalesce_runs(srcs, d0s, d1s)
        if runs is None:
            runs = [(s.data_ptr(), a.data_ptr(), b.data_ptr(), s.numel()) for s, a, b in zip(srcs, d0s, d1s)]
        self.entries = len(srcs)
        self.runs = runs
        self.single = bool(coalesce) and len(runs) == 1
        col = list(zip(*runs)) if runs else [[], [], [], []]
        self.src, self.d0, self.d1, self.ns = (torch.tensor(list(c), dtype=torch.int64).to(dev) for c in col)
        self.count = len(runs)
        self.max_n = max((r[3] for r in runs), default=0)

    def args(self):
        return self.src.data_ptr(), self.d0.data_ptr(), self.d1.data_ptr(), self.ns.data_ptr(), \
            self.count, self.max_n


def encode_batched_into(tables: BatchTables, dtype_code: int, decrease_precision=False, stream=None):
    stream = stream if stream is not None else stream_handle()
    if tables.count == 0:
        return
    if tables.single:
        s, a, b, n = tables.runs[0]
        check(_lib.efl_fxp_encode(s, dtype_code, a, b, n, int(bool(decrease_precision)), stream))
        return
    src, d0, d1, ns, count, max_n = tables.args()
    check(_lib.efl_fxp_encode_batched(src, dtype_code, d0, d1, ns, count, max_n,
                                      int(bool(decrease_precision)), stream))


def decode_batched_into(tables: BatchTables, dtype_code: int, flags=0, stream=None):
    stream = stream if stream is not None else stream_handle()
    if tables.count == 0:
        return
    if tables.single:
        m, e, y, n = tables.runs[0]
        check(_lib.efl_fxp_decode(m, e, y, dtype_code, n, n, flags, stream))
        return
    src, d0, d1, ns, count, max_n = tables.args()
    check(_lib.efl_fxp_decode_batched(src, d0, d1, dtype_code, ns, count, max_n, flags, stream))


def batched_tile(direction: str):
    """(lanes, pairs per lane) of the fp32 batched kernel of `direction` ("encode" / "decode"):
    efl_fxp_tune kinds 10-13 read with value -1."""
    k = 10 if direction == "encode" else 12
    return _lib.efl_fxp_tune(k, -1), _lib.efl_fxp_tune(k + 1, -1)


def fixed_point_to_float_point_batched(mantissas, exponents, dtype=torch.float32, flush_denormal=None):
    """One launch decoding a list of (mantissa, exponent) int64 device tensor pairs. Each pair is
    checked like efl_fxp_decode checks one (same size, fixed_point.cc:230-232) and made contiguous
    first, so a strided view is decoded from its own elements."""
    if len(mantissas) != len(exponents):
        raise errors.InvalidArgumentError("batched decode: as many exponents as mantissas")
    if not mantissas:
        return []
    dtype = to_torch_dtype(dtype)
    if dtype not in (torch.float32, torch.float64):
        raise errors.InvalidArgumentError(f"FixedPointToFloatPoint: dtype must be float or double, got {dtype}")
    dev = mantissas[0].device
    if dev.type != "cuda":
        raise errors.InvalidArgumentError("batched ops take device tensors")
    ms, es = [], []
    for i, (m, e) in enumerate(zip(mantissas, exponents)):
        if m.dtype != torch.int64 or e.dtype != torch.int64:
            raise errors.InvalidArgumentError(f"batched decode: pair {i}: mantissa and exponent must be int64")
        if m.device != dev or e.device != dev:
            raise errors.InvalidArgumentError(f"batched decode: pair {i} is not on {dev}")
        if m.numel() != e.numel():
            raise errors.InvalidArgumentError(f"batched decode: pair {i}: mantissa and exponent should be the same size.")
        ms.append(m.contiguous())
        es.append(e.contiguous())
    ftz = _flush_denormal if flush_denormal is None else bool(flush_denormal)
    ys = _carve(ms, dtype, dev)
    tables = BatchTables(ms, es, ys)
    decode_batched_into(tables, dt_code(dtype), 1 if ftz else 0, stream_handle(dev))
    return ys


ops = types.SimpleNamespace(
    convert_to_fixed_point=convert_to_fixed_point,
    fixed_point_to_float_point=fixed_point_to_float_point,
    convert_to_fixed_point_batched=convert_to_fixed_point_batched,
    fixed_point_to_float_point_batched=fixed_point_to_float_point_batched,
)
