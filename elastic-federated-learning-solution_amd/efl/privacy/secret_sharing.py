"""Secret-sharing layers: additive float masks applied before the communicator sends a share
cross-silo.

Reference: efls-train/python/efl/privacy/secret_sharing.py
  generate_suitable_noise (:26-27), _matmul modes A/B/C (:30-77), matmul + custom gradient
  (:80-109), SecretSharingDense (:112-149), dense (:152-155), share (:158-168), reveal (:171-194).

Every per-element mask runs in one HIP kernel of libefl_hip.so (csrc/mask.hip: efl_ss_noise,
efl_ss_mask_cols, efl_ss_mask_rows) that reads the tensor once and writes every share the
protocol needs, instead of TF's chain of uniform/mul/slice/add/concat ops. The products
(`(a - e) @ b1 + ...`) are plain library GEMMs (torch.matmul -> hipBLASLt). No CPU fallback.

Randomness. The reference's `tf.random.uniform` is unseeded; here the uniform is the same
construction (Philox4x32-10 + Uint32ToFloat) from a per-process `NoiseStream`: a 64-bit key drawn
from os.urandom unless `set_seed` fixes it, and a counter that advances by ceil(n/4) Philox blocks
per call, so no two masks of a process reuse a draw.

Differences from the reference, all deliberate:
  * a mode-A party passes the peer's matrix shape as `b` (a mode-B party: as `a`), which is what
    the reference indexes (`b[0] * 3 // 2`, :38) -- a tensor is accepted too and only its shape used;
  * the Dense weight noise is a constant draw for autograd (the reference differentiates through
    `uniform * kernel`, giving the kernel a random gradient factor (1 + U/d)/2 instead of 1/2).
"""
from __future__ import annotations

import os
import threading

import torch

from efl import errors, exporter, lib
from efl.privacy.encryptor_utils import Role, SecretSharingMatmulMode as Mode


class NoiseStream:
    """Philox key + block counter of this process's masks (thread-safe)."""

    def __init__(self, seed: int | None = None, counter: int = 0):
        self._lock = threading.Lock()
        self.reset(seed, counter)

    def reset(self, seed: int | None = None, counter: int = 0):
        with self._lock:
            self.seed = int.from_bytes(os.urandom(8), "little") if seed is None else int(seed) & (2**64 - 1)
            self.counter = int(counter)

    def take(self, n: int) -> tuple[int, int]:
        """(seed, ctr0) for a call over n elements; advances the counter by ceil(n / 4)."""
        with self._lock:
            ctr0 = self.counter
            self.counter = (self.counter + (n + 3) // 4) & (2**64 - 1)
            return self.seed, ctr0


_stream = NoiseStream()


@exporter.export("secret_sharing.set_seed")
def set_seed(seed: int | None, counter: int = 0) -> None:
    """Fix (or, with None, re-randomise) the mask stream of this process."""
    _stream.reset(seed, counter)


def noise_stream() -> NoiseStream:
    return _stream


def _f32_on_device(t):
    t = lib.as_tensor(t)
    if t.dtype != torch.float32:
        raise errors.InvalidArgumentError(f"secret sharing masks are float32 (tf.random.uniform), got {t.dtype}")
    x, home = lib.on_device(t.detach())
    if x.data_ptr() % 16:
        x = x.clone()
    return x, home


def _noise(t, op, divisor=1.0, stream=None):
    x, home = _f32_on_device(t)
    seed, ctr0 = (stream or _stream).take(x.numel())
    o0 = torch.empty_like(x)
    o1 = torch.empty_like(x) if op else o0
    lib.check(lib.raw().efl_ss_noise(x.data_ptr(), o0.data_ptr(), o1.data_ptr(), x.numel(), op, seed, ctr0,
                                     float(divisor), lib.stream_handle(x.device)))
    if op == 0:
        return lib.back(o0, home)
    return lib.back(o0, home), lib.back(o1, home)


@exporter.export("secret_sharing.generate_suitable_noise")
def generate_suitable_noise(t, stream=None):
    """tf.random.uniform(tf.shape(t)) * t (secret_sharing.py:26-27)."""
    return _noise(t, 0, stream=stream)


def split_share(t, stream=None):
    """(a, t - a) with a = noise(t): share()'s sent and kept parts (secret_sharing.py:162-168)."""
    return _noise(t, 1, stream=stream)


def weight_noise(w, divisor, stream=None):
    """(w - noise(w)/d, w + noise(w)/d): SecretSharingDense's sent and kept weights (:137-143)."""
    return _noise(w, 2, divisor, stream=stream)


def mask_cols(a, stream=None):
    """Mode-A side of _matmul (:31-35): e = noise(a) ->
    (send [R, 3C/2] = [a + e | e_even + e_odd], a - e, e_odd - e_even)."""
    x, home = _f32_on_device(a)
    if x.dim() != 2:
        raise errors.InvalidArgumentError(f"secret_sharing.matmul: a must be 2-D, got {tuple(x.shape)}")
    R, C = x.shape
    if C % 2:
        raise errors.InvalidArgumentError(f"secret_sharing.matmul: columns of a must be even, got {C}")
    seed, ctr0 = (stream or _stream).take(x.numel())
    send = torch.empty((R, C * 3 // 2), dtype=torch.float32, device=x.device)
    k0 = torch.empty_like(x)
    k1 = torch.empty((R, C // 2), dtype=torch.float32, device=x.device)
    lib.check(lib.raw().efl_ss_mask_cols(x.data_ptr(), send.data_ptr(), k0.data_ptr(), k1.data_ptr(), R, C,
                                         seed, ctr0, lib.stream_handle(x.device)))
    return lib.back(send, home), lib.back(k0, home), lib.back(k1, home)


def mask_rows(b, stream=None):
    """Mode-B side of _matmul (:43-47): f = noise(b) ->
    (send [3K/2, N] = [b/2 - f ; f_even - f_odd], b/2 + f, f_odd + f_even)."""
    x, home = _f32_on_device(b)
    if x.dim() != 2:
        raise errors.InvalidArgumentError(f"secret_sharing.matmul: b must be 2-D, got {tuple(x.shape)}")
    K, N = x.shape
    if K % 2:
        raise errors.InvalidArgumentError(f"secret_sharing.matmul: rows of b must be even, got {K}")
    seed, ctr0 = (stream or _stream).take(x.numel())
    send = torch.empty((K * 3 // 2, N), dtype=torch.float32, device=x.device)
    k0 = torch.empty_like(x)
    k1 = torch.empty((K // 2, N), dtype=torch.float32, device=x.device)
    lib.check(lib.raw().efl_ss_mask_rows(x.data_ptr(), send.data_ptr(), k0.data_ptr(), k1.data_ptr(), K, N,
                                         seed, ctr0, lib.stream_handle(x.device)))
    return lib.back(send, home), lib.back(k0, home), lib.back(k1, home)


def _shape(m):
    if isinstance(m, torch.Tensor):
        return tuple(int(s) for s in m.shape)
    return tuple(int(s) for s in m)


def _recv(communicator, name, shape, like):
    t = communicator.recv(name, shape=shape, dtype=torch.float32)
    return t.to(like.device)


def _matmul(a, b, communicator, name, mode):
    """secret_sharing.py:30-77. Mode A: this party holds a, `b` is the peer's shape. Mode B: holds
    b, `a` is the peer's shape. Mode C: holds both; the result summed over the two parties is
    (a_0 + a_1) @ (b_0 + b_1)."""
    mode = Mode(mode) if not isinstance(mode, Mode) else mode
    if mode == Mode.A:
        K, N = _shape(b)
        send_t, a_minus_e, eo_minus_ee = mask_cols(a)
        h = communicator.send(name + "_a1_and_e1", send_t)
        b1_and_f1 = _recv(communicator, name + "_b1_and_f1", (K * 3 // 2, N), send_t)
        b1, f1 = b1_and_f1[:K], b1_and_f1[K:]
        h.result()
        return a_minus_e @ b1 + eo_minus_ee @ f1
    if mode == Mode.B:
        R, C = _shape(a)
        send_t, half_plus_f, fo_plus_fe = mask_rows(b)
        h = communicator.send(name + "_b1_and_f1", send_t)
        a1_and_e1 = _recv(communicator, name + "_a1_and_e1", (R, C * 3 // 2), send_t)
        a1, e1 = a1_and_e1[:, :C], a1_and_e1[:, C:]
        h.result()
        return a1 @ half_plus_f - e1 @ fo_plus_fe
    if mode == Mode.C:
        if a.dtype != b.dtype:
            raise TypeError("The dtypes of a and b must be the same.")
        R, C = a.shape
        N = b.shape[1]
        z = a @ b
        a_send, a_minus_e, eo_minus_ee = mask_cols(a)
        b_send, half_plus_f, fo_plus_fe = mask_rows(b)
        send_t = torch.cat([a_send, b_send.t()], dim=0)
        h = communicator.send(name + "_a1_e1_b1_f1", send_t)
        recv = _recv(communicator, name + "_a1_e1_b1_f1", (R + N, C * 3 // 2), send_t)
        a1_e1, b1_f1 = recv[:R], recv[R:].t()
        ra1, re1 = a1_e1[:, :C], a1_e1[:, C:]
        rb1, rf1 = b1_f1[:C], b1_f1[C:]
        h.result()
        z1 = a_minus_e @ rb1 + eo_minus_ee @ rf1
        z2 = ra1 @ half_plus_f - re1 @ fo_plus_fe
        return z + z1 + z2
    raise ValueError(str(mode) + ": No such mode.")


def _grad_c(a, b, dy, communicator, name, combine_gradients):
    """The mode-C backward of matmul (secret_sharing.py:83-106)."""
    if combine_gradients:
        B, U = dy.shape
        R, C = a.shape
        z = dy.new_zeros
        dy_at = torch.cat([torch.cat([dy, z((B, B))], dim=1),
                           torch.cat([torch.zeros_like(b), a.t()], dim=1)], dim=0)
        bt_dy = torch.cat([torch.cat([b.t(), z((U, U))], dim=1),
                           torch.cat([torch.zeros_like(a), dy], dim=1)], dim=0)
        da_db = _matmul(dy_at, bt_dy, communicator, name + "_gradient", Mode.C)
        return da_db[:R, :C], da_db[-C:, -U:]
    da = _matmul(dy, b.t().contiguous(), communicator, name + "_da", Mode.C)
    db = _matmul(a.t().contiguous(), dy, communicator, name + "_db", Mode.C)
    return da, db


class _SSMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, communicator, name, mode, combine_gradients):
        ctx.save_for_backward(a, b)
        ctx.args = (communicator, name, mode, combine_gradients)
        return _matmul(a, b, communicator, name, mode)

    @staticmethod
    def backward(ctx, dy):
        communicator, name, mode, combine_gradients = ctx.args
        if mode == Mode.A:
            raise ValueError("Please switch from mode A to mode C, because mode A is equivalent to mode C "
                             "when the gradients need to be computed.")
        if mode == Mode.B:
            raise ValueError("Please switch from mode B to mode C, because mode B is equivalent to mode C "
                             "when the gradients need to be computed.")
        a, b = ctx.saved_tensors
        da, db = _grad_c(a, b, dy.contiguous(), communicator, name, combine_gradients)
        return da, db, None, None, None, None


@exporter.export("secret_sharing.matmul")
def matmul(a, b, communicator, name, mode, combine_gradients=False):
    """secret_sharing.py:80-109: the secret-shared product, differentiable in mode C."""
    mode = Mode(mode) if not isinstance(mode, Mode) else mode
    if mode == Mode.C and (a.requires_grad or b.requires_grad) and torch.is_grad_enabled():
        return _SSMatmul.apply(a, b, communicator, name, mode, combine_gradients)
    if mode == Mode.C:
        return _matmul(a, b, communicator, name, mode)
    if mode == Mode.A and isinstance(a, torch.Tensor) and a.requires_grad and torch.is_grad_enabled():
        return _ModeAB.apply(a, communicator, name, mode, _shape(b))
    if mode == Mode.B and isinstance(b, torch.Tensor) and b.requires_grad and torch.is_grad_enabled():
        return _ModeAB.apply(b, communicator, name, mode, _shape(a))
    return _matmul(a, b, communicator, name, mode)


matmul.Mode = Mode   # the reference exports the enum as secret_sharing.matmul.Mode


class _ModeAB(torch.autograd.Function):
    """Modes A and B forward; their backward raises as the reference's grad does (:84-87)."""

    @staticmethod
    def forward(ctx, held, communicator, name, mode, peer_shape):
        ctx.mode = mode
        if mode == Mode.A:
            return _matmul(held, peer_shape, communicator, name, mode)
        return _matmul(peer_shape, held, communicator, name, mode)

    @staticmethod
    def backward(ctx, dy):
        letter = "A" if ctx.mode == Mode.A else "B"
        raise ValueError(f"Please switch from mode {letter} to mode C, because mode {letter} is equivalent "
                         "to mode C when the gradients need to be computed.")


class _Share(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, communicator, name):
        ctx.args = (communicator, name)
        a, kept = split_share(inputs)
        communicator.send(name, a).result()
        return kept

    @staticmethod
    def backward(ctx, dy):
        communicator, name = ctx.args
        return dy + _recv(communicator, name + "_grad", tuple(dy.shape), dy), None, None


@exporter.export("secret_sharing.share")
def share(inputs, communicator, name):
    """secret_sharing.py:158-168: send a = noise(inputs) to the peer, keep inputs - a. The gradient
    adds the peer's gradient share received as name + '_grad'."""
    return _Share.apply(inputs, communicator, name)


class _Reveal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, communicator, name, role):
        ctx.args = (communicator, name, role)
        if role == Role.SENDER:
            communicator.send(name, inputs).result()
            return inputs.clone()
        if role == Role.RECEIVER:
            return inputs + _recv(communicator, name, tuple(inputs.shape), inputs)
        raise ValueError(str(role) + ": No such role.")

    @staticmethod
    def backward(ctx, dy):
        communicator, name, role = ctx.args
        if role == Role.RECEIVER:
            a, kept = split_share(dy.contiguous())
            communicator.send(name + "_grad", a).result()
            return kept, None, None, None
        return _recv(communicator, name + "_grad", tuple(dy.shape), dy), None, None, None


@exporter.export("secret_sharing.reveal")
def reveal(inputs, communicator, name, role):
    """secret_sharing.py:171-194: the sender sends its share, the receiver adds it; backward the
    receiver re-shares its gradient (noise sent as name + '_grad')."""
    if role not in (Role.SENDER, Role.RECEIVER):
        raise ValueError(str(role) + ": No such role.")
    return _Reveal.apply(inputs, communicator, name, role)


@exporter.export("secret_sharing.Dense")
class SecretSharingDense(torch.nn.Module):
    """secret_sharing.py:112-149 (a tf.layers.Dense): outputs = matmul(inputs, kernel, mode C) + bias.
    The kernel [in, units] is built on the first call from inputs' last dimension, like a Keras
    layer; `kernel_initializer(tensor)` fills it in place (default glorot-uniform as TF's)."""

    def __init__(self, communicator, prefix, units, noise_divisor=None, combine_gradients=False,
                 use_bias=True, kernel_initializer=None, bias_initializer=None, **kwargs):
        super().__init__()
        self._communicator = communicator
        self._prefix = prefix
        self.units = int(units)
        self._noise_divisor = noise_divisor
        self._combine_gradients = combine_gradients
        self.use_bias = use_bias
        self._kernel_init = kernel_initializer
        self._bias_init = bias_initializer
        self.kernel = None
        self.bias = None

    def _build(self, inputs):
        fan_in = int(inputs.shape[-1])
        w = torch.empty((fan_in, self.units), dtype=torch.float32, device=inputs.device)
        if self._kernel_init is not None:
            with torch.no_grad():
                self._kernel_init(w)
        else:
            torch.nn.init.xavier_uniform_(w)
        self.kernel = torch.nn.Parameter(w)
        if self.use_bias:
            bias = torch.zeros(self.units, dtype=torch.float32, device=inputs.device)
            if self._bias_init is not None:
                with torch.no_grad():
                    self._bias_init(bias)
            self.bias = torch.nn.Parameter(bias)

    def forward(self, inputs):
        if inputs.dim() > 2:
            raise ValueError("SecretSharingDense hasn't support broadcasting yet.")
        if self.kernel is None:
            self._build(inputs)
        kernel = self.kernel
        if self._noise_divisor is not None:
            sent, kept = weight_noise(kernel.detach(), self._noise_divisor)
            h = self._communicator.send(self._prefix + "_weights", sent)
            peer = _recv(self._communicator, self._prefix + "_weights", tuple(kernel.shape), kernel)
            h.result()
            kernel = (kernel + (kept - kernel.detach()) + peer) / 2
        outputs = matmul(inputs, kernel, self._communicator, self._prefix, Mode.C,
                         combine_gradients=self._combine_gradients)
        if self.use_bias:
            outputs = outputs + self.bias
        return outputs

    def apply(self, inputs):
        return self(inputs)


@exporter.export("secret_sharing.dense")
def dense(inputs, communicator, prefix, units, noise_divisor=None, combine_gradients=False, **kwargs):
    """secret_sharing.py:152-155. Returns (outputs, layer), as efl.paillier.*.dense do: a torch
    tensor cannot carry the layer's variables the way a TF graph collection does."""
    layer = SecretSharingDense(communicator, prefix, units, noise_divisor=noise_divisor,
                               combine_gradients=combine_gradients, **kwargs)
    return layer(inputs), layer
