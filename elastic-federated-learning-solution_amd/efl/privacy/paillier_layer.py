"""Two-party Paillier layers — the call sites of the forward-encryption path.

Port of the protocol of efls-train/python/efl/privacy/paillier_layer.py to torch autograd: the
same messages, names, order of sends/receives and noise masking, with the arithmetic on the MI355X:

  sender (key owner, `paillier.sender.Dense`, :26-85)      receiver (`paillier.recver.Dense`, :96-163)
  forward: encode(x), encrypt -> send [x]_mantissa/_exponent
                                                           recv [x]; z = [x] @ encode(W, dp=True)
                                                           n1 ~ N(0,1); send [z+n1]
           recv [z+n1], decrypt, decode, + x @ w_s
           send z+n1                                        recv z+n1; return z+n1 - n1
  backward: send [nw]; recv [dw+n2] -> decrypt -> + nf     [dw] = [x]^T @ encode(dy); send [dw+n2]
           send dw+n2; recv [dx] -> decrypt -> dx          recv dw+n2 -> dw; recv [nw];
                                                           [dx] = [nw] @ encode(dy)^T + dy W^T; send [dx]
Weight variants (:209-360) use an element-wise product instead of the matmul.

Every message crosses `efl.Communicator` (gRPC, DT_STRING hex ciphertexts) exactly as the
reference sends them, so either side can talk to a reference peer.
"""
from __future__ import annotations

import torch

from efl import exporter
from efl.privacy.paillier import FixedPointTensor, fixedpoint_encode
from efl.privacy.paillier_cipher import PaillierTensor


def _decrypt_decode(keypair, m, e):
    return FixedPointTensor(keypair.decrypt(m), e).decode()


def _wait(handles):
    for h in handles:
        h.result()


class _SenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, w, layer):
        kp, comm, p = layer.keypair, layer.communicator, layer.prefix
        x = fixedpoint_encode(inputs)
        x.mantissa = kp.encrypt(x.mantissa)
        hs = [comm.send(p + "_[x]_mantissa", x.mantissa.tensor), comm.send(p + "_[x]_exponent", x.exponent)]
        z_add_n1 = layer.local(inputs, w)
        shape = tuple(z_add_n1.shape)
        m = comm.recv(p + "_[z+n1]_mantissa", shape=shape, dtype="string")
        e = comm.recv(p + "_[z+n1]_exponent", shape=shape, dtype=torch.int64)
        z_add_n1 = z_add_n1 + _decrypt_decode(kp, m, e).to(z_add_n1.device)
        hs.append(comm.send(p + "_z+n1", z_add_n1))
        _wait(hs)
        ctx.layer = layer
        ctx.save_for_backward(inputs, w)
        return z_add_n1.clone()

    @staticmethod
    def backward(ctx, dy):
        layer = ctx.layer
        inputs, w = ctx.saved_tensors
        kp, comm, p = layer.keypair, layer.communicator, layer.prefix
        shape = tuple(w.shape)
        nw = fixedpoint_encode(w)
        nw.mantissa = kp.encrypt(nw.mantissa)
        nf = torch.randn(shape, generator=layer.generator, device="cpu").to(w.device) + \
            10 * torch.sigmoid(inputs.sum())
        hs = [comm.send(p + "_[nw]_mantissa", nw.mantissa.tensor), comm.send(p + "_[nw]_exponent", nw.exponent)]
        m = comm.recv(p + "_[dw+n2]_mantissa", shape=shape, dtype="string")
        e = comm.recv(p + "_[dw+n2]_exponent", shape=shape, dtype=torch.int64)
        dw_add_n2 = _decrypt_decode(kp, m, e).to(w.device) + nf
        hs.append(comm.send(p + "_dw+n2", dw_add_n2))
        ishape = tuple(inputs.shape)
        m = comm.recv(p + "_[dx]_mantissa", shape=ishape, dtype="string")
        e = comm.recv(p + "_[dx]_exponent", shape=ishape, dtype=torch.int64)
        dx = _decrypt_decode(kp, m, e).to(inputs.device)
        _wait(hs)
        return dx, -nf, None


class _ReceiverFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_exponent, w, layer):
        kp, comm, p = layer.keypair, layer.communicator, layer.prefix
        shape = tuple(x_exponent.shape)
        x_mantissa = comm.recv(p + "_[x]_mantissa", shape=shape, dtype="string")
        x = FixedPointTensor(PaillierTensor(kp, kp._cipher(x_mantissa)), x_exponent)
        z = layer.cipher_product(x, fixedpoint_encode(w, decrease_precision=True))
        n1 = torch.randn(tuple(z.exponent.shape), generator=layer.generator).to(w.device)
        z_add_n1 = z + n1
        hs = [comm.send(p + "_[z+n1]_mantissa", z_add_n1.mantissa.tensor),
              comm.send(p + "_[z+n1]_exponent", z_add_n1.exponent)]
        z_add_n1 = comm.recv(p + "_z+n1", shape=tuple(z.exponent.shape)).to(w.device)
        _wait(hs)
        ctx.layer, ctx.x = layer, x
        ctx.save_for_backward(x_exponent, w)
        return z_add_n1 - n1

    @staticmethod
    def backward(ctx, dy):
        layer, x = ctx.layer, ctx.x
        x_exponent, w = ctx.saved_tensors
        kp, comm, p = layer.keypair, layer.communicator, layer.prefix
        dw = layer.cipher_grad_w(x, dy)
        n2 = torch.randn(tuple(w.shape), generator=layer.generator).to(w.device)
        dw_add_n2 = dw + n2
        hs = [comm.send(p + "_[dw+n2]_mantissa", dw_add_n2.mantissa.tensor),
              comm.send(p + "_[dw+n2]_exponent", dw_add_n2.exponent)]
        dw = comm.recv(p + "_dw+n2", shape=tuple(w.shape)).to(w.device) - n2
        dx_plain = layer.plain_grad_x(dy, w)
        nw_m = comm.recv(p + "_[nw]_mantissa", shape=tuple(w.shape), dtype="string")
        nw_e = comm.recv(p + "_[nw]_exponent", shape=tuple(w.shape), dtype=torch.int64)
        nw = FixedPointTensor(PaillierTensor(kp, kp._cipher(nw_m)), nw_e)
        dx = layer.cipher_grad_x(nw, dy) + dx_plain
        hs += [comm.send(p + "_[dx]_mantissa", dx.mantissa.tensor), comm.send(p + "_[dx]_exponent", dx.exponent)]
        _wait(hs)
        return torch.zeros_like(x_exponent, dtype=torch.float32), dw, None


class _LayerBase(torch.nn.Module):
    def __init__(self, keypair, communicator, prefix, units, seed=None):
        super().__init__()
        self.keypair, self.communicator, self.prefix, self.units = keypair, communicator, prefix, units
        self.generator = torch.Generator()
        if seed is not None:
            self.generator.manual_seed(seed)


@exporter.export("paillier.sender.Dense")
class PaillierActiveDense(_LayerBase):
    """paillier_layer.py:26-85: kernel zeros, not trainable through the optimizer."""

    def __init__(self, keypair, communicator, prefix, units, name=None, _reuse=None, seed=None):
        super().__init__(keypair, communicator, prefix, units, seed)
        self.kernel = None

    def local(self, inputs, w):
        return inputs @ w

    def forward(self, inputs):
        if inputs.dim() > 2:
            raise ValueError("PaillierDense hasn't support broadcasting yet.")
        if self.kernel is None:
            self.kernel = torch.nn.Parameter(torch.zeros(inputs.shape[-1], self.units, device=inputs.device))
        return _SenderFn.apply(inputs, self.kernel, self)


@exporter.export("paillier.recver.Dense")
class PaillierPassiveDense(_LayerBase):
    """paillier_layer.py:96-163. Input: the received [x]_exponent; output x @ W."""

    def __init__(self, keypair, communicator, prefix, units, kernel_initializer=None, name=None, dtype=None,
                 _scope=None, _reuse=None, seed=None):
        super().__init__(keypair, communicator, prefix, units, seed)
        self.kernel = None
        self._init = kernel_initializer

    def cipher_product(self, x, fw):
        return x @ fw

    def cipher_grad_w(self, x, dy):
        fpdy = fixedpoint_encode(dy, decrease_precision=True)
        xt = FixedPointTensor(PaillierTensor(self.keypair, x.mantissa.tensor.transpose()), x.exponent.t())
        return xt @ fpdy

    def plain_grad_x(self, dy, w):
        return dy @ w.t()

    def cipher_grad_x(self, nw, dy):
        fpdy = fixedpoint_encode(dy, decrease_precision=True)
        fp = nw @ FixedPointTensor(fpdy.mantissa.t().contiguous(), fpdy.exponent.t().contiguous())
        return FixedPointTensor(PaillierTensor(self.keypair, fp.mantissa.tensor.transpose()), fp.exponent.t())

    def forward(self, x_exponent):
        if x_exponent.dim() > 2:
            raise ValueError("PaillierDense hasn't support broadcasting yet.")
        if self.kernel is None:
            w = torch.empty(x_exponent.shape[-1], self.units)          # host draw: seeded generator
            if self._init is None:
                torch.nn.init.xavier_uniform_(w, generator=self.generator)
            else:
                self._init(w)
            self.kernel = torch.nn.Parameter(w.to(x_exponent.device))
        return _ReceiverFn.apply(x_exponent, self.kernel, self)


@exporter.export("paillier.sender.Weight")
class PaillierActiveWeight(PaillierActiveDense):
    """paillier_layer.py:209-270: element-wise weight of shape (units,)."""

    def local(self, inputs, w):
        return inputs * w

    def forward(self, inputs):
        if inputs.dim() > 2:
            raise ValueError("PaillierDense hasn't support broadcasting yet.")
        if self.kernel is None:
            self.kernel = torch.nn.Parameter(torch.zeros(self.units, device=inputs.device))
        return _SenderFn.apply(inputs, self.kernel, self)


@exporter.export("paillier.recver.Weight")
class PaillierPassiveWeight(PaillierPassiveDense):
    """paillier_layer.py:279-346: z = [x] * encode(w); dw = sum_rows([x] * encode(dy))."""

    def cipher_product(self, x, fw):
        return x * fw

    def cipher_grad_w(self, x, dy):
        """dw = the column sums of [x] * encode(dy). The reference adds the rows one at a time in a
        tf.while_loop (:297-310): acc + row aligns the two exponents to their minimum and multiplies,
        so after all rows the mantissa is prod_r [x dy]_rc^(2^(e_rc - min_r e_rc)) mod n^2 with
        exponent min_r e_rc, whatever the order. That is exactly a PaillierMatmul of [x dy]^T by a
        column of ones with exponent 0 (paillier.cc:915-1053): one Straus multi-exponentiation per
        column (max_r d squarings instead of sum_r d), one launch instead of rows - 1 adds; the same
        ciphertext bits (tests/test_paillier_layer_gpu.py checks them against the sequential sum)."""
        dw = x * fixedpoint_encode(dy, decrease_precision=True)
        return column_sum(self.keypair, dw)

    def plain_grad_x(self, dy, w):
        return dy * w

    def cipher_grad_x(self, nw, dy):
        return nw * dy

    def forward(self, x_exponent):
        if self.kernel is None:
            w = torch.zeros(self.units, device=x_exponent.device)
            if self._init is not None:
                self._init(w)
            self.kernel = torch.nn.Parameter(w)
        return _ReceiverFn.apply(x_exponent, self.kernel, self)


def _device_of(inputs):
    """The receiver's kernel lives where its plaintext inputs are, else on the GPU the cipher runs on."""
    if inputs is not None:
        return inputs.device
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def column_sum(keypair, fp):
    """sum over rows of a FixedPointTensor with an encrypted [rows, cols] mantissa -> [cols]
    (PaillierPassiveWeight's gradient reduction, paillier_layer.py:297-310), as one
    PaillierMatmul by ones: [cols, rows] x [rows, 1]."""
    m = fp.mantissa.tensor
    rows, cols = m.shape
    e = torch.as_tensor(fp.exponent).to(m.limbs.device, torch.int64)
    ones = torch.ones((rows, 1), dtype=torch.int64, device=m.limbs.device)
    zm, ze = keypair.matmul(m.transpose(), e.t().contiguous(), ones, torch.zeros_like(ones))
    return FixedPointTensor(PaillierTensor(keypair, zm.reshape((cols,))), ze.reshape(cols))


def sequential_column_sum(keypair, fp):
    """The reference's row-by-row loop (paillier_layer.py:297-310) over FixedPointTensor.__add__:
    the definition column_sum is tested against."""
    from efl.privacy.paillier_cipher import CipherTensor
    m = fp.mantissa.tensor
    rows, cols = m.shape

    def row(i):
        return CipherTensor(m.limbs[i * cols:(i + 1) * cols].contiguous(), (cols,), m.key)
    acc = FixedPointTensor(PaillierTensor(keypair, row(0)), fp.exponent[0])
    for i in range(1, rows):
        acc = acc + FixedPointTensor(PaillierTensor(keypair, row(i)), fp.exponent[i])
    return acc


# ----------------------------------------------------------------------------------------------
# functional forms. TF1 runs them once, while building the graph, and tf.layers keeps their
# variables by scope name (`name`, `_reuse`, paillier_layer.py:166-203). Eagerly they run every
# step, so each layer (and the receiver's plaintext Dense) is built once per (communicator,
# function, prefix, name) and found again on later calls: its weights persist and train.
# ----------------------------------------------------------------------------------------------

def cached_layers(communicator) -> dict:
    """The layers the functional forms built on `communicator`, keyed (function, prefix, name);
    collect their parameters for the optimizer from here."""
    reg = getattr(communicator, "_efl_paillier_layers", None)
    if reg is None:
        reg = {}
        setattr(communicator, "_efl_paillier_layers", reg)
    return reg


def _cached(communicator, key, build, keypair=None, units=None):
    """The layer built for `key` on this communicator (built on first use). A later call with a
    different keypair object (a rotated key) re-points the layer at it; one with a different
    `units` is an error, as TF's variable reuse with a mismatched shape is."""
    reg = cached_layers(communicator)
    layer = reg.get(key)
    if layer is None:
        layer = reg[key] = build()
        return layer
    if units is not None and getattr(layer, "units", units) != units:
        from efl import errors
        raise errors.InvalidArgumentError(f"layer {key} was built with units={layer.units}, called with {units}")
    if keypair is not None and getattr(layer, "keypair", keypair) is not keypair:
        layer.keypair = keypair
    return layer


def _plain_dense(in_features, units, use_bias, kernel_initializer, bias_initializer, device):
    """tf.layers.Dense(units) of the receiver's own features: kernel glorot-uniform (TF's default)
    unless kernel_initializer is given (a callable filling a [in, units] tensor in place, TF's
    orientation), bias zeros unless bias_initializer is given."""
    lin = torch.nn.Linear(in_features, units, bias=use_bias)
    with torch.no_grad():
        w = torch.empty(in_features, units)
        if kernel_initializer is None:
            torch.nn.init.xavier_uniform_(w)
        else:
            kernel_initializer(w)
        lin.weight.copy_(w.t())
        if use_bias:
            if bias_initializer is None:
                lin.bias.zero_()
            else:
                bias_initializer(lin.bias)
    return lin.to(device)


@exporter.export("paillier.sender.dense")
def dense_send(inputs, keypair, communicator, prefix, units, name=None, reuse=None, seed=None):
    layer = _cached(communicator, ("sender.dense", prefix, name),
                    lambda: PaillierActiveDense(keypair, communicator, prefix, units, name=name, _reuse=reuse,
                                                seed=seed), keypair, units)
    return layer(inputs), layer.kernel


@exporter.export("paillier.recver.dense")
def dense_recv(inputs, keypair, communicator, prefix, recv_shape, units, activation=None, use_bias=True,
               kernel_initializer=None, bias_initializer=None, name=None, reuse=None, seed=None, **_unused):
    layer = _cached(communicator, ("recver.dense", prefix, name),
                    lambda: PaillierPassiveDense(keypair, communicator, prefix, units,
                                                 kernel_initializer=kernel_initializer, seed=seed), keypair, units)
    x_exponent = communicator.recv(prefix + "_[x]_exponent", shape=recv_shape, dtype=torch.int64)
    y = layer(x_exponent.to(_device_of(inputs)))
    if inputs is not None:
        lin = _cached(communicator, ("recver.dense.plain", prefix, name),
                      lambda: _plain_dense(inputs.shape[-1], units, use_bias, kernel_initializer,
                                           bias_initializer, inputs.device))
        y = y + lin(inputs)
    if activation is not None:
        y = activation(y)
    return y, layer.kernel


@exporter.export("paillier.sender.weight")
def weight_send(inputs, keypair, communicator, prefix, units, seed=None):
    layer = _cached(communicator, ("sender.weight", prefix, None),
                    lambda: PaillierActiveWeight(keypair, communicator, prefix, units, seed=seed), keypair, units)
    return layer(inputs), layer.kernel


@exporter.export("paillier.recver.weight")
def weight_recv(inputs, keypair, communicator, prefix, units, kernel_initializer=None, seed=None):
    layer = _cached(communicator, ("recver.weight", prefix, None),
                    lambda: PaillierPassiveWeight(keypair, communicator, prefix, units,
                                                  kernel_initializer=kernel_initializer, seed=seed), keypair, units)
    x_exponent = communicator.recv(prefix + "_[x]_exponent", shape=(-1, units), dtype=torch.int64)
    y = layer(x_exponent.to(_device_of(inputs)))
    if inputs is not None:
        y = y + inputs
    return y, layer.kernel
