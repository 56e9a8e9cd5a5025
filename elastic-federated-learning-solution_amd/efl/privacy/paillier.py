"""efl.paillier — fixed-point codec and Paillier cipher of the forward-encryption path.

Drop-in for efls-train/python/efl/privacy/paillier.py:29-205 (same exported names, argument order
and meaning), over torch tensors; the arithmetic runs in libefl_hip.so on the MI355X.

Reference call site of the forward path (efls-train/python/efl/privacy/paillier_layer.py:64-67):
    x = fixedpoint_encode(inputs)
    x.mantissa = keypair.encrypt(x.mantissa)
    communicator.send(prefix + '_[x]_mantissa', x.mantissa.tensor)
    communicator.send(prefix + '_[x]_exponent', x.exponent)
"""
from __future__ import annotations

import torch

from efl import exporter
from efl.lib import ops as fed_ops


@exporter.export("paillier.fixedpoint.Tensor")
class FixedPointTensor(object):
    """value = mantissa * 2 ** exponent (paillier.py:107-145)."""

    def __init__(self, mantissa, exponent):
        self.mantissa = mantissa
        self.exponent = exponent

    def decode(self, dtype=torch.float32):
        m = self.mantissa
        from efl.privacy.paillier_cipher import PaillierTensor
        if isinstance(m, PaillierTensor):
            raise TypeError("decode() of an encrypted mantissa: decrypt it first")
        return fed_ops.fixed_point_to_float_point(m, self.exponent, dtype=dtype)

    # homomorphic arithmetic lives with the cipher (paillier.py:116-145)
    def __add__(self, another):
        from efl.privacy.paillier_cipher import fixedpoint_add
        return fixedpoint_add(self, another)

    def __mul__(self, another):
        from efl.privacy.paillier_cipher import fixedpoint_mul
        return fixedpoint_mul(self, another)

    def __matmul__(self, another):
        from efl.privacy.paillier_cipher import fixedpoint_matmul
        return fixedpoint_matmul(self, another)

    def __repr__(self):
        return f"FixedPointTensor(mantissa={self.mantissa!r}, exponent={self.exponent!r})"


@exporter.export("paillier.fixedpoint.encode")
def fixedpoint_encode(t, decrease_precision=None):
    """ConvertToFixedPoint (paillier.py:148-150 -> fixed_point.cc:24-199)."""
    return FixedPointTensor(*fed_ops.convert_to_fixed_point(t, decrease_precision=decrease_precision))


@exporter.export("paillier.fixedpoint.decode")
def fixedpoint_decode(fp, dtype=torch.float32):
    """FixedPointToFloatPoint (paillier.py:153-155 -> fixed_point.cc:201-287)."""
    return fed_ops.fixed_point_to_float_point(fp.mantissa, fp.exponent, dtype=dtype)
