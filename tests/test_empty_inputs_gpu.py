"""Empty tensors through every op of the path: the reference's kernels loop over zero elements and
return empty outputs of the input's shape (fixed_point.cc:100-101 allocate_output(shape), the
Paillier ops' Shard over 0 elements); so must the build, with no launch of a zero-sized grid."""
import json
import os

import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "paillier_kat.json")) as f:
    KAT = json.load(f)


@pytest.fixture(scope="module")
def efl():
    import efl as _efl
    _efl.lib.require_gpu()
    return _efl


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
@pytest.mark.parametrize("shape", [(0,), (3, 0), (0, 5)])
def test_fixed_point_codec_empty(efl, dtype, shape):
    x = torch.empty(shape, dtype=dtype, device="cuda")
    fp = efl.paillier.fixedpoint.encode(x)
    assert tuple(fp.mantissa.shape) == shape and tuple(fp.exponent.shape) == shape
    assert fp.mantissa.dtype == torch.int64 and fp.exponent.dtype == torch.int64
    if dtype in (torch.float32, torch.float64):
        y = efl.paillier.fixedpoint.decode(fp, dtype=dtype)
        assert tuple(y.shape) == shape and y.dtype == dtype
    # host tensors take the same path back to the host
    fph = efl.paillier.fixedpoint.encode(x.cpu())
    assert fph.mantissa.device.type == "cpu" and tuple(fph.mantissa.shape) == shape


def test_batched_codec_empty_lists_and_entries(efl):
    assert efl.lib.ops.convert_to_fixed_point_batched([]) == ([], [])
    assert efl.lib.ops.fixed_point_to_float_point_batched([], []) == []
    xs = [torch.empty(0, device="cuda"), torch.randn(5, device="cuda"), torch.empty(0, device="cuda")]
    Ms, Es = efl.lib.ops.convert_to_fixed_point_batched(xs)
    ys = efl.lib.ops.fixed_point_to_float_point_batched(Ms, Es)
    assert [y.numel() for y in ys] == [0, 5, 0] and torch.equal(ys[1], xs[1])
    Ms, Es = efl.lib.ops.convert_to_fixed_point_batched([torch.empty(0, device="cuda")])
    assert Ms[0].numel() == 0


@pytest.mark.parametrize("private", [True, False])
def test_paillier_ops_empty(efl, private):
    k = next(k for k in KAT["keys"] if k["n_bytes"] == 128)
    kp = efl.paillier.Keypair(seed=3)
    kp.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1,
                     int(k["p"], 16), int(k["q"], 16))
    pub = efl.paillier.Keypair(seed=3)
    pub.set_keys_ints(int(k["n"], 16), int(k["hs"], 16), k["a_bits"] // 8, 1)
    enc_kp = kp if private else pub
    m = torch.empty((2, 0), dtype=torch.int64)
    ct = enc_kp.encrypt(m)
    assert tuple(ct.shape) == (2, 0)
    assert len(ct.tensor.to_hex().strings()) == 0
    d = kp.decrypt(ct, dtype=torch.int64)
    assert d.numel() == 0
    assert len(kp.decrypt(ct).strings()) == 0
    z = enc_kp.add(ct.tensor, ct.tensor)
    assert z.numel() == 0
    assert enc_kp.mul_scalar(ct.tensor, torch.empty((2, 0), dtype=torch.int64)).numel() == 0
    assert enc_kp.mul_exp2(ct.tensor, torch.empty((2, 0), dtype=torch.int64)).numel() == 0
    assert enc_kp.invert(ct.tensor).numel() == 0
    assert enc_kp.fbpowm(n=0).numel() == 0
    # the fixed-point layer ops on an empty activation
    a = torch.empty(0, 4, device="cuda")
    fa = efl.paillier.fixedpoint.encode(a)
    fa.mantissa = enc_kp.encrypt(fa.mantissa)
    c = fa + torch.empty(0, 4, device="cuda")
    assert tuple(c.mantissa.shape) == (0, 4)
    c3 = fa @ torch.randn(4, 3, device="cuda")
    assert tuple(c3.mantissa.shape) == (0, 3)
