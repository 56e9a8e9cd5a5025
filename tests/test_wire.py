"""CPU: efl.framework.wire is byte-compatible with the reference's protobuf messages.

The expected side is the protobuf runtime itself, with descriptors declared from the reference's
.proto field numbers (efls-train/protos/trainer_service.proto:13-22; vendored
tensorflow/core/framework/tensor.proto:15-64, tensor_shape.proto, types.proto).
"""
import numpy as np
import pytest
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

import efl
from efl.framework import wire

F = descriptor_pb2.FieldDescriptorProto


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="efl_test_wire.proto", package="efltest", syntax="proto3")
    dim = fd.message_type.add(name="Dim")
    dim.field.add(name="size", number=1, type=F.TYPE_INT64, label=F.LABEL_OPTIONAL)
    dim.field.add(name="name", number=2, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    shp = fd.message_type.add(name="TensorShapeProto")
    shp.field.add(name="dim", number=2, type=F.TYPE_MESSAGE, type_name=".efltest.Dim", label=F.LABEL_REPEATED)
    shp.field.add(name="unknown_rank", number=3, type=F.TYPE_BOOL, label=F.LABEL_OPTIONAL)
    tp = fd.message_type.add(name="TensorProto")
    tp.field.add(name="dtype", number=1, type=F.TYPE_INT32, label=F.LABEL_OPTIONAL)   # enum DataType
    tp.field.add(name="tensor_shape", number=2, type=F.TYPE_MESSAGE, type_name=".efltest.TensorShapeProto",
                 label=F.LABEL_OPTIONAL)
    tp.field.add(name="version_number", number=3, type=F.TYPE_INT32, label=F.LABEL_OPTIONAL)
    tp.field.add(name="tensor_content", number=4, type=F.TYPE_BYTES, label=F.LABEL_OPTIONAL)
    tp.field.add(name="float_val", number=5, type=F.TYPE_FLOAT, label=F.LABEL_REPEATED)
    tp.field.add(name="double_val", number=6, type=F.TYPE_DOUBLE, label=F.LABEL_REPEATED)
    tp.field.add(name="int_val", number=7, type=F.TYPE_INT32, label=F.LABEL_REPEATED)
    tp.field.add(name="string_val", number=8, type=F.TYPE_BYTES, label=F.LABEL_REPEATED)
    tp.field.add(name="int64_val", number=10, type=F.TYPE_INT64, label=F.LABEL_REPEATED)
    mr = fd.message_type.add(name="MessageRequest")
    mr.field.add(name="name", number=1, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    mr.field.add(name="step", number=2, type=F.TYPE_UINT64, label=F.LABEL_OPTIONAL)
    mr.field.add(name="tensor", number=3, type=F.TYPE_MESSAGE, type_name=".efltest.TensorProto", label=F.LABEL_OPTIONAL)
    rs = fd.message_type.add(name="MessageResponse")
    rs.field.add(name="code", number=1, type=F.TYPE_INT32, label=F.LABEL_OPTIONAL)   # enum error.Code
    rs.field.add(name="msg", number=2, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName("efltest." + n)) for n in
            ("TensorProto", "MessageRequest", "MessageResponse")}


PB = _build()

CASES = [
    ("x_[x]_exponent", 0, np.arange(12, dtype=np.int64).reshape(3, 4) - 5),
    ("t", 7, np.random.default_rng(0).standard_normal((2, 3, 5)).astype(np.float32)),
    ("d", 2**40 + 3, np.array(3.5)),                                  # scalar
    ("empty", 1, np.zeros((0, 4), np.float32)),                        # zero-size dim
    ("i32", 12, np.array([-1, 2, -2**31], np.int32)),
    ("u8", 3, np.array([0, 255, 7], np.uint8)),
]


@pytest.mark.parametrize("name,step,arr", CASES, ids=[c[0] for c in CASES])
def test_request_matches_protobuf(name, step, arr):
    dt = wire.DT_OF_NP[arr.dtype]
    ours = wire.message_request(name, step, dt, arr.shape, arr.tobytes())
    m = PB["MessageRequest"]()
    m.name, m.step = name, step
    m.tensor.dtype = dt
    m.tensor.tensor_shape.SetInParent()       # TF: shape_.AsProto(proto->mutable_tensor_shape())
    for d in arr.shape:
        m.tensor.tensor_shape.dim.add(size=d)
    if arr.size:
        m.tensor.tensor_content = arr.tobytes()
    assert ours == m.SerializeToString()
    n2, s2, t2 = wire.parse_message_request(m.SerializeToString())
    assert (n2, s2, t2.dtype, t2.shape) == (name, step, dt, arr.shape)
    assert np.array_equal(t2.to_numpy(), arr)


def test_string_tensor_content_matches_tf_encoding():
    strs = ["1f" * 40, "", "-abc", "0"] * 50
    hx = efl.HexTensor.from_strings(np.array(strs, dtype=object).reshape(20, 10))
    body = hx.to_tensor_content()
    # EncodeStringList: every varint32 length first, then the bytes
    lens = b"".join(wire.varint(len(s)) for s in strs)
    assert body == lens + "".join(strs).encode()
    req = wire.message_request("c", 1, wire.DT_STRING, hx.shape, body)
    m = PB["MessageRequest"].FromString(req)
    assert m.tensor.dtype == 7 and bytes(m.tensor.tensor_content) == body
    _, _, t = wire.parse_message_request(req)
    back = efl.HexTensor.from_tensor_content(bytes(t.content), t.shape)
    assert back == hx and back.strings() == strs


def test_string_length_varints_vectorised():
    """The numpy varint32 codec of DT_STRING lengths equals the scalar protobuf varint at every
    width boundary, parses back, and rejects truncated or over-long headers."""
    from efl.privacy import hex_tensor as ht
    edges = [0, 1, 127, 128, 16383, 16384, 2**21 - 1, 2**21, 2**28 - 1, 2**28, 2**32 - 1]
    rng = np.random.default_rng(4)
    lens = np.array(edges + rng.integers(0, 2**32, 300).tolist() + rng.integers(0, 600, 300).tolist(), np.int64)
    enc = ht._varint32_encode(lens)
    assert enc.tobytes() == b"".join(wire.varint(int(v)) for v in lens)
    tail = np.frombuffer(b"\x05\x80abc", np.uint8)            # bytes after the header do not matter
    vals, used = ht._varint32_decode(np.concatenate([enc, tail]), lens.size)
    assert np.array_equal(vals, lens) and used == enc.size
    with pytest.raises(ValueError):
        ht._varint32_decode(enc[:-1], lens.size)               # last length cut off
    with pytest.raises(ValueError):
        ht._varint32_decode(np.array([0x80] * 6 + [1], np.uint8), 1)
    with pytest.raises(ValueError):
        ht._varint32_encode(np.array([2**32]))
    with pytest.raises(ValueError):                             # lengths promise more bytes than sent
        efl.HexTensor.from_tensor_content(b"\x05ab", (1,))


def test_typed_fields_like_tf_fromproto():
    m = PB["MessageRequest"](name="v", step=1)
    m.tensor.dtype = wire.DT_FLOAT
    for d in (2, 3):
        m.tensor.tensor_shape.dim.add(size=d)
    m.tensor.float_val.extend([1.5, -2.0])      # fewer values than elements: last one repeats
    _, _, t = wire.parse_message_request(m.SerializeToString())
    assert np.array_equal(t.to_numpy(), np.array([[1.5, -2, -2], [-2, -2, -2]], np.float32))
    m2 = PB["MessageRequest"](name="s")
    m2.tensor.dtype = wire.DT_STRING
    m2.tensor.tensor_shape.dim.add(size=2)
    m2.tensor.string_val.extend([b"ab", b"-1"])
    _, _, t2 = wire.parse_message_request(m2.SerializeToString())
    assert t2.typed == [b"ab", b"-1"]
    m3 = PB["MessageRequest"](name="l")
    m3.tensor.dtype = wire.DT_INT64
    m3.tensor.tensor_shape.dim.add(size=3)
    m3.tensor.int64_val.extend([-5, 2**62, 0])
    _, _, t3 = wire.parse_message_request(m3.SerializeToString())
    assert np.array_equal(t3.to_numpy(), np.array([-5, 2**62, 0]))


@pytest.mark.parametrize("code,msg", [(0, ""), (15, "Tensor named a expects step 1, but given step 2."), (4, "x")])
def test_response_matches_protobuf(code, msg):
    ours = wire.message_response(code, msg)
    assert ours == PB["MessageResponse"](code=code, msg=msg).SerializeToString()
    assert wire.parse_message_response(ours) == (code, msg)


def test_message_assembled_in_place_from_mixed_parts():
    """message_request builds the request in one new bytes object: host parts, torch uint8 tensors
    (device text in production) and a split tensor_content give the same bytes as a plain join."""
    import numpy as np
    import torch
    from efl.framework import wire
    from efl.privacy.hex_tensor import HexTensor
    hx = HexTensor.from_strings(["1f", "abcdef", "-3", "0" * 300])
    head, text = hx.tensor_content_parts()
    want = wire.message_request("x_[x]_mantissa", 7, wire.DT_STRING, hx.shape, bytes(head) + bytes(text))
    got = wire.message_request("x_[x]_mantissa", 7, wire.DT_STRING, hx.shape, (head, torch.from_numpy(text.copy())))
    assert isinstance(got, bytes) and got == want
    got2 = wire.message_request("x_[x]_mantissa", 7, wire.DT_STRING, hx.shape, [memoryview(head), text])
    assert got2 == want
    # tiny messages never write into the interpreter's shared 0/1-byte objects
    assert wire._assemble([b""], 0) == b"" and wire._assemble([b"a"], 1) == b"a"
    t = torch.arange(10, dtype=torch.int64)
    assert wire.message_request("t", 0, wire.DT_INT64, (10,), t.numpy()) == \
        wire.message_request("t", 0, wire.DT_INT64, (10,), t.numpy().tobytes())
    name, step, msg = wire.parse_message_request(got)
    assert (name, step) == ("x_[x]_mantissa", 7)
    assert HexTensor.from_tensor_content(msg.content, msg.shape).strings() == hx.strings()
    assert np.array_equal(np.frombuffer(bytes(b"ab"), np.uint8), np.array([97, 98], np.uint8))
