"""efl — MI355X-native drop-in for the forward-encryption path of EFLS-train.

Public names mirror efls-train/python/efl (exporter registry, efl/__init__.py:47):
  efl.paillier.fixedpoint.{encode, decode, Tensor}, efl.paillier.{Keypair, Tensor}
  efl.Communicator (gRPC TrainerService, pre-send/post-recv hooks), efl.privacy.FixedPointHook
  efl.FederalModel (create_keypair, paillier_{sender,recver}_{dense,weight}, minimize), efl.MODE
  efl.secret_sharing.{matmul, Dense, dense, share, reveal}
  efl.privacy.{DPGradientDescentGaussianOptimizer, DPAdamOptimizer, ..., make_optimizer_class}
  efl.HexTensor (the DT_STRING stand-in), efl.lib.ops (the `fed_ops` namespace)
The kernels live in libefl_hip.so (C ABI: include/efl_hip.h); there is no CPU fallback.
"""
from efl import exporter
from efl import errors
from efl import lib
from efl.lib import set_flush_denormal, flush_denormal
from efl.privacy import dp_optimizer
from efl.privacy import encryptor_utils
from efl.privacy import paillier
from efl.privacy import paillier_cipher
from efl.privacy import paillier_layer
from efl.privacy import secret_sharing
from efl.privacy.hex_tensor import HexTensor
from efl.framework import communicator
from efl.framework import encrypt_hook
from efl.framework.communicator import Communicator, TensorHook
from efl.framework import task_scope as _task_scope
from efl.framework import model
from efl.framework.task_scope import MODE
from efl.framework.model import FederalModel

exporter.filldict(globals())

__version__ = "0.1.0"
