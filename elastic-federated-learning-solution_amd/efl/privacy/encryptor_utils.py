"""Roles of the two parties of a Paillier layer (efls-train/python/efl/privacy/encryptor_utils.py)."""
from enum import Enum

from efl import exporter


@exporter.export("privacy.Role")
class Role(Enum):
    SENDER = 0
    RECEIVER = 1


class SecretSharingMatmulMode(Enum):
    """efls-train/python/efl/privacy/encryptor_utils.py:29-33 (exported there as
    secret_sharing.matmul.Mode; here reachable as efl.secret_sharing.matmul.Mode)."""
    A = 0
    B = 1
    C = 2
