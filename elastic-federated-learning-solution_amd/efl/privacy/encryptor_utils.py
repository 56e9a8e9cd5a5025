"""Roles of the two parties of a Paillier layer (efls-train/python/efl/privacy/encryptor_utils.py)."""
from enum import Enum

from efl import exporter


@exporter.export("privacy.Role")
class Role(Enum):
    SENDER = 0
    RECEIVER = 1
