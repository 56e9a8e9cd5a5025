"""MODE and task scopes (efls-train/python/efl/framework/common_define.py:22,
efls-train/python/efl/framework/task_scope.py:26-67): the (mode, task) key FederalModel files its
Paillier kernels and outputs under."""
from __future__ import annotations

import contextlib
import copy
import enum

from efl import exporter

MODE = enum.Enum("MODE", ("TRAIN", "EVAL"))
exporter.export("MODE")(MODE)


class TaskScope(object):
    def __init__(self, mode=None, task=None):
        self._mode = mode
        self._task = task

    @property
    def mode(self):
        return self._mode

    @property
    def task(self):
        return self._task

    def __str__(self):
        return "{}_{}".format(self.mode, self.task)

    def __hash__(self):
        return hash(str(self))

    def __eq__(self, other):
        return (self.mode, self.task) == (other.mode, other.task)


_CURRENT = TaskScope()


@exporter.export("task_scope")
@contextlib.contextmanager
def task_scope(mode=None, task=None):
    global _CURRENT
    old = _CURRENT
    _CURRENT = TaskScope(mode, task)
    try:
        yield
    finally:
        _CURRENT = old


@exporter.export("current_task_scope")
def current_task_scope():
    return copy.deepcopy(_CURRENT)
