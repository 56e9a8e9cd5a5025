"""FederalModel — the Paillier entry points of efls-train's model API and the learning-rate update
of the Paillier kernels (efls-train/python/efl/framework/model.py:490-815).

The reference's FederalModel is a TF1 graph builder (loss_fn / optimizer_fn / compile / fit over a
MonitoredTrainingSession); only its Paillier surface and its send/recv sit on the forward-encryption
path, and that is what this class carries, eagerly, over torch:

  create_keypair(name, role, ...)                  model.py:543-570  keypair + PaillierHook
  paillier_sender_dense / paillier_recver_dense    model.py:572-625  register (kernel, learning_rate)
  paillier_sender_weight / paillier_recver_weight  model.py:627-677
  send / recv                                      model.py:679-716
  minimize(optimizer, loss)                        model.py:718-815  (the Paillier part of _minimize)

Why the kernels get their own update. Both parties' Paillier kernels are created trainable=False
(paillier_layer.py:29-30, 104-110), so the user's optimizer never sees them; `_minimize` adds them to
the variables it differentiates and applies `lr * grad` with a separate GradientDescentOptimizer(1.)
(model.py:808-814), each kernel with the learning rate it was registered with. The sender's kernel is
a zero-initialised share whose gradient is -nf (its mask), registered with the PEER's learning rate;
the receiver's kernel gets dw + nf. After the update
    W_recv + w_send  ->  W_recv + w_send - lr * dw,
plain SGD of x @ (W_recv + w_send), while neither party ever holds dw or the sum in the clear.
"""
from __future__ import annotations

import collections

import torch

from efl import exporter
from efl.framework.communicator import Communicator
from efl.framework.task_scope import MODE, current_task_scope
from efl.privacy.paillier_cipher import PaillierHook, PaillierKeypair
from efl.privacy.paillier_layer import dense_recv, dense_send, weight_recv, weight_send


@exporter.export("FederalModel")
class FederalModel(object):
    """model.py:490-515. `communicator` is an efl.Communicator (connected by `initialize()` if it is
    not yet); without one, the keyword arguments build it the way the reference does from its flags
    (federal_role, peer_addr, local_addr, ...)."""

    def __init__(self, communicator=None, federal_role=None, peer_addr=None, local_addr=None, task_index=0,
                 worker_num=1, client_thread_num=None, server_thread_num=None, scanning_interval_milliseconds=None,
                 default_timeout_milliseconds=None, **communicator_kwargs):
        if communicator is None:
            if federal_role not in ("leader", "follower"):
                raise ValueError("federal_role must be set one of [leader/follower] in FederalModel.")
            communicator = Communicator(federal_role, task_index, worker_num, peer_addr, local_addr,
                                        client_thread_num=client_thread_num, server_thread_num=server_thread_num,
                                        scanning_interval_milliseconds=scanning_interval_milliseconds,
                                        default_timeout_milliseconds=default_timeout_milliseconds,
                                        **communicator_kwargs)
        self._communicator = communicator
        self._federal_role = communicator._federal_role
        self._recv_grad_ops = collections.defaultdict(list)
        self._require_grad_ops = collections.defaultdict(list)
        self._hooks = collections.defaultdict(list)
        self._keypairs = {}
        self._paillier_vars_and_lrs = collections.defaultdict(list)
        self._paillier_outputs = collections.defaultdict(list)
        self._session_started = False

    # ---------------------------------------------------------------------------- properties
    @property
    def recv_grad_ops(self):
        return self._recv_grad_ops

    @property
    def require_grad_ops(self):
        return self._require_grad_ops

    @property
    def federal_role(self):
        return self._federal_role

    @property
    def communicator(self):
        return self._communicator

    @property
    def keypairs(self):
        return self._keypairs

    def keypair(self, name):
        return self._keypairs[name]

    def paillier_vars_and_lrs(self, task=None):
        """[(kernel, learning_rate)] registered under `task` (model.py:514)."""
        return list(self._paillier_vars_and_lrs[self._task(task)])

    def paillier_outputs(self, task=None):
        return list(self._paillier_outputs[self._task(task)])

    # ------------------------------------------------------------------------ session / hooks
    def add_hooks(self, hooks, mode=MODE.TRAIN, task=None):
        """Session hooks (PaillierHook, ...): after_create_session runs in initialize(), before_run /
        after_run around every step (begin_step / end_step)."""
        self._hooks[(mode, task)].extend(hooks)
        if self._session_started:
            for h in hooks:
                h.after_create_session()

    def _all_hooks(self):
        return [h for hs in self._hooks.values() for h in hs]

    def initialize(self):
        """The part of MonitoredTrainingSession creation the path needs: connect the communicator
        (CommunicatorHook.after_create_session, communicator.py:139-140), then every hook's
        after_create_session — the Paillier key exchange (paillier.py:190-193)."""
        if self._communicator._status == "CREATED":
            self._communicator.initialize()
        self._session_started = True
        for h in self._all_hooks():
            h.after_create_session()

    def begin_step(self):
        for h in self._all_hooks():
            h.before_run()

    def end_step(self):
        """after_run of every hook, then the communicator's step (CommunicatorHook.after_run,
        communicator.py:145-146): the rendezvous key of the next step's messages."""
        for h in self._all_hooks():
            h.after_run()
        self._communicator.add_step()

    # --------------------------------------------------------------------- Paillier surface
    def create_keypair(self, name, role, update_step_interval=None, n_bytes=None, a_bytes=None, reps=None,
                       group_size=None, seed=None):
        """model.py:543-570: a keypair named `name` plus the PaillierHook that generates it (SENDER)
        or installs the peer's public key (RECEIVER) when the session starts, and again every
        update_step_interval steps. `seed` keys the keypair's encryption randomness (Philox; None =
        os.urandom)."""
        keypair = PaillierKeypair(seed=seed)
        self._keypairs[name] = keypair
        hook = PaillierHook(keypair, self._communicator, role, name, update_step_interval=update_step_interval,
                            n_bytes=n_bytes, a_bytes=a_bytes, reps=reps, group_size=group_size)
        self.add_hooks([hook])
        return keypair

    def _kp(self, keypair_or_name):
        return self._keypairs[keypair_or_name] if isinstance(keypair_or_name, str) else keypair_or_name

    def _task(self, task):
        return task if task else current_task_scope().task

    def _register(self, kernel, learning_rate, trainable, task):
        """The reference registers each kernel once, when the graph is built; eagerly the layer runs
        every step, so a kernel already registered under the task only has its rate refreshed."""
        if not trainable:
            return
        regs = self._paillier_vars_and_lrs[self._task(task)]
        for i, (k, _) in enumerate(regs):
            if k is kernel:
                regs[i] = (kernel, learning_rate)
                return
        regs.append((kernel, learning_rate))

    def paillier_sender_dense(self, inputs, keypair_or_name, prefix, learning_rate, units, mode=MODE.TRAIN,
                              task=None, name=None, reuse=None, trainable=True, seed=None):
        """model.py:572-601. learning_rate is the PEER's (the receiver's) learning rate. Returns the
        layer output (the reference files it under the task's Paillier outputs and returns None;
        returning it lets an eager caller use it — minimize() finds it either way)."""
        outputs, kernel = dense_send(inputs, self._kp(keypair_or_name), self._communicator, prefix, units,
                                     name=name, reuse=reuse, seed=seed)
        self._register(kernel, learning_rate, trainable, task)
        if mode == MODE.TRAIN:
            self._paillier_outputs[self._task(task)].append(outputs)
        return outputs

    def paillier_recver_dense(self, inputs, keypair_or_name, prefix, learning_rate, units, recv_shape, task=None,
                              **kwargs):
        """model.py:603-625: kwargs are dense_recv's (activation, use_bias, kernel_initializer, ...)."""
        trainable = kwargs.pop("trainable", True)
        outputs, kernel = dense_recv(inputs, self._kp(keypair_or_name), self._communicator, prefix, recv_shape,
                                     units, **kwargs)
        self._register(kernel, learning_rate, trainable, task)
        return outputs

    def paillier_sender_weight(self, inputs, keypair_or_name, prefix, learning_rate, units, mode=MODE.TRAIN,
                               task=None, trainable=True, seed=None):
        """model.py:627-653."""
        outputs, kernel = weight_send(inputs, self._kp(keypair_or_name), self._communicator, prefix, units,
                                      seed=seed)
        self._register(kernel, learning_rate, trainable, task)
        if mode == MODE.TRAIN:
            self._paillier_outputs[self._task(task)].append(outputs)
        return outputs

    def paillier_recver_weight(self, inputs, keypair_or_name, prefix, learning_rate, units, task=None,
                               kernel_initializer=None, trainable=True, seed=None):
        """model.py:655-677."""
        outputs, kernel = weight_recv(inputs, self._kp(keypair_or_name), self._communicator, prefix, units,
                                      kernel_initializer=kernel_initializer, seed=seed)
        self._register(kernel, learning_rate, trainable, task)
        return outputs

    # --------------------------------------------------------------------------- send / recv
    def send(self, name, tensor, require_grad=False, mode=MODE.TRAIN, task=None):
        """model.py:679-699. With require_grad the gradient of `tensor` comes back from the peer as
        `name + '_grad'` in minimize()."""
        handle = self._communicator.send(name, tensor)
        if require_grad:
            self._require_grad_ops[self._task(task)].append((name, tensor))
        return handle

    def recv(self, name, shape=None, dtype=torch.float32, require_grad=False, task=None):
        """model.py:701-716. With require_grad the received tensor is a leaf that requires grad, and
        minimize() sends its gradient back as `name + '_grad'`."""
        t = self._communicator.recv(name, shape=shape, dtype=dtype)
        if require_grad:
            t = t.detach().requires_grad_(True)
            self._recv_grad_ops[self._task(task)].append((name, t))
        return t

    # ------------------------------------------------------------------------------ training
    def minimize(self, optimizer, loss=None, task=None):
        """One backward + update of `task`, model.py:718-815 over torch autograd:

        * loss None (a sender with no loss of its own) or one of the task's Paillier outputs: the
          Paillier outputs are differentiated with unit upstream gradients (`grad_loss=None` in the
          reference; the sender's backward only waits on dy, paillier_layer.py:43). Otherwise the
          loss (reduced by mean if it is not a scalar) and the Paillier outputs together.
        * received tensors marked require_grad send their gradients back as `<name>_grad`; tensors
          sent with require_grad get theirs from the peer and are differentiated with it.
        * `optimizer.step()` for the caller's own variables (it never holds the Paillier kernels:
          they are created trainable=False), then `kernel -= learning_rate * kernel.grad` for every
          registered Paillier kernel — GradientDescentOptimizer(1.) on lr * grad (model.py:808-814).
        Returns the list of send handles of the gradient messages."""
        task = self._task(task)
        outs = self._paillier_outputs[task]
        roots, grads = [], []
        if loss is None or any(loss is o for o in outs):
            for o in outs:
                roots.append(o)
                grads.append(torch.ones_like(o))
        else:
            if loss.dim() != 0:
                loss = loss.mean()
            roots.append(loss)
            grads.append(None)
            for o in outs:
                roots.append(o)
                grads.append(torch.ones_like(o))
        for name, t in self._require_grad_ops[task]:
            g = self._communicator.recv(name + "_grad", shape=tuple(t.shape), dtype=t.dtype).to(t.device)
            roots.append(t)
            grads.append(g)
        handles = []
        if roots:
            torch.autograd.backward(roots, grads)
        for name, t in self._recv_grad_ops[task]:
            g = t.grad if t.grad is not None else torch.zeros_like(t)
            handles.append(self._communicator.send(name + "_grad", g))
            t.grad = None
        if optimizer is not None:
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
        self.apply_paillier_gradients(task)
        self._paillier_outputs[task] = []
        self._require_grad_ops[task] = []
        self._recv_grad_ops[task] = []
        return handles

    def apply_paillier_gradients(self, task=None):
        """model.py:808-814: kernel -= lr * grad for every registered Paillier kernel (each once,
        however many times its layer ran this step; a kernel without a gradient is left alone)."""
        seen = set()
        with torch.no_grad():
            for kernel, lr in self._paillier_vars_and_lrs[self._task(task)]:
                if id(kernel) in seen or kernel is None:
                    continue
                seen.add(id(kernel))
                if kernel.grad is None:
                    continue
                lr = float(lr() if callable(lr) else lr)
                kernel.sub_(lr * kernel.grad)
                kernel.grad = None

    def paillier_kernels(self, task=None):
        """The distinct registered kernels (for checkpointing or inspection)."""
        out, seen = [], set()
        for kernel, lr in self._paillier_vars_and_lrs[self._task(task)]:
            if id(kernel) not in seen:
                seen.add(id(kernel))
                out.append((kernel, lr))
        return out

