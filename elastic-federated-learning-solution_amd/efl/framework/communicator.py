"""efl.Communicator — the cross-silo tensor channel with a pre-send / post-recv hook.

Drop-in for efls-train/python/efl/framework/communicator.py:34-149 (same constructor arguments and
send/recv signatures) over the reference's own gRPC service and wire format
(efls-train/protos/trainer_service.proto:44-49; MessageRequest bytes from efl.framework.wire), so a
build peer and a reference peer speak the same protocol.

Semantics kept from the C++ resource (efls-train/cc/efl/communicator/communicator_ops.cc):
  * send(name, t) completes when the PEER's recv consumed the tensor (the server answers the
    SendMessage RPC from the receive callback, :235-261 / communication_service.cc:216-248);
    here send() returns a handle immediately (TF runs send ops asynchronously) and
    handle.result() waits for that acknowledgement.
  * rendezvous by name and step: a parked message whose step differs from the receiver's step
    fails both sides with DataLoss (:271-279); a receive past `default_timeout_milliseconds`
    fails with DeadlineExceeded (Monitor, monitor.cc:47-97).
  * the follower connects to the leader with retries on UNAVAILABLE (communicator.py:104-116).
  * env vars EFL_CLIENT_MAX_{SEND,RECEIVE}_MESSAGE_SIZE / EFL_SERVER_MAX_{SEND,RECEIVE}_MESSAGE_SIZE
    (default 1 GiB), EFL_PEER_CERTS_FILENAME, EFL_SSL_TARGET_NAME_OVERRIDE, EFL_MY_CERTS_FILENAME,
    EFL_MY_KEY_FILENAME (communicator_ops.cc:430-441, communication_service.cc:62-71).
Differences: names need not be pre-registered (eager mode has no graph to collect
them from; `strict_names=True` restores NotFound for unregistered names), and several messages of
one name may wait in FIFO order instead of overwriting each other.

The hook (`hooks=[...]`) is where the forward-encryption transform plugs in: a hook's pre_send
turns one logical tensor into the wire tensors (e.g. fixed-point mantissa + exponent computed on the
MI355X) and its post_recv reassembles them, so callers of send/recv need no change.
"""
from __future__ import annotations

import collections
import logging
import os
import threading
import time
import warnings
import zlib
from concurrent import futures

import grpc
import numpy as np
import torch

from efl import errors, exporter
from efl.framework import wire

log = logging.getLogger("efl.communicator")

_SERVICE = "efl.TrainerService"
_SEND = f"/{_SERVICE}/SendMessage"
_CONNECT = f"/{_SERVICE}/Connect"
_GET_READER_STATE = f"/{_SERVICE}/GetReaderState"
_GET_CKPT = f"/{_SERVICE}/GetCheckpointVersion"

_TORCH_OF_DT = {wire.DT_FLOAT: torch.float32, wire.DT_DOUBLE: torch.float64, wire.DT_INT32: torch.int32,
                wire.DT_UINT8: torch.uint8, wire.DT_INT16: torch.int16, wire.DT_INT8: torch.int8,
                wire.DT_INT64: torch.int64, wire.DT_BOOL: torch.bool}
_DT_OF_TORCH = {v: k for k, v in _TORCH_OF_DT.items()}


def _env_int(name, default):
    v = os.environ.get(name, "")
    return int(v) if v else default


_PAIR_SUFFIXES = ("_mantissa", "_exponent")


def channel_of(name: str, nchan: int) -> int:
    """The client connection a message name always travels on: a stable hash of the name, so two
    sends of one name keep their order (the receiver parks each name's messages FIFO). A hook's
    '<x>_mantissa' / '<x>_exponent' pair hashes '<x>' and takes adjacent channels, so the two large
    payloads of one send still cross on two connections at once."""
    if nchan <= 1:
        return 0
    for i, suf in enumerate(_PAIR_SUFFIXES):
        if name.endswith(suf):
            return (zlib.crc32(name[:-len(suf)].encode()) + i) % nchan
    return zlib.crc32(name.encode()) % nchan


def _http2_opts():
    """HTTP/2 transport options for the large-message path (both server and client). Frame size:
    the largest the protocol allows instead of 16 KiB, so a 512 MiB message is 32 frames, not
    32 Ki (EFL_GRPC_MAX_FRAME_SIZE, 0 = gRPC's default)."""
    frame = _env_int("EFL_GRPC_MAX_FRAME_SIZE", 0)
    out = []
    if frame:
        out.append(("grpc.http2.max_frame_size", frame))
    extra = os.environ.get("EFL_GRPC_OPTIONS", "")
    for kv in filter(None, extra.split(",")):
        k, v = kv.split("=", 1)
        out.append((k, int(v)))
    return out


def _read(path):
    with open(path, "rb") as f:
        return f.read()


class _Parked:
    """A received SendMessage waiting for the local recv (the RPC is held open until then)."""
    __slots__ = ("step", "payload", "done", "code", "msg")

    def __init__(self, step, payload):
        self.step, self.payload = step, payload
        self.done = threading.Event()
        self.code, self.msg = 0, ""

    def finish(self, code=0, msg=""):
        self.code, self.msg = code, msg
        self.done.set()


class _Waiter:
    __slots__ = ("ready", "parked")

    def __init__(self):
        self.ready = threading.Event()
        self.parked = None


class SendHandle:
    """Completion of one send: result() blocks until the peer consumed the tensor."""

    def __init__(self, parts):
        self._parts = parts   # [(name, grpc future)]

    def result(self, timeout=None):
        for name, fut in self._parts:
            try:
                resp = fut.result(timeout=timeout)
            except grpc.RpcError as e:
                raise errors.from_code(e.code().value[0], f"send {name}: {e.details()}") from None
            code, msg = wire.parse_message_response(resp)
            if code:
                raise errors.from_code(code, msg)
        return None

    def done(self):
        return all(f.done() for _, f in self._parts)


class TensorHook:
    """Pre-send / post-recv transform. pre_send returns the wire tensors [(name, tensor)];
    post_recv pulls the wire tensors with `raw_recv(name, dtype)` and returns the logical tensor.
    Return None from either to pass the tensor through unchanged."""

    def pre_send(self, name, tensor):
        return None

    def post_recv(self, name, shape, dtype, raw_recv):
        return None


@exporter.export("Communicator")
class Communicator(object):
    def __init__(self, federal_role, worker_index, worker_num, peer_addr, local_addr,
                 client_thread_num=None, server_thread_num=None,
                 scanning_interval_milliseconds=None, default_timeout_milliseconds=None,
                 hooks=None, strict_names=False, connect_retry_seconds=10.0, channels=None):
        if federal_role not in ("leader", "follower"):
            raise ValueError("federal_role must be set one of [leader/follower] in Communicator")
        self._federal_role = federal_role
        self._worker_index = worker_index
        self._worker_num = worker_num
        self._peer_addr = peer_addr
        self._local_addr = local_addr
        self._server_threads = server_thread_num or 64
        self._timeout = (default_timeout_milliseconds or 600000) / 1000.0
        self._hooks = list(hooks or [])
        self._strict = strict_names
        self._retry = connect_retry_seconds
        # client connections to the peer (the reference opens one channel per peer,
        # communicator_ops.cc:462); EFL_CHANNELS overrides. Any count speaks the same protocol.
        # Two: a hook's mantissa and exponent messages (512 MiB each at config 5) travel on two TCP
        # connections at once, 1.26-1.34 -> 1.44-1.45 GB/s on the MI355X box's host
        # (tools/grpc_probe.py, profiles/r03/grpc_probe.jsonl); four was no faster.
        self._nchan = max(1, int(channels if channels is not None else _env_int("EFL_CHANNELS", 2)))
        self._local_step = [0] * worker_num
        self._recv_set = set()
        self._lock = threading.Lock()
        self._parked = collections.defaultdict(collections.deque)   # name -> deque[_Parked]
        self._waiters = {}                                           # (name, step) -> _Waiter
        self._connected = threading.Event()
        self._leader_ready = threading.Event()
        self._server = None
        self._channel = None
        self._status = "CREATED"

    # ------------------------------------------------------------------ reference surface
    @property
    def step(self):
        return self._local_step[self._worker_index]

    def add_step(self):
        self._local_step[self._worker_index] += 1
        return self.step

    def add_hook(self, hook: TensorHook):
        self._hooks.append(hook)

    def send(self, name, tensor):
        """Send `tensor` to the peer under `name` at the current step (async; see SendHandle)."""
        self._require_connected()
        for h in self._hooks:
            parts = h.pre_send(name, tensor)
            if parts is not None:
                return SendHandle([p for n, t in parts for p in self._send_raw(n, t)._parts])
        return self._send_raw(name, tensor)

    def recv(self, name, shape=None, dtype=torch.float32):
        """Receive the tensor the peer sent as `name` at the current step (blocking)."""
        self._require_connected()
        self._recv_set.add(name)
        for h in self._hooks:
            out = h.post_recv(name, shape, dtype, self._recv_raw)
            if out is not None:
                return out
        t = self._recv_raw(name, dtype)
        if shape is not None and not isinstance(t, dict):
            t = t.reshape(tuple(int(s) for s in shape))
        return t

    def initialize(self, sess=None):
        """CreateCommunicator + Response/RequestConnection (communicator.py:104-116)."""
        if self._status != "CREATED":
            raise errors.FailedPreconditionError("Already Connected.")
        self._start_server()
        self._start_client()
        if self._federal_role == "leader":
            self._leader_ready.set()
            if not self._connected.wait(self._timeout):
                raise errors.DeadlineExceededError("no Connect from the follower")
        else:
            connect = self._channel.unary_unary(_CONNECT)
            while True:
                try:
                    connect(b"", timeout=self._timeout)
                    break
                except grpc.RpcError as e:
                    if e.code() != grpc.StatusCode.UNAVAILABLE:
                        raise errors.from_code(e.code().value[0], e.details()) from None
                    log.info("Connecting failed with leader, wait %.1f second.", self._retry)
                    time.sleep(self._retry)
            self._connected.set()
        self._status = "CONNECTED"
        log.info("Connect with Peer.")

    def shutdown(self, sess=None):
        if self._status != "CONNECTED":
            raise errors.FailedPreconditionError("Already Closed.")
        with self._lock:
            for q in self._parked.values():
                for p in q:
                    p.finish(1, "communicator shut down")   # CANCELLED
        if self._server is not None:
            self._server.stop(grace=1.0).wait()
        for ch in getattr(self, "_channels", []):
            ch.close()
        self._status = "CLOSED"

    @property
    def hook(self):
        if not hasattr(self, "_hook"):
            self._hook = CommunicatorHook(self)
        return self._hook

    # the data-alignment / failover RPCs are outside the forward-encryption scope
    def send_ckpt_version(self, sess, version):
        raise errors.UnimplementedError("checkpoint-version handshake is out of scope")

    def recv_ckpt_version(self, sess):
        raise errors.UnimplementedError("checkpoint-version handshake is out of scope")

    def send_reader_state(self, name, block_id, sample_index):
        raise errors.UnimplementedError("reader-state handshake is out of scope")

    def recv_reader_state(self, name):
        raise errors.UnimplementedError("reader-state handshake is out of scope")

    # ------------------------------------------------------------------------- internals
    def _require_connected(self):
        if self._status != "CONNECTED":
            raise errors.FailedPreconditionError("Haven't connected with peer worker.")

    def _start_server(self):
        opts = [("grpc.max_send_message_length", _env_int("EFL_SERVER_MAX_SEND_MESSAGE_SIZE", 1 << 30)),
                ("grpc.max_receive_message_length", _env_int("EFL_SERVER_MAX_RECEIVE_MESSAGE_SIZE", 1 << 30))]
        opts += _http2_opts()
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=self._server_threads), options=opts)
        handlers = {
            "SendMessage": grpc.unary_unary_rpc_method_handler(self._on_send_message),
            "Connect": grpc.unary_unary_rpc_method_handler(self._on_connect),
        }
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(_SERVICE, handlers),))
        certs, keyf = os.environ.get("EFL_MY_CERTS_FILENAME", ""), os.environ.get("EFL_MY_KEY_FILENAME", "")
        if certs and keyf:
            peer = os.environ.get("EFL_PEER_CERTS_FILENAME", "")
            creds = grpc.ssl_server_credentials([(_read(keyf), _read(certs))],
                                                root_certificates=_read(peer) if peer else None,
                                                require_client_auth=False)
            port = server.add_secure_port(self._local_addr, creds)
        else:
            port = server.add_insecure_port(self._local_addr)
        if port == 0:
            raise errors.UnavailableError(f"cannot listen on {self._local_addr}")
        server.start()
        self._server = server

    def _start_client(self):
        opts = [("grpc.max_send_message_length", _env_int("EFL_CLIENT_MAX_SEND_MESSAGE_SIZE", 1 << 30)),
                ("grpc.max_receive_message_length", _env_int("EFL_CLIENT_MAX_RECEIVE_MESSAGE_SIZE", 1 << 30))]
        opts += _http2_opts()
        override = os.environ.get("EFL_SSL_TARGET_NAME_OVERRIDE", "")
        if override:
            opts.append(("grpc.ssl_target_name_override", override))
        peer_certs = os.environ.get("EFL_PEER_CERTS_FILENAME", "")

        def channel(k):
            # a local subchannel pool per channel: each is its own TCP connection (channels with
            # equal arguments would otherwise share one connection through the global pool)
            o = opts + ([("grpc.use_local_subchannel_pool", 1), ("efl.channel_index", k)] if self._nchan > 1 else [])
            if peer_certs:
                return grpc.secure_channel(
                    self._peer_addr, grpc.ssl_channel_credentials(root_certificates=_read(peer_certs)), o)
            return grpc.insecure_channel(self._peer_addr, o)
        self._channels = [channel(k) for k in range(self._nchan)]
        self._channel = self._channels[0]
        self._send_rpcs = [ch.unary_unary(_SEND) for ch in self._channels]
        self._send_rpc = self._send_rpcs[0]
        self._inflight = {}

    # server side ---------------------------------------------------------------------
    def _on_connect(self, request, context):
        # the leader answers once its own initialize() ran (connect_cb_, communicator_ops.cc:209-217)
        self._leader_ready.wait(self._timeout)
        self._connected.set()
        return b""

    def _on_send_message(self, request, context):
        name, step, tensor = wire.parse_message_request(request)
        log.debug("%s: arrived %s step %d", self._federal_role, name, step)
        p = _Parked(step, tensor)
        with self._lock:
            w = self._waiters.pop((name, step), None)
            if w is None and self._strict and name not in self._recv_set:
                return wire.message_response(5, f"Tensor named {name} not registed.")   # NOT_FOUND
            if w is not None:
                w.parked = p
                w.ready.set()
            else:
                q = self._parked[name]
                q.append(p)
                # a receiver of this name waiting for another step: wake it for the DataLoss check
                for (wn, _ws), ww in list(self._waiters.items()):
                    if wn == name and ww.parked is None:
                        ww.ready.set()
        if not p.done.wait(self._timeout):
            return wire.message_response(4, f"Send Tensor {name}, step {step} Timeout.")
        return wire.message_response(p.code, p.msg)

    # client side ---------------------------------------------------------------------
    def _send_raw(self, name, t):
        from efl.privacy.hex_tensor import HexTensor
        if hasattr(t, "tensor") and hasattr(t, "keypair"):      # PaillierTensor
            t = t.tensor
        if hasattr(t, "to_hex"):                                  # CipherTensor: DT_STRING on the wire
            t = t.to_hex()
        if isinstance(t, HexTensor):
            dtype, shape, content = wire.DT_STRING, t.shape, t.wire_parts()
        else:
            if not isinstance(t, torch.Tensor):
                t = torch.as_tensor(np.asarray(t))
            if t.is_cuda:
                t = t.cpu()
            t = t.contiguous()
            dtype = _DT_OF_TORCH.get(t.dtype)
            if dtype is None:
                raise errors.InvalidArgumentError(f"cannot send dtype {t.dtype}")
            shape = tuple(t.shape)
            content = t.view(torch.uint8).numpy().reshape(-1) if t.numel() else b""
        req = wire.message_request(name, self.step, dtype, shape, content)
        return SendHandle([(name, self._send_ordered(name, req))])

    def _send_ordered(self, name, req):
        """Issue the SendMessage RPC for `name`, after the previous send of the same name completed
        if one is still in flight. Concurrent unary RPCs are not ordered on the server (a small
        message overtakes a large one even on one connection), and the receiver hands a name's
        parked messages over FIFO; the reference keeps one in-flight message per name at all
        (communication_service.cc:236-238 replaces the parked call). A send completes when the peer
        has received it, so chaining costs nothing unless one name is sent twice before the first
        is consumed."""
        rpc = self._send_rpcs[channel_of(name, len(self._send_rpcs))]
        timeout = self._timeout
        with self._lock:
            prev = self._inflight.get(name)
            if prev is None or prev.done():
                fut = rpc.future(req, timeout=timeout)
            else:
                fut = futures.Future()

                def relay(g):
                    e = g.exception()
                    if e is not None:
                        fut.set_exception(e)
                    else:
                        fut.set_result(g.result())

                def start(_):
                    try:
                        rpc.future(req, timeout=timeout).add_done_callback(relay)
                    except Exception as e:       # noqa: BLE001 - surfaced by SendHandle.result
                        fut.set_exception(e)
                prev.add_done_callback(start)
            self._inflight[name] = fut

        def forget(_):
            # compare-and-pop under the lock: a send of the same name may store its successor
            # between the check and the pop, and popping that successor would let a third send
            # run beside it. Never re-entered with the lock held: forget is attached only here,
            # after the `with` block, and nothing completes `fut` under the lock afterwards.
            with self._lock:
                if self._inflight.get(name) is fut:
                    del self._inflight[name]
        fut.add_done_callback(forget)
        return fut

    def _take(self, name, step):
        """Pop the parked message for (name, step) or register a waiter; called under the lock."""
        q = self._parked.get(name)
        if q:
            p = q.popleft()
            return p, None
        w = _Waiter()
        self._waiters[(name, step)] = w
        return None, w

    def _recv_raw(self, name, dtype=None, readonly=False):
        """readonly=True (hooks that only read the payload, e.g. to copy it to the GPU): the
        tensor is a view of the received message bytes instead of a private copy; it must not be
        written to."""
        step = self.step
        log.debug("%s: waiting %s step %d", self._federal_role, name, step)
        deadline = time.monotonic() + self._timeout
        with self._lock:
            p, w = self._take(name, step)
        while p is None:
            left = deadline - time.monotonic()
            if left <= 0 or not w.ready.wait(left):
                with self._lock:
                    self._waiters.pop((name, step), None)
                raise errors.DeadlineExceededError(f"Receive Tensor {name}, step {step} Timeout.")
            with self._lock:
                if w.parked is not None:
                    p = w.parked
                else:   # a message of this name arrived for another step
                    w.ready.clear()
                    q = self._parked.get(name)
                    if q:
                        p = q.popleft()
                        self._waiters.pop((name, step), None)
        if p.step != step:
            msg = f"Tensor named {name} expects step {step}, but given step {p.step}."
            p.finish(15, msg)   # DATA_LOSS to the sender
            raise errors.DataLossError(msg)
        try:
            out = self._materialize(p.payload, dtype, readonly)
        except Exception as e:   # deserialize error -> Unknown to both sides (:241-246)
            p.finish(2, f"Tensor named {name} deserialize error.")
            raise errors.UnknownError(f"Tensor named {name} deserialize error: {e}") from None
        p.finish(0, "")
        return out

    @staticmethod
    def _materialize(msg: wire.TensorMsg, dtype, readonly=False):
        from efl.privacy.hex_tensor import HexTensor
        if msg.dtype == wire.DT_STRING:
            if msg.content is not None and len(msg.content):
                return HexTensor.from_tensor_content(msg.content, msg.shape)
            return HexTensor.from_strings(np.array(msg.typed, dtype=object).reshape(msg.shape))
        arr = msg.to_numpy()
        if arr.flags.writeable:
            return torch.from_numpy(arr)
        if not readonly:
            return torch.from_numpy(arr.copy())
        # a view of the (immutable) message bytes: torch warns that it cannot mark it read-only
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            return torch.from_numpy(arr)


class CommunicatorHook(object):
    """Session hook equivalent (communicator.py:134-149): initialize on session creation, step
    after every run, shutdown at the end."""

    def __init__(self, communicator):
        self._communicator = communicator

    def after_create_session(self, sess=None, coord=None):
        self._communicator.initialize(sess)

    def before_run(self, run_context=None):
        return None

    def after_run(self, run_context=None, run_values=None):
        self._communicator.add_step()

    def end(self, sess=None):
        self._communicator.shutdown(sess)
