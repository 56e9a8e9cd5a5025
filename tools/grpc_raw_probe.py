#!/usr/bin/env python3
"""A bare grpcio unary call with a 512 MiB bytes payload over loopback (no efl code): the transport
ceiling of config 5's gRPC leg on this host. Server and client in one process, generic handlers, the
same 1 GiB message limits as efl.Communicator. Prints one JSON line."""
import json
import time
from concurrent import futures

import grpc

N = 512 << 20
OPTS = [("grpc.max_send_message_length", 1 << 30), ("grpc.max_receive_message_length", 1 << 30)]


def main():
    srv = grpc.server(futures.ThreadPoolExecutor(8), options=OPTS)
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
        "S", {"M": grpc.unary_unary_rpc_method_handler(lambda req, ctx: b"")}),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    ch = grpc.insecure_channel(f"127.0.0.1:{port}", OPTS)
    rpc = ch.unary_unary("/S/M")
    payload = bytes(N)
    rpc(b"x")
    ms = []
    for _ in range(4):
        t0 = time.monotonic()
        rpc(payload)
        ms.append((time.monotonic() - t0) * 1e3)
    ms = sorted(ms[1:])
    print(json.dumps({"probe": "bare grpcio unary call, 512 MiB bytes, loopback, one process",
                      "ms": [round(v, 1) for v in ms], "GBs": round(N / (ms[len(ms) // 2] * 1e-3) / 1e9, 3)}))
    ch.close()
    srv.stop(0)


if __name__ == "__main__":
    main()
