#!/usr/bin/env python3
"""Config 5's transport ceiling under gRPC channel/server options: the bare grpcio unary call of
tools/grpc_raw_probe.py (512 MiB bytes payload, loopback, one process) with each option set in a
fresh process. Prints one JSON line per variant (GB/s of the median of three calls after a warm-up).

    python tools/grpc_options_probe.py [variant ...]
"""
import json
import os
import subprocess
import sys
import time
from concurrent import futures

N = 512 << 20
BASE = [("grpc.max_send_message_length", 1 << 30), ("grpc.max_receive_message_length", 1 << 30)]
READ = [("grpc.experimental.tcp_read_chunk_size", 1 << 20), ("grpc.experimental.tcp_min_read_chunk_size", 1 << 20),
        ("grpc.experimental.tcp_max_read_chunk_size", 1 << 24)]
FRAME = [("grpc.http2.max_frame_size", (1 << 24) - 1)]
VARIANTS = {
    "base": ([], {}),
    "frame16M": (FRAME, {}),
    "read_chunk": (READ, {}),
    "frame+read": (FRAME + READ, {}),
    "bdp_off_lookahead": ([("grpc.http2.bdp_probe", 0), ("grpc.http2.lookahead_bytes", 1 << 26)], {}),
    "write_buffer": ([("grpc.http2.write_buffer_size", 1 << 24)], {}),
    "frame+read+wbuf": (FRAME + READ + [("grpc.http2.write_buffer_size", 1 << 24)], {}),
    "poll_epoll1": ([], {"GRPC_POLL_STRATEGY": "epoll1"}),
}


def one(name):
    import grpc
    extra, _ = VARIANTS[name]
    opts = BASE + extra
    srv = grpc.server(futures.ThreadPoolExecutor(8), options=opts)
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
        "S", {"M": grpc.unary_unary_rpc_method_handler(lambda req, ctx: b"")}),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    ch = grpc.insecure_channel(f"127.0.0.1:{port}", opts)
    rpc = ch.unary_unary("/S/M")
    payload = bytes(N)
    rpc(payload)
    ms = []
    for _ in range(3):
        t0 = time.monotonic()
        rpc(payload)
        ms.append((time.monotonic() - t0) * 1e3)
    ms.sort()
    ch.close()
    srv.stop(0)
    print(json.dumps({"variant": name, "options": extra, "env": VARIANTS[name][1], "ms": [round(v, 1) for v in ms],
                      "GBs": round(N / (ms[1] * 1e-3) / 1e9, 3), "grpc": grpc.__version__}), flush=True)


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--one":
        one(sys.argv[2])
        return
    for name in sys.argv[1:] or list(VARIANTS):
        env = dict(os.environ, **VARIANTS[name][1])
        subprocess.run([sys.executable, __file__, "--one", name], env=env, check=True, timeout=120)


if __name__ == "__main__":
    main()
