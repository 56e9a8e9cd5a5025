"""The fed_ops codec called on HOST tensors (how a reference caller, whose ops are CPU ops, hands
them over): 256 MiB fp32 pageable in -> (M, E) on the host -> fp32 on the host. Times both
directions with the pinned three-stream pipeline (efl.lib.HOST_PIPELINE_MIN_ELEMS, default) and
with the plain path (one pageable H2D, the kernel, pageable D2H), alternating in one process.
One JSON line per (path, rep); GiB/s of plaintext per leg."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "elastic-federated-learning-solution_amd"))

import torch  # noqa: E402


def main():
    import efl
    efl.lib.require_gpu()
    ops = efl.lib.ops
    x = torch.randn(65536, 1024, generator=torch.Generator().manual_seed(0))
    on = efl.lib.HOST_PIPELINE_MIN_ELEMS
    for rep in range(3):
        for path, thr in (("pipeline", on), ("plain", 1 << 62)):
            efl.lib.HOST_PIPELINE_MIN_ELEMS = thr
            ops.convert_to_fixed_point(x)                       # warm allocations
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            M, E = ops.convert_to_fixed_point(x)
            t1 = time.perf_counter()
            y = ops.fixed_point_to_float_point(M, E)
            t2 = time.perf_counter()
            assert y.device.type == "cpu" and torch.equal(y, x)
            gib = x.numel() * 4 / 2**30
            print(json.dumps({"path": path, "rep": rep, "encode_ms": round((t1 - t0) * 1e3, 1),
                              "decode_ms": round((t2 - t1) * 1e3, 1),
                              "encode_GiBs": round(gib / (t1 - t0), 2), "decode_GiBs": round(gib / (t2 - t1), 2)}),
                  flush=True)
            del M, E, y
    efl.lib.HOST_PIPELINE_MIN_ELEMS = on


if __name__ == "__main__":
    main()
