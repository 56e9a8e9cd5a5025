"""GPU, two processes: BASELINE config 5 at its own size — one step of the two-party loopback end to
end with the full 256 MiB fp32 tensor [65536, 1024]:

  follower: pinned host fp32 -> FixedPointHook (H2D | encode | D2H pipeline) -> gRPC: two 512 MiB
            MessageRequests (M, E; the reference's 1 GiB cap, communicator_ops.cc:437-440)
  leader:   gRPC -> FixedPointHook (H2D | decode | D2H, reading the message bytes in place) -> host

Checks, inside the leader (nothing of 256 MiB crosses back to pytest):
  * every received M / E element of a 1 % sample (plus the first and last 4 Ki elements) equals the
    oracle's ConvertToFixedPoint of the same input element;
  * the decoded tensor is the FTZ round trip of the input on EVERY element: bit-identical to x
    wherever x is a normal float other than +-2^23, and equal to the oracle's decode elsewhere."""
import multiprocessing as mp

import numpy as np
import pytest
import torch

from test_communicator import free_port

pytestmark = pytest.mark.gpu

ROWS, COLS = 65536, 1024


def _x():
    x = torch.randn(ROWS, COLS, generator=torch.Generator().manual_seed(2025))
    x[0, :6] = torch.tensor([0.0, -0.0, 8388608.0, -1.5e-40, float("inf"), 1e-38])
    x[-1] = torch.relu(x[-1])
    return x


def party(role, my, peer, q):
    try:
        import efl
        from oracle import fxp

        class RecordingHook(efl.privacy.FixedPointHook):
            """FixedPointHook that also keeps a sample of the wire M / E it received."""
            sample = None

            def post_recv(self, name, shape, dtype, raw_recv):
                def rec(n, readonly=False):
                    t = raw_recv(n, readonly=readonly)
                    self.wire[n] = t.reshape(-1)[self.sample].clone()
                    return t
                return super().post_recv(name, shape, dtype, rec)

        n = ROWS * COLS
        rng = np.random.default_rng(7)
        idx = np.unique(np.concatenate([np.arange(4096), np.arange(n - 4096, n),
                                        rng.integers(0, n, n // 100)]))
        hook = RecordingHook(reuse_buffers=True)
        hook.wire, hook.sample = {}, torch.from_numpy(idx)
        c = efl.Communicator(role, 0, 1, f"127.0.0.1:{peer}", f"127.0.0.1:{my}", hooks=[hook],
                             default_timeout_milliseconds=300000, connect_retry_seconds=0.2)
        c.initialize()
        x = _x()
        out = {}
        if role == "follower":
            c.send("act_[x]", x.pin_memory()).result(timeout=300)
        else:
            y = c.recv("act_[x]", shape=(ROWS, COLS))
            out["pinned"] = bool(y.is_pinned())
            xf = x.reshape(-1).numpy()
            yb = y.reshape(-1).numpy().view(np.uint32)
            xb = xf.view(np.uint32)
            M = hook.wire["act_[x]_mantissa"].reshape(-1).numpy()
            E = hook.wire["act_[x]_exponent"].reshape(-1).numpy()
            Mo, Eo = fxp.encode(xf[idx])
            out["sample"] = int(idx.size)
            out["me_equal"] = bool(np.array_equal(M, Mo) and np.array_equal(E, Eo))
            keep = (np.abs(xf) >= np.float32(1.1754944e-38)) & (np.abs(xf) != np.float32(8388608.0)) & np.isfinite(xf)
            out["identity_count"] = int(keep.sum())
            out["identity_equal"] = bool(np.array_equal(yb[keep], xb[keep]))
            rest = np.flatnonzero(~keep)
            Mr, Er = fxp.encode(xf[rest])
            out["rest"] = int(rest.size)
            out["rest_equal"] = bool(np.array_equal(yb[rest], fxp.decode(Mr, Er, np.float32, ftz=True).view(np.uint32)))
        c.add_step()
        c.shutdown()
        q.put((role, out, None))
    except BaseException:  # pragma: no cover - reported to the parent
        import traceback
        q.put((role, None, traceback.format_exc()[-3000:]))


def test_config5_full_size_two_process_loopback():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pl, pf = free_port(), free_port()
    procs = [ctx.Process(target=party, args=("leader", pl, pf, q)),
             ctx.Process(target=party, args=("follower", pf, pl, q))]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            role, out, err = q.get(timeout=400)
            assert err is None, (role, err)
            res[role] = out
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    r = res["leader"]
    assert r["pinned"]
    assert r["sample"] > ROWS * COLS // 100 - 100000 and r["me_equal"]
    assert r["identity_count"] > ROWS * COLS - 2000 and r["identity_equal"]
    assert r["rest"] >= 400 and r["rest_equal"]          # the ReLU zeros of the last row + the specials
