"""ORACLE — test infrastructure only (tests/, smoke(), bench.py's cpu_baseline leg). Never imported
by the product.

numpy restatement of the secret-sharing masks of efls-train/python/efl/privacy/secret_sharing.py:
  generate_suitable_noise(t) = tf.random.uniform(tf.shape(t)) * t          (secret_sharing.py:26-27)
  share(): send a = noise(x), keep x - a                                  (:158-168)
  SecretSharingDense(noise_divisor): send w - noise/d, keep w + noise/d   (:137-143)
  _matmul mode A: e = noise(a); send [a + e | e_even + e_odd]; keep a - e, e_odd - e_even   (:30-41)
  _matmul mode B: f = noise(b); send [b/2 - f ; f_even - f_odd]; keep b/2 + f, f_odd + f_even (:42-53)
The uniform is TF's: Philox4x32-10 words through Uint32ToFloat (tensorflow/core/lib/random/
random_distributions.h: exponent 127 over the low 23 bits, minus 1.0). TF's own stream is unseeded, so
the reference pins only the distribution; the build fixes the counter layout (element i = word i % 4
of block ctr0 + i / 4, key = seed) and this oracle follows it, so kernel outputs compare bit for bit.
The fp32 arithmetic is done in numpy float32 (IEEE round-to-nearest, same as the kernels).

DP-SGD noise (efls-train/python/efl/privacy/dp_optimizer.py:60-73; tensorflow_privacy 0.3.0
GaussianSumQuery): tf.random.normal is TF's NormalDistribution over the same Philox words --
Box-Muller on word pairs (0, 1), (2, 3) of each block (BoxMullerFloat: u1 = max(U(x0), 1e-7),
v1 = float(2 pi * U(x1)) in double, r = sqrt(-2 log u1), (r sin v1, r cos v1)). log/sin/cos here are
float64 rounded to float32 (correctly rounded); the kernels use the device's logf / sincosf, so the
normals agree to a few ulp, not bit for bit (the tests state the tolerance). Parity with the
reference is statistical only: its stream is unseeded.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox_blocks(seed: int, ctr0: int, nblocks: int) -> np.ndarray:
    """[nblocks, 4] uint32 Philox4x32-10 outputs for counters (ctr0 + b, 0, 0) under key seed
    (the same rounds as oracle/philox.py, vectorised)."""
    ctr = (np.uint64(ctr0) + np.arange(nblocks, dtype=np.uint64))
    c0 = ctr & MASK
    c1 = ctr >> np.uint64(32)
    c2 = np.zeros(nblocks, np.uint64)
    c3 = np.zeros(nblocks, np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)) & MASK, p1 & MASK, \
            ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)) & MASK, p0 & MASK
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def uniform(seed: int, ctr0: int, n: int) -> np.ndarray:
    """U[0,1) float32 for elements 0..n-1 of one call."""
    w = philox_blocks(seed, ctr0, (n + 3) // 4).reshape(-1)[:n]
    bits = (np.uint32(0x3F800000) | (w & np.uint32(0x7FFFFF))).view(np.float32)
    return (bits - np.float32(1.0)).astype(np.float32)


def noise(x: np.ndarray, seed: int, ctr0: int, op: int = 0, divisor: float = 1.0):
    """efl_ss_noise: op 0 -> n; op 1 -> (n, x - n); op 2 -> (x - n, x + n); n = U * x / divisor."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = uniform(seed, ctr0, x.size).reshape(x.shape)
    n = (u * x).astype(np.float32)
    if divisor != 1.0:
        n = (n / np.float32(divisor)).astype(np.float32)
    if op == 0:
        return n
    if op == 1:
        return n, (x - n).astype(np.float32)
    return (x - n).astype(np.float32), (x + n).astype(np.float32)


def mask_cols(a: np.ndarray, seed: int, ctr0: int):
    """Mode A side: (send [R, 3C/2], keep0 [R, C], keep1 [R, C/2])."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    R, C = a.shape
    assert C % 2 == 0
    e = (uniform(seed, ctr0, a.size).reshape(a.shape) * a).astype(np.float32)
    e_odd, e_even = e[:, 1::2], e[:, ::2]
    send = np.concatenate([a + e, e_even + e_odd], axis=1).astype(np.float32)
    return send, (a - e).astype(np.float32), (e_odd - e_even).astype(np.float32)


def mask_rows(b: np.ndarray, seed: int, ctr0: int):
    """Mode B side: (send [3K/2, N], keep0 [K, N], keep1 [K/2, N])."""
    b = np.ascontiguousarray(b, dtype=np.float32)
    K, N = b.shape
    assert K % 2 == 0
    f = (uniform(seed, ctr0, b.size).reshape(b.shape) * b).astype(np.float32)
    f_odd, f_even = f[1::2], f[::2]
    half = (b / np.float32(2)).astype(np.float32)
    send = np.concatenate([half - f, f_even - f_odd], axis=0).astype(np.float32)
    return send, (half + f).astype(np.float32), (f_odd + f_even).astype(np.float32)


def normal(seed: int, ctr0: int, n: int) -> np.ndarray:
    """N(0, 1) float32 for elements 0..n-1 of one call (TF's Box-Muller over Philox word pairs)."""
    nb = (n + 3) // 4
    w = philox_blocks(seed, ctr0, nb)
    u = (np.uint32(0x3F800000) | (w & np.uint32(0x7FFFFF))).view(np.float32) - np.float32(1.0)
    u = u.astype(np.float32)
    out = np.empty((nb, 4), np.float32)
    for a, b in ((0, 1), (2, 3)):
        u1 = np.maximum(u[:, a], np.float32(1.0e-7)).astype(np.float32)
        v1 = (2.0 * np.pi * u[:, b].astype(np.float64)).astype(np.float32)
        lg = np.log(u1.astype(np.float64)).astype(np.float32)
        r = np.sqrt((np.float32(-2.0) * lg).astype(np.float32).astype(np.float64)).astype(np.float32)
        sn = np.sin(v1.astype(np.float64)).astype(np.float32)
        cs = np.cos(v1.astype(np.float64)).astype(np.float32)
        out[:, a] = sn * r
        out[:, b] = cs * r
    return out.reshape(-1)[:n]


def dp_noise(x: np.ndarray, seed: int, ctr0: int, mode: int, sigma: float, divisor: float, z=None):
    """efl_dp_noise: mode 0 (x + z x sigma) / d; mode 1 (x + (z sigma + 0)) / d (float32 steps).
    `z` overrides the normals (to isolate the arithmetic from log/sin/cos rounding)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    z = normal(seed, ctr0, x.size).reshape(x.shape) if z is None else np.asarray(z, np.float32).reshape(x.shape)
    s = np.float32(sigma)
    with np.errstate(all="ignore"):          # inf * 0 and overflow behave as the fp32 ops do
        if mode == 0:
            nz = ((z * x).astype(np.float32) * s).astype(np.float32)
        else:
            nz = ((z * s).astype(np.float32) + np.float32(0.0)).astype(np.float32)
        return ((x + nz).astype(np.float32) / np.float32(divisor)).astype(np.float32)
