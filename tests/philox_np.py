"""NumPy restatement of the device sampler (test infrastructure, not a test module).

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC 2011; Random123's reference constants) and the draw of
``sample_kernel`` (flow-q-learning_amd/csrc/kernels.hip, section "sampling"),
which replaces the reference's minibatch draw ``np.random.randint(size, B)`` +
``arr[idxs]`` ([EXT] Dataset.sample, called at task/offline_task_real.py:38-43)
and the update's noise draws ([EXT] FQLAgent.update's jax.random splits):

* row b of member m at update count c: counter (b, c, salt, 0) under the member's
  sampler key (``sample_key``) gives word 0 -> row index (w0 * N) >> 32 and word 1
  -> flow time t = (w1 >> 8) / 2^24;
* counters (b, c, salt, 1 + q) give the normals 2q, 2q + 1 by Box-Muller
  (r = sqrt(-2 ln((w0 >> 8) + 1) / 2^24), angle 2 pi (w1 >> 8) / 2^24);
  normal i of 4A belongs to z_next / x0 / z_d / z_metric (i // A), action i % A.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
SALT_TRAIN, SALT_VAL = 0x51A7, 0x5A1D
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: (k0, k1). Returns uint32 [..., 4]."""
    c = np.asarray(ctr, dtype=np.uint64).copy()
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[..., 0]
        p1 = M1 * c[..., 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c[..., 1] ^ np.uint64(k0)
        n2 = hi0 ^ c[..., 3] ^ np.uint64(k1)
        c = np.stack([n0, lo1, n2, lo0], axis=-1)
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c.astype(np.uint32)


def sample_key(seed: int, alpha: float) -> int:
    """runtime.cpp sample_key: splitmix64 finaliser of seed ^ (bits(float32 alpha) << 32 | golden)."""
    ab = int(np.array([alpha], dtype=np.float32).view(np.uint32)[0])
    m = (1 << 64) - 1
    z = (int(seed) ^ ((ab << 32) | 0x9E3779B9)) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _u01(x):
    return (x >> np.uint32(8)).astype(np.float64) * (1.0 / 16777216.0)


def _u01_open_closed(x):
    return ((x >> np.uint32(8)).astype(np.float64) + 1.0) * (1.0 / 16777216.0)


def draw(key: int, count: int, B: int, n_rows: int, A: int, salt: int = SALT_TRAIN):
    """(idx [B] int64, noise dict of the oracle's keys) that sample_kernel draws for one
    member at update count ``count``."""
    k = (key & 0xFFFFFFFF, key >> 32)
    b = np.arange(B, dtype=np.uint32)
    ctr = np.stack([b, np.full(B, count, np.uint32), np.full(B, salt, np.uint32), np.zeros(B, np.uint32)], -1)
    w = philox4x32_10(ctr, k)
    idx = ((w[:, 0].astype(np.uint64) * np.uint64(n_rows)) >> np.uint64(32)).astype(np.int64)
    t = _u01(w[:, 1])
    normals = np.zeros((B, 4 * A))
    for q in range(2 * A):
        ctr[:, 3] = 1 + q
        wq = philox4x32_10(ctr, k)
        r = np.sqrt(-2.0 * np.log(_u01_open_closed(wq[:, 0])))
        ang = 2.0 * np.pi * _u01(wq[:, 1])
        normals[:, 2 * q] = r * np.cos(ang)
        if 2 * q + 1 < 4 * A:
            normals[:, 2 * q + 1] = r * np.sin(ang)
    noise = {"z_next": normals[:, 0:A], "x0": normals[:, A:2 * A], "t": t.reshape(B, 1),
             "z_d": normals[:, 2 * A:3 * A], "z_metric": normals[:, 3 * A:4 * A]}
    return idx, noise
