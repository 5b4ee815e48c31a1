"""Philox4x32-10 (Salmon, Moraes, Dror, Shaw — SC'11, Random123 constants) in numpy, and the
exact draw schedule the HIP kernels use.  TEST INFRASTRUCTURE ONLY.

The reference draws env noise from torch's global generator (humanoid_env.py:624-631, :868,
:1038-1044, :1053-1066, :1018-1032, :665-681), which a GPU cannot reproduce; the build keys a
counter-based generator by (seed, env, step, block, purpose) instead, identically in the HIP path
(csrc/hg_common.h) and here, so oracle and GPU draws agree bit for bit.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)

ACT_DELAY, ACT_NOISE, OBS_NOISE, CMD, PUSH, RESET_DOF, RESET_ROOT, TERRAIN = 1, 2, 3, 4, 5, 6, 7, 8


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over arrays of uint32 counters; returns 4 uint32 arrays."""
    c = [np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3)]
    k0 = np.uint64(k0) & MASK
    k1 = np.uint64(k1) & MASK
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [(hi1 ^ c[1] ^ k0) & MASK, lo1, (hi0 ^ c[3] ^ k1) & MASK, lo0]
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return [x.astype(np.uint32) for x in c]


def u01(x):
    return ((x >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def u01_open0(x):
    return (((x >> np.uint32(8)) + np.uint32(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def rng4(seed, env, step, block, purpose):
    """Same counter packing as rng4() in csrc/hg_common.h."""
    env = np.asarray(env, dtype=np.uint64)
    step = np.uint64(step)
    c1 = np.full(env.shape, step & MASK, dtype=np.uint64)
    c2 = np.full(env.shape, (np.uint64(block) & np.uint64(0xFFFF)) | ((step >> np.uint64(32)) << np.uint64(16)),
                 dtype=np.uint64)
    c3 = np.full(env.shape, purpose, dtype=np.uint64)
    return philox4x32_10(env, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def normals4(r):
    """Box-Muller, as normals4() in hg_common.h (float32)."""
    r0 = np.sqrt(np.float32(-2.0) * np.log(u01_open0(r[0])))
    r1 = np.sqrt(np.float32(-2.0) * np.log(u01_open0(r[2])))
    a0 = np.float32(6.283185307179586) * u01(r[1])
    a1 = np.float32(6.283185307179586) * u01(r[3])
    return np.stack([r0 * np.cos(a0), r0 * np.sin(a0), r1 * np.cos(a1), r1 * np.sin(a1)], 1).astype(np.float32)


def normals(seed, env, step, purpose, count):
    blocks = (count + 3) // 4
    return np.concatenate([normals4(rng4(seed, env, step, b, purpose)) for b in range(blocks)], 1)[:, :count]
