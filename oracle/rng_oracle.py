"""numpy restatement of the device's counter-based draws (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module.  It recomputes, on the host, the N(0,1)
turbulence noise that the kernels draw with Philox4x32-10 (Salmon et al., SC'11)
and Box-Muller (csrc/fw_device.hpp philox/normal4, csrc/fw_kernels.hip noise4):
sample k of episode e of global env g is

    philox(key = (seed & 0xffffffff, seed >> 32), counter = (g, e, 1, k)) -> 4 x u32
    z[2j], z[2j+1] = sqrt(-2 ln u1) (cos, sin)(2 pi u2),
        u1 = r[2j] 2^-32 + 2^-33,  u2 = r[2j+1] 2^-32

for the four Dryden input channels (dryden.py:166-172 draws them from
RandomState.standard_normal instead; the reference's generator cannot run on a
GPU lane).  Episode e counts the env's resets (1 after the first).
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32(k0, k1, c0, c1, c2, c3):
    """Vectorised Philox4x32-10; every argument broadcastable uint32 arrays."""
    k0, k1 = np.uint32(k0), np.uint32(k1)
    c = [np.asarray(x, dtype=np.uint32) for x in np.broadcast_arrays(c0, c1, c2, c3)]
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c[0].astype(np.uint64)
            p1 = M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c


def normal4(r):
    """Box-Muller of one Philox block -> 4 standard normals (fp64)."""
    z = []
    for j in range(2):
        u1 = r[2 * j].astype(np.float64) * 2.3283064365386963e-10 + 1.1641532182693481e-10
        u2 = r[2 * j + 1].astype(np.float64) * 2.3283064365386963e-10
        rad = np.sqrt(-2.0 * np.log(u1))
        ang = 6.283185307179586 * u2
        z += [rad * np.cos(ang), rad * np.sin(ang)]
    return z


def turbulence_noise(seed, env_ids, episode, length):
    """[len(env_ids)][4][length] N(0,1) Dryden input noise the device draws in ``episode``."""
    seed = int(seed) % (1 << 64)
    g = np.asarray(env_ids, dtype=np.uint32)[:, None]
    k = np.arange(length, dtype=np.uint32)[None, :]
    r = philox4x32(seed & 0xFFFFFFFF, seed >> 32, g, np.uint32(episode), np.uint32(1), k)
    return np.stack(normal4(r), axis=1)
