"""Philox4x32-10 known-answer vectors (Random123 kat_vectors) for the oracle generator."""
import numpy as np

import rng_ref as R


def test_philox_kat():
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in cases:
        out = R.philox4x32_10(*[np.array([c], np.uint32) for c in ctr], *key)
        assert tuple(int(o[0]) for o in out) == want


def test_normals_moments():
    z = R.normals(5, np.arange(20000), 7, R.OBS_NOISE, 8).ravel()
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
