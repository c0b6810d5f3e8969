"""Philox4x32-10 (the Glorot initialiser's RNG, csrc/hip/common.h) against
the Random123 known-answer vectors, and the host entry point of the HIP init
kernel against a pure-Python model of the same draw."""
import math

import pytest

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox(c, k0, k1):
    c = list(c)
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c[3] ^ k1) & MASK, p0 & MASK]
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c


def test_random123_known_answers():
    assert philox([0, 0, 0, 0], 0, 0) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert philox([MASK] * 4, MASK, MASK) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]


def _py_draw(key, lin, tag, limit):
    c = philox([lin & MASK, lin >> 32, tag, 0x676c6f72], key & MASK, key >> 32)
    u = (c[0] >> 8) * (1.0 / 16777216.0)
    return (2.0 * u - 1.0) * limit


def test_host_reference_matches_python_model():
    try:
        from gentun_amd.ops import cnn_kernels as K
        L = K.lib()
    except Exception as exc:      # noqa: BLE001
        pytest.skip("HIP library not loadable here: {}".format(exc))
    for key, lin, tag, lim in [(0, 0, 0, 1.0), (123456789012345, 77, 3, 0.25), ((1 << 63) - 1, 1 << 33, 9, 0.1)]:
        got = L.gt_glorot_ref(key, lin, tag, lim)
        assert math.isclose(got, _py_draw(key, lin, tag, lim), rel_tol=1e-6, abs_tol=1e-7)
