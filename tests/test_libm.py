"""The restated glibc float libm the texture maps use (pt_device.h libm_atan2f,
libm_asinf, libm_logf: SphericalCoordinatesSkymapTexture's std::atan2 / std::asin
on floats, transform_texture.h:73-85, and LogTexture's std::log, filter_texture.h:
62-67) against this machine's own glibc atan2f / asinf / logf, called through
ctypes: random operands over the unit range the texture maps see, wide-exponent
operands, the branches uniform operands miss (exponent gaps beyond +-26 and
+-60, signed zeros, infinities, NaN, subnormals).  A different glibc on the
host (say, a correctly rounded one) fails here before any render differs.
The CPU half checks tools/libm's restatements the same way (no GPU)."""
import ctypes
import ctypes.util
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _f, _n in (("atan2f", 2), ("asinf", 1), ("logf", 1)):
    getattr(_libm, _f).restype = ctypes.c_float
    getattr(_libm, _f).argtypes = [ctypes.c_float] * _n


def operands(n=200000, seed=11):
    rng = np.random.default_rng(seed)
    y = rng.uniform(-1, 1, n).astype(np.float32)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    # wide exponents, both signs
    k = n // 4
    y[:k] = (np.ldexp(rng.uniform(1, 2, k), rng.integers(-149, 128, k)) * rng.choice([-1, 1], k)).astype(np.float32)
    x[k:2 * k] = (np.ldexp(rng.uniform(1, 2, k), rng.integers(-149, 128, k)) *
                  rng.choice([-1, 1], k)).astype(np.float32)
    sp = np.array([0.0, -0.0, 1.0, -1.0, 2.0 ** -30, -2.0 ** -30, 2.0 ** -149, -2.0 ** -149, 2.0 ** 100, np.inf,
                   -np.inf, np.nan, 0.5, 1.5, 2.0 ** -126, 3.4e38], dtype=np.float32)
    gy, gx = np.meshgrid(sp, sp)
    # exponent gaps of 20..70 both ways, x negative and positive
    ey = np.arange(-70, 71)
    gap_y = np.concatenate([np.ldexp(1.5, ey), -np.ldexp(1.25, ey), np.ones(141), -np.ones(141)]).astype(np.float32)
    gap_x = np.concatenate([-np.ones(141), np.ones(141), -np.ldexp(1.5, ey), np.ldexp(1.75, ey)]).astype(np.float32)
    y = np.concatenate([y, gy.ravel(), gap_y])
    x = np.concatenate([x, gx.ravel(), gap_x])
    return np.stack([y, x], axis=1).astype(np.float32)


def host_libm(ops):
    out = np.empty((len(ops), 3), dtype=np.float32)
    for i, (y, x) in enumerate(ops.tolist()):
        out[i] = (_libm.atan2f(y, x), _libm.asinf(y), _libm.logf(x))
    return out


def same_bits(a, b):
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


@pytest.mark.gpu
def test_device_libm_matches_host_glibc(built):
    from pathtrace import _lib
    ops = operands()
    dev = _lib.selftest_libm(ops)
    ref = host_libm(ops)
    ok = same_bits(dev, ref)
    for c, name in enumerate(("atan2f", "asinf", "logf")):
        bad = np.nonzero(~ok[:, c])[0]
        assert bad.size == 0, "%s: %d of %d differ, e.g. ops %s dev %s glibc %s" % (
            name, bad.size, len(ops), ops[bad[:3]], dev[bad[:3], c], ref[bad[:3], c])


@pytest.mark.slow
@pytest.mark.parametrize("tool,args", [("atan2f_restated.c", []), ("asinf_restated.c", []),
                                       ("logf_restated.c", ["97"])])
def test_restated_libm_matches_glibc_on_cpu(tmp_path, tool, args):
    """tools/libm's CPU restatements (the device algorithms, line for line)
    against glibc: atan2f on 2e7 random + 2.4e6 edge operand pairs, asinf on
    every float in [-1, 1], logf on every 97th non-negative float (the full
    sweep of all 2^31 takes ~1 min: profiles/round4/logf_restated_vs_glibc.txt)."""
    exe = str(tmp_path / "chk")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tools", "libm", tool), "-lm", "-o",
                    exe], check=True)
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
