"""The per-(pixel, sample) engine (include/pt/pt_engine.h) against an
independent pure-Python model, the oracle, and the reference driver's KAT
stream; and the O(1) jump the GPU bursts rely on against plain stepping."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
M64 = (1 << 64) - 1
MULT = 6364136223846793005


def splitmix(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class PyEngine:
    def __init__(self, seed, pixel, sample):
        key = splitmix(seed) ^ (pixel << 20) ^ sample
        self.s = splitmix(key)
        self.inc = ((splitmix(key ^ 0xD1B54A32D192ED03) << 1) | 1) & M64

    def __call__(self):
        old = self.s
        self.s = (old * MULT + self.inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF


def jump(k):
    a, g = 1, 0
    for _ in range(k):
        a, g = (a * MULT) & M64, (g * MULT + 1) & M64
    return a, g


def test_python_model_matches_reference_driver_stream():
    kat = np.load(os.path.join(GOLD, "kat.npy"))
    e = PyEngine(0x5EED, 7, 3)
    assert [e() for _ in range(16)] == [int(v) for v in kat[15:31]]


def test_jump_equals_stepping():
    e = PyEngine(1, 2, 3)
    s0, inc = e.s, e.inc
    for k in [0, 1, 3, 5, 64, 189, 192]:
        a, g = jump(k)
        f = PyEngine(1, 2, 3)
        for _ in range(k):
            f()
        assert (a * s0 + g * inc) & M64 == f.s


@pytest.fixture(scope="module")
def header_probe(tmp_path_factory):
    """Compile a host program against the product header pt_engine.h."""
    d = tmp_path_factory.mktemp("eng")
    src = d / "probe.c"
    src.write_text(r'''
#include <stdio.h>
#include "pt/pt_engine.h"
int main(void) {
    for (unsigned k = 0; k <= 200; k++) {
        uint64_t a, g; pt_pcg_jump_coeffs(k, &a, &g);
        printf("%u %llu %llu\n", k, (unsigned long long)a, (unsigned long long)g);
    }
    uint64_t st, inc; pt_engine_seed(pt_sample_key(0x5EED, 7, 3), &st, &inc);
    for (int i = 0; i < 16; i++) { uint64_t o = st; st = o * PT_PCG_MULT + inc; printf("o %u\n", pt_pcg_output(o)); }
    return 0;
}''')
    exe = d / "probe"
    subprocess.check_call(["gcc", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    return subprocess.check_output([str(exe)], text=True).split("\n")


def test_header_jump_coefficients(header_probe):
    for line in header_probe:
        if line and not line.startswith("o"):
            k, a, g = map(int, line.split())
            assert (a, g) == jump(k)


def test_header_engine_stream(header_probe):
    outs = [int(l.split()[1]) for l in header_probe if l.startswith("o")]
    e = PyEngine(0x5EED, 7, 3)
    assert outs == [e() for _ in range(16)]


def test_streams_of_adjacent_samples_are_unrelated():
    a, b = PyEngine(0x5EED, 10, 0), PyEngine(0x5EED, 10, 1)
    xa = np.array([a() for _ in range(4096)], dtype=np.float64)
    xb = np.array([b() for _ in range(4096)], dtype=np.float64)
    assert abs(np.corrcoef(xa, xb)[0, 1]) < 0.05
    assert abs(xa.mean() / 2 ** 32 - 0.5) < 0.02
