"""rt_sincosf (one shared reduction) is bit-identical to rt_sinf / rt_cosf — the pinned
Cephes-style builtins of include/rt_math.h the parity model rests on.  Host build of the
header with the system C++ compiler (the device uses the same source)."""
from __future__ import annotations

import subprocess

import numpy as np

from conftest import ROOT

SRC = r'''
#include <cstdio>
#include <cstring>
#include <cstdint>
#include "rt_math.h"
int main() {
    uint32_t bad = 0, n = 0;
    for (uint64_t k = 0; k < (1ull << 32); k += 4099) { /* strided over every float bit pattern */
        uint32_t u = (uint32_t)k; float x; std::memcpy(&x, &u, 4);
        float s, c; rt_sincosf(x, &s, &c);
        const float s2 = rt_sinf(x), c2 = rt_cosf(x);
        uint32_t a, b, d, e; std::memcpy(&a, &s, 4); std::memcpy(&b, &s2, 4); std::memcpy(&d, &c, 4); std::memcpy(&e, &c2, 4);
        if ((a != b && !(x != x)) || (d != e && !(x != x))) ++bad;
        ++n;
    }
    for (int i = -200000; i <= 200000; ++i) { /* dense around the sampling range 2 pi [0, 1) */
        const float x = (float)i * 1.0e-4f;
        float s, c; rt_sincosf(x, &s, &c);
        if (std::memcmp(&s, &(const float &)rt_sinf(x), 4) || std::memcmp(&c, &(const float &)rt_cosf(x), 4)) ++bad;
        ++n;
    }
    std::printf("%u %u\n", n, bad);
    return 0;
}
'''


def test_sincos_matches_sin_and_cos(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", f"-I{ROOT / 'include'}", str(src), "-o",
                    str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True, timeout=300).stdout.split()
    n, bad = int(out[0]), int(out[1])
    assert n > 1_000_000 and bad == 0
