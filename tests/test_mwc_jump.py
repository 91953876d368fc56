"""The arithmetic behind the speculated mesh pixels' chunk seeds (rt_kernels.hip
`mwc_jump`, rt_host.cpp `spec_setup`): each of frand's two MWC generators (rng.h:9-47,
x <- A (x & 0xffff) + (x >> 16)) is x <- A x mod M, M = A 2^16 - 1, on the states below M, so k
draws are one multiplication by A^k mod M; states at or above M reach that range within 2 steps
(M itself is a fixed point), and A^-1 = 2^16 mod M undoes the canonicalising steps.  CPU-only:
the kernel's use of it is pinned by the GPU split tests against the oracle."""
import numpy as np
import pytest

GENERATORS = (36969, 18000)


def step(x, a):
    return (a * (x & 0xFFFF) + (x >> 16)) & 0xFFFFFFFF


def jump(x, k, a):
    """mwc_jump's rule: small k stepped; else canonicalise, then one multiplication."""
    m = a * 65536 - 1
    if k <= 16:
        for _ in range(k):
            x = step(x, a)
        return x
    k0 = 0
    while x > m:
        x = step(x, a)
        k0 += 1
    if x == m:
        return m
    mul = pow(a, k, m)
    for _ in range(k0):
        mul = mul * 65536 % m
    return x * mul % m


@pytest.mark.parametrize("a", GENERATORS)
def test_jump_equals_stepping(a):
    rng = np.random.default_rng(a)
    m = a * 65536 - 1
    starts = [int(v) for v in rng.integers(0, 2**32, 100)] + [0, 1, 2, m - 1, m, m + 1, 2**32 - 1, 2**31 - 1]
    for x0 in starts:
        for k in (1, 7, 16, 17, 64, 255, 1024):
            x = x0
            for _ in range(k):
                x = step(x, a)
            assert jump(x0, k, a) == x, (x0, k)


@pytest.mark.parametrize("a", GENERATORS)
def test_states_below_m_stay_and_others_arrive_within_two_steps(a):
    m = a * 65536 - 1
    assert step(m, a) == m  # the fixed point
    assert a * 65536 % m == 1  # a^-1 = 2^16 mod M
    # states above M (the only ones that need canonicalising: the 2^20 just above M and just
    # below 2^32, and a random 2^22 between), and a random sample below M: the step keeps states
    # below M, and the others are below M or at the fixed point within 2 steps (rt_kernels.hip's
    # loop bound; every 32-bit state was checked once)
    rng = np.random.default_rng(a)
    above = np.concatenate([np.arange(m + 1, m + 1 + 2**20, dtype=np.uint64),
                            np.arange(2**32 - 2**20, 2**32, dtype=np.uint64),
                            rng.integers(m + 1, 2**32, 2**22, dtype=np.uint64)])
    x = above
    for _ in range(2):
        x = np.where(x > m, (a * (x & 0xFFFF) + (x >> 16)) & 0xFFFFFFFF, x)
    assert not (x > m).any()
    below = np.random.default_rng(1).integers(0, m, 2**22, dtype=np.uint64)
    assert ((a * (below & 0xFFFF) + (below >> 16)) < m).all()
