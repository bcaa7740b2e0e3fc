"""Portable, bit-reproducible inputs for the large golden fixture.

The fixture's inputs (1.5M edges, F = 128) are too large to commit, so they
are regenerated from a counter-based integer hash (splitmix64) with uint64
arithmetic only: no libm, no RNG library, hence the same bits on every
numpy/CPU. The fixture stores the SHA-256 of the generated arrays, so any
drift of this generator is caught before outputs are compared.

Graph ``reddit_rows``: N = 32,768 nodes, E = 1,500,000 edges in edge-id
order. Destinations are power-law at Reddit row lengths and beyond (a
destination's id is drawn below 2^s for s uniform in 2..15, then a fixed
bijection of [0, N) scatters the hubs): the four longest rows have ~53k
in-edges each, the next four ~27k, then ~13k, ... (Reddit's largest
in-degree is 21,657). Sources follow the same law with s in 0..15, so hub pairs
repeat thousands of times: heavy parallel (multigraph) duplicates, which the
reference's uncoalesced COO keeps (src/graph/graph.cc:509-524).
"""
import hashlib

import numpy as np

N = 1 << 15
E = 1_500_000
F = 128

def splitmix64(stream, count):
    """``count`` uint64 words of stream ``stream`` (splitmix64 of a counter)."""
    with np.errstate(over="ignore"):
        x = (np.arange(count, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        x = x + np.uint64(stream) * np.uint64(0xD1B54A32D192ED03)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _powerlaw_ids(stream, count, s_lo, s_hi, mult, add):
    z = splitmix64(stream, count)
    s = np.uint64(s_lo) + (z >> np.uint64(32)) % np.uint64(s_hi - s_lo + 1)
    v = (z & np.uint64(N - 1)) & ((np.uint64(1) << s) - np.uint64(1))
    # fixed bijection of [0, 2^15): odd multiplier + offset, mod 2^15
    return ((v * np.uint64(mult) + np.uint64(add)) & np.uint64(N - 1)).astype(np.int64)


def uniform_f32(stream, shape, lo, hi):
    """Uniform floats k / 2^23 * (hi - lo) + lo, k < 2^23: exact in fp32 for
    the power-of-two widths used here (2 and 1)."""
    count = int(np.prod(shape))
    k = (splitmix64(stream, count) >> np.uint64(41)).astype(np.int64)  # 23 bits
    width = hi - lo
    return (k.astype(np.float32) * np.float32(width / float(1 << 23)) + np.float32(lo)) \
        .astype(np.float32).reshape(shape)


def reddit_rows():
    """(src, dst, H, W, G): int64[E] x2, fp32 (N, F), fp32 (E,), fp32 (N, F)."""
    dst = _powerlaw_ids(1, E, 2, 15, 40503, 12345)
    src = _powerlaw_ids(2, E, 0, 15, 22937, 777)
    H = uniform_f32(3, (N, F), -1.0, 1.0)
    W = uniform_f32(4, (E,), 0.5, 1.5)
    G = uniform_f32(5, (N, F), -1.0, 1.0)
    return src, dst, H, W, G


def digest(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()
