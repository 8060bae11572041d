"""Pure-Python Flink/Java hashing (oracle twin of csrc/mxs_common.h).

key group  = murmurHash(key.hashCode()) % maxParallelism        (KeyGroupRangeAssignment)
subtask    = keyGroup * parallelism / maxParallelism           (computeOperatorIndexForKeyGroup)
maxParallelism default = min(max(roundUpToPow2(p + p/2), 128), 32768)
Verified against the README's `N>` prefixes in SURVEY.md Appendix A.5.
"""
from __future__ import annotations

M32 = 0xFFFFFFFF


def _i32(x: int) -> int:
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def _rotl(x: int, r: int) -> int:
    x &= M32
    return ((x << r) | (x >> (32 - r))) & M32


def java_string_hash(s: str) -> int:
    h = 0
    for unit in _utf16_units(s):
        h = (31 * h + unit) & M32
    return _i32(h)


def _utf16_units(s: str):
    b = s.encode("utf-16-le", errors="surrogatepass")
    for i in range(0, len(b), 2):
        yield b[i] | (b[i + 1] << 8)


def java_long_hash(v: int) -> int:
    u = v & 0xFFFFFFFFFFFFFFFF
    return _i32(u ^ (u >> 32))


def java_int_hash(v: int) -> int:
    return _i32(v)


def java_double_hash(v: float) -> int:
    import struct

    bits = struct.unpack("<q", struct.pack("<d", v))[0]
    if v != v:  # canonical NaN
        bits = 0x7FF8000000000000
    return java_long_hash(bits)


def java_hash(v) -> int:
    """hashCode() of the Java boxed type the value models (str, int->Long, float->Double)."""
    if isinstance(v, str):
        return java_string_hash(v)
    if isinstance(v, bool):
        return 1231 if v else 1237
    if isinstance(v, int):
        return java_long_hash(v)
    if isinstance(v, float):
        return java_double_hash(v)
    if isinstance(v, tuple):  # TupleN.hashCode: 31 * result + field hash
        h = 0
        for i, f in enumerate(v):
            fh = java_hash(f)
            h = fh if i == 0 else _i32(31 * h + fh)
        return h
    raise TypeError(f"no Java hash for {type(v).__name__}")


def flink_murmur(code: int) -> int:
    h = code & M32
    h = (h * 0xCC9E2D51) & M32
    h = _rotl(h, 15)
    h = (h * 0x1B873593) & M32
    h = _rotl(h, 13)
    h = (h * 5 + 0xE6546B64) & M32
    h ^= 4
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    c = _i32(h)
    if c >= 0:
        return c
    if c != -(1 << 31):
        return -c
    return 0


def key_groups_of_java_hashes(hashes, max_parallelism: int = 128):
    """flink_murmur(h) % max_parallelism of an int32 array of Java hashes (numpy, vectorised;
    the per-key Python path of flink_murmur for whole dictionaries)."""
    import numpy as np

    h = np.asarray(hashes).astype(np.int64) & M32

    def rotl(x, r):
        return ((x << r) | (x >> (32 - r))) & M32

    h = (h * 0xCC9E2D51) & M32
    h = rotl(h, 15)
    h = (h * 0x1B873593) & M32
    h = rotl(h, 13)
    h = (h * 5 + 0xE6546B64) & M32
    h ^= 4
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    c = np.where(h >= 1 << 31, h - (1 << 32), h)  # as int32
    c = np.where(c == -(1 << 31), 0, np.abs(c))
    return (c % max_parallelism).astype(np.int32)


def default_max_parallelism(p: int) -> int:
    x = p + p // 2
    pow2 = 1 << (max(x, 1) - 1).bit_length()
    return min(max(pow2, 128), 32768)


def key_group(key, max_parallelism: int = 128) -> int:
    return flink_murmur(java_hash(key)) % max_parallelism


def subtask_of(key, parallelism: int, max_parallelism: int = 128) -> int:
    return key_group(key, max_parallelism) * parallelism // max_parallelism
