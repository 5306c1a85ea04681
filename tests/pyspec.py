"""Independent pure-Python statement of SURVEY.md Appendix A (small inputs only).

A second, separately written restatement used to cross-check oracle/csum_oracle.c
on random buffers, including the cases where the reference's exact two-fold
differs from a full RFC 1071 fold (raw sums >= 2^32).
"""
import struct


def pseudo(saddr_be: int, daddr_be: int, len_be: int) -> int:
    raw = struct.pack("<IIBBH", saddr_be, daddr_be, 0, 6, len_be)
    return sum(struct.unpack("<6H", raw))


def csum_continue(sum_start: int, p: bytes, nbytes: int) -> int:
    s = sum_start if sum_start < 2**63 else sum_start - 2**64    # C `long`
    n = max(nbytes, 0)
    even = n & ~1
    s += sum(p[k] | (p[k + 1] << 8) for k in range(0, even, 2))
    if n & 1:
        s += p[n - 1]
    s = (s >> 16) + (s & 0xFFFF)
    s = s + (s >> 16)
    return (~s) & 0xFFFF


def exact_sum(sum_start: int, p: bytes) -> int:
    return sum_start + sum(p[k] * (1 if k % 2 == 0 else 256) for k in range(len(p)))
