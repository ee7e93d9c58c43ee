"""Mirror of the reference crc.py (crc.py:1-79): CRC-14 (poly 0x2757) of FT8/FT4 messages.

compute_crc runs in the k_crc14 HIP kernel; the decode path computes the same CRC inside the BP
epilogue of csrc/bp.hip.
"""
from __future__ import annotations

from . import _device

CRC_WIDTH = 14
CRC_POLYNOMIAL = 0x2757
TOPBIT = 1 << (CRC_WIDTH - 1)


def compute_crc(message, num_bits: int) -> int:
    """crc.py:11-39."""
    if num_bits > 96:
        raise ValueError("compute_crc supports messages of at most 96 bits")
    nbytes = (num_bits + 7) // 8
    if len(message) < nbytes:
        raise IndexError("message shorter than num_bits")
    return _device.crc14([bytes(message[:nbytes])], [num_bits])[0]


def extract_crc(a91) -> int:
    """crc.py:41-54: the 14 CRC bits that follow the 77-bit payload."""
    return ((a91[9] & 0x07) << 11) | (a91[10] << 3) | (a91[11] >> 5)


def add_crc(payload, a91) -> None:
    """crc.py:56-79: a91 <- payload (77 bits) + CRC-14 over 82 bits."""
    for i in range(10):
        a91[i] = payload[i]
    a91[9] &= 0xF8
    a91[10] = 0
    a91[11] = 0
    checksum = compute_crc(a91, 82)
    a91[9] |= checksum >> 11
    a91[10] = (checksum >> 3) & 0xFF
    a91[11] = (checksum << 5) & 0xE0
