"""Mirror of the reference ldpc_decoder.py (ldpc_decoder.py:33-113), run on the GPU.

bp_decode and ldpc_check call the k_bp / k_ldpc_check HIP kernels (csrc/bp.hip): float64 sum-product
BP with the reference's rational tanh/atanh and evaluation order, bit-identical hard decisions.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from . import _device
from .constants import FTX_LDPC_M, FTX_LDPC_N, kFTX_LDPC_Mn, kFTX_LDPC_Nm, kFTX_LDPC_Num_rows  # noqa: F401


def ldpc_check(codeword: np.ndarray) -> int:
    """ldpc_decoder.py:33-52: number of unsatisfied parity checks of a 174-bit codeword."""
    return int(_device.ldpc_check(np.asarray(codeword).reshape(1, FTX_LDPC_N))[0])


def bp_decode(codeword: np.ndarray, max_iterations: int) -> Tuple[np.ndarray, int]:
    """ldpc_decoder.py:54-113: (hard decision of the last evaluated iteration, min parity errors)."""
    plain, rec = _device.bp(np.asarray(codeword, dtype=np.float64).reshape(1, FTX_LDPC_N), max_iterations)
    return plain[0].astype(np.uint8), int(rec[0]["ldpc_errors"])


def bp_decode_batch(codewords: np.ndarray, max_iterations: int):
    """Batched bp_decode: LLRs [n, 174] -> (plain [n, 174] uint8, min_errors [n])."""
    plain, rec = _device.bp(np.asarray(codewords, dtype=np.float64).reshape(-1, FTX_LDPC_N), max_iterations)
    return plain, rec["ldpc_errors"].astype(np.int64)
