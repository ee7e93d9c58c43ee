"""ft8_demodulator_amd -- MI355X-native FT8 receive path (drop-in for Rintazero/ft8_demodulator).

Public API mirrors the reference's ft8_demodulator package (src/ft8_tools/ft8_demodulator):
decode_ft8_message, calculate_spectrogram, select_frequency_band,
create_waterfall_from_spectrogram, ft8_find_candidates, ft8_decode_candidate, bp_decode,
ldpc_check, compute_crc/extract_crc/add_crc and the FT8* dataclasses -- plus the WAV entry
point (from_wave) and a batched slot decoder (SlotDecoder, decode_slots).  Every numeric stage runs in
hand-written HIP kernels (csrc/) reached through the C-ABI library libft8hip.so; there is no
CPU fallback: calls fail loudly when the library or a GPU is missing.
"""
__version__ = "0.1.0"

from .ftx_types import FT8Candidate, FT8DecodeStatus, FT8Message, FT8Protocol, FT8Waterfall  # noqa: E402,F401
from .spectrogram_analyse import calculate_spectrogram, select_frequency_band  # noqa: E402,F401
from .ft8_decode import (  # noqa: E402,F401
    create_waterfall_from_spectrogram, decode_ft8_message, ft8_decode_candidate, ft8_extract_likelihood,
    ft8_find_candidates, ft8_score_grid, ft8_sync_score, ftx_normalize_logl, pack_bits)
from .ldpc_decoder import bp_decode, ldpc_check  # noqa: E402,F401
from .crc import add_crc, compute_crc, extract_crc  # noqa: E402,F401
from .from_wave import decode_ft8_from_wave, read_wave_file  # noqa: E402,F401
from ._pipeline import SlotDecoder, decode_slots  # noqa: E402,F401
