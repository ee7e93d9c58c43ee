"""Batched decode of independent 15-s slots (the data-parallel unit of this path).

    dec = SlotDecoder(sample_rate=12000, max_candidates=300, min_score=2)
    per_slot = dec.decode(samples)          # samples: torch [B, N] on the GPU (float32/int16/...)

decode_slots() is the one-call form.  See _pipeline.SlotDecoder.
"""
from ._pipeline import SlotDecoder  # noqa: F401


def decode_slots(samples, sample_rate=12000, **kwargs):
    """samples [B, N] -> list (per slot) of decode_ft8_message-style 5-tuples."""
    return SlotDecoder(sample_rate=sample_rate, **kwargs).decode(samples)
