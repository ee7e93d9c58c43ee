"""The reference's decode-a-WAV entry point (src/tests/demodulator/from_wave.py:24-234), drop-in.

read_wave_file keeps the reference semantics (stdlib `wave`, widths 1/2/4 -> uint8/int16/int32,
channel 0 of stereo, float32 / iinfo.max).  decode_ft8_from_wave uploads 16-bit PCM as int16 and
lets the STFT kernel apply the float32 x/32767 scaling on the device (bit-identical to
read_wave_file, half the host->device bytes); other widths are converted on the host as the
reference does.  `python -m ft8_demodulator_amd.from_wave file.wav [flags]` is the CLI.
"""
from __future__ import annotations

import argparse
import os
import sys
import wave

import numpy as np

from .ft8_decode import decode_ft8_message


def _read_raw(wave_path: str, verbose: bool = False):
    with wave.open(wave_path, "rb") as wf:
        n_channels = wf.getnchannels()
        sample_width = wf.getsampwidth()
        sample_rate = wf.getframerate()
        n_frames = wf.getnframes()
        if verbose:
            print(f"n_channels: {n_channels}")
            print(f"sample_width: {sample_width}")
            print(f"sample_rate: {sample_rate}")
            print(f"n_frames: {n_frames}")
        raw = wf.readframes(n_frames)
    if sample_width == 1:
        dtype = np.uint8
    elif sample_width == 2:
        dtype = np.int16
    elif sample_width == 4:
        dtype = np.int32
    else:
        raise ValueError(f"Unsupported sample width: {sample_width}")
    data = np.frombuffer(raw, dtype=dtype)
    if n_channels == 2:
        data = data[::2]
    return data, dtype, sample_rate


def read_wave_file(wave_path: str, verbose: bool = False) -> tuple:
    """from_wave.py:24-69 -> (float32 samples in [-1, 1], sample_rate)."""
    data, dtype, sample_rate = _read_raw(wave_path, verbose)
    x = data.astype(np.float32)
    x /= np.iinfo(dtype).max
    return x, sample_rate


def decode_ft8_from_wave(wave_path: str, freq_min: float = None, freq_max: float = None, time_min: float = None,
                         time_max: float = None, bins_per_tone: int = 2, steps_per_symbol: int = 2,
                         max_candidates: int = 20, min_score: float = 10, max_iterations: int = 20,
                         correction: bool = False, device=None, verbose: bool = False) -> list:
    """from_wave.py:71-178."""
    if correction:
        # from_wave.py:105-159 passes an FT8Waterfall as correct_frequency_drift's `params`, whose
        # default filling (frequency_correction.py:164-166) raises TypeError: the reference CLI's
        # correction path never decodes.  Same error here; the correction itself is available as
        # ft8_demodulator_amd.frequency_correction.correct_frequency_drift (GPU).
        raise TypeError("argument of type 'FT8Waterfall' is not iterable "
                        "(from_wave.py:152-158 passes a waterfall as correct_frequency_drift's params)")
    data, dtype, sample_rate = _read_raw(wave_path, verbose)
    if dtype == np.int16:
        import torch
        from . import _lib
        from ._pipeline import SlotDecoder, make_plan, records_to_results
        _lib.require_gpu()
        dev = torch.device("cuda", _lib.device_index(device))
        x = torch.from_numpy(np.array(data, copy=True)).to(dev)
        plan = make_plan(int(x.shape[0]), sample_rate, bins_per_tone, steps_per_symbol, freq_min, freq_max,
                         time_min, time_max)
        if plan.empty or max_candidates <= 0:
            return []
        dec = SlotDecoder(sample_rate, bins_per_tone, steps_per_symbol, max_candidates, min_score, max_iterations,
                          freq_min, freq_max, time_min, time_max, device=dev)
        recs = dec.records(x.unsqueeze(0), code=_lib.FT8_I16)[0]
        return records_to_results(recs, sample_rate, bins_per_tone, False)
    x = data.astype(np.float32)
    x /= np.iinfo(dtype).max
    return decode_ft8_message(x, sample_rate, bins_per_tone=bins_per_tone, steps_per_symbol=steps_per_symbol,
                              max_candidates=max_candidates, min_score=min_score, max_iterations=max_iterations,
                              freq_min=freq_min, freq_max=freq_max, time_min=time_min, time_max=time_max,
                              device=device)


def _print_results(results):
    if not results:
        print("No FT8 messages decoded")
        return
    print("\nDecoded FT8 messages:")
    print("-" * 50)
    for message, status, time_sec, freq_hz, score in results:
        print(f"Time: {time_sec:.2f} seconds")
        print(f"Frequency: {freq_hz:.1f} Hz")
        print(f"Score: {score:.1f}")
        print(f"Payload: {message.payload.hex()}")
        print(f"CRC check: {status.crc_calculated}")
        print(f"LDPC errors: {status.ldpc_errors}")
        print("-" * 50)


def _decode_many(args):
    """Several files (build-defined extension of the reference CLI): 16-bit PCM files of one sample
    rate and length are decoded as batches through the streaming path (stream.decode_wave_files);
    any other file -- and every file with --correction -- one at a time.  Results per file, in order."""
    from .stream import decode_wave_files
    kw = dict(freq_min=args.freq_min, freq_max=args.freq_max, time_min=args.time_min, time_max=args.time_max,
              bins_per_tone=args.bins_per_tone, steps_per_symbol=args.steps_per_symbol,
              max_candidates=args.max_candidates, min_score=args.min_score, max_iterations=args.max_iterations)
    out = [None] * len(args.wave_file)
    groups = {}
    for i, path in enumerate(args.wave_file):
        raw, dt, fs = _read_raw(path)
        if args.correction or dt != np.int16:
            out[i] = decode_ft8_from_wave(path, correction=args.correction, **kw)
        else:
            groups.setdefault((fs, raw.shape[0]), []).append(i)
    for idx in groups.values():
        res = decode_wave_files([args.wave_file[i] for i in idx], **kw)
        for i, r in zip(idx, res):
            out[i] = r
    return out


def main(argv=None):
    """from_wave.py:180-229 (same flags).  Several wave files may be given (decoded as batches)."""
    parser = argparse.ArgumentParser(description="Decode FT8 signals from a wave file (MI355X GPU path)")
    parser.add_argument("wave_file", nargs="+", help="input wave file(s)")
    parser.add_argument("--freq-min", type=float, help="minimum frequency (Hz)")
    parser.add_argument("--freq-max", type=float, help="maximum frequency (Hz)")
    parser.add_argument("--time-min", type=float, help="minimum time (s)")
    parser.add_argument("--time-max", type=float, help="maximum time (s)")
    parser.add_argument("--bins-per-tone", type=int, default=2)
    parser.add_argument("--steps-per-symbol", type=int, default=2)
    parser.add_argument("--max-candidates", type=int, default=20)
    parser.add_argument("--min-score", type=float, default=10)
    parser.add_argument("--max-iterations", type=int, default=20)
    parser.add_argument("--correction", type=bool, default=False)
    args = parser.parse_args(argv)
    for path in args.wave_file:
        if not os.path.exists(path):
            print(f"Error: File {path} does not exist")
            sys.exit(1)
    if len(args.wave_file) > 1:
        per_file = _decode_many(args)
        for path, results in zip(args.wave_file, per_file):
            print(f"\n== {path}")
            _print_results(results)
        return per_file
    args.wave_file = args.wave_file[0]
    results = decode_ft8_from_wave(args.wave_file, freq_min=args.freq_min, freq_max=args.freq_max,
                                   time_min=args.time_min, time_max=args.time_max,
                                   bins_per_tone=args.bins_per_tone, steps_per_symbol=args.steps_per_symbol,
                                   max_candidates=args.max_candidates, min_score=args.min_score,
                                   max_iterations=args.max_iterations, correction=args.correction)
    _print_results(results)
    return results


if __name__ == "__main__":
    main()
