"""Streaming decode of slots that arrive in host memory ("WAV ingestion + H2D
pipelining").

Batches of 15-s slots -- typically 16-bit PCM straight from WAV files -- are staged in pinned host
memory and uploaded on a dedicated copy stream into one of depth + 2 device buffers: the copy stream
uploads batch k + depth + 1 while batches k + 1 .. k + depth decode and batch k's results are
converted on the host; results come back through pinned host buffers.  Consecutive batches decode on
`depth` decoders (default 2), each with its own library context and compute stream, so the next
batch's front end (STFT, sync, selection) runs in the CUs the previous batch's k_bp tail leaves --
the bench's `--depth` pattern (bench.py).  int16 PCM
is uploaded as-is (half the PCIe bytes of float32) and scaled by the STFT kernel exactly as
read_wave_file does (from_wave.py:59-67).

    sd = StreamDecoder(n_samples=180000, max_candidates=300, min_score=2)
    for per_slot in sd.decode_batches(batches):      # each batch: np.int16 [B, n_samples], or a
        ...                                          # pinned torch int16 tensor (no staging copy)

decode_wave_files() is the one-call form for a list of WAV files of equal length and rate.
"""
from __future__ import annotations

from typing import Iterable, Iterator, List

import numpy as np

from . import _lib
from ._pipeline import SlotDecoder, records_to_results, warn_truncated


class StreamDecoder:
    """Host -> device upload on a copy stream overlapped with ft8_decode_batch on `depth` decoders
    (own context and compute stream each; depth 1 = one decoder on the current stream).

    Memory: depth + 2 device and depth + 2 pinned host sample buffers of max_batch x n_samples
    (int16 PCM: 2 B per sample; float32: 4 B), plus depth + 2 pinned result buffers, plus one library
    context per decoder beyond the first (its own scratch: waterfall, scores, LLRs of max_batch
    slots).  At max_batch 256 and 180 000 int16 samples a sample buffer is 92 MB, so the default
    depth 2 holds 4 x 92 MB on the device and 4 x 92 MB pinned, against 3 x 92 MB each at depth 1,
    and creates one extra context (~0.5 GB of decode scratch at 256 slots).  Choose depth 1 for one
    or two batches: there is nothing to overlap."""

    def __init__(self, n_samples: int, sample_rate: int = 12000, max_batch: int = 256, pcm16: bool = True,
                 device=None, depth: int = 2, **decoder_kw):
        torch = _lib.require_gpu()
        self.torch = torch
        self.dev = torch.device("cuda", _lib.device_index(device))
        self.n = int(n_samples)
        self.fs = sample_rate   # as given (int or float Hz): result times are abs_time / fs
        self.max_batch = int(max_batch)
        self.pcm16 = bool(pcm16)
        self.dtype = torch.int16 if pcm16 else torch.float32
        self.depth = int(depth)
        if self.depth < 1:
            raise ValueError("depth must be >= 1")
        self.NBUF = self.depth + 2   # depth decoding + one uploading + the one being collected
        self.dec = SlotDecoder(sample_rate=sample_rate, device=self.dev, **decoder_kw)
        # decoders 1 .. depth-1 own a context each: decoders sharing one would be ordered across
        # their streams by the library (one chain again)
        self.decs = [self.dec] + [SlotDecoder(sample_rate=sample_rate, device=self.dev,
                                              context=_lib.Context(self.dev.index), **decoder_kw)
                                  for _ in range(self.depth - 1)]
        self.bpt = self.dec.kw["bins_per_tone"]
        self.code = _lib.FT8_I16 if pcm16 else _lib.FT8_F32
        self.copy_stream = torch.cuda.Stream(self.dev)
        self.computes = ([torch.cuda.current_stream(self.dev)] if self.depth == 1 else
                         [torch.cuda.Stream(self.dev) for _ in range(self.depth)])
        self.compute = self.computes[0]
        self.uploaded = [None] * self.NBUF   # copy-stream event: dbuf[i] holds its batch
        self.dbuf = [torch.empty((self.max_batch, self.n), dtype=self.dtype, device=self.dev) for _ in range(self.NBUF)]
        self.hbuf = [torch.empty((self.max_batch, self.n), dtype=self.dtype, pin_memory=True) for _ in range(self.NBUF)]
        self.freed = [None] * self.NBUF   # compute-stream event: decode done with dbuf[i]
        cap = self.dec.cap * _lib.RESULT_DTYPE.itemsize
        self.hout = [torch.empty(self.max_batch * cap, dtype=torch.uint8, pin_memory=True) for _ in range(self.NBUF)]
        self.hcnt = [torch.empty(self.max_batch, dtype=torch.int32, pin_memory=True) for _ in range(self.NBUF)]
        self.ready = [None] * self.NBUF   # compute-stream event: results copied to hout/hcnt[i]
        self.caller_upload = None   # copy-stream event of an in-place upload of a caller's pinned tensor

    def _stage(self, i: int, batch) -> int:
        """Start the upload of a host batch into device buffer i.  A pinned torch tensor is uploaded
        in place; anything else is first copied into pinned buffer i."""
        torch = self.torch
        if isinstance(batch, torch.Tensor) and batch.device.type == "cpu" and batch.is_pinned():
            src = batch if batch.dim() == 2 else batch.unsqueeze(0)
            if src.dtype != self.dtype or src.shape[1] != self.n or src.shape[0] > self.max_batch:
                raise ValueError(f"pinned batch must be {self.dtype} [<= {self.max_batch}, {self.n}]")
            nb = src.shape[0]
            if self.freed[i] is not None:
                self.freed[i].synchronize()
            with torch.cuda.stream(self.copy_stream):
                self.dbuf[i][:nb].copy_(src, non_blocking=True)
                up = torch.cuda.Event()
                up.record(self.copy_stream)
            self.uploaded[i] = up
            self.caller_upload = up  # the caller's buffer is read until this completes
            return nb
        b = np.asarray(batch)
        if b.ndim == 1:
            b = b[None, :]
        if b.shape[1] != self.n or b.shape[0] > self.max_batch:
            raise ValueError(f"batch must be [<= {self.max_batch}, {self.n}]")
        want = np.int16 if self.pcm16 else np.float32
        if b.dtype != want:
            raise TypeError(f"batch dtype must be {np.dtype(want).name}")
        nb = b.shape[0]
        if self.freed[i] is not None:
            self.freed[i].synchronize()          # the decode that last read dbuf[i] is done
        self.hbuf[i][:nb].numpy()[...] = b
        with torch.cuda.stream(self.copy_stream):
            self.dbuf[i][:nb].copy_(self.hbuf[i][:nb], non_blocking=True)
            up = torch.cuda.Event()
            up.record(self.copy_stream)
        self.uploaded[i] = up
        return nb

    def _launch(self, i: int, nb: int, k: int):
        """Decode buffer i (batch k) on decoder / stream k % depth, after its upload."""
        torch = self.torch
        st = self.computes[k % self.depth]
        dec = self.decs[k % self.depth]
        st.wait_event(self.uploaded[i])
        with torch.cuda.stream(st):
            out, cnt = dec.run(self.dbuf[i][:nb], code=self.code)
            ev = torch.cuda.Event()
            ev.record(st)
            self.freed[i] = ev
            cap = dec.cap * _lib.RESULT_DTYPE.itemsize
            self.hout[i][: nb * cap].copy_(out[: nb * cap], non_blocking=True)
            self.hcnt[i][:nb].copy_(cnt[:nb], non_blocking=True)
            r = torch.cuda.Event()
            r.record(st)
            self.ready[i] = r

    def _collect(self, i: int, nb: int) -> List[list]:
        self.ready[i].synchronize()
        cap = self.dec.cap
        recs = self.hout[i][: nb * cap * _lib.RESULT_DTYPE.itemsize].numpy().view(_lib.RESULT_DTYPE).reshape(nb, cap)
        raw = self.hcnt[i][:nb].numpy()
        warn_truncated(raw, cap, stacklevel=3)
        cnt = np.minimum(raw, cap)
        out = [[] for _ in range(nb)]
        # every decode of the batch converted in one call (slot-major, candidate order), then dealt
        sel = np.arange(cap)[None, :] < cnt[:, None]
        res = records_to_results(recs[sel], self.fs, self.bpt, False)
        pos = 0
        for s in np.flatnonzero(cnt > 0).tolist():
            c = int(cnt[s])
            out[s] = res[pos: pos + c]
            pos += c
        return out

    def decode_batches(self, batches: Iterable, borrow: bool = False) -> Iterator[List[list]]:
        """Yield per-slot results of each batch, in order.  depth + 2 batches are in flight on the
        device: when batch k's decode ends, batches k + 1 .. k + depth decode (on their own
        streams, overlapping) while batch k + depth + 1 uploads and batch k's results are converted.  A
        pinned caller tensor is uploaded in place, and its upload has completed before control
        returns to the caller (who may refill it).  borrow=True: a pinned caller tensor is instead
        lent to the decoder until its own batch's results are yielded (a caller cycling through at
        least depth + 3 pinned buffers, or never rewriting them, may pass it), so no upload is
        waited for on the host and the copy stream runs uploads back to back."""
        it = iter(batches)
        end = object()
        launched = []   # (buffer, n_slots), oldest first
        count = 0

        def start(batch):
            nonlocal count
            i = count % self.NBUF
            count += 1
            self.caller_upload = None
            nb = self._stage(i, batch)
            self._launch(i, nb, count - 1)
            launched.append((i, nb))
            return self.caller_upload

        for _ in range(self.NBUF - 1):      # prime the pipeline
            batch = next(it, end)
            if batch is end:
                break
            up = start(batch)
            if up is not None and not borrow:
                up.synchronize()
        while launched:
            i, nb = launched[0]
            # the next upload goes out before the oldest batch is waited for: its buffer's previous
            # batch was collected last iteration, so the copy stream never idles behind a decode
            batch = next(it, end)
            up = start(batch) if batch is not end else None
            self.ready[i].synchronize()     # the oldest batch's decode and result copy are done
            done = self._collect(i, nb)     # conversion overlaps the new upload
            launched.pop(0)
            if up is not None and not borrow:
                up.synchronize()
            yield done


def decode_wave_files(paths: List[str], batch: int = 256, device=None, depth=None, **decoder_kw) -> List[list]:
    """Decode many 16-bit PCM WAV files of one sample rate and length -> results per file.
    depth: StreamDecoder's; by default 2 when there are more than two batches (upload and decodes
    overlap), else 1 (no second context, fewer buffers)."""
    from .from_wave import _read_raw
    if not paths:
        return []
    first, dt, fs = _read_raw(paths[0])
    if dt != np.int16:
        raise TypeError("decode_wave_files expects 16-bit PCM")
    n = first.shape[0]

    def batches():
        for b0 in range(0, len(paths), batch):
            arr = np.empty((min(batch, len(paths) - b0), n), dtype=np.int16)
            for j, p in enumerate(paths[b0:b0 + arr.shape[0]]):
                d, dt2, fs2 = _read_raw(p)
                if dt2 != np.int16 or fs2 != fs or d.shape[0] != n:
                    raise ValueError(f"{p}: every file must be 16-bit PCM at {fs} Hz with {n} samples")
                arr[j] = d
            yield arr

    n_batches = -(-len(paths) // batch)
    if depth is None:
        depth = 2 if n_batches > 2 else 1
    sd = StreamDecoder(n, sample_rate=fs, max_batch=min(batch, len(paths)), pcm16=True, device=device,
                       depth=depth, **decoder_kw)
    out: List[list] = []
    for res in sd.decode_batches(batches()):
        out.extend(res)
    return out
