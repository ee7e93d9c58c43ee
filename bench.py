"""Benchmark: 15-s FT8 slots/s (full decode) on MI355X, BASELINE.json config 3 per GPU.

One step = one ft8_decode_batch over a batch of 256 independent synthetic 15-s slots at 12 kHz
(50 GFSK signals per slot at SNR U(-24, -10) dB, full-band convention; K=300, min_score=2,
20 BP iterations): STFT -> Costas sync -> selection -> LLR -> BP -> CRC, samples already
resident in HBM.  With N > 1 GPUs each rank decodes its own 256 slots (weak scaling) and the
step ends with an RCCL all-gather of every rank's decodes, packed on the device (the path's one
exchange; no host sync inside the step).  Consecutive steps alternate over --depth (default 2)
decoders, each with its own context and stream, so one step's front end overlaps the previous
step's k_bp tail; every step decodes the whole batch (`depth.one_chain`: the same steps as one chain).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--slots S] [--no-cpu] [--gather]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N ranks
itself (a torch.distributed.run child, before this process touches the GPU) and exits with its
code; it exits non-zero when fewer than N GPUs are visible or when WORLD_SIZE disagrees with --gpus.
Rank r decodes global slots [256 r, 256 (r + 1)) (per-slot seeds 100000 + slot), so the N = 1 batch
is the first shard of every larger run.

Prints ONE JSON line on rank 0.  Besides the contract fields it carries:
  depth         contexts / streams the timed steps alternate over; one_chain: the same K steps on one
                context and one stream, timed after the loop (N=1)
  settle        untimed steps run before the W warmup steps until consecutive blocks' GPU times agree
                within 1.5 % (k_bp's clock ramp), their block times; --settle_max 0 turns it off
  roofline      the dominant kernel (k_bp: LLR + float64 BP + CRC), FLOP-rate vs the FP64 vector peak
  roofline_hbm  the HBM-bound STFT kernel, GB/s vs the 8 TB/s HBM peak
  stages_ms     per-kernel device time per step (HIP events on the decode stream)
  bp_stress     BASELINE config 4 first pass: 100k LLR vectors x 50 BP iterations, candidates/s (N=1)
  subtract_redecode  BASELINE config 4 with the subtract-and-redecode second pass: 334 crowded
                slots x K=300 (top-k), 50 iterations, both passes, candidates/s (N=1)
  geometries    the reference's other geometries (20 kHz, the bundled recording's rate; 12 kHz at
                bins_per_tone = steps_per_symbol = 10, its decode test's): slots/s, stage times, the
                generic STFT / score kernels' HBM rooflines (N=1)
  drift_correct the beacon receiver's frequency-drift correction on a batch of 256
                complex128 beacon signals (12 kHz, 3 x 12.64 s, steps_per_symbol 8): signals/s, the
                dominant kernel's roofline and the oracle port's CPU rate (N=1)
  h2d_stream    the same slots as int16 PCM in pinned host memory, upload overlapped with decode (N=1)
  cpu_baseline  the oracle port (oracle/, C + scipy) on the first slots of rank 0's own batch -- the
                same bytes the GPU decodes (rank 0, N=1)
  parity        those slots' GPU decodes vs the oracle's: payload + CRC multisets, ordered lists
  gather        (N > 1 or --gather) the last timed step's decode exchange: backend, rows and bytes per rank
  gather_n1     (N = 1) steps with vs without the N > 1 exchange (device pack + RCCL all-gather over a
                world-size-1 group), interleaved blocks: its cost per step
  sensitivity   the reference's own sensitivity harness (test_ft8_standard.py:43-123, the source of its
                only published number) on the GPU: per sample rate the minimum
                full-band SNR for >= 50 % decodes, next to the xlsx table, with an oracle-checked sample (N=1)
  reference_measured  the reference's own single-thread figure, for context
"""
import argparse
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "15-s FT8 slots/sec (full decode) + LDPC candidates/sec, 1/2/4/8 MI355X"
FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (AMD spec; k_bp issues no MFMA)
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X FP32 vector
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec


def bp_flops_per_pass():
    """Algorithmic float64 FLOPs of one message-passing sweep of bp_decode (ldpc_decoder.py:88-108):
    per edge V->C: 2 adds + 1 scale + fast_tanh (x^2, 4 num, 4 den, 1 div) = 13;
    per edge C->V: (deg-1) products + fast_atanh (10) + 1 scale; plus the per-iteration hard
    decision (3 adds per bit, counted separately)."""
    from ft8_demodulator_amd import _ldpc_tables as T
    f = 0
    for m in range(83):
        d = T.CHK_START[m + 1] - T.CHK_START[m]
        f += d * 13 + d * ((d - 1) + 10 + 1)
    return f


def host_cores():
    """Worker processes for the CPU legs: the host cores this process may use -- sched_getaffinity,
    bounded by the cgroup CPU quota and by OMP_NUM_THREADS when set (the GPU box sets it to this
    job's CPU share; affinity there lists the whole machine).  -> (cores, basis string)."""
    aff = len(os.sched_getaffinity(0))
    n, basis = aff, [f"sched_getaffinity={aff}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
            n = min(n, max(1, int(quota)))
            basis.append(f"cgroup cpu.max={quota:g}")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        basis.append(f"OMP_NUM_THREADS={omp}")
    return max(1, n), "min(" + ", ".join(basis) + ")"


def _worker_init():
    import torch
    torch.set_num_threads(1)


def cpu_synth_worker(args):
    """One slot of the benchmark workload synthesised on the CPU (synth.make_slots, per-slot seed)."""
    from ft8_demodulator_amd import synth
    seed, signals = args
    x, _ = synth.make_slots(1, signals, fs=12000, snr_db=(-24.0, -10.0), seeds=[seed], device="cpu")
    return x[0].numpy()


def cpu_worker(args):
    from oracle import oracle as O
    x, kw = args
    return [(bytes(r[0]).hex(), int(r[1]), float(r[5]), float(r[6]), float(r[7]))
            for r in O.decode_ft8_message(x, 12000, **kw)]


def cpu_baseline(kw, n_slots, procs, basis, seed0, signals):
    """Oracle port (oracle/, C + scipy) on the first n_slots slots of rank 0's batch, `procs` worker
    processes.  The slots are synthesised here on the CPU and then uploaded as the first n_slots
    rows of the GPU batch, so the CPU and the GPU decode the SAME bytes (the decodes are compared
    in the `parity` object).  Runs before this process touches the GPU, so the forked workers
    inherit no device state.  -> (baseline dict, [n_slots, N] float32 samples, per-slot decodes)."""
    import multiprocessing as mp
    import numpy as np
    from oracle import oracle as O
    O.lib()
    ctx = mp.get_context("fork")
    with ctx.Pool(procs, initializer=_worker_init) as pool:
        t0 = time.perf_counter()
        xs = pool.map(cpu_synth_worker, [(seed0 + b, signals) for b in range(n_slots)], chunksize=1)
        t_syn = time.perf_counter() - t0
        pool.map(cpu_worker, [(xs[0], kw)] * procs)  # warm the workers (imports, scipy plans)
        t0 = time.perf_counter()
        decodes = pool.map(cpu_worker, [(x, kw) for x in xs], chunksize=1)
        dt = time.perf_counter() - t0
    base = {"value": n_slots / dt, "unit": "slots/s", "cores": procs, "cores_basis": basis, "kind": "port",
            "sample": f"the first {n_slots} slots of rank 0's GPU batch (the same float32 bytes; K=300, min_score=2, "
                      f"20 iters); oracle/ft8_oracle.c + scipy STFT, {procs} processes, {dt:.2f} s wall",
            "wall_s": dt, "synth_wall_s": t_syn}
    return base, np.stack(xs), decodes


def parity_check(gpu_recs, cpu_decodes, bpt=2):
    """GPU records (SlotDecoder.records) vs the oracle's decodes of the same slots: payload + CRC
    multisets per slot (the contract), ordered (payload, crc, time, freq) lists, score deltas."""
    mism, ordered, dmax, ng, nc = [], 0, 0.0, 0, 0
    for s, (g, c) in enumerate(zip(gpu_recs, cpu_decodes)):
        gl = [(bytes(r["payload"]).hex(), int(r["crc_calculated"]), int(r["abs_time"]) / 12000,
               (int(r["abs_freq"]) / bpt) * 6.25, float(r["score"])) for r in g]
        ng, nc = ng + len(gl), nc + len(c)
        if sorted(x[:2] for x in gl) != sorted(x[:2] for x in c):
            mism.append(s)
        if [x[:4] for x in gl] == [x[:4] for x in c]:
            ordered += 1
            for a, b in zip(gl, c):
                dmax = max(dmax, abs(a[4] - b[4]))
    return {"slots": len(cpu_decodes), "decodes_gpu": ng, "decodes_cpu": nc,
            "payload_crc_multiset_equal": not mism, "mismatching_slots": mism,
            "ordered_lists_equal_slots": ordered, "max_abs_score_diff": dmax,
            "note": "CPU = oracle port with scipy's pocketfft STFT; GPU = this build's STFT (dB within "
                    "1e-3 on strong bins, SURVEY 8(a)): a candidate whose score lies within that error of "
                    "min_score or of a selection boundary can enter or leave the list; "
                    "tests/test_gpu_bench_parity.py checks every slot of this batch stage by stage"}


def gather_check(flat, counts, totals, S, world, decoded, cap):
    """The resolved all-gather of one step (N > 1) against the decode count all ranks reported:
    rank r's records are its totals[r] rows, their slot ids lie in [r S, (r + 1) S) in nondecreasing
    order, each global slot appears exactly counts[r][slot] times (capped counts), and the totals
    add up to the all-reduced decode count.  flat: structured ft8_result array, rank-major."""
    import numpy as np
    tot = [int(t) for t in totals]
    cnt = np.minimum(np.asarray(counts)[:, :S].astype(np.int64), cap)
    slots = np.asarray(flat["slot"], dtype=np.int64)
    per_slot = np.bincount(slots, minlength=world * S) if len(slots) else np.zeros(world * S, np.int64)
    ok_range = bool(len(slots) == 0 or (slots.min() >= 0 and slots.max() < world * S))
    ok_order = bool(np.all(np.diff(slots) >= 0)) if len(slots) else True
    ok_counts = ok_range and per_slot.shape[0] == world * S and bool(np.array_equal(per_slot, cnt.reshape(-1)))
    ok_rank = True
    off = 0
    for r in range(world):
        seg = slots[off:off + tot[r]]
        ok_rank &= bool(len(seg) == 0 or (seg.min() >= r * S and seg.max() < (r + 1) * S))
        off += tot[r]
    ok_total = sum(tot) == int(decoded) == len(slots) == int(cnt.sum())
    return {"gather_ok": bool(ok_range and ok_order and ok_counts and ok_rank and ok_total),
            "records": len(slots), "sum_totals": sum(tot), "decodes_all_reduced": int(decoded),
            "slot_ids_in_range": ok_range, "slot_order": ok_order, "per_slot_counts_match": bool(ok_counts),
            "rank_ranges": bool(ok_rank)}


def shard_sample(flat, lo, m):
    """The gathered records of global slots [lo, lo + m) -> per-slot lists (as SlotDecoder.records)."""
    sl = flat["slot"]
    return [flat[sl == lo + i] for i in range(m)]


def bp_parity(llr, x, plain, res, iters, n_sample):
    """bp_stress's launch vs the oracle (oracle/ft8_oracle.c, pinned to the reference's bp_decode)
    on n_sample evenly spaced vectors: normalised LLRs, hard decisions and min_errors bit-exact,
    CRC status and payload of every vector equal to the oracle's decode tail."""
    import numpy as np
    from ft8_demodulator_amd import _lib
    from oracle import oracle as O
    n = llr.shape[0]
    idx = np.unique(np.linspace(0, n - 1, min(n_sample, n)).astype(np.int64))
    xs = x[idx].cpu().numpy()
    ps = plain[idx].cpu().numpy()
    rec = res.view(-1, _lib.RESULT_DTYPE.itemsize)[idx].cpu().numpy().reshape(-1).view(_lib.RESULT_DTYPE)
    t0 = time.perf_counter()
    bad_norm, bad_bp, bad_tail = [], [], []
    for j, i in enumerate(idx):
        xr = O.normalize(llr[i])
        if not np.array_equal(xs[j].view(np.uint64), xr.view(np.uint64)):
            bad_norm.append(int(i))
        pr, er = O.bp_decode(xr, iters)
        if er != int(rec[j]["ldpc_errors"]) or not np.array_equal(pr, ps[j]):
            bad_bp.append(int(i))
        ok, pay, _ce, cc = O.decode_tail(pr, er)
        if bool(rec[j]["ok"]) != ok or int(rec[j]["crc_calculated"]) != cc or (ok and bytes(rec[j]["payload"]) != pay):
            bad_tail.append(int(i))
    return {"vectors": int(len(idx)), "sample": f"every {n // max(len(idx), 1)}th of the {n} launch vectors",
            "normalize_bit_exact": not bad_norm, "bp_bit_exact": not bad_bp, "crc_payload_equal": not bad_tail,
            "mismatches": {"normalize": bad_norm[:10], "bp": bad_bp[:10], "tail": bad_tail[:10]},
            "oracle_s": time.perf_counter() - t0, "oracle": "oracle/ft8_oracle.c (bp_decode, ldpc_decoder.py:54-113)"}


def _oracle_bp_chunk(args):
    from oracle import oracle as O
    xs, iters = args
    for v in xs:
        O.bp_decode(v, iters)
    return len(xs)


def bp_cpu_baseline(xn, iters, procs, n_total):
    """The oracle's bp_decode (oracle/ft8_oracle.c, pinned to ldpc_decoder.py:54-113) on the given
    normalised LLR vectors, `procs` threads (ctypes releases the GIL), extrapolated to the GPU
    launch's n_total vectors ("time 1 000 candidates and extrapolate")."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    O.lib()
    n = xn.shape[0]
    chunks = [(xn[i::procs], iters) for i in range(procs)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(procs) as ex:
        done = sum(ex.map(_oracle_bp_chunk, chunks))
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "candidates/s", "cores": procs, "kind": "port",
            "sample": f"{done} of the launch's normalised LLR vectors x {iters} BP iterations through "
                      f"oracle/ft8_oracle.c bp_decode on {procs} threads, {dt:.2f} s wall",
            "extrapolated_s_per_launch": n_total / (done / dt),
            "extrapolation": f"linear in vectors: {n_total} vectors / the sample's rate"}


def bp_stress(ctx, dev, n=100000, iters=50, reps=3, sigma=0.85, n_sample=2000, procs=1, n_cpu=2000):
    """BASELINE config 4 (first pass): n LLR vectors from codewords of random payloads,
    (2b-1) + sigma N(0,1), ftx_normalize_logl on the device, then ft8_bp with `iters` iterations.
    Returns candidates/s and the k_bp roofline for this launch shape."""
    import torch
    from ft8_demodulator_amd import _lib, synth
    llr, _ = synth.bp_stress_llrs(n, sigma=sigma)
    a = torch.from_numpy(llr).to(dev)
    x = torch.empty_like(a)
    res = torch.zeros(n * _lib.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    L, st = _lib.lib(), _lib.stream_handle()
    ctx.check(L.ft8_normalize(ctx.handle, _lib.ptr(a), n, _lib.ptr(x), st), "ft8_normalize")

    def run():
        ctx.check(L.ft8_bp(ctx.handle, _lib.ptr(x), n, iters, None, _lib.ptr(res), st), "ft8_bp")

    ctx.set_timing(True)   # allocates the BP work counters (events are not used below)
    ctx.set_timing(False)
    run()
    torch.cuda.synchronize()
    ctx.counters(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cn = ctx.counters(reset=True)
    bp_ms = dt / reps * 1e3  # one k_bp launch (+ its 4-byte counter reset) per call, back to back
    flops = (cn["passes"] * bp_flops_per_pass() + cn["iterations"] * 174 * 3) / reps
    tf = flops / (bp_ms * 1e-3) / 1e12
    # parity of this very launch shape, after the timing: the same call once more with the hard
    # decisions written out, and an evenly spaced sample checked against the oracle
    plain = torch.empty((n, 174), dtype=torch.uint8, device=dev)
    ctx.check(L.ft8_bp(ctx.handle, _lib.ptr(x), n, iters, _lib.ptr(plain), _lib.ptr(res), st), "ft8_bp")
    torch.cuda.synchronize()
    parity = bp_parity(llr, x, plain, res, iters, n_sample)
    cpu = bp_cpu_baseline(x[:n_cpu].cpu().numpy(), iters, procs, n) if n_cpu > 0 else None
    return {"workload": f"BASELINE config 4 first pass: {n} LLR vectors (codewords of random payloads, "
                        f"(2b-1)+{sigma}*N(0,1), normalised), {iters} BP iterations",
            "candidates_per_s": n * reps / dt, "ms_per_launch": bp_ms, "timing": "wall clock over back-to-back launches",
            "converged_frac": cn["converged"] / max(cn["candidates"], 1),
            "sweeps_per_launch": cn["passes"] / reps,
            "roofline": {"kernel": "k_bp", "bound": "fp64-valu", "achieved": tf, "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": tf / FP64_VECTOR_PEAK_TFLOPS},
            "parity": parity, "cpu_baseline": cpu}


SUB_SEED0 = 200000


def subtract_oracle_worker(args):
    """One slot of the subtract leg through oracle/subtract.py (CPU, float64 NumPy restatement of
    FT8_FLAG_SUBTRACT): the slot synthesised on the CPU, top-k pass 1, a fit per decode (record order
    = the selection's order), the residual, top-k pass 2 -> (samples, pass-1 payloads, new payloads)."""
    import numpy as np
    from ft8_demodulator_amd import synth
    from oracle import subtract as OS
    from ft8_demodulator_amd._pipeline import make_plan
    seed, signals, iters = args
    x, _ = synth.make_slots(1, signals, fs=12000, snr_db=(-24.0, -10.0), seeds=[seed], device="cpu")
    xs = x[0].numpy()
    t0 = time.perf_counter()
    plan = make_plan(xs.shape[0], 12000)
    d1 = OS.decode_topk(xs, 12000, 300, 2, iters)
    recs = np.zeros(len(d1), dtype=[("payload", "u1", 10), ("ok", "u1"), ("abs_time", "<i4"), ("abs_freq", "<i4")])
    for i, (pay, at, af) in enumerate(d1):
        recs[i] = (np.frombuffer(pay, np.uint8), 1, at, af)
    ofit = OS.fits(xs, recs, 12000, plan.nperseg, plan.hop, plan.nfft, plan.t_lo, plan.f_lo)
    res = OS.residual(xs, ofit, plan.nperseg, 12000).astype(np.float32)
    p1 = {pay for pay, _, _ in d1}
    new = {pay for pay, _, _ in OS.decode_topk(res, 12000, 300, 2, iters)} - p1
    t_dec = time.perf_counter() - t0
    from oracle import oracle as O
    n_pass = int((O.score_grid(O.waterfall(xs, 12000, 2, 2), 2, 2) >= 2).sum())  # k_topkc's input size
    return xs, sorted(p.hex() for p in p1), sorted(p.hex() for p in new), sum(f is not None for f in ofit), n_pass, t_dec


def subtract_oracle(n, procs, signals=50, iters=50):
    """The first n slots of the subtract leg through oracle/subtract.py, `procs` processes, before
    the GPU is touched -> (samples [n, N] float32, per-slot (pass-1, new) payload hex lists, info)."""
    import multiprocessing as mp
    import numpy as np
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    cores = min(procs, n)
    with ctx.Pool(cores, initializer=_worker_init) as pool:
        out = pool.map(subtract_oracle_worker, [(SUB_SEED0 + b, signals, iters) for b in range(n)], chunksize=1)
    t_dec = sum(o[5] for o in out)
    return (np.stack([o[0] for o in out]), [(o[1], o[2]) for o in out],
            {"fits": sum(o[3] for o in out), "oracle_wall_s": time.perf_counter() - t0,
             "passing_scores_per_slot": float(np.mean([o[4] for o in out])),
             "cpu_baseline": {"value": n / t_dec * cores, "unit": "slots/s", "cores": cores, "kind": "port",
                              "sample": f"{n} slots of this leg through oracle/subtract.py (both passes: top-k decode, "
                                        f"fits, residual, top-k decode; {iters} BP iterations), one slot per process, "
                                        f"{t_dec / n:.2f} s per slot (decode only, synthesis excluded)",
                              "candidates_per_s": 2 * 300 * n / t_dec * cores}})


def subtract_redecode(dev, n_slots=334, signals=50, iters=50, reps=3, oracle_sample=None):
    """BASELINE config 4 with the subtract-and-redecode second pass (build-defined):
    334 crowded slots x K=300 candidates = 100 200 LDPC candidates per pass, 50 BP iterations,
    top-k candidate selection (FT8_FLAG_TOPK) and FT8_FLAG_SUBTRACT: pass 1, fit + subtract every
    decoded message, pass 2 on the residual.  candidates/s counts the BP candidates of both passes."""
    import numpy as np
    import torch
    from ft8_demodulator_amd import _lib, synth
    from ft8_demodulator_amd._pipeline import SlotDecoder
    x, truths = synth.make_slots(n_slots, signals, fs=12000, snr_db=(-24.0, -10.0), seed=SUB_SEED0, device=dev)
    n_or = 0
    if oracle_sample is not None:
        # the oracle's slots were synthesised on the CPU: decode those very bytes
        n_or = oracle_sample[0].shape[0]
        x[:n_or] = torch.from_numpy(oracle_sample[0]).to(dev)
    dec = SlotDecoder(12000, 2, 2, max_candidates=300, min_score=2, max_iterations=iters, device=dev,
                      flags=_lib.FT8_FLAG_TOPK | _lib.FT8_FLAG_SUBTRACT)
    recs = dec.records(x, _lib.FT8_F32)
    true1 = true2 = false = 0
    for s in range(n_slots):
        tr = set(bytes(p) for p in truths[s].payloads)
        g1 = set(bytes(r["payload"]) for r in recs[s] if r["pass_index"] == 0)
        g2 = set(bytes(r["payload"]) for r in recs[s] if r["pass_index"] == 1)
        true1, true2, false = true1 + len(g1 & tr), true2 + len(g2 & tr), false + len((g1 | g2) - tr)
    parity = None
    if n_or:
        mism1, mism2, n1, n2 = [], [], 0, 0
        for s_ in range(n_or):
            # payload SETS: a message decoded at two candidates appears twice in the records
            g1 = sorted({bytes(r["payload"]).hex() for r in recs[s_] if r["pass_index"] == 0})
            g2 = sorted({bytes(r["payload"]).hex() for r in recs[s_] if r["pass_index"] == 1})
            o1, o2 = oracle_sample[1][s_]
            n1, n2 = n1 + len(o1), n2 + len(o2)
            if g1 != o1:
                mism1.append(s_)
            if g2 != o2:
                mism2.append(s_)
        parity = {"slots": n_or, "oracle_pass1_decodes": n1, "oracle_pass2_new_decodes": n2,
                  "oracle_fits": oracle_sample[2]["fits"], "oracle_wall_s": oracle_sample[2]["oracle_wall_s"],
                  "pass1_payloads_equal": not mism1, "pass2_new_payloads_equal": not mism2,
                  "mismatching_slots_pass1": mism1, "mismatching_slots_pass2": mism2,
                  "oracle": "oracle/subtract.py (CPU float64 restatement of the build-defined second pass; the "
                            "reference has no second pass, so pass 2 is pinned to the restatement, not the reference)",
                  "from": "the first slots of this leg's batch, synthesised on the CPU and uploaded (same bytes)"}
    cpu = oracle_sample[2].get("cpu_baseline") if oracle_sample is not None else None
    ctx = dec.ctx
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.timing(reset=True)
    ctx.counters(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        dec.run(x, _lib.FT8_F32)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    tm = ctx.timing(reset=True)
    cn = ctx.counters(reset=True)
    n_samp = int(x.shape[1])
    del x
    # rooflines of the second-pass kernels (algorithmic work per unit).  Fits:
    # one per distinct pass-1 payload of a slot (k_sub_est skips failed records and repeats)
    fits = sum(len({bytes(r["payload"]) for r in recs[s_] if r["pass_index"] == 0}) for s_ in range(n_slots))
    nsps, Q, hop = 1920, 32, 960
    D = nsps // Q
    Mt = -(-(hop // 2) // D)
    nT, nF, Mz = 2 * Mt + 1, 5, 79 * Q + 2 * (Mt + 1)
    est_flops = Mz * D * 10 + nF * 79 * (Q * 14 + (nT - 1) * 19 + nT * 3) + 79 * nsps * 16
    app_flops = 79 * nsps * 28
    FP32_PEAK = FP32_VECTOR_PEAK_TFLOPS

    def ms_of(k_):
        v = tm.get(k_, (0.0, 0))
        return v[0] / max(v[1], 1)
    est_ms, app_ms, sel_ms = ms_of("sub_est"), ms_of("sub_apply"), ms_of("select")
    rl = {}
    if est_ms > 0:
        a_ = fits * est_flops / (est_ms * 1e-3) / 1e12
        rl["k_sub_est"] = {"bound": "fp32-valu", "achieved": a_, "peak": FP32_PEAK, "unit": "TFLOP/s",
                           "frac": a_ / FP32_PEAK, "flops_per_fit": est_flops, "fits_per_launch": fits,
                           "launch_ms": est_ms}
    if app_ms > 0:
        a_ = fits * app_flops / (app_ms * 1e-3) / 1e12
        hbm_b = n_slots * n_samp * 8  # samples read + residual written once
        rl["k_sub_apply"] = {"bound": "fp32-valu", "achieved": a_, "peak": FP32_PEAK, "unit": "TFLOP/s",
                             "frac": a_ / FP32_PEAK, "flops_per_fit": app_flops, "fits_per_launch": fits,
                             "launch_ms": app_ms, "hbm_bytes_per_launch": hbm_b,
                             "hbm_frac": hbm_b / (app_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    if sel_ms > 0 and oracle_sample is not None:
        nseg = 88 * 15
        npass = oracle_sample[2]["passing_scores_per_slot"]
        b_ = n_slots * (nseg * 16 + npass * 4 + 300 * 16)
        rl["k_topkc"] = {"bound": "hbm", "achieved": b_ / (sel_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": b_ / (sel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_per_launch": b_,
                         "launch_ms": sel_ms,
                         "bytes": "per slot: 1320 segment masks x 16 B + passing scores x 4 B (mean of the oracle "
                                  "sample's slots) + 300 candidates x 16 B written"}
    return {"workload": f"BASELINE config 4 with subtract-and-redecode: {n_slots} crowded slots x K=300 "
                        f"(top-k selection) = {n_slots * 300} candidates per pass, {iters} BP iterations, "
                        "pass 1 -> fit and subtract every decoded message -> pass 2 on the residual",
            "candidates_per_s": cn["candidates"] / dt, "bp_candidates_per_launch": cn["candidates"] / reps,
            "slots_per_s": n_slots * reps / dt, "ms_per_launch": dt / reps * 1e3,
            "true_decodes_per_slot_pass1": true1 / n_slots, "true_decodes_per_slot_pass2": true2 / n_slots,
            "false_decodes": int(false),
            "parity": parity,
            "cpu_baseline": cpu,
            "rooflines": rl,
            "stages_ms": {k: v[0] / reps for k, v in tm.items() if v[1] > 0},
            "data": "synthetic (ft8_demodulator_amd.synth, seeds 200000..); the reference has no second pass: "
                    "pass 2 is pinned against the CPU restatement oracle/subtract.py "
                    "(tests/test_gpu_subtract_oracle.py)"}


# the reference's own geometries besides the 12 kHz production one: the bundled recording's 20 kHz
# (from_wave.py:24-69, src/ft8_tools/ft8_beacon_receiver/data/raw/ft8_fs20k_f0_550_id_1.wav) and its
# decode test's 12 kHz at bins_per_tone = steps_per_symbol = 10 (test_spectrogram_analyse.py:128-163)
GEOMETRIES = (("fs20k_bpt2", 20000, 2, 2, 256), ("fs12k_bpt10", 12000, 10, 10, 32))


def geometry_legs(dev, reps=5):
    """Decode throughput at the reference's other geometries (K=300, min_score=2, 20 iterations),
    with the per-stage event times and the HBM rooflines of the generic STFT and score kernels they
    run.  Parity at these geometries is the test suite's (tests/test_gpu_reftests.py: the
    reference's own outputs)."""
    import torch
    from ft8_demodulator_amd import SlotDecoder, synth, _lib
    out = {}
    for name, fs, bpt, sps, n in GEOMETRIES:
        x, _ = synth.make_slots(n, 50, fs=fs, snr_db=(-24.0, -10.0), seed=300000, device=dev)
        dec = SlotDecoder(fs, bpt, sps, 300, 2, 20, device=dev)
        ctx = dec.ctx
        ctx.set_timing(True)
        ctx.set_timing(False)
        for _ in range(3):
            _, counts = dec.run(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            _, counts = dec.run(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        decodes = int(counts.sum())
        stages = {}
        for st in ("stft", "score", "select", "llr", "bp"):
            ctx.timing(reset=True)
            ctx.set_timing(True, stages=[st])
            for _ in range(3):
                dec.run(x)
            torch.cuda.synchronize()
            ctx.set_timing(False)
            v = ctx.timing(reset=True)[st]
            stages[st] = v[0] / max(v[1], 1)
        ctx.set_timing(False, stages=None)
        N = int(x.shape[1])
        pl = dec.plan(N)
        method = _lib.lib().ft8_stft_method(ctx.handle, fs, bpt, sps, N, _lib.FT8_F32)
        wf_bytes = n * pl.T * pl.F * 4
        stft_b = n * N * 4 + wf_bytes
        out[name] = {
            "workload": f"{n} synthetic 15-s slots at {fs} Hz, bins_per_tone {bpt}, steps_per_symbol {sps} "
                        f"(nfft {pl.nfft}, hop {pl.hop}: {pl.T} frames x {pl.F} bins), 50 signals/slot, "
                        "K=300, min_score=2, 20 iterations",
            "slots_per_s": n / dt, "ms_per_batch": dt * 1e3, "decodes_per_batch": decodes,
            "stft_method": {0: "stockham", 1: "packed3840", 2: "chirp-z", 3: "direct DFT"}.get(method, method),
            "score_kernel": "k_score2" if bpt == sps and (bpt <= 4 or bpt == 10) else "k_score",
            "stages_ms": stages,
            "roofline_stft": {"kernel": {"fs20k_bpt2": "k_stft_pk<3200: 16 8 5 5>",
                                         "fs12k_bpt10": "k_stft_pk<9600: 16 8 15 5>"}.get(name, "k_stft"),
                              "bound": "hbm", "bytes_per_launch": stft_b, "launch_ms": stages["stft"],
                              "achieved": stft_b / (stages["stft"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": stft_b / (stages["stft"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                              "bytes": "samples read once (4 B) + dB waterfall written once (4 B per kept bin)"},
            "roofline_score": {"bound": "hbm", "bytes_per_launch": wf_bytes, "launch_ms": stages["score"],
                               "achieved": wf_bytes / (stages["score"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": wf_bytes / (stages["score"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                               "bytes": "the waterfall read once (score writes not counted)"},
            "data": "synthetic (ft8_demodulator_amd.synth, seeds 300000..)"}
        del x, dec
        torch.cuda.empty_cache()
    return out


DRIFT_PARAMS = {"bins_per_tone": 2, "steps_per_symbol": 8}  # the reference test's correction params


def drift_worker(args):
    from oracle import drift as OD
    hexp, f0, fc, drift, seed = args
    x = OD.beacon_input(hexp, 12000, f0, fc, drift, 28.0, seed)
    t0 = time.perf_counter()
    OD.correct_frequency_drift(x, 12000, 6.25, 0.16, params=dict(DRIFT_PARAMS))
    return time.perf_counter() - t0


def drift_signal_params(n, seed=4242):
    import numpy as np
    rng = np.random.default_rng(seed)
    return [(bytes(rng.integers(0, 256, 10, dtype=np.uint8)).hex(), float(rng.uniform(200, 500)),
             float(rng.uniform(300, 700)), float(rng.uniform(50, 150)), int(seed + i)) for i in range(n)]


def drift_cpu_baseline(procs, n=32):
    """oracle/drift.py (NumPy/SciPy restatement of correct_frequency_drift) on n signals of the
    drift workload, `procs` processes; each worker times only the correction (not the synthesis)."""
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    work = drift_signal_params(n)
    with ctx.Pool(procs) as pool:
        pool.map(drift_worker, work[:procs])  # warm imports / FFT plans
        t0 = time.perf_counter()
        per = pool.map(drift_worker, work, chunksize=1)
        dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "signals/s", "cores": procs, "kind": "port",
            "sample": f"{n} beacon signals of the drift workload, oracle/drift.py (NumPy + scipy "
                      f"spectrogram), {procs} processes, {dt:.2f} s wall, {sum(per) / n:.2f} s per signal",
            "wall_s": dt}


def drift_32k(dev, n_sig=16, reps=3):
    """The reference drift test's own rate (test_correction.py:93): 32 768 Hz complex128 beacons,
    nfft 10 485 = 3^2 5 233 -- an FFT length the Stockham plans cannot take, so both STFT-argmax
    passes run the chirp-z transform (ft8_stft_method).  Per-signal time of ft8_drift_correct."""
    import ctypes
    import numpy as np
    import torch
    from ft8_demodulator_amd import _lib, ft8_generator as G
    from ft8_demodulator_amd.frequency_correction import _drift_params, DEFAULT_PARAMS
    fs = 32768
    nsps = int(0.16 * fs)
    L = 79 * nsps
    n = 3 * L
    prm = drift_signal_params(n_sig, seed=32768)
    pays = np.frombuffer(b"".join(bytes.fromhex(p[0]) for p in prm), dtype=np.uint8).reshape(-1, 10)
    _, _, tones = G.encode_batch(pays, device=dev)
    sig = np.array([(p[1] + p[2], 1.0, 0.0, L, i, 0) for i, p in enumerate(prm)], dtype=_lib.TX_SIGNAL_DTYPE)
    x = G.synthesize(tones, sig, n_sig, n, fs, _lib.FT8_TX_REFERENCE, dtype=torch.complex128, device=dev)
    t = torch.arange(n, device=dev, dtype=torch.float64)
    k = torch.tensor([p[3] for p in prm], device=dev, dtype=torch.float64)[:, None] / fs
    x *= torch.polar(torch.ones((), device=dev, dtype=torch.float64), 2 * np.pi * k * t * t / (2 * fs))
    g = torch.Generator(device=dev)
    g.manual_seed(8)
    sd = torch.sqrt((x.abs() ** 2).mean(dim=1, keepdim=True) / 10 ** 2.8 * fs / 2)
    x += torch.complex(torch.randn(x.shape, generator=g, device=dev, dtype=torch.float64),
                       torch.randn(x.shape, generator=g, device=dev, dtype=torch.float64)) * sd
    del t
    ctx = _lib.context(dev)
    out = torch.empty_like(x)
    res = torch.zeros(n_sig * _lib.DRIFT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    p = _drift_params(dict(DEFAULT_PARAMS, **DRIFT_PARAMS), fs, 6.25, 0.16)
    st = _lib.stream_handle(dev)
    method = _lib.lib().ft8_stft_method(ctx.handle, fs, DRIFT_PARAMS["bins_per_tone"], DRIFT_PARAMS["steps_per_symbol"],
                                        n, _lib.FT8_C128)

    def run():
        ctx.check(_lib.lib().ft8_drift_correct(ctx.handle, _lib.ptr(x), _lib.FT8_C128, n, n_sig, n, ctypes.byref(p),
                                               _lib.ptr(out), _lib.ptr(res), st), "ft8_drift_correct")

    run()
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(_lib.DRIFT_RESULT_DTYPE)
    ok = r["status"] == _lib.FT8_DRIFT_FULL
    est = np.asarray(r["rate_per_sample"]) * fs
    true = np.array([p_[3] for p_ in prm])
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    del x, out
    return {"workload": f"correct_frequency_drift on {n_sig} complex128 beacons at 32768 Hz x {n} samples "
                        "(the reference drift test's rate: nfft 10485 = 3^2 5 233)",
            "stft_method": {0: "stockham", 1: "packed3840", 2: "chirp-z", 3: "direct DFT"}.get(method, method),
            "ms_per_signal": dt / n_sig * 1e3, "signals_per_s": n_sig / dt, "full_fits": int(ok.sum()),
            "median_abs_rate_err_hz_per_s": float(np.median(np.abs(est[ok] - true[ok]))) if ok.any() else None}


# the reference's only published result, the minimum SNR (full band, B = fs/2)
# for >= 50 % decodes, snr_vs_freq_analysis.xlsx sheet1 rows 3-14, keyed by sample rate fs = 2 B
XLSX_MIN_SNR_DB = {2000: -9, 3000: -11, 4000: -12, 5000: -13, 6000: -13, 7000: -14, 8000: -14, 9000: -16,
                   10000: -16, 11000: -17, 12000: -17, 13000: -17}
SENSITIVITY_RATES = sorted(set(range(2000, 10001, 500)) | {11000, 12000, 13000})


def _oracle_decode_payloads(args):
    from oracle import oracle as O
    x, fs = args
    return [bytes(r[0]).hex() for r in O.decode_ft8_message(x, fs, 2, 2, 20, 1, 20)]


def sensitivity(dev, rates=None, snr_lo=-24.0, snr_hi=-5.0, step=0.2, rounds=20, seed=31337, chunk=2048,
                oracle_per_rate=2, procs=1):
    """The reference's sensitivity harness on the GPU (test_ft8_standard.py:43-123): at each sample
    rate, for SNR from snr_lo to snr_hi in `step` dB, `rounds` independent test_step's -- a random
    payload (np.random.randint(0, 256, 10)) -> the reference-timing GFSK waveform with f0 = fc = 0
    (ft8_synthesize, FT8_TX_REFERENCE: modulator.py:27-90, float64) -> white noise at the SNR of the
    full band (signal power = mean(wave^2), :51-54) -> decode_ft8_message(bins_per_tone =
    steps_per_symbol = 2, max_candidates 20, min_score 1, 20 iterations) -> success if anything
    decodes.  The minimum SNR is the first (lowest) SNR whose success ratio reaches 0.5 (:99-107; the
    reference stops a point early once 11 of 20 failed, which cannot change that test).  All points
    and rounds of a rate are one float64 batch on the GPU.  A sample of slots per rate (the two
    rounds at the rate's threshold SNR) is decoded again by the oracle (C + scipy) from the same
    float64 bytes: `parity`."""
    import numpy as np
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from ft8_demodulator_amd import SlotDecoder, _lib
    from ft8_demodulator_amd import ft8_generator as G
    rates = rates or SENSITIVITY_RATES
    snrs = np.round(np.arange(snr_lo, snr_hi + step / 2, step), 6)
    n_pts = len(snrs)
    gen = torch.Generator(device=dev)
    rng = np.random.default_rng(seed)
    table, samples, t_dec, n_dec_slots = [], [], 0.0, 0
    for fs in rates:
        nsps = int(0.16 * fs)
        n = 79 * nsps
        n_slots = n_pts * rounds
        snr_of = np.repeat(snrs, rounds)        # slot i: SNR point i // rounds
        pay = rng.integers(0, 256, size=(n_slots, 10), dtype=np.uint8)
        _, _, tones = G.encode_batch(pay, 10, device=dev)
        dec = SlotDecoder(fs, 2, 2, max_candidates=20, min_score=1, max_iterations=20, device=dev)
        success = np.zeros(n_slots, dtype=bool)
        keep = {}
        for c0 in range(0, n_slots, chunk):
            c1 = min(n_slots, c0 + chunk)
            sig = np.zeros(c1 - c0, dtype=_lib.TX_SIGNAL_DTYPE)
            sig["amplitude"], sig["slot"] = 1.0, np.arange(c1 - c0)
            clean = G.synthesize(tones[c0:c1], sig, c1 - c0, n, fs, _lib.FT8_TX_REFERENCE, dtype=torch.float64,
                                 device=dev)
            gen.manual_seed(seed * 1000003 + fs * 1009 + c0)
            p_sig = (clean * clean).mean(dim=1)
            snr_t = torch.as_tensor(snr_of[c0:c1], dtype=torch.float64, device=dev)
            x = clean + torch.sqrt(p_sig / 10.0 ** (snr_t / 10.0))[:, None] * torch.randn(
                clean.shape, dtype=torch.float64, device=dev, generator=gen)
            del clean
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, counts = dec.run(x, _lib.FT8_F64)
            torch.cuda.synchronize()
            t_dec += time.perf_counter() - t0
            n_dec_slots += c1 - c0
            success[c0:c1] = counts.cpu().numpy() > 0
            # the oracle sample is picked once the threshold is known: the chunk stays on the device
            # until then (a rate's batch is a few GB at most)
            keep[c0] = x
        ok = success.reshape(n_pts, rounds).sum(axis=1)
        hit = np.nonzero(ok >= rounds * 0.5)[0]
        thr = float(snrs[hit[0]]) if hit.size else None
        # 50 % crossing by linear interpolation of the success ratio (a finer figure than the grid's)
        ratio = ok / rounds
        cross = None
        if hit.size and hit[0] > 0:
            j = hit[0]
            r0, r1 = ratio[j - 1], ratio[j]
            cross = float(snrs[j - 1] + (0.5 - r0) / (r1 - r0) * (snrs[j] - snrs[j - 1])) if r1 > r0 else float(snrs[j])
        # the reference harness's own rule on its own grid (test_ft8_standard.py:74-76, 81-82:
        # np.arange(-21, -10, 0.2); 3 when no point reaches 50 %) -- the wider grid is an extension
        on_ref = (snrs >= -21.0 - 1e-9) & (snrs < -10.0 - 1e-9)
        hit_ref = np.nonzero(on_ref & (ok >= rounds * 0.5))[0]
        ref_rule = float(snrs[hit_ref[0]]) if hit_ref.size else 3.0
        row = {"fs": fs, "bandwidth_hz": fs / 2, "min_snr_db": thr, "ref_rule_min_snr_db": ref_rule,
               "crossing_50pct_db": cross,
               "xlsx_min_snr_db": XLSX_MIN_SNR_DB.get(fs),
               "success_per_point": {f"{s_:.1f}": int(k_) for s_, k_ in zip(snrs, ok) if 0 < k_ < rounds}}
        table.append(row)
        # oracle sample: the first `oracle_per_rate` rounds at the threshold point (or the top point)
        jp = hit[0] if hit.size else n_pts - 1
        for r_ in range(min(oracle_per_rate, rounds)):
            i = jp * rounds + r_
            c0 = (i // chunk) * chunk
            x_host = keep[c0][i - c0].cpu().numpy()
            gpu_pay = [bytes(p_).hex() for p_ in dec.records(keep[c0][i - c0:i - c0 + 1], _lib.FT8_F64)[0]["payload"]]
            samples.append((fs, float(snr_of[i]), x_host, gpu_pay))
        del keep
        torch.cuda.empty_cache()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max(1, procs)) as ex:   # ctypes and scipy release the GIL
        cpu = list(ex.map(_oracle_decode_payloads, [(x_, fs_) for fs_, _s, x_, _g in samples]))
    t_cpu = time.perf_counter() - t0
    mism = [{"fs": fs_, "snr_db": s_, "gpu": g_, "oracle": c_} for (fs_, s_, _x, g_), c_ in zip(samples, cpu) if g_ != c_]
    return {"method": "test_ft8_standard.py:43-123 on the GPU: f0 = fc = 0, bins_per_tone = steps_per_symbol = 2, "
                      "K = 20, min_score 1, 20 iterations, float64 input; SNR over the full band (B = fs / 2); "
                      f"{snr_lo} .. {snr_hi} dB in {step} dB steps (an extension of the reference's "
                      f"np.arange(-21, -10, 0.2) grid), {rounds} rounds per point; min_snr_db = the first point with "
                      ">= 50 % decodes on the wide grid; ref_rule_min_snr_db = the reference's rule on its own grid "
                      "(3 when no point of it reaches 50 %); crossing_50pct_db = the linear interpolation of the "
                      "success ratio at 0.5",
            "rounds": rounds, "slots": n_dec_slots, "decode_slots_per_s": n_dec_slots / t_dec if t_dec else None,
            "table": table,
            "parity": {"slots": len(samples), "equal": len(samples) - len(mism), "mismatches": mism[:8],
                       "what": "payload lists, GPU vs oracle on the same float64 bytes (the rounds at each "
                               "rate's threshold SNR)", "oracle_threads": procs, "oracle_wall_s": t_cpu},
            "cpu_baseline": {"value": len(samples) / t_cpu if t_cpu else None, "unit": "slots/s",
                             "cores": procs, "kind": "port",
                             "sample": f"the {len(samples)} parity slots above, oracle/ft8_oracle.c + scipy, "
                                       f"{procs} threads"}}


def drift_correct(dev, n_sig=256, reps=5):
    """The beacon receiver's correct_frequency_drift (frequency_correction.py:118-659) on a batch of
    n_sig independent complex128 beacons: 12 kHz, the reference test's layout (12.64 s of signal
    between two 12.64 s zero-signal pads, 455 040 samples), drift U(50, 150) Hz/s, Es/N0 28 dB,
    bins_per_tone 2, steps_per_symbol 8, poly_degree 2, precise sync.  Inputs resident in HBM."""
    import ctypes
    import numpy as np
    import torch
    from ft8_demodulator_amd import _lib, ft8_generator as G
    from ft8_demodulator_amd.frequency_correction import _drift_params, DEFAULT_PARAMS
    fs, nsps = 12000, 1920
    L = 79 * nsps
    n = 3 * L
    prm = drift_signal_params(n_sig)
    pays = np.frombuffer(b"".join(bytes.fromhex(p[0]) for p in prm), dtype=np.uint8).reshape(-1, 10)
    _, _, tones = G.encode_batch(pays, device=dev)
    sig = np.array([(p[1] + p[2], 1.0, 0.0, L, i, 0) for i, p in enumerate(prm)], dtype=_lib.TX_SIGNAL_DTYPE)
    x = G.synthesize(tones, sig, n_sig, n, fs, _lib.FT8_TX_REFERENCE, dtype=torch.complex128, device=dev)
    t = torch.arange(n, device=dev, dtype=torch.float64)
    k = torch.tensor([p[3] for p in prm], device=dev, dtype=torch.float64)[:, None] / fs
    x *= torch.polar(torch.ones((), device=dev, dtype=torch.float64), 2 * np.pi * k * t * t / (2 * fs))
    es = (x.abs() ** 2).mean(dim=1, keepdim=True)
    sd = torch.sqrt(es / 10 ** 2.8 * fs / 2)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    x += torch.complex(torch.randn(x.shape, generator=g, device=dev, dtype=torch.float64),
                       torch.randn(x.shape, generator=g, device=dev, dtype=torch.float64)) * sd
    del t
    ctx = _lib.context(dev)
    out = torch.empty_like(x)
    res = torch.zeros(n_sig * _lib.DRIFT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    p = _drift_params(dict(DEFAULT_PARAMS, **DRIFT_PARAMS), fs, 6.25, 0.16)
    st = _lib.stream_handle(dev)

    def run():
        ctx.check(_lib.lib().ft8_drift_correct(ctx.handle, _lib.ptr(x), _lib.FT8_C128, n, n_sig, n, ctypes.byref(p),
                                               _lib.ptr(out), _lib.ptr(res), st), "ft8_drift_correct")

    run()
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(_lib.DRIFT_RESULT_DTYPE)
    est = np.asarray(r["rate_per_sample"]) * fs
    true = np.array([p_[3] for p_ in prm])
    ok = r["status"] == _lib.FT8_DRIFT_FULL
    ctx.set_timing(True)
    ctx.timing(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    tm = ctx.timing(reset=True)
    stages = {k_: v[0] / reps for k_, v in tm.items() if v[1] > 0 and k_.startswith("drift")}
    _, hop, nfft, T = _lib.geometry(fs, 2, 8, n)
    # algorithmic work of one STFT-argmax launch: a 3840-point complex float64 FFT per frame
    # (5 N log2 N flops) + window (6 N) + |X|^2 of the kept half (3 N/2); 2 launches per call
    fft_flops = n_sig * T * (5 * nfft * np.log2(nfft) + 6 * nfft + 1.5 * nfft)
    stft_ms = tm["drift_stft_argmax"][0] / max(tm["drift_stft_argmax"][1], 1)
    tf = fft_flops / (stft_ms * 1e-3) / 1e12
    # de-rotation: stage 1 reads 16 B and writes 16 B per sample, stage 2 reads and writes 16 B
    rot_bytes = n_sig * n * 64
    rot_ms = tm["drift_derotate"][0] / reps
    # the complex128 STFT-argmax decides frames in float32 where its error bound settles them and
    # redoes the rest in float64 (stft.hip, launch_c3840_screened): the last call's split
    n_re, n_fr = ctypes.c_int64(0), ctypes.c_int64(0)
    ctx.check(_lib.lib().ft8_stft_screen_stats(ctx.handle, ctypes.byref(n_re), ctypes.byref(n_fr)), "ft8_stft_screen_stats")
    redo_share = n_re.value / max(n_fr.value, 1)
    t_peak = fft_flops / (FP32_VECTOR_PEAK_TFLOPS * 1e12) + fft_flops * redo_share / (FP64_VECTOR_PEAK_TFLOPS * 1e12)
    peak_mix = fft_flops / t_peak / 1e12
    del x, out
    return {"workload": f"correct_frequency_drift on {n_sig} complex128 beacons x {n} samples (12 kHz, "
                        "signal between two zero-signal pads as in test_correction.py), drift U(50,150) Hz/s, "
                        "Es/N0 28 dB, bins_per_tone 2, steps_per_symbol 8, poly_degree 2, precise_sync",
            "signals_per_s": n_sig * reps / dt, "ms_per_launch": dt / reps * 1e3,
            "full_fits": int(ok.sum()), "median_abs_rate_err_hz_per_s": float(np.median(np.abs(est[ok] - true[ok]))),
            "stages_ms": stages,
            "stft_screen": {"frames": int(n_fr.value), "redone_f64": int(n_re.value),
                            "what": "the last STFT-argmax call's frames, and those the float32 pass left to float64"},
            # every frame is transformed in float32 and the redone share again in float64: the peak
            # is the rate at which those two amounts of work would run at the FP32 and FP64 peaks
            "roofline": {"kernel": "k_stftc3840 (argmax epilogue, complex128: float32 screening + float64 redo)",
                         "bound": "fp32-valu + fp64-valu", "achieved": tf, "peak": peak_mix, "unit": "TFLOP/s",
                         "frac": tf / peak_mix, "flops_per_launch": fft_flops, "launch_ms": stft_ms,
                         "flops_f32_per_launch": fft_flops, "flops_f64_per_launch": fft_flops * redo_share},
            "roofline_derotate": {"kernel": "k_derotate1 + k_derotate2", "bound": "hbm",
                                  "achieved": rot_bytes / (rot_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": rot_bytes / (rot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_per_call": rot_bytes},
            "data": "synthetic (HIP transmit chain, reference GFSK timing; seeded drift and noise)"}


def settled(prev_ms, cur_ms, tol=0.015):
    """The settle phase's stop rule: a block's GPU time within `tol` of the previous block's."""
    return prev_ms is not None and abs(cur_ms - prev_ms) <= tol * prev_ms


def h2d_stream(x, steps, kw, depth=2):
    """Slots handed over as 16-bit PCM in pinned host memory (the WAV ingestion path): the upload of
    batch k+depth on a copy stream overlaps the decodes of the batches before it, which alternate
    over `depth` decoders/streams as the headline's steps do.  PCIe-inclusive slots/s -- reported
    beside `value`, never as it -- with the leg's two bounds: the upload alone (PCIe) and the same
    pipeline at depth 1."""
    import torch
    from ft8_demodulator_amd.stream import StreamDecoder
    pcm = torch.clamp(torch.round(x / x.abs().amax() * 30000.0), -32767, 32767).to(torch.int16).cpu().pin_memory()
    S = pcm.shape[0]

    def run(sd, borrow=False):
        for _ in sd.decode_batches([pcm] * 6, borrow=borrow):  # warm-up: one-time costs of a first stream
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = []
        for _ in sd.decode_batches([pcm] * steps, borrow=borrow):
            ts.append(time.perf_counter())
        torch.cuda.synchronize()
        # steady state: the spacing of batches' results once the pipeline is full (after the first
        # NBUF yields, before the drain's last ones, which come back to back)
        lo, hi = sd.NBUF, steps - sd.NBUF
        steady = (ts[hi] - ts[lo]) / (hi - lo) if hi > lo else None
        return (time.perf_counter() - t0) / steps, steady

    sd = StreamDecoder(pcm.shape[1], max_batch=S, depth=depth, **kw)
    dt, steady = run(sd)
    # the same batches lent to the decoder (borrow=True: the pinned batch is never rewritten, so no
    # upload is waited for on the host)
    dtb, steadyb = run(sd, borrow=True)
    del sd
    dt1, steady1 = run(StreamDecoder(pcm.shape[1], max_batch=S, depth=1, **kw)) if depth > 1 else (dt, steady)
    # the PCIe bound: the same pinned batch uploaded back to back on its own
    dbuf = torch.empty(pcm.shape, dtype=pcm.dtype, device=x.device)
    for _ in range(3):
        dbuf.copy_(pcm, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dbuf.copy_(pcm, non_blocking=True)
    torch.cuda.synchronize()
    up = (time.perf_counter() - t0) / steps
    del dbuf
    nbytes = int(pcm.numel() * 2)
    return {"workload": f"{steps} batches of {S} int16 PCM slots handed over in pinned host memory "
                        f"(ft8_demodulator_amd.stream.StreamDecoder, depth {depth}): batch k+{depth + 1} uploads on "
                        f"a copy stream while batches k+1..k+{depth} decode on {depth} contexts/streams "
                        "and batch k's results are copied back to pinned host memory and converted to the "
                        "reference's result tuples",
            "slots_per_s": S / dt, "ms_per_batch": dt * 1e3, "depth": depth,
            "timing": f"wall clock over the {steps} batches (pipeline fill and drain included)",
            "steady": None if steady is None else {
                "slots_per_s": S / steady, "ms_per_batch": steady * 1e3,
                "what": "spacing of consecutive batches' results with the pipeline full"},
            "borrow": {"slots_per_s": S / dtb, "ms_per_batch": dtb * 1e3,
                       "steady_ms_per_batch": None if steadyb is None else steadyb * 1e3,
                       "what": "decode_batches(borrow=True): pinned batches lent until their results "
                               "are yielded, uploads not waited for on the host"},
            "depth1": {"slots_per_s": S / dt1, "ms_per_batch": dt1 * 1e3,
                       "steady_ms_per_batch": None if steady1 is None else steady1 * 1e3},
            "h2d_bytes_per_batch": nbytes,
            "upload_alone": {"ms_per_batch": up * 1e3, "gb_per_s": nbytes / up / 1e9,
                             "slots_per_s": S / up,
                             "what": "the pinned batch copied to the device back to back, nothing else running"}}


def single_call(x, calls=50):
    """The drop-in call itself: decode_ft8_message on one host-memory slot (numpy float32, upload
    and result conversion included), warm, at the reference's defaults and at config 2's K=300."""
    from ft8_demodulator_amd import decode_ft8_message
    import torch
    slot = x[0].cpu().numpy()
    out = {"workload": "decode_ft8_message(numpy float32 15-s slot, 12 kHz) called back to back on one slot "
                       "of the batch (host -> device upload, decode, results as the reference's tuples)"}
    for name, kw in (("defaults_ms", {}), ("k300_min2_ms", dict(max_candidates=300, min_score=2))):
        for _ in range(5):
            decode_ft8_message(slot, 12000, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            decode_ft8_message(slot, 12000, **kw)
        out[name] = (time.perf_counter() - t0) / calls * 1e3
    return out


REFERENCE_MEASURED = {
    "value": 1.0 / 30.5, "unit": "slots/s", "cores": 1,
    "what": "the reference's own decode_ft8_message (Python/NumPy/SciPy) on one config-2-like slot (50 signals, "
            "K=300, min_score=2): 30.5 s per slot single-threaded, measured in the survey container (8-core "
            "Xeon VM, numpy 2.2.6, scipy 1.15.3; SURVEY.md section 6, BASELINE.md section 2) -- not a same-node run"}

STAGE_ORDER = ("stft", "score", "select", "llr", "bp", "compact")


def gpu_clock_ghz(device=0):
    """The shader clock of this box (tools/probe/clock.hip: clock64 cycles over the constant-rate
    wall clock): {"light": one wave spinning, "loaded": four FP64-FMA waves per SIMD on every CU,
    k_bp's issue load} in GHz, or None.  Boxes differ: the same build's k_bp takes the same cycles at
    1.8-2.1 GHz ("Boxes and clocks")."""
    import ctypes
    try:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libclockprobe.so"))
    except OSError:
        return None
    fn = lib.ft8probe_clock_ghz
    fn.argtypes, fn.restype = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)], ctypes.c_int
    out = {}
    for name, loaded in (("light", 0), ("loaded", 1)):
        g = ctypes.c_double(0.0)
        out[name] = round(g.value, 3) if fn(int(device), loaded, ctypes.byref(g)) == 0 and g.value > 0 else None
    return out


def counters_for_build(pattern, build_id):
    """The newest committed profiles/<pattern> summary whose build_id equals the running library's
    -> (kernels dict, relative path); (None, "stale: <newest file> (build <id>)") when none matches,
    (None, None) when there is none."""
    import glob

    def _rv(p_):  # rNN[_vK]_... -> (NN, K)
        parts = os.path.basename(p_)[1:].split("_")
        return int(parts[0]), int(parts[1][1:]) if parts[1].startswith("v") and parts[1][1:].isdigit() else -1
    # only the headline passes' summaries, r<round>_v<k>_<suffix> (not a leg's, e.g. r4_v23_sub_...)
    rx = re.compile(r"^r\d+_v\d+_" + re.escape(pattern.rsplit("*_", 1)[1]) + "$")
    files = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", pattern)) if rx.match(os.path.basename(f))),
                   key=_rv)
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("build_id") == build_id:
            return d.get("kernels", {}), os.path.relpath(f, ROOT)
    if files:
        with open(files[-1]) as fh:
            old = json.load(fh).get("build_id")
        return None, f"stale: {os.path.relpath(files[-1], ROOT)} (build {old}); no summary of this build"
    return None, None


def rccl_world1(dev):
    """A world-size-1 RCCL ("nccl") process group on `dev` (127.0.0.1 rendezvous)."""
    import socket
    import torch.distributed as dist
    if dist.is_initialized():
        return
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)


def gather_leg(dec, x, dev, S, steps, rounds=3):
    """N = 1: the cost of the N > 1 step's exchange, on this GPU -- blocks of `steps` plain steps and
    of `steps` steps that also pack the decodes (ft8_pack_decodes) and all-gather them over a
    world-size-1 RCCL group, interleaved `rounds` times; ms per step of each (best block)."""
    import torch
    import torch.distributed as dist
    from ft8_demodulator_amd.distributed import DecodeGatherer
    rccl_world1(dev)
    g = DecodeGatherer(S, dec.cap)
    last = []

    def block(with_gather):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out, counts = dec.run(x)
            if with_gather:
                last[:] = [g.start(out, counts)]
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    block(True)
    plain, gath = [], []
    for _ in range(rounds):
        plain.append(block(False))
        gath.append(block(True))
    recs, _, tot = last[0].resolve()
    ok = recs.shape[1] == int(tot[0])
    dist.destroy_process_group()
    return {"backend": "nccl (RCCL), world size 1", "steps_per_block": steps, "rounds": rounds,
            "ms_per_step_plain": min(plain), "ms_per_step_with_gather": min(gath),
            "overhead_pct": (min(gath) / min(plain) - 1.0) * 100.0,
            "blocks_plain_ms": plain, "blocks_gather_ms": gath,
            "rows_per_rank_sent": g.capacity, "decodes_gathered_last_step": int(tot[0]), "resolved_ok": bool(ok),
            "what": "each gather step: ft8_pack_decodes (one HIP kernel) + dist.all_gather_into_tensor of the "
                    "packed buffer on the decode stream, no host sync; the last step's exchange resolved after"}


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N ranks under torch.distributed.run as a child
    process (this process never touches the GPU) and return its exit code."""
    import socket
    import subprocess
    import torch
    n_dev = torch.cuda.device_count()  # does not initialise HIP on this image (asserted below)
    # the ranks are started as child processes; a parent that had initialised the GPU must not
    # spawn them (exec from a GPU-initialised process is forbidden on this pool)
    if torch.cuda.is_initialized():
        print("bench.py: the launcher process initialised HIP before spawning its ranks", file=sys.stderr)
        return 2
    if n_dev < (1 if args.share_gpu else args.gpus):
        print(f"bench.py: --gpus {args.gpus} requested but only {n_dev} GPU(s) are visible", file=sys.stderr)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


class StepLoop:
    """The bench's step sequence.  Step k runs decoder k % D inside stream context k % D (a factory:
    torch.cuda.stream of that decoder's stream on the GPU; contextlib.nullcontext on the CPU), then -- with a
    gatherer (N > 1 or --gather) -- packs and issues that step's decode exchange on the same stream,
    with no host sync.  Kept steps' exchanges are resolved after the loop, in issue order: they are
    collectives, so every rank issues and resolves them in the same order (tests/test_distributed_gloo.py
    drives this loop at world size 2 with fake decoders)."""

    def __init__(self, decs, stream_ctxs, x, gatherer=None):
        self.decs, self.ctxs, self.x, self.gatherer = decs, stream_ctxs, x, gatherer
        self.handles = []

    def step(self, k, keep=False, ev=None):
        D = len(self.decs)
        with self.ctxs[k % D]():
            out, counts = self.decs[k % D].run(self.x)
            if self.gatherer is not None:
                h = self.gatherer.start(out, counts)
                if keep:
                    self.handles.append(h)   # every timed step's exchange is resolved after the loop
            if ev is not None:
                ev.record()                  # on this step's stream, after its work
        return counts

    def resolve(self):
        """Resolve every kept exchange in issue order -> [(records, counts, totals, capacity)]."""
        out = []
        for h in self.handles:
            out.append((*h.resolve(), h.capacity))
        self.handles.clear()
        return out


LINE_MAX = 4096   # bytes of the stdout line; the driver's parser gave up on the 23.8 KB r05 line


def _strict(o, nd=None):
    """JSON-safe copy: NaN / +-inf -> None (strict JSON), numpy scalars -> Python, floats rounded to
    `nd` significant digits when given (the compact line)."""
    import math
    if isinstance(o, dict):
        return {str(k): _strict(v, nd) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_strict(v, nd) for v in o]
    if hasattr(o, "item") and not isinstance(o, (str, bytes)):
        try:
            o = o.item()
        except (TypeError, ValueError):
            return str(o)
    if isinstance(o, bool) or o is None or isinstance(o, (int, str)):
        return o
    if isinstance(o, float):
        if not math.isfinite(o):
            return None
        return float(f"{o:.{nd}g}") if nd else o
    return str(o)


def write_legs(full, path):
    """The full record (every leg, step times, per-rank shard parity) -> `path` (relative to the repo
    root unless absolute), strict JSON.  -> the path as the line names it (None if unwritable)."""
    p = path if os.path.isabs(path) else os.path.join(ROOT, path)
    try:
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        with open(p, "w") as f:
            json.dump(_strict(full), f, allow_nan=False, indent=1)
    except OSError as e:
        print(f"bench.py: could not write {p}: {e}", file=sys.stderr)
        return None
    return path


def _pick(d, keys):
    return None if d is None else {k: d.get(k) for k in keys if k in d}


def compact_line(full, legs_path):
    """The one stdout line: the contract fields, roofline, cpu_baseline, a parity summary, settle steps,
    the one-chain rate, build id and (N > 1) the exchange's two verdicts; per-leg headline numbers
    only, every leg's full record in the side file `legs`.  Strict JSON, <= LINE_MAX bytes."""
    rf = full.get("roofline") or {}
    clk = rf.get("clock") or {}
    rh = full.get("roofline_hbm") or {}
    par = full.get("parity")
    one = (full.get("depth") or {}).get("one_chain")
    line = {k: full.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup")}
    line["settle_steps"] = full.get("settle_steps", (full.get("settle") or {}).get("steps", 0))
    for k in ("ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        line[k] = full.get(k)
    if "rehearsal" in full:
        line["rehearsal"] = full["rehearsal"]
    cfg = full.get("config") or {}
    line["config"] = {k: cfg.get(k) for k in ("workload", "slots_per_gpu", "sample_rate", "max_candidates",
                                              "min_score", "max_iterations", "pipeline_depth", "parallelism")
                      if k in cfg}
    line["ldpc_candidates_per_s"] = full.get("ldpc_candidates_per_s")
    line["decodes_per_step"] = full.get("decodes_per_step")
    iss = rf.get("issue") or {}
    line["roofline"] = {**_pick(rf, ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
                                     "traffic_source", "launch_ms", "flops_per_launch")),
                        "clock_effective_ghz": clk.get("effective_ghz"),
                        # the issue side of the bound (the committed SQ pass of this build): the exact
                        # FP64 stream is ~0.5 of FLOP peak when the VALU is 100 % busy
                        "valu_busy": iss.get("valu_busy_per_simd"),
                        "valu_instructions_per_sweep": iss.get("valu_instructions_per_sweep")}
    line["roofline_hbm"] = _pick(rh, ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
                                      "launch_ms", "bytes_per_launch"))
    line["cpu_baseline"] = _pick(full.get("cpu_baseline"), ("value", "unit", "cores", "kind", "sample"))
    line["parity"] = None if par is None else {
        "slots": par.get("slots"), "equal": par.get("payload_crc_multiset_equal"),
        "decodes_gpu": par.get("decodes_gpu"), "decodes_cpu": par.get("decodes_cpu"),
        "ordered_equal_slots": par.get("ordered_lists_equal_slots")}
    line["depth"] = {"contexts": (full.get("depth") or {}).get("contexts"),
                     "one_chain_value": None if one is None else one.get("value")}
    g = full.get("gather")
    if g is not None:
        line["gather"] = {"backend": g.get("backend"), "world": g.get("world"), "gather_ok": g.get("gather_ok"),
                          "shard_parity_ok": g.get("shard_parity_ok")}
    gn = full.get("gather_n1")
    if gn:
        line["gather_n1_ms_per_step"] = {k: gn.get(k) for k in ("ms_per_step_plain", "ms_per_step_with_gather")
                                         if k in gn}
    legs = {}
    bs = full.get("bp_stress")
    if bs:
        legs["bp_stress_candidates_per_s"] = bs.get("candidates_per_s")
    sr = full.get("subtract_redecode")
    if sr:
        legs["subtract_redecode_candidates_per_s"] = sr.get("candidates_per_s")
    hs = full.get("h2d_stream")
    if hs:
        legs["h2d_stream_slots_per_s"] = hs.get("slots_per_s")
    dc = full.get("drift_correct")
    if dc:
        legs["drift_signals_per_s"] = dc.get("signals_per_s")
    if legs:
        line["legs_summary"] = legs
    line["build_id"] = full.get("build_id")
    line["gpu_clock_ghz"] = full.get("gpu_clock_ghz")
    line["legs"] = legs_path
    out = _strict(line, nd=6)
    s = json.dumps(out, allow_nan=False, separators=(",", ":"))
    # over budget (long free-text fields): shed the descriptive strings first, never the numbers
    for k in ("data", "legs_summary", "roofline_hbm"):
        if len(s.encode()) <= LINE_MAX:
            break
        out.pop(k, None)
        s = json.dumps(out, allow_nan=False, separators=(",", ":"))
    if len(s.encode()) > LINE_MAX and out.get("cpu_baseline"):
        out["cpu_baseline"].pop("sample", None)
        s = json.dumps(out, allow_nan=False, separators=(",", ":"))
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # warm-up: k_bp settles over ~15 launches (2.35 -> 2.02 ms per 256-slot launch as the clocks
    # settle under the FP64 load; profiles/r2_v1_steps.json), so the timed steps start after 20
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--slots", type=int, default=256, help="slots per GPU per step")
    ap.add_argument("--settle_max", type=int, default=96,
                    help="untimed steps at most before the warmup, until the GPU time of consecutive "
                         "blocks of 4*depth steps agrees within 1.5%% (k_bp's clock ramp); 0 = off")
    ap.add_argument("--depth", type=int, default=2,
                    help="consecutive steps alternate over this many contexts, each on its own stream, so one "
                         "step's STFT / sync can start while the previous step's k_bp retires its last waves "
                         "(1: one chain on one stream)")
    ap.add_argument("--signals", type=int, default=50)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-slots", type=int, default=256)
    ap.add_argument("--shard-parity-slots", type=int, default=32,
                    help="N > 1: slots of each rank's shard decoded by the oracle before the GPU is touched and "
                         "compared with the gathered records of the last timed step")
    ap.add_argument("--stage-steps", type=int, default=10, help="steps per single-stage event pass")
    ap.add_argument("--no-bp-stress", action="store_true", help="skip the config-4 BP stress leg")
    ap.add_argument("--no-h2d", action="store_true", help="skip the PCIe-inclusive streaming leg")
    ap.add_argument("--no-single-call", action="store_true",
                    help="skip the single-slot decode_ft8_message leg (its 1-slot k_bp launches would mix into a "
                         "kernel-trace summary of the headline)")
    ap.add_argument("--no-subtract", action="store_true", help="skip the config-4 subtract-and-redecode leg")
    ap.add_argument("--subtract-oracle-slots", type=int, default=8,
                    help="slots of the subtract leg checked against oracle/subtract.py (0: none)")
    ap.add_argument("--no-drift", action="store_true", help="skip the frequency-drift correction leg")
    ap.add_argument("--no-geometries", action="store_true", help="skip the 20 kHz / bpt=10 geometry legs")
    ap.add_argument("--no-sensitivity", action="store_true", help=argparse.SUPPRESS)  # the leg is opt-in now
    ap.add_argument("--sensitivity", action="store_true",
                    help="also run the reference's sensitivity harness (test_ft8_standard.py) on the GPU "
                         "(~36k float64 slot decodes + an oracle sample; opt-in, into the legs file)")
    ap.add_argument("--gather", action="store_true",
                    help="N = 1: every timed step also packs its decodes and all-gathers them over a world-size-1 "
                         "RCCL group (the per-step exchange of the N > 1 path)")
    ap.add_argument("--no-gather-leg", action="store_true",
                    help="skip the N = 1 leg that times steps with and without the RCCL exchange")
    ap.add_argument("--legs-out", default=os.path.join("gpurun_out", "bench_legs.json"),
                    help="side file (relative to the repo root unless absolute) that receives the full record: "
                         "every leg, step times, per-rank shard parity; the stdout line names it")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, gloo instead of "
                         "RCCL (exercises the launch, sharding and decode gather; not a measurement)")
    args = ap.parse_args()

    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)
    elif args.gpus > 1:
        sys.exit(launch_ranks(args))
    else:
        world = 1
    if args.gpus < 1:
        sys.exit(2)

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    kw = dict(max_candidates=300, min_score=2, max_iterations=20)
    S = args.slots
    seed0 = 100000 + rank * S  # global slot g uses seed 100000 + g
    cpu = drift_cpu_port = None
    cpu_x = cpu_dec = None
    shard_sample_wall = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_slots > 0:
        procs, basis = host_cores()
        cpu, cpu_x, cpu_dec = cpu_baseline(kw, min(args.cpu_slots, S), procs, basis, seed0, args.signals)
        if not args.no_drift:
            drift_cpu_port = drift_cpu_baseline(procs)
    sub_oracle = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.no_subtract and args.subtract_oracle_slots > 0:
        sub_oracle = subtract_oracle(args.subtract_oracle_slots, host_cores()[0])
    if world > 1 and args.shard_parity_slots > 0:
        # every rank: the oracle decodes the first slots of this rank's own shard (global seeds
        # 100000 + g) on its share of the host cores, before the GPU is touched; those bytes are
        # the first rows of the rank's batch, so the gathered records of the last timed step are
        # checked against them (gather.shard_parity)
        procs, basis = host_cores()
        procs = max(1, procs // world)
        base_, cpu_x, cpu_dec = cpu_baseline(kw, min(args.shard_parity_slots, S), procs,
                                             basis + f" // {world} ranks", seed0, args.signals)
        shard_sample_wall = base_["wall_s"]
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    elif args.gather:
        rccl_world1(dev)

    from ft8_demodulator_amd import SlotDecoder, synth, _lib
    from ft8_demodulator_amd.distributed import DecodeGatherer

    # the batch: slots synthesised on the CPU for the CPU leg are uploaded as-is (same bytes), the
    # rest synthesised on the GPU with the same per-slot seeds
    n_cpu = 0 if cpu_x is None else cpu_x.shape[0]
    parts = []
    if n_cpu:
        parts.append(torch.from_numpy(cpu_x).to(dev))
    if S > n_cpu:
        xg, _ = synth.make_slots(S - n_cpu, args.signals, fs=12000, snr_db=(-24.0, -10.0),
                                 seeds=[seed0 + b for b in range(n_cpu, S)], device=dev)
        parts.append(xg)
    x = torch.cat(parts) if len(parts) > 1 else parts[0]
    del parts
    torch.cuda.synchronize()
    dec = SlotDecoder(12000, 2, 2, device=dev, **kw)
    ctx = dec.ctx
    # --depth D: step k runs on decoder k % D -- its own context (scratch, BP claim counters) and its
    # own stream -- so consecutive steps overlap only where the hardware lets them (the next step's
    # front end filling the CUs k_bp's last waves leave); every step still decodes the whole batch
    D = max(1, args.depth)
    decs = [dec] + [SlotDecoder(12000, 2, 2, device=dev, context=_lib.Context(local), **kw) for _ in range(D - 1)]
    streams = [torch.cuda.current_stream(dev)] if D == 1 else [torch.cuda.Stream(dev) for _ in range(D)]
    for d_ in decs:
        d_.ctx.set_timing(True)   # allocates the device BP work counters; no events in the timed loop
        d_.ctx.set_timing(False)

    # N > 1 (or --gather): every step ends with the decode exchange -- ft8_pack_decodes on the device,
    # one all-gather of the packed buffer, no host sync (distributed.DecodeGatherer); the last
    # step's exchange is resolved after the timed loop.  Records carry global slot ids.
    exchange = world > 1 or args.gather
    gatherer = DecodeGatherer(S, dec.cap, slot_offset=rank * S) if exchange else None
    loop = StepLoop(decs, [lambda st_=st_: torch.cuda.stream(st_) for st_ in streams], x, gatherer)
    step = loop.step

    # clock settling before the W warmup steps: k_bp's shader clock ramps over its first launches
    # (step_times of the driver's --warmup 5 lines: the first timed pairs 10 % slower than the last),
    # so untimed blocks of 4 D steps run until a block's GPU time is within 1.5 % of the one before
    # (at most --settle_max steps; 0 = off).  Reported in the line as `settle`.
    settle = {"steps": 0, "block_ms": [], "max_steps": args.settle_max}
    if args.settle_max > 0:
        blk = 4 * D
        ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        prev = None
        while settle["steps"] + blk <= args.settle_max:
            torch.cuda.synchronize()
            ev_a.record()
            for k_ in range(blk):
                step(k_)
            for st_ in streams:
                torch.cuda.current_stream(dev).wait_stream(st_)
            ev_b.record()
            torch.cuda.synchronize()
            t_ = ev_a.elapsed_time(ev_b)
            settle["steps"] += blk
            settle["block_ms"].append(round(t_, 4))
            done_ = settled(prev, t_)
            if world > 1:   # every rank runs the same settle steps (each step's exchange is a collective)
                flag_ = torch.tensor([0.0 if done_ else 1.0],
                                     device="cpu" if dist.get_backend() == "gloo" else dev)
                dist.all_reduce(flag_, op=dist.ReduceOp.MAX)
                done_ = flag_.item() == 0.0
            if done_:
                break
            prev = t_
    n_warm = max(args.warmup, D)
    for k_ in range(n_warm):
        step(k_)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # one HIP event after every timed step (recorded on the step's stream, no host sync): the
    # per-step GPU periods show whether the timed steps had settled (k_bp's clock ramps over its
    # first launches); with D > 1 a period is the spacing of consecutive steps' completions
    step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    step_ev[0].record()
    for i_ in range(args.steps):
        counts = step(n_warm + i_, keep=True, ev=step_ev[i_ + 1])   # the alternation continues
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = [step_ev[i_].elapsed_time(step_ev[i_ + 1]) for i_ in range(args.steps)]
    # the same K steps as one chain (D = 1) right after, on the first decoder and the default
    # stream: what the overlap of consecutive steps is worth on this box
    depth1 = None
    if D > 1 and world == 1:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            dec.run(x)
        torch.cuda.synchronize()
        dt1 = (time.perf_counter() - t1) / args.steps
        depth1 = {"ms_per_step": dt1 * 1e3, "value": S / dt1,
                  "what": "the same steps on one context and one stream, timed after the line's loop"}
    decoded = int(counts.sum().item())
    gather = None
    gather_last = None
    if exchange:
        from ft8_demodulator_amd.distributed import gathered_records, pack_bytes
        rows_sent = gatherer.capacity
        # resolve every timed step's exchange in issue order (collectives: all ranks do the same);
        # a step whose total exceeded the capacity runs its overflow exchange here and grows it
        over_steps = 0
        for recs_g, cnts_g, totals_g, cap_ in loop.resolve():
            over_steps += int(int(totals_g.max()) > cap_)
        gather_last = (gathered_records(recs_g, totals_g), cnts_g.cpu().numpy(), totals_g.cpu().tolist())
        gather = {"backend": dist.get_backend(), "world": world,
                  "rows_per_rank_sent": rows_sent, "bytes_per_rank_sent": pack_bytes(gatherer.S_pad, rows_sent),
                  "decodes_per_rank_last_step": gather_last[2], "steps_over_capacity": over_steps,
                  "capacity_grown": gatherer.grown, "capacity_after": gatherer.capacity,
                  "host_sync_per_step": False}

    # per-kernel durations inside the real step sequence: one pass of `stage_steps` steps per stage,
    # with HIP events bracketing only that stage's kernel (the rest of the step runs undisturbed);
    # the BP work counters of the k_bp pass give its algorithmic FLOPs per launch
    R = max(1, args.stage_steps)
    stage_ms = {}
    for st in STAGE_ORDER:
        ctx.timing(reset=True)
        if st == "bp":
            ctx.counters(reset=True)
            ctx.bp_clock(reset=True)
        ctx.set_timing(True, stages=[st])
        for _ in range(R):
            step(0)   # the first decoder (this context), one chain
        torch.cuda.synchronize()
        ctx.set_timing(False)
        tm = ctx.timing(reset=True)[st]
        stage_ms[st] = tm[0] / max(tm[1], 1)
        if st == "bp":
            cn = ctx.counters(reset=True)
            bclk = ctx.bp_clock(reset=True)
    ctx.set_timing(False, stages=None)
    # the STFT is the first kernel of a step, so an event placed before it also times the host's
    # launch gap; its launch duration comes from back-to-back re-launches of the step's STFT instead
    # (ft8_replay_stage), events only around the whole run
    stft_reps = 20
    ctx.replay("stft", 2)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ctx.replay("stft", stft_reps)
    e1.record()
    torch.cuda.synchronize()
    stft_replay_ms = e0.elapsed_time(e1) / stft_reps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        d = torch.tensor([decoded], dtype=torch.int64, device=dev)
        dist.all_reduce(d)
        decoded = int(d.item())

    parity = None
    if cpu_dec is not None and world == 1:
        parity = parity_check(dec.records(x[:n_cpu]), cpu_dec)
    if gather is not None:
        flat, cnts_np, tot_l = gather_last
        gather.update(gather_check(flat, cnts_np, tot_l, S, world, decoded, dec.cap))
        mine = None
        if cpu_dec is not None:
            # this rank's oracle sample against the gathered records of its global slots
            mine = parity_check(shard_sample(flat, rank * S, n_cpu), cpu_dec)
            mine = {"rank": rank, "global_slots": [rank * S, rank * S + n_cpu], "oracle_wall_s": shard_sample_wall,
                    **{k: mine[k] for k in ("slots", "decodes_gpu", "decodes_cpu", "payload_crc_multiset_equal",
                                            "mismatching_slots", "ordered_lists_equal_slots", "max_abs_score_diff")}}
        per_rank = [mine]
        if world > 1:
            per_rank = [None] * world
            dist.all_gather_object(per_rank, mine)
        gather["shard_parity"] = per_rank
        # None when no rank had an oracle sample (e.g. --no-cpu at N = 1): nothing was compared
        gather["shard_parity_ok"] = (None if all(p_ is None for p_ in per_rank) else
                                     all(p_ is not None and p_["payload_crc_multiset_equal"] for p_ in per_rank))

    total_slots = S * world * args.steps
    value = total_slots / elapsed
    K = args.steps
    bp_ms = stage_ms["bp"]
    stft_ms = stft_replay_ms
    # dominant kernel: k_bp.  Algorithmic FLOPs per launch from the device counters.
    f_pass = bp_flops_per_pass()
    f_hd = 174 * 3
    flops = (cn["passes"] * f_pass + cn["iterations"] * f_hd) / R
    ach_tf = flops / (bp_ms * 1e-3) / 1e12
    # STFT: samples read once (f32) + dB waterfall written once
    from ft8_demodulator_amd._pipeline import make_plan
    plan = make_plan(x.shape[1], 12000)
    stft_bytes = S * (x.shape[1] * 4 + plan.T * plan.F * 4)
    stft_gbs = stft_bytes / (stft_ms * 1e-3) / 1e9
    cand_per_s = cn["candidates"] / R * world / (elapsed / K)
    # BASELINE.md's whole-step figure: B_slot = N s_in + 2 F T 4 + K (58 8 4 + 174 8 2 + 40)
    # algorithmic bytes per slot; slots/s x B_slot vs the 8 TB/s HBM peak
    b_slot = x.shape[1] * 4 + 2 * plan.F * plan.T * 4 + kw["max_candidates"] * (58 * 8 * 4 + 174 * 8 * 2 + 40)
    step_gbs = value / world * b_slot / 1e9

    # k_bp's own clock (ft8_get_bp_clock, the same R launches the events timed): every persistent
    # wave reads the shader-clock and wall-clock counters at start and retire.  Cycles per launch do
    # not depend on the box's clock; cycles / wall time is the clock k_bp itself ran at, so a change
    # of k_bp time between lines splits into "more cycles" or "lower clock" from the line alone
    bp_clock = None
    if bclk["waves"] and bclk["wave_wall_ticks"] and bclk["wall_clock_khz"]:
        waves_per_launch = bclk["waves"] / R
        mean_wave_cycles = bclk["wave_cycles"] / bclk["waves"]
        bp_clock = {"mean_wave_cycles": mean_wave_cycles, "max_wave_cycles": bclk["max_wave_cycles"],
                    "waves_per_launch": waves_per_launch,
                    "effective_ghz": bclk["wave_cycles"] / (bclk["wave_wall_ticks"] / (bclk["wall_clock_khz"] * 1e3)) / 1e9,
                    "cycles_per_event_ms_ghz": mean_wave_cycles / (bp_ms * 1e-3) / 1e9,
                    "wave_busy_vs_event": (bclk["wave_wall_ticks"] / bclk["waves"] / (bclk["wall_clock_khz"] * 1e3))
                    / (bp_ms * 1e-3),
                    "note": "mean_wave_cycles ~ k_bp's cycles per launch (persistent waves live for the launch); "
                            "effective_ghz = summed wave cycles / summed wave wall time; wave_busy_vs_event = mean "
                            "wave lifetime / event-timed launch"}
    q1 = max(1, K // 4)
    step_times = {"ms": [round(v_, 4) for v_ in step_ms],
                  "first_quarter_mean_ms": sum(step_ms[:q1]) / q1, "last_quarter_mean_ms": sum(step_ms[-q1:]) / q1,
                  "from": "HIP events between consecutive timed steps (GPU periods; the line's ms_per_step is the "
                          "host wall clock around all of them)"}

    stress = None
    if world == 1 and not args.no_bp_stress:
        stress = bp_stress(ctx, dev, procs=host_cores()[0])
    stream = None
    if world == 1 and not args.no_h2d:
        stream = h2d_stream(x, 40, kw, depth=D)
    call = single_call(x) if world == 1 and not args.no_single_call else None
    drift = None
    if world == 1 and not args.no_drift:
        drift = drift_correct(dev)
        drift["cpu_baseline"] = drift_cpu_port
        drift["rate_32768"] = drift_32k(dev)
    geoms = None
    if world == 1 and not args.no_geometries:
        geoms = geometry_legs(dev)
    sens = None
    if world == 1 and args.sensitivity:
        sens = sensitivity(dev, procs=host_cores()[0])
    sub = None
    if world == 1 and not args.no_subtract:
        sub = subtract_redecode(dev, oracle_sample=sub_oracle)

    # HBM bytes and issue counters per launch from the committed rocprofv3 PMC summaries
    # (tools/pmc_traffic.py: FETCH_SIZE / WRITE_SIZE passes; tools/pmc_sq_json.py: the SQ pass), each
    # stamped with the build_id it measured: only a summary of THIS build is reported, else null
    gather_n1 = None
    if world == 1 and not args.gather and not args.no_gather_leg:
        gather_n1 = gather_leg(dec, x, dev, S, args.steps)
    build_id = _lib.lib().ft8_build_id().decode()
    traffic, tsrc = counters_for_build("r*_pmc_traffic.json", build_id)
    qdata, qsrc = counters_for_build("r*_v*_pmc.json", build_id)
    issue = None
    q = (qdata or {}).get("k_bp<false>")
    if q and cn["passes"]:
        issue = {"valu_busy_per_simd": q.get("valu_busy_per_simd"),
                 "valu_instructions_per_sweep": q["SQ_INSTS_VALU"] / (cn["passes"] / R),
                 "source": qsrc,
                 "note": "the exact (uncontracted, correctly rounded) FP64 instruction stream carries "
                         "~245 algorithmic flops per lane per sweep; frac at 100% VALU busy would be "
                         "~frac / valu_busy (DESIGN.md section 3)"}
    elif qsrc:
        issue = {"source": qsrc}
    traffic = traffic or {}

    def hbm(kernel_prefix):
        for k, v in traffic.items():
            if k.startswith(kernel_prefix):
                return v.get("hbm_bytes")
        return None

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "slots/s",
        "n_gpus": world,
        **({"rehearsal": "--share-gpu: every rank on cuda:0 over gloo; not a measurement"} if args.share_gpu else {}),
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (STFT, sync score) / f64 (LLR, BP)",
        "data": "synthetic (ft8_demodulator_amd.synth: 50 GFSK signals/slot, SNR U(-24,-10) dB, unit noise; "
                "per-slot seeds 100000 + global slot)",
        "config": {"workload": "BASELINE config 3: batch of 256 independent 15-s slots per GPU, 12 kHz, "
                               "K=300 candidates, min_score=2, 20 BP iterations (config 5 shape at N>1)",
                   "slots_per_gpu": S, "sample_rate": 12000, "samples_per_slot": int(x.shape[1]),
                   "max_candidates": 300, "min_score": 2, "max_iterations": 20,
                   "pipeline_depth": D,
                   "parallelism": f"slot-sharded x{world}" + (
                       (", one all-gather per step of the device-packed decodes over "
                        + ("gloo (--share-gpu rehearsal, every rank on cuda:0)" if args.share_gpu else "RCCL")
                        + (" (world size 1, --gather)" if world == 1 else ""))
                       if exchange else "")},
        "ldpc_candidates_per_s": cand_per_s,
        "decodes_per_step": decoded,  # successful decodes in one step's batch (every step decodes the same batch)
        "roofline": {"kernel": "k_bp (float64 BP + CRC)", "bound": "fp64-valu",
                     "achieved": ach_tf, "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": ach_tf / FP64_VECTOR_PEAK_TFLOPS, "traffic": hbm("ft8::k_bp"), "traffic_source": tsrc,
                     "flops_per_launch": flops, "launch_ms": bp_ms,
                     "launch_ms_from": f"HIP events around k_bp alone in {R} full steps after the timed loop",
                     "bp_passes_per_launch": cn["passes"] / R, "candidates_per_launch": cn["candidates"] / R,
                     "clock": bp_clock, "issue": issue},
        "step_times": step_times,
        "depth": {"contexts": D, "streams": D if D > 1 else 1, "one_chain": depth1},
        "settle": settle,
        "step_hbm": {"what": "BASELINE.md whole-step accounting: slots/s per GPU x B_slot algorithmic bytes "
                             "(the step is FP64-VALU bound in k_bp, so this fraction is low by construction)",
                     "bytes_per_slot": b_slot, "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": step_gbs / HBM_PEAK_GBS},
        "roofline_hbm": {"kernel": "k_stft", "bound": "hbm", "achieved": stft_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": stft_gbs / HBM_PEAK_GBS,
                         "traffic": hbm("ft8::k_stft"), "traffic_source": tsrc,
                         "bytes_per_launch": stft_bytes, "launch_ms": stft_ms,
                         "launch_ms_from": f"{stft_reps} back-to-back re-launches of the step's STFT "
                                           "(ft8_replay_stage), HIP events around the run"},
        "stages_ms": stage_ms,
        "stages_sum_ms": sum(stage_ms.values()),
        "bp_stress": stress,
        "h2d_stream": stream,
        "single_call": call,
        "subtract_redecode": sub,
        "drift_correct": drift,
        "geometries": geoms,
        "sensitivity": sens,
        "cpu_baseline": cpu,
        "parity": parity,
        "reference_measured": REFERENCE_MEASURED,
        "build_id": build_id,
        # the shader clock of this box, measured after the timed work (boxes differ by up to ~15 %)
        "gpu_clock_ghz": gpu_clock_ghz(local),
    }
    if gather is not None:
        line["gather"] = gather
    if gather_n1 is not None:
        line["gather_n1"] = gather_n1
    line["settle_steps"] = settle["steps"]
    if rank == 0:
        # every leg goes to the side file; stdout gets ONE compact line (<= LINE_MAX bytes, strict JSON)
        legs_path = write_legs(line, args.legs_out)
        print(compact_line(line, legs_path), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
