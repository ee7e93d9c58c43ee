"""Reconcile a rocprofv3 kernel trace of `bench.py` with its timed loop.

    python tools/trace_steps.py <run_kernel_trace.csv> <bench json line file> [--warmup W] [-o out.json]

Finds the decode steps in dispatch order on each stream (k_stft* -> k_score* -> k_select -> k_llr ->
k_bp -> k_compact; with `--depth D` consecutive steps run on D streams), orders them by their first
dispatch, takes steps W .. W+K-1 as the timed loop (W = the line's settle steps + max(its warmup, depth), K = its
`steps`), and reports per timed step the sum of kernel durations and the device span (first kernel
start -> last kernel end), and for the loop its device period (first timed kernel start -> last
timed kernel end, / K), against the line's ms_per_step; then every k_bp dispatch in order (decode
steps and the bench's back-to-back re-launches), so the roofline's launch_ms can be checked
against the profiler's own clock.
"""
import argparse
import csv
import json
import os
import statistics as st

STEP = ("k_stft", "k_score", "k_select", "k_llr", "k_bp", "k_compact")


def short(name):
    n = name.replace("ft8::(anonymous namespace)::", "").replace("ft8::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("line")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    with open(a.line) as f:
        line = next(json.loads(l) for l in f if l.startswith("{"))
    # round 6: the stdout line is compact; the full record (stages_ms, settle, ...) is in its legs file
    legs = line.get("legs")
    if legs:
        base = os.path.dirname(os.path.abspath(a.line))
        for cand in (legs, os.path.join(base, os.path.basename(legs))):
            if os.path.exists(cand):
                with open(cand) as f:
                    line = {**json.load(f), **{k: v for k, v in line.items() if k not in ("roofline", "depth")}}
                break
    depth = int(line.get("depth", {}).get("contexts", 1) or 1)
    # steps before the timed loop: the clock-settle phase's (bench `settle`, round 5), then the warmup
    settle = int(line.get("settle_steps", (line.get("settle") or {}).get("steps", 0)) or 0)
    W = settle + max(line["warmup"], depth) if a.warmup is None else a.warmup
    K = line["steps"]
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         short(r["Kernel_Name"]), int(r.get("Stream_Id") or 0)))
    # submission order: a kernel's start timestamp can precede its predecessor's end (and even
    # start) by a few microseconds in the trace, so sorting by start misorders steps
    rows = sorted(rows)
    ft8 = [r for r in rows if r[3].startswith("k_")]
    # decode steps, per stream: a k_stft followed (next ft8 kernels of that stream) by score,
    # select, llr, bp, compact; then all streams' steps in order of their first dispatch
    steps = []
    for sid in sorted({r[4] for r in ft8}):
        q = [r for r in ft8 if r[4] == sid]
        i = 0
        while i < len(q):
            seq = [r[3] for r in q[i:i + 6]]
            if len(seq) == 6 and all(s.startswith(p) for s, p in zip(seq, STEP)):
                steps.append(q[i:i + 6])
                i += 6
            else:
                i += 1
    steps.sort(key=lambda s: s[0][0])
    steps = [[(b, e, k) for _, b, e, k, _ in s] for s in steps]
    timed = steps[W:W + K]
    per = []
    for s in timed:
        t0, t1 = s[0][0], s[-1][1]
        per.append({"kernel_sum_ms": sum(e - b for b, e, _ in s) / 1e6, "span_ms": (t1 - t0) / 1e6,
                    "kernels_ms": {k: (e - b) / 1e6 for b, e, k in s}})
    loop_ms = ((max(s[-1][1] for s in timed) - min(s[0][0] for s in timed)) / 1e6) if timed else None
    # with depth > 1 the timed steps overlap, so their kernels' start -> end spans include time spent
    # waiting for CUs the other stream holds; the bench's `depth.one_chain` loop right after the
    # timed loop (the same K steps on the first decoder alone) gives the per-kernel durations
    after = [{k: (e - b) / 1e6 for b, e, k in s} for s in steps[W + K:W + 2 * K]] if depth > 1 else []
    one_chain_ms = ((steps[W + 2 * K - 1][-1][1] - steps[W + K][0][0]) / 1e6 / K
                    if depth > 1 and len(steps) >= W + 2 * K else None)
    ft8 = [(b, e, k) for _, b, e, k, _ in ft8]
    bp_all = [(b, (e - b) / 1e6) for b, e, k in ft8 if k == "k_bp"]
    in_steps = {s[4][0] for s in steps}
    bp_step = [d for b, d in bp_all if b in in_steps]
    bp_replay = [d for b, d in bp_all if b not in in_steps]
    out = {
        "trace": a.trace, "line_ms_per_step": line["ms_per_step"], "line_bp_launch_ms": line["roofline"]["launch_ms"],
        "decode_steps_found": len(steps), "timed_steps": len(timed), "warmup": W, "depth": depth,
        "timed_kernel_sum_ms_mean": st.mean(p["kernel_sum_ms"] for p in per) if per else None,
        "timed_span_ms_mean": st.mean(p["span_ms"] for p in per) if per else None,
        "timed_period_ms_mean": loop_ms / len(timed) if timed else None,
        "timed_kernels_ms_mean": {k: st.mean(p["kernels_ms"][k] for p in per) for k in per[0]["kernels_ms"]} if per else {},
        "timed_kernels_note": ("depth 1: per-kernel durations of the timed steps" if depth == 1 else
                               f"depth {depth}: OVERLAP-INFLATED start->end spans of kernels whose steps overlap "
                               "(they include time spent waiting for CUs the other stream holds) -- not per-kernel "
                               "costs; use one_chain_kernels_ms_mean for those"),
        "k_bp_in_steps_ms": bp_step, "k_bp_replays_ms": bp_replay,
        "k_bp_replay_mean_ms": st.mean(bp_replay) if bp_replay else None,
        "k_bp_timed_mean_ms": st.mean(p["kernels_ms"]["k_bp"] for p in per) if per else None,
        "one_chain_steps_after_loop": len(after), "one_chain_period_ms_mean": one_chain_ms,
        "line_one_chain_ms_per_step": (line.get("depth", {}).get("one_chain") or {}).get("ms_per_step"),
        "one_chain_kernels_ms_mean": {k: st.mean(a_[k] for a_ in after) for k in after[0]} if after else {},
    }
    if per:
        names = {"stft": "k_stft", "score": "k_score", "select": "k_select", "llr": "k_llr", "bp": "k_bp",
                 "compact": "k_compact"}
        # per-kernel comparison against the line: the timed steps at depth 1, the one-chain steps
        # after the loop at depth > 1
        km = out["timed_kernels_ms_mean"] if depth == 1 or not after else out["one_chain_kernels_ms_mean"]
        out["kernels_compared"] = "timed steps" if km is out["timed_kernels_ms_mean"] else "one-chain steps after the loop"
        out["line_stage_vs_trace_timed"] = {
            st: line["stages_ms"][st] / next(v for k, v in km.items() if k.startswith(pre))
            for st, pre in names.items() if st in line.get("stages_ms", {})}
        bp_ms = next(v for k, v in km.items() if k.startswith("k_bp"))
        out["line_bp_vs_trace_bp"] = line["roofline"]["launch_ms"] / bp_ms
        out["trace_frac"] = (line["roofline"]["flops_per_launch"] / (bp_ms * 1e-3) / 1e12 / line["roofline"]["peak"])
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
