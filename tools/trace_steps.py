"""Reconcile a rocprofv3 kernel trace of `bench.py` with its timed loop.

    python tools/trace_steps.py <run_kernel_trace.csv> <bench json line file> [--warmup W] [-o out.json]

Finds the decode steps in dispatch order (k_stft* -> k_score* -> k_select -> k_llr -> k_bp ->
k_compact), takes steps W .. W+K-1 as the timed loop (K = the line's `steps`), and reports per timed
step: the sum of kernel durations, the device span (first kernel start -> last kernel end) and the
gap to the next step, against the line's ms_per_step; then every k_bp dispatch in order (decode
steps and the bench's back-to-back re-launches), so the roofline's launch_ms can be checked
against the profiler's own clock.
"""
import argparse
import csv
import json
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
    W = line["warmup"] if a.warmup is None else a.warmup
    K = line["steps"]
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         short(r["Kernel_Name"])))
    # submission order: a kernel's start timestamp can precede its predecessor's end (and even
    # start) by a few microseconds in the trace, so sorting by start misorders steps
    rows = [r[1:] for r in sorted(rows)]
    ft8 = [r for r in rows if r[2].startswith("k_")]
    # decode steps: a k_stft followed (next ft8 kernels) by score, select, llr, bp, compact
    steps = []
    i = 0
    while i < len(ft8):
        seq = [k for _, _, k in ft8[i:i + 6]]
        if len(seq) == 6 and all(s.startswith(p) for s, p in zip(seq, STEP)):
            steps.append(ft8[i:i + 6])
            i += 6
        else:
            i += 1
    timed = steps[W:W + K]
    per = []
    for j, s in enumerate(timed):
        t0, t1 = s[0][0], s[-1][1]
        nxt = timed[j + 1][0][0] if j + 1 < len(timed) else None
        per.append({"kernel_sum_ms": sum(e - b for b, e, _ in s) / 1e6, "span_ms": (t1 - t0) / 1e6,
                    "period_ms": (nxt - t0) / 1e6 if nxt else None,
                    "kernels_ms": {k: (e - b) / 1e6 for b, e, k in s}})
    periods = [p["period_ms"] for p in per if p["period_ms"]]
    bp_all = [(b, (e - b) / 1e6) for b, e, k in ft8 if k == "k_bp"]
    in_steps = {s[4][0] for s in steps}
    bp_step = [d for b, d in bp_all if b in in_steps]
    bp_replay = [d for b, d in bp_all if b not in in_steps]
    out = {
        "trace": a.trace, "line_ms_per_step": line["ms_per_step"], "line_bp_launch_ms": line["roofline"]["launch_ms"],
        "decode_steps_found": len(steps), "timed_steps": len(timed), "warmup": W,
        "timed_kernel_sum_ms_mean": st.mean(p["kernel_sum_ms"] for p in per) if per else None,
        "timed_span_ms_mean": st.mean(p["span_ms"] for p in per) if per else None,
        "timed_period_ms_mean": st.mean(periods) if periods else None,
        "timed_kernels_ms_mean": {k: st.mean(p["kernels_ms"][k] for p in per) for k in per[0]["kernels_ms"]} if per else {},
        "k_bp_in_steps_ms": bp_step, "k_bp_replays_ms": bp_replay,
        "k_bp_replay_mean_ms": st.mean(bp_replay) if bp_replay else None,
        "k_bp_timed_mean_ms": st.mean(p["kernels_ms"]["k_bp"] for p in per) if per else None,
    }
    if per:
        names = {"stft": "k_stft", "score": "k_score", "select": "k_select", "llr": "k_llr", "bp": "k_bp",
                 "compact": "k_compact"}
        km = out["timed_kernels_ms_mean"]
        out["line_stage_vs_trace_timed"] = {
            st: line["stages_ms"][st] / next(v for k, v in km.items() if k.startswith(pre))
            for st, pre in names.items() if st in line.get("stages_ms", {})}
        out["line_bp_vs_trace_timed_bp"] = line["roofline"]["launch_ms"] / out["k_bp_timed_mean_ms"]
        out["trace_frac"] = (line["roofline"]["flops_per_launch"] / (out["k_bp_timed_mean_ms"] * 1e-3) / 1e12
                             / line["roofline"]["peak"])
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
