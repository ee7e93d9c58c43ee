"""tools/trace_steps.py on synthetic kernel traces: one chain, and two streams whose steps overlap
(bench --depth 2) followed by the one-chain loop -- the tool must find every step on its own
stream, take the timed ones after max(warmup, depth), and report the loop period."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("ft8::k_stft3840p<float, true>", "ft8::k_score2<2, 2, true>", "ft8::k_select<float>",
           "ft8::k_llr<float>", "ft8::k_bp<false>", "ft8::k_compact")
DUR = (150, 220, 30, 80, 1500, 5)  # us


def _write(tmp, steps, depth, warmup, K, settle=None, compact=False):
    """steps: list of (stream, t0_us) -> trace csv + bench line."""
    rows, did = [], 0
    for sid, t0 in steps:
        t = t0
        for name, d in zip(KERNELS, DUR):
            did += 1
            rows.append({"Kind": "KERNEL_DISPATCH", "Stream_Id": sid, "Dispatch_Id": did, "Kernel_Name": name,
                         "Start_Timestamp": int(t * 1000), "End_Timestamp": int((t + d) * 1000)})
            t += d
    trace = os.path.join(tmp, "trace.csv")
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    line = {"warmup": warmup, "steps": K, "ms_per_step": 1.9, "depth": {"contexts": depth},
            "roofline": {"launch_ms": 1.5, "flops_per_launch": 2.3e10, "peak": 78.6},
            "stages_ms": {"stft": 0.15, "score": 0.22, "select": 0.03, "llr": 0.08, "bp": 1.5, "compact": 0.005}}
    if settle is not None:
        line["settle"] = {"steps": settle, "block_ms": [], "max_steps": 96}
    if compact:
        # round 6's stdout line: settle_steps inline, stages_ms only in the legs file it names
        with open(os.path.join(tmp, "legs.json"), "w") as f:
            json.dump(line, f)
        line = {k: line[k] for k in ("warmup", "steps", "ms_per_step", "depth", "roofline")}
        line["settle_steps"] = settle or 0
        line["legs"] = "gpurun_out/legs.json"   # resolved next to the line file when not found as given
    lf = os.path.join(tmp, "line.log")
    with open(lf, "w") as f:
        f.write(json.dumps(line) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_steps.py"), trace, lf],
                         capture_output=True, text=True, check=True)
    return json.loads(out.stdout)


def test_one_chain(tmp_path):
    step = sum(DUR)
    steps = [(0, i * step) for i in range(3 + 4)]
    d = _write(str(tmp_path), steps, depth=1, warmup=3, K=4)
    assert d["timed_steps"] == 4 and d["decode_steps_found"] == 7
    assert abs(d["timed_period_ms_mean"] - step / 1000) < 1e-9
    assert d["kernels_compared"] == "timed steps"
    assert abs(d["timed_kernels_ms_mean"]["k_bp"] - 1.5) < 1e-9


def test_two_streams_then_one_chain(tmp_path):
    step = sum(DUR)
    period = 1800  # overlapped steps: a new one every 1.8 ms on alternating streams
    W, K = 5, 6
    steps = [(1 + (i % 2), i * period) for i in range(W + K)]
    t = (W + K) * period + step
    steps += [(0, t + i * step) for i in range(K)]          # the one-chain loop after it
    d = _write(str(tmp_path), steps, depth=2, warmup=W, K=K)
    assert d["depth"] == 2 and d["timed_steps"] == K and d["decode_steps_found"] == W + 2 * K
    assert abs(d["timed_period_ms_mean"] - ((K - 1) * period + step) / K / 1000) < 1e-9
    assert abs(d["one_chain_period_ms_mean"] - step / 1000) < 1e-9
    assert d["kernels_compared"] == "one-chain steps after the loop" and d["one_chain_steps_after_loop"] == K


def test_settle_steps_precede_the_warmup(tmp_path):
    """The bench's clock-settle steps (line `settle.steps`) run before the warmup: the timed loop
    starts after settle + max(warmup, depth) steps.  Settle steps here are spaced 3 ms apart, the
    rest one step apart, so a wrong offset shows in the period."""
    step = sum(DUR)
    S, W, K = 8, 3, 4
    steps = [(0, i * 3000) for i in range(S)]
    t0 = S * 3000
    steps += [(0, t0 + i * step) for i in range(W + K)]
    d = _write(str(tmp_path), steps, depth=1, warmup=W, K=K, settle=S)
    assert d["warmup"] == S + W and d["timed_steps"] == K and d["decode_steps_found"] == S + W + K
    assert abs(d["timed_period_ms_mean"] - step / 1000) < 1e-9


def test_compact_line_with_legs_file(tmp_path):
    """The compact stdout line (settle_steps inline, stages_ms in the legs file it names) gives the
    same reconciliation as the full line; depth-2 per-kernel means are labelled overlap-inflated."""
    step = sum(DUR)
    S, W, K = 8, 3, 4
    steps = [(0, i * 3000) for i in range(S)] + [(0, S * 3000 + i * step) for i in range(W + K)]
    d = _write(str(tmp_path), steps, depth=1, warmup=W, K=K, settle=S, compact=True)
    assert d["warmup"] == S + W and d["timed_steps"] == K
    assert "line_stage_vs_trace_timed" in d and abs(d["line_stage_vs_trace_timed"]["bp"] - 1.0) < 1e-9
    period = 1800
    steps = [(1 + (i % 2), i * period) for i in range(5 + 6)]
    t = 11 * period + step
    steps += [(0, t + i * step) for i in range(6)]
    d = _write(str(tmp_path), steps, depth=2, warmup=5, K=6, compact=True)
    assert "OVERLAP-INFLATED" in d["timed_kernels_note"]
