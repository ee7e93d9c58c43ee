"""k_bp lane layout (csrc/ft8_bp_layout.h): which variable each (lane, slot j) of the variable-major
phases owns, and the row order m' of the checks in the message array.

k_bp keeps the 522 edge messages in one LDS array, row-position-major (bp.hip: edge (m', q) at index
83 q + m', q < 6, or 498 + m').  The edge-major phases address it contiguously, but the
variable-major phases (the tov reads of phase A, the toc stores of phase C) gather each lane's
variable's three edges: nine ds_read_b64 and nine ds_write_b64 per sweep at scattered addresses.
A ds_read_b64 is serviced as two 32-lane groups and conflicts where two lanes of a group hit one
bank pair (index mod 32); a ds_write_b64 as four 16-lane groups (index mod 16).  Which variable a
lane owns and the order of the checks inside each degree class are free (the sums and products are
formed per variable / per check in the reference's order either way), so this tool searches both
(simulated annealing on swaps) to minimise the modelled conflict cycles, and writes the tables.

The model counts extra LDS cycles exactly as SQ_LDS_BANK_CONFLICT does: with round 4's layout it
gives 31 (phase A) + 58 (phase C) + 36 (phase D, fixed by the layout) = 125 per sweep and wave, the
measured 181.8 M cycles over 1.455 M sweeps of the headline launch (profiles/r4_v19_pmc.json).

  python tools/gen_bp_layout.py [--iters N] [--seed S]     -> rewrites csrc/ft8_bp_layout.h
  python tools/gen_bp_layout.py --check                     -> the committed tables' cost
"""
import argparse
import math
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ft8_demodulator_amd import _ldpc_tables as T  # noqa: E402

N, M, E, W = 174, 83, 522, 64
CS, VE = T.CHK_START, T.VAR_EDGE
DEG = [CS[m + 1] - CS[m] for m in range(M)]
EDGE_CHK = [m for m in range(M) for _ in range(CS[m], CS[m + 1])]
ONE = 583  # the constant 1.0 the padding variables read
HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ft8_demodulator_amd", "csrc",
                   "ft8_bp_layout.h")


def idx_of(e, rank):
    m = EDGE_CHK[e]
    q, r = e - CS[m], rank[m]
    return q * 83 + r if q < 6 else 498 + r


def group_cost(addrs, size, banks):
    c = 0
    for g in range(0, W, size):
        seen = {}
        for a in addrs[g:g + size]:
            if a is not None:
                seen.setdefault(a % banks, set()).add(a)
        c += max((len(s) for s in seen.values()), default=1) - 1
    return c


def cost(slots, rank):
    rc = wc = 0
    for j in range(3):
        for m in range(3):
            a = [idx_of(VE[3 * v + m], rank) if v is not None else None for v in slots[j]]
            rc += group_cost([x if x is not None else ONE for x in a], 32, 32)   # ds_read_b64
            wc += group_cost(a, 16, 16)                                          # ds_write_b64
    return rc, wc


def default_layout():
    slots = [[(l + W * j) if l + W * j < N else None for l in range(W)] for j in range(3)]
    rank, c7, c6 = [0] * M, 0, 24
    for m in range(M):
        if DEG[m] == 7:
            rank[m], c7 = c7, c7 + 1
        else:
            rank[m], c6 = c6, c6 + 1
    return slots, rank


def search(iters, seed):
    rnd = random.Random(seed)
    slots, rank = default_layout()
    real = [(j, l) for j in range(3) for l in range(W) if l + W * j < N]  # padding stays at j = 2, lanes >= 46
    d7 = [m for m in range(M) if DEG[m] == 7]
    d6 = [m for m in range(M) if DEG[m] == 6]
    cur = sum(cost(slots, rank))
    best, best_l = cur, ([r[:] for r in slots], rank[:])
    for it in range(iters):
        t = 2.0 * (1 - it / iters) + 0.02
        if rnd.random() < 0.8:
            (j1, l1), (j2, l2) = rnd.sample(real, 2)
            slots[j1][l1], slots[j2][l2] = slots[j2][l2], slots[j1][l1]
            c = sum(cost(slots, rank))
            if c <= cur or rnd.random() < math.exp((cur - c) / t):
                cur = c
            else:
                slots[j1][l1], slots[j2][l2] = slots[j2][l2], slots[j1][l1]
        else:
            a, b = rnd.sample(d7 if rnd.random() < 0.3 else d6, 2)
            rank[a], rank[b] = rank[b], rank[a]
            c = sum(cost(slots, rank))
            if c <= cur or rnd.random() < math.exp((cur - c) / t):
                cur = c
            else:
                rank[a], rank[b] = rank[b], rank[a]
        if cur < best:
            best, best_l = cur, ([r[:] for r in slots], rank[:])
    return best_l


def write_header(slots, rank, note):
    slot_var = [v if v is not None else 255 for j in range(3) for v in slots[j]]
    var_slot = [0] * N
    for s, v in enumerate(slot_var):
        if v != 255:
            var_slot[v] = s
    assert sorted(v for v in slot_var if v != 255) == list(range(N))
    assert all(slot_var[s] == 255 for s in range(128 + 46, 192)) and all(v != 255 for v in slot_var[:174])
    assert sorted(rank[m] for m in range(M) if DEG[m] == 7) == list(range(24))
    fmt = lambda xs: "{" + ", ".join(str(x) for x in xs) + "}"  # noqa: E731
    with open(HDR, "w") as f:
        f.write("// Generated by tools/gen_bp_layout.py -- do not edit.  " + note + "\n")
        f.write("// k_bp lane layout: FT8_BP_SLOT_VAR[64 j + lane] = the variable lane owns in variable slot j\n")
        f.write("// (255: padding), FT8_BP_VAR_SLOT its inverse, FT8_BP_CHK_RANK[m] = the row m' of check m in the\n")
        f.write("// message array (degree-7 checks take 0..23).\n#pragma once\n")
        f.write("#define FT8_BP_SLOT_VAR_INIT " + fmt(slot_var) + "\n")
        f.write("#define FT8_BP_VAR_SLOT_INIT " + fmt(var_slot) + "\n")
        f.write("#define FT8_BP_CHK_RANK_INIT " + fmt(rank) + "\n")


def read_header():
    vals = {}
    for line in open(HDR):
        if line.startswith("#define FT8_BP_"):
            name, body = line.split(None, 2)[1], line.split(None, 2)[2]
            vals[name] = [int(x) for x in body.strip().strip("{}").split(",")]
    sv, rank = vals["FT8_BP_SLOT_VAR_INIT"], vals["FT8_BP_CHK_RANK_INIT"]
    slots = [[(sv[W * j + l] if sv[W * j + l] != 255 else None) for l in range(W)] for j in range(3)]
    return slots, rank


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200000)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    d = cost(*default_layout())
    if a.check:
        print("default layout (read, write) extra cycles per sweep:", d, " committed:", cost(*read_header()))
        sys.exit(0)
    sl, rk = search(a.iters, a.seed)
    c = cost(sl, rk)
    write_header(sl, rk, "seed %d, %d iterations: modelled conflict cycles per sweep (read, write) %s, "
                 "default layout %s" % (a.seed, a.iters, c, d))
    print("wrote", HDR, c)
