"""k_bp's lane layout tables (csrc/ft8_bp_layout.h, tools/gen_bp_layout.py): a permutation of the 174
variables over the real variable slots (padding kept at slot 2, lanes >= 46), the degree-7 checks on
rows 0..23, and fewer modelled LDS bank-conflict cycles than the plain order."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gen_bp_layout as G  # noqa: E402


def test_layout_tables_are_permutations():
    slots, rank = G.read_header()
    flat = [v for j in range(3) for v in slots[j]]
    assert sorted(v for v in flat if v is not None) == list(range(G.N))
    assert all(v is None for v in flat[128 + 46:]) and all(v is not None for v in flat[:128 + 46])
    assert sorted(rank) == list(range(G.M))
    assert {rank[m] for m in range(G.M) if G.DEG[m] == 7} == set(range(24))


def test_layout_cuts_modelled_conflicts():
    default = G.cost(*G.default_layout())
    assert default == (31, 58)  # the model reproduces round 4's measured 125 cycles per sweep with phase D's 36
    rc, wc = G.cost(*G.read_header())
    assert rc + wc < sum(default)
