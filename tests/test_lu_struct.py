"""CPU tests of the tracker LU's column-group classes (hc_lu.hpp, round 5).

The sparse LU tests, per pivot step, whether a column group can be non-zero
in a pivot row of the wave.  For trifocal_2op1p_30x30 the library compiles in
which groups never pass that test (a symbolic fill-in bound over every pivot
order) and which always do (measured on datasets 000/001/002,
profiles/r5lv_live.jsonl); these tests recompute the structure and the bound
from the problem's own dH/dx index and check the library's tables against
them.  Parity of the resulting solves is tests/test_gpu_parity.py's."""
import pytest

from conftest import ROOT  # noqa: F401

NV = 30


def structural_patterns(problem):
    """Row r, bit c: entry (r, c) of dH/dx has terms (the reference's padded
    index, Data_Reader.cpp:167-189: [column][term][part][row])."""
    U = problem.dHdx_index
    pat = [0] * NV
    for r in range(NV):
        for c in range(NV):
            if any(U[(c * 8 + j) * 5 * NV + r] != 0 for j in range(8)):
                pat[r] |= 1 << c
    return pat


def fill_bounds(pat):
    """Upper bound S_I of the pivot rows' patterns at step I (columns > I) over
    every pivot order, and a lower bound (columns every candidate row holds)."""
    cur = list(pat)
    upper, lower = [], []
    for i in range(NV):
        rows = [r for r in range(NV) if (cur[r] >> i) & 1]
        above = ((0xFFFFFFFF << (i + 1)) & ((1 << NV) - 1))
        u, lo = 0, (1 << NV) - 1
        for r in rows:
            u |= cur[r]
            lo &= pat[r]
        upper.append(u & above)
        lower.append(lo & above if rows else 0)
        for r in rows:
            cur[r] |= u & above
    return upper, lower


def chunks(i, ch=2):
    single = 1 if ((i + 1) & 1) and (i + 1 < NV) else 0
    out = [(i + 1, 1)] if single else []
    j = i + 1 + single
    while j < NV:
        out.append((j, min(ch, NV - j)))
        j += ch
    return out


@pytest.fixture(scope="module")
def lib():
    from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
    return _abi.lib()


def test_compiled_structure_is_the_problems(lib, problem):
    pat = structural_patterns(problem)
    assert [int(lib.hc_lu_struct_pattern(r)) for r in range(NV)] == pat
    assert int(lib.hc_lu_struct_pattern(NV)) == 0 and int(lib.hc_lu_struct_pattern(-1)) == 0


def test_dead_groups_are_exactly_the_symbolic_bound(lib, problem):
    upper, _ = fill_bounds(structural_patterns(problem))
    n = {0: 0, 1: 0, 2: 0}
    for i in range(NV - 1):
        for k, (st, ln) in enumerate(chunks(i)):
            cls = int(lib.hc_lu_group_class(i, k))
            dead = (upper[i] & (((1 << ln) - 1) << st)) == 0
            assert (cls == 1) == dead, (i, k, cls)
            n[cls] += 1
        assert int(lib.hc_lu_group_class(i, len(chunks(i)))) == -1
    assert int(lib.hc_lu_group_class(NV - 1, 0)) == -1
    assert sum(n.values()) == 225 and n[1] == 101 and n[2] == 40 and n[0] == 84


def test_provably_live_groups_run_unconditionally(lib, problem):
    """Every group each candidate pivot row holds structurally is live in every
    solve; the library runs those (and the measured ones) without a test."""
    _, lower = fill_bounds(structural_patterns(problem))
    proven = 0
    for i in range(NV - 1):
        for k, (st, ln) in enumerate(chunks(i)):
            if lower[i] & (((1 << ln) - 1) << st):
                proven += 1
                assert int(lib.hc_lu_group_class(i, k)) == 2, (i, k)
    assert proven == 16


def test_pivot_search_spans_cover_the_candidate_rows(lib, problem):
    """The tracker's pivot search at step I reduces over the DPP group that
    holds every row that may hold column I (the others hold exact zeros)."""
    pat = structural_patterns(problem)
    cur = list(pat)
    spans = []
    for i in range(NV):
        rows = [r for r in range(NV) if (cur[r] >> i) & 1]
        assert int(lib.hc_lu_candidates(i)) == sum(1 << r for r in rows), i
        lo, hi = min(rows), max(rows)
        span = 1 if lo >> 2 == hi >> 2 else 2 if lo >> 3 == hi >> 3 else 3 if lo >> 4 == hi >> 4 else 4
        assert int(lib.hc_lu_search_span(i)) == span, i
        spans.append(span)
        above = ((0xFFFFFFFF << (i + 1)) & ((1 << NV) - 1))
        u = 0
        for r in rows:
            u |= cur[r]
        for r in rows:
            cur[r] |= u & above
    assert spans[:18] == [3, 4, 1, 3, 4, 1, 3, 4, 2, 1, 1, 2, 3, 3, 3, 3, 3, 3] and set(spans[18:]) == {4}
    assert int(lib.hc_lu_search_span(NV)) == -1 and int(lib.hc_lu_candidates(-1)) == 0
