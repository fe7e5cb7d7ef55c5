"""Packed GPU neighbor-list codec (csrc/include/sphx/packed_list.hpp; Python mirror in ops/neighbors.py): 16-bit
delta slots with jump slots for large steps, per-group rows. The GPU search writes this format and the pair loops
decode it (tests/test_gpu_parity.py compares the decoded GPU lists with the CPU search)."""

import numpy as np
import pytest

from sphexa_amd.ops.neighbors import (GROUP, decode_packed, encode_step, pack_lists, packed_rows_max,
                                      packed_table_ints)


def _roundtrip(lists, first, ngmax=150):
    nl = pack_lists(lists, first, ngmax)
    idx, valid = decode_packed(nl)
    for t, lst in enumerate(lists):
        assert idx[t][valid[t]].tolist() == [int(v) for v in lst]
    return nl, idx, valid


def test_small_steps_one_slot_each():
    for d in (1, -1, 16383, -16384, 7, -300):
        assert len(encode_step(d)) == 1
    for d in (16384, -16385, 1 << 27, -(1 << 27)):
        assert len(encode_step(d)) == 2
    assert len(encode_step(1 << 30)) >= 3  # beyond one jump's +-2^28


def test_roundtrip_random_lists():
    rng = np.random.default_rng(3)
    first = 1000
    n = 3 * GROUP + 17  # partial last group
    lists = []
    for t in range(n):
        k = int(rng.integers(0, 120))
        near = first + t + rng.integers(-3000, 3000, size=k)
        far = rng.integers(0, 1 << 30, size=int(rng.integers(0, 4)))
        lst = np.unique(np.concatenate([near, far]).clip(0, None))
        lst = lst[lst != first + t][:140]
        lists.append(lst.tolist())
    nl, idx, valid = _roundtrip(lists, first)
    assert nl.rows_used <= n * packed_rows_max(150)


def test_unsorted_and_descending_entries():
    _roundtrip([[5, 2, 900000, 1, 2 ** 31 - 2, 3], [], [7]], first=10)


def test_rows_follow_the_longest_lane_of_a_group():
    lists = [[1]] * GROUP
    lists[5] = list(range(100, 130))  # 30 entries -> 4 rows of 8 slots
    nl = pack_lists(lists, 0, 150)
    assert nl.nidx[0].item() == 4 and nl.rows_used == 4
    assert packed_table_ints(150) % 4 == 0


def test_list_too_long_is_rejected():
    with pytest.raises(ValueError):
        pack_lists([list(range(1, 2 ** 30, 2 ** 22))], 0, 150)  # 256 jump+emit pairs
