"""Chunk-coded GPU neighbor-list codec (csrc/include/sphx/packed_list.hpp; Python mirror in ops/neighbors.py): 16-bit
codes slot | k << 10 decoded through a per-group chunk table (slot 0 = the group's first particle, so padding decodes
to the target itself), 8 codes per lane and block, one 1-KiB row per block index of a group. The GPU search writes
this format and the pair loops decode it (tests/test_gpu_parity.py compares the decoded GPU lists with the CPU search)."""

import numpy as np
import pytest

from sphexa_amd.ops.neighbors import (CHUNK_CAP, GROUP, decode_packed, group_rows, list_blocks_max, pack_lists,
                                      packed_rows_max, packed_table_ints, packed_table_region)


def _roundtrip(lists, first, ngmax=150):
    nl = pack_lists(lists, first, ngmax)
    idx, valid = decode_packed(nl)
    for t, lst in enumerate(lists):
        assert idx[t][valid[t]].tolist() == [int(v) for v in lst]
    return nl, idx, valid


def test_roundtrip_random_lists():
    rng = np.random.default_rng(3)
    first = 1000
    n = 3 * GROUP + 17  # partial last group
    lists = []
    for t in range(n):
        k = int(rng.integers(0, 120))
        near = first + t + rng.integers(-3000, 3000, size=k)
        lst = np.unique(near.clip(0, None))
        lst = lst[lst != first + t][:140]
        lists.append(lst.tolist())
    nl, idx, valid = _roundtrip(lists, first)
    assert nl.rows_used <= ((n + GROUP - 1) // GROUP) * packed_rows_max(150)


def test_unsorted_and_far_entries():
    _roundtrip([[5, 2, 900000, 1, 2 ** 31 - 2, 3], [], [7]], first=10)


def test_padding_and_self_entries_are_not_valid():
    lists = [[0, 3]] * 3  # target 0 lists itself: the codec keeps it, the decoder reports it as the target
    nl = pack_lists(lists, 0, 150)
    idx, valid = decode_packed(nl)
    assert idx[0][valid[0]].tolist() == [3]
    assert idx[1][valid[1]].tolist() == [0, 3]
    # padding past the two entries decodes to the target itself
    assert (idx[2][2:8] == 2).all() and not valid[2][2:8].any()


def test_rows_follow_the_longest_lane_of_a_group():
    lists = [[1]] * GROUP
    lists[5] = list(range(100, 130))  # 30 entries -> 4 list blocks, + 1 chunk-table row + 1 mask row
    nl = pack_lists(lists, 0, 150)
    assert nl.nidx[0].item() == 4 and nl.rows_used == 6
    T = packed_table_ints(150)
    assert group_rows(nl.nidx[:T].view(1, T)).item() == 6
    assert packed_table_ints(150) % 4 == 0


def test_chunk_table_over_one_row():
    # 300 distinct 64-aligned chunks in one group: the table takes two rows
    lists = [[64 * k for k in range(300)][t::GROUP] for t in range(GROUP)]
    nl, _, _ = _roundtrip(lists, 10 ** 6)
    w = nl.nidx[1].item()
    assert (w & 0x3FF) == 301 and ((w >> 10) & 0x3F) == 2 and (w >> 16) == 2 + 3  # bases: 2 rows, masks: 3 rows


def test_masks_cover_every_code():
    # the staged-source mask of a slot has the bit of every source a list names (packed_list.hpp)
    rng = np.random.default_rng(3)
    lists = [sorted(set(rng.integers(0, 5000, 40).tolist())) for _ in range(GROUP)]
    nl = pack_lists(lists, 0, 150)
    buf = nl.nidx.numpy()
    T_I = packed_table_ints(150)
    w = int(buf[1])
    nch, tc = w & 0x3FF, (w >> 10) & 0x3F
    region = packed_table_region(1, 150)
    rows = buf[region:].reshape(-1, 256)
    r = buf[2:2 + (w >> 16)]
    bases = [int(rows[r[e // 256], e % 256]) for e in range(nch)]
    masks = [int(np.uint32(rows[r[tc + e // 128], 2 * (e % 128)])) | int(np.uint32(rows[r[tc + e // 128], 2 * (e % 128) + 1])) << 32
             for e in range(nch)]
    union = {bases[e] + k for e in range(1, nch) for k in range(64) if masks[e] >> k & 1}
    assert union == {j for lst in lists for j in lst}
    assert T_I % 4 == 0


def test_limits_are_rejected():
    with pytest.raises(ValueError):
        pack_lists([list(range(0, 8 * list_blocks_max(150) + 1))], 0, 150)
    with pytest.raises(ValueError):
        pack_lists([[64 * k for k in range(CHUNK_CAP)]], 0, 150)
