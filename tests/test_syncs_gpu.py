"""Host synchronizations per time step (verdict r2 item 5): counted with torch's sync-debug mode by
scripts/sync_inventory.py; several ranks share the GPU over gloo and the gloo bounce copies (comm._stage_host /
_stage_dev, absent with RCCL) are not counted. Ceilings in a step without a tree rebalance (a step that rebalances a
per-step octree runs the synchronous rebalance loop: a few more): 2 (Sedov) / 3 (Evrard: + open-box extent) on one
rank; 4 / 4 for any number of ranks (the global leaf counts, which also give the migration counts; the halo and
multipole count table; the time-step packet; the conserved quantities). The box extents of several ranks stay on the
device for the keys and the remote LET tree is planned and built on the device (csrc/hip/let_tree.hip): neither
waits. In the bench.py / CLI configuration (Propagator.defer_host) the last two are collected one step late through
events: 2 / 2. Multi-rank: measured over 4 steps, the median step must meet the ceiling."""

import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


@pytest.mark.parametrize("init,ceiling", [("sedov", 2), ("evrard", 3)])
def test_syncs_one_rank(gpu, init, ceiling):
    import sync_inventory as S

    sites, _ = S.inventory(init, 30)
    assert sum(sites.values()) <= ceiling, dict(sites)


@pytest.mark.parametrize("ranks", [2, 8])
@pytest.mark.parametrize("init,ceiling", [("sedov", 4), ("evrard", 4)])
def test_syncs_multi_rank(gpu, ranks, init, ceiling):
    import sync_inventory as S

    for rank, steps, staged, _ in S.multi_rank(ranks, init, 40, steps=4):
        counts = sorted(sum(s.values()) for s in steps)
        assert counts[len(counts) // 2 - 1] <= ceiling, (rank, counts, steps)
        assert counts[-1] <= ceiling + 6, (rank, counts, steps)


@pytest.mark.parametrize("init", ["sedov", "evrard"])
def test_syncs_multi_rank_deferred(gpu, init):
    """the bench.py / CLI configuration on 2 ranks: 2 counted synchronizations per step (leaf counts, count table)"""
    import sync_inventory as S

    for rank, steps, staged, events in S.multi_rank(2, init, 40, steps=4, defer=True):
        counts = sorted(sum(s.values()) for s in steps)
        assert counts[len(counts) // 2 - 1] <= 2, (rank, counts, steps, events)
