"""Debug helper (GPU): search a small jittered Sedov lattice on the GPU and the CPU and print where the decoded GPU
lists differ (entries, codes, chunk tables of the first differing target)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from test_gpu_parity import _setup  # noqa: E402

from sphexa_amd.ops import neighbors as N  # noqa: E402


def main():
    gpu = torch.device("cuda", 0)
    dc, pc, domc = _setup("cpu", 16, jitter=0.01)
    dg, pg, domg = _setup(gpu, 16, jitter=0.01)
    pc.sync(domc, dc)
    pg.sync(domg, dg)
    nlc = N.find_neighbors(dc, domc.octree, domc.box, 0, dc.size)
    nlg = N.find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    print("nc equal", torch.equal(dc["nc"], dg["nc"].cpu()))
    idx, valid = N.decode_packed(nlg)
    ncc = dc["nc"]
    buf = nlg.nidx.cpu()
    groups = (dg.size + 63) // 64
    TI = N.packed_table_ints(nlg.ngmax)
    tab = buf[:groups * TI].view(groups, TI)
    bad = 0
    for t in range(dg.size):
        g_set = idx[t][valid[t]].tolist()
        c_set = nlc.nidx[t * nlc.ngmax:t * nlc.ngmax + int(ncc[t]) - 1].tolist()
        if sorted(g_set) != sorted(c_set):
            bad += 1
            if bad <= 2:
                g = t // 64
                print(f"target {t}: gpu {len(g_set)} cpu {len(c_set)}")
                print("  extra", sorted(set(g_set) - set(c_set))[:40])
                print("  missing", sorted(set(c_set) - set(g_set))[:40])
                print("  dup", len(g_set) - len(set(g_set)))
                print("  tab", tab[g].tolist())
                print("  idx", idx[t].tolist()[:130])
    print("bad targets", bad, "of", dg.size)


if __name__ == "__main__":
    main()
