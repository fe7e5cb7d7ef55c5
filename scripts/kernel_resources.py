"""Per-kernel resources from a gfx950 assembly listing (hipcc -S --cuda-device-only): VGPRs, SGPRs, LDS bytes,
scratch, and the waves per SIMD those allow (512 VGPRs per SIMD lane, 160 KiB LDS per CU, 4 SIMDs per CU).

usage: python scripts/kernel_resources.py file.s [nameSubstring ...]
"""
import re
import sys


def parse(path):
    txt = open(path).read()
    meta = txt[txt.find("amdhsa.kernels:"):]
    out = []
    for blk in re.split(r"\n  - ", meta)[1:]:
        def f(key):
            m = re.search(r"\.%s:\s+(\S+)" % key, blk)
            return m.group(1) if m else None
        name = f("name")
        if name is None:
            continue
        out.append(dict(name=name, vgpr=int(f("vgpr_count") or 0), agpr=int(f("agpr_count") or 0),
                        sgpr=int(f("sgpr_count") or 0), lds=int(f("group_segment_fixed_size") or 0),
                        scratch=int(f("private_segment_fixed_size") or 0),
                        wg=int(f("max_flat_workgroup_size") or 256)))
    return out


def waves_per_simd(k):
    regs = k["vgpr"] + k["agpr"]
    by_v = 8 if regs == 0 else min(8, 512 // (((regs + 7) // 8) * 8))
    waves_wg = max(k["wg"] // 64, 1)
    by_l = 8 if k["lds"] == 0 else min(8, (160 * 1024 // k["lds"]) * waves_wg // 4)
    return min(by_v, by_l), by_v, by_l


def main():
    ks = parse(sys.argv[1])
    subs = sys.argv[2:]
    for k in ks:
        if subs and not any(s in k["name"] for s in subs):
            continue
        w, wv, wl = waves_per_simd(k)
        print(f"{k['name'][:90]:90s} vgpr {k['vgpr']:3d} agpr {k['agpr']:3d} sgpr {k['sgpr']:3d} "
              f"lds {k['lds']:6d} scratch {k['scratch']:4d} waves/SIMD {w} (vgpr {wv}, lds {wl})")


if __name__ == "__main__":
    main()
