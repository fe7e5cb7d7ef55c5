"""Count instructions per innermost loop of a kernel in a gfx950 assembly listing (hipcc -S --cuda-device-only).

usage: python scripts/loop_valu.py file.s kernelSubstring [kernelSubstring ...]
"""
import re
import sys


def kernel_body(lines, name):
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l):
            for j in range(i, len(lines)):
                if "s_endpgm" in lines[j]:
                    return lines[i:j + 1]
    return []


def main():
    lines = open(sys.argv[1]).read().split("\n")
    for name in sys.argv[2:]:
        body = kernel_body(lines, name)
        for i, l in enumerate(body):
            m = re.match(r"^\.(LBB\w+):.*Loop Header: Depth=(\d)", l)
            if not m:
                # nested headers carry the label on the previous line
                m2 = re.match(r"^\s*; =>.*Loop Header: Depth=(\d)", l)
                if not m2 or i == 0:
                    continue
                ml = re.match(r"^\.(LBB\w+):", body[i - 1])
                if not ml:
                    continue

                class _M:
                    def __init__(self, a, b):
                        self.g = (a, b)

                    def group(self, k):
                        return self.g[k - 1]

                m = _M(ml.group(1), m2.group(1))
            tag = "Header=" + m.group(1)[1:] if m.group(1).startswith("L") else m.group(1)
            tag = "Header=" + m.group(1).replace("LBB", "BB")
            # every block of the loop carries "in Loop: Header=BBx_y" (or is the header): gather their instructions
            seg, inside = [], False
            for x in body:
                xs = x.strip()
                if re.match(r"^(\.LBB\w+:|; %bb\.\d+:)", xs):
                    inside = (tag in xs) or (xs.startswith("." + m.group(1) + ":"))
                    continue
                if inside and xs and not xs.startswith((";", ".")):
                    seg.append(xs)
            lab = m.group(1)
            cnt = {}
            for x in seg:
                op = x.split()[0]
                key = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
                       "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else
                       "lds" if op.startswith("ds_") else "other")
                cnt[key] = cnt.get(key, 0) + 1
            movs = sum(1 for x in seg if x.startswith("v_mov"))
            trans = sum(1 for x in seg if re.match(r"v_(sin|cos|exp|log|sqrt|rsq|rcp)_", x))
            pk = sum(1 for x in seg if x.startswith("v_pk_"))
            print(f"{name} loop {lab} depth {m.group(2)}: {cnt} movs {movs} trans {trans} pk {pk}")


if __name__ == "__main__":
    main()
