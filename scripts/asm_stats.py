"""Instruction statistics of one kernel in a hipcc --save-temps .s file (which waits, how many MFMAs / LDS reads /
LDS-DMA loads / barriers, and the hot loop's body).

    python scripts/asm_stats.py build/x.s gemm_big_kernelILb0ELb0 [--loop]
"""
import re
import sys
from collections import Counter


def kernel_body(s: str, pat: str) -> tuple:
    names = [n for n in re.findall(r"^(\S+):\s*;\s*@", s, re.M) if pat in n]
    if not names:
        raise SystemExit(f"no kernel matching {pat}")
    name = names[0]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    return name, s[i:j]


def main(argv):
    path, pat = argv[0], argv[1]
    s = open(path).read()
    name, body = kernel_body(s, pat)
    lines = body.split("\n")
    ins = [l.strip() for l in lines if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
    c = Counter(x.split()[0] for x in ins)
    print(name, "instructions:", len(ins))
    for k in sorted(c, key=lambda k: -c[k])[:40]:
        print(f"  {k:34s} {c[k]}")
    print("waits:", Counter(x for x in ins if x.startswith("s_waitcnt")).most_common(20))
    if "--loop" in argv:
        # the loop = the basic block(s) between a label and the backward branch to it holding the most MFMAs
        labels = {m.group(1): idx for idx, l in enumerate(lines) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
        best = None
        for idx, l in enumerate(lines):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l) or re.search(r"s_branch\s+(\.LBB\w+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < idx:
                seg = lines[labels[m.group(1)]:idx + 1]
                n = sum("v_mfma" in x for x in seg)
                if best is None or n > best[0]:
                    best = (n, seg)
        if best:
            print(f"---- loop ({best[0]} MFMAs, {len(best[1])} lines)")
            print("\n".join(best[1]))


if __name__ == "__main__":
    main(sys.argv[1:])
