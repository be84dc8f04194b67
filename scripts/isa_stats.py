#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (gfx950).

usage: isa_stats.py LISTING.s SYMBOL_SUBSTRING [--top 40]

Counts mnemonics between the kernel's label and its .Lfunc_end, grouped into
VALU / SALU / LDS / VMEM / branch classes, plus the kernel's resource
metadata (vgpr/agpr/sgpr counts, scratch, LDS).  Static counts only: loops are
counted once (the wide kernels are fully unrolled per work item, so per-item
counts equal the static counts of the item body)."""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.rstrip().endswith(":") and not l.startswith("\t")))
    name = lines[start].split(":")[0]
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cnt = collections.Counter()
    for l in lines[start + 1:end]:
        s = l.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        cnt[s.split()[0]] += 1
    cls = collections.Counter()
    for m, c in cnt.items():
        if m.startswith("v_"):
            k = "VALU-trans" if re.match(r"v_(log|exp|rcp|rsq|sqrt|sin|cos)_", m) else "VALU"
        elif m.startswith("s_"):
            k = "branch/wait" if re.match(r"s_(cbranch|branch|waitcnt|barrier|nop|sleep|setprio)", m) else "SALU"
        elif m.startswith("ds_"):
            k = "LDS"
        elif m.startswith(("buffer_", "global_", "flat_", "scratch_")):
            k = "VMEM"
        else:
            k = "other"
        cls[k] += c
    print(name)
    for k, c in sorted(cls.items(), key=lambda x: -x[1]):
        print(f"  {k:12s} {c}")
    print("top mnemonics:")
    for m, c in cnt.most_common(top):
        print(f"  {m:28s} {c}")
    meta = "\n".join(lines[end:end + 400])
    for key in ("NumVgprs", "NumAgprs", "NumSgprs", "ScratchSize", "Occupancy", "LDSByteSize", "TotalNumVgprs"):
        m = re.search(rf"; {key}: (\d+)", meta)
        if m:
            print(f"  {key}: {m.group(1)}")


if __name__ == "__main__":
    main()
