"""Flag >64-bit vector-memory stores whose data VGPRs the very next VALU instruction
overwrites (the gfx950 store-data hazard hipcc does not pad; see buf_store_f32x4 in
rfanalyzer_amd/csrc/fft_common.h).  usage: store_hazard_check.py LISTING.s [...]"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


bad = 0
for path in sys.argv[1:]:
    lines = [l.strip() for l in open(path)]
    for i, l in enumerate(lines):
        if not re.match(r"(buffer|global|flat)_store_dwordx[34]", l):
            continue
        data = regs(l.split()[1].rstrip(","))
        j = i + 1
        while j < len(lines) and (not lines[j] or lines[j].startswith((";", ".", "s_nop")) is False and lines[j].startswith((";", "."))):
            j += 1
        nxt = lines[j] if j < len(lines) else ""
        if nxt.startswith("v_"):
            dst = regs(nxt.split()[1].rstrip(","))
            if dst & data:
                bad += 1
                print(f"{path}:{i + 1}: {l}  ->  {nxt}")
print(f"{bad} hazards")
sys.exit(1 if bad else 0)
