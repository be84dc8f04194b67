"""Per-kernel instruction statistics of a gfx950 assembly file (hipcc -S).
usage: asm_stats.py FILE.s [substring filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    ins = re.findall(r"\n\s+([a-z_0-9]+)", body)
    c = lambda p: sum(1 for i in ins if i.startswith(p))
    vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", body)
    sc = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", body)
    print(f"{name[-48:]:48s} valu {c('v_'):5d} pk {c('v_pk_'):5d} ds {c('ds_'):4d} buffer {c('buffer_'):4d} "
          f"waitcnt {c('s_waitcnt'):4d} vgpr {vg and vg.group(1)} scratch {sc and sc.group(1)}")
