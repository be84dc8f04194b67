#!/usr/bin/env python3
"""Instruction budget table from scripts/r06_sq_table.sh's PMC passes.

Per (format, N): SQ wave-instruction counts of the main FFT kernel per launch, per sample in lane
instructions (x 64 lanes / samples), the VALU busy fraction (SQ_ACTIVE_INST_VALU x 4 cycles / 1024
SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)), the wave wait fraction, and the kernel time (HIP events).
From them the VALU-issue floor of the launch (every SIMD issuing VALU every 4 cycles: SQ_ACTIVE_INST_VALU
x 4 / 1024 SIMDs / 2.4 GHz) and the HBM fraction that floor allows:
  frac_valu_ceiling = alg bytes / VALU floor / 8 TB/s
-- the highest fraction this arithmetic allows if memory, LDS and VALU overlapped perfectly."""
import csv
import glob
import os
import re
import sys

BPS = {"s8": 2, "f32": 8}
CLK = 2.4e9


def main():
    d = sys.argv[1]
    rows = []
    for p in sorted(glob.glob(os.path.join(d, "p_*"))):
        if not os.path.isdir(p):
            continue
        tag = os.path.basename(p)[2:]
        fmt, n = tag.split("_")[0], int(tag.split("_")[1])
        acc = {}
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "fft_" in r["Kernel_Name"]:
                    acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        c = {k: sum(v) / len(v) for k, v in acc.items()}
        if not c:
            continue
        t = open(os.path.join(d, f"t_{tag}.log")).read()
        m = re.search(r"kernel\s+([\d.]+) us", t)
        kus = float(m.group(1)) if m else float("nan")
        samples = 32768000
        lane = lambda k: c.get(k, 0) * 64 / samples
        busy = c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8)
        wait = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        floor_us = c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / CLK * 1e6
        alg = samples * (BPS[fmt] + 4)
        rows.append((fmt, n, "state" in tag, lane("SQ_INSTS_VALU"), lane("SQ_INSTS_LDS"),
                     lane("SQ_INSTS_VMEM_RD") + lane("SQ_INSTS_VMEM_WR"), lane("SQ_INSTS_SALU"), busy, wait, kus,
                     alg / kus / 1e3 / 8000, floor_us, alg / floor_us / 1e3 / 8000))
    print("# per sample: lane instructions (wave instructions x 64 / samples); 500 x 64 K = 32.8 M samples per launch")
    print("# fmt   N        VALU    LDS   VMEM   SALU | VALU busy  wait | kernel us  frac | VALU floor us  frac ceiling")
    for r in rows:
        print(f"  {r[0]:4s} {r[1]:6d}{' ring' if r[2] else '     '} {r[3]:6.2f} {r[4]:6.2f} {r[5]:6.2f} {r[6]:6.2f} |"
              f"   {r[7]:.3f}  {r[8]:.3f} | {r[9]:9.1f} {r[10]:.3f} | {r[11]:12.1f}  {r[12]:.3f}")


if __name__ == "__main__":
    main()
