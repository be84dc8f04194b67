#!/bin/bash
# Copy the judged records of one r04_evidence.sh / final_evidence.sh call from gpurun_out/ into
# profiles/TAG/ (tracked).  usage: scripts/collect_evidence.sh TAG
set -eu
cd "$(dirname "$0")/.."
T=$1; D=profiles/$T; G=gpurun_out
mkdir -p $D
cp $G/bench_$T.json $D/bench.json
cp $G/pytest_gpu_$T.log $D/pytest_gpu.txt
cp $G/smoke_$T.log $D/smoke.txt
cp $G/kbench_$T.txt $D/kbench.txt
cp $G/prof_$T/run_kernel_stats.csv $D/rocprof_kernel_stats.csv
[ -f $G/pmc_traffic_$T.json ] && cp $G/pmc_traffic_$T.json $D/pmc.json
[ -f $G/sq_$T.txt ] && cp $G/sq_$T.txt $D/sq_counters_fft64k.txt
[ -f $G/bench_shard_$T.json ] && cp $G/bench_shard_$T.json $D/bench_shard_config4.json
[ -f $G/prof_shard_$T/run_kernel_stats.csv ] && cp $G/prof_shard_$T/run_kernel_stats.csv $D/rocprof_kernel_stats_config4_shard.csv
[ -f $G/seed_sweep_$T.txt ] && grep -v amdgpu.ids $G/seed_sweep_$T.txt > $D/config3_seed_sweep.txt
ls $D
# the sha-tagged records bench.py attaches to roofline.traffic / roofline.valu (used only while
# the in-tree librfa.so is the build they were measured on)
python3 - "$T" <<'PY'
import ast, json, sys
t = sys.argv[1]
pmc = json.load(open(f"profiles/{t}/pmc.json"))
key = "s8_65536_500"
rec = dict(pmc[key]); rec["source"] = f"profiles/{t}"
json.dump({key: rec}, open("profiles/pmc_traffic.json", "w"), indent=1, sort_keys=True)
line = [l for l in open(f"profiles/{t}/sq_counters_fft64k.txt") if l.startswith(t + " {")][0]
c = ast.literal_eval(line[len(t) + 1:])
sq = {"kernel": rec["kernel"], "librfa_sha16": rec["librfa_sha16"],
      "valu_busy_frac": round(c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8), 4),
      "wave_wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
      "valu_wave_insts_per_launch": c["SQ_INSTS_VALU"], "lds_bank_conflicts": c["SQ_LDS_BANK_CONFLICT"],
      "source": f"profiles/{t}/sq_counters_fft64k.txt",
      "formula": "VALUBusy = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs); wave_wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES"}
json.dump({key: sq}, open("profiles/sq_valu.json", "w"), indent=1)
print("records:", rec["librfa_sha16"], sq["valu_busy_frac"], sq["wave_wait_frac"])
PY
