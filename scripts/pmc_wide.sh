# PMC passes for the 16K s8 wide vs narrow kernel (one counter group per pass)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in wide narrow; do
 for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" "GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM"; do
  RFA_KERNEL=$k timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$k -o p -- python3 scripts/kbench.py --sizes 16384 --formats s8 --iters 3 > /dev/null 2>&1 || { echo "pmc fail $k $grp"; break; }
  python3 - "$k" <<'PY'
import csv, glob, sys, collections
f = sorted(glob.glob(f"gpurun_out/pmc_{sys.argv[1]}/**/*counter_collection.csv", recursive=True))
rows = list(csv.DictReader(open(f[-1])))
acc = collections.defaultdict(list)
for r in rows:
    if "fft_" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1], {k: round(sum(v)/len(v)) for k, v in acc.items()})
PY
  rm -rf gpurun_out/pmc_$k
 done
done
