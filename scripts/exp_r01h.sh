STEPS=test bash scripts/gpu_check.sh r01h
for k in wide narrow; do echo "== KERNEL $k"; RFA_KERNEL=$k timeout -k 10 120 python scripts/kbench.py --sizes 8192,16384,65536 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/exp_r01h.txt 2>&1
cat gpurun_out/exp_r01h.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_h -o p -- python3 scripts/kbench.py --sizes 16384 --formats s8 --iters 3 > /dev/null 2>&1
python3 -c "
import csv,glob,collections
f=sorted(glob.glob('gpurun_out/pmc_h/**/*counter_collection.csv',recursive=True))[-1]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'fft_' in r['Kernel_Name']: acc[r['Counter_Name']].append(float(r['Counter_Value']))
print({k: round(sum(v)/len(v)) for k,v in acc.items()})"
rm -rf gpurun_out/pmc_h
