STEPS=test bash scripts/gpu_check.sh r01d
for m in 14 13; do echo "== MAX_LOGM $m"; RFA_MAX_LOGM=$m timeout -k 10 120 python scripts/kbench.py --sizes 16384,32768,65536 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/exp_r01d.txt 2>&1
cat gpurun_out/exp_r01d.txt
