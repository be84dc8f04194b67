STEPS=test bash scripts/gpu_check.sh r01e
for k in wide narrow; do echo "== KERNEL $k"; RFA_KERNEL=$k timeout -k 10 120 python scripts/kbench.py --sizes 8192,16384,32768,65536,131072 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/exp_r01e.txt 2>&1
cat gpurun_out/exp_r01e.txt
