STEPS=test bash scripts/gpu_check.sh r01g
for k in wide narrow; do echo "== KERNEL $k"; RFA_KERNEL=$k timeout -k 10 120 python scripts/kbench.py --sizes 8192,16384,65536 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/exp_r01g.txt 2>&1
cat gpurun_out/exp_r01g.txt
