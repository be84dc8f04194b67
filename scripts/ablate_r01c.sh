STEPS=test bash scripts/gpu_check.sh r01c
for d in 0 1 2 3 4 6 7; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 16384,65536 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/ablate_r01c.txt 2>&1
cat gpurun_out/ablate_r01c.txt
timeout -k 10 200 python scripts/kbench.py --sizes 256,1024,4096,8192,16384,32768,65536,131072 --formats s8,f32 > gpurun_out/kbench_r01c.txt 2>&1; cat gpurun_out/kbench_r01c.txt
