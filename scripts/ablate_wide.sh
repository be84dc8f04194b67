for d in 0 1 2 3 16 19 4 8 12 31; do echo "== DIAG $d"; RFA_DIAG=$d timeout -k 10 120 python scripts/kbench.py --sizes 16384 --formats s8 --iters 10 2>&1 | grep -v amdgpu.ids || break; done > gpurun_out/ablate_wide.txt 2>&1
cat gpurun_out/ablate_wide.txt
