run() { echo "== $*"; env "$@" timeout -k 10 120 python scripts/kbench.py --sizes 16384,65536 --iters 10 2>&1 | grep -v amdgpu.ids; }
{ run RFA_PERSIST=0
  run RFA_PERSIST=2 RFA_STAGGER_NS=0
  run RFA_PERSIST=2 RFA_STAGGER_NS=3000
  run RFA_PERSIST=2 RFA_STAGGER_NS=6000
  run RFA_PERSIST=2 RFA_STAGGER_NS=10000
  run RFA_PERSIST=1
} > gpurun_out/exp_stagger.txt 2>&1
cat gpurun_out/exp_stagger.txt
