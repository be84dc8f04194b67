set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 ./tools/call_bench 4000 1 > gpurun_out/r05a_call1.json 2>&1 && cat gpurun_out/r05a_call1.json &&
timeout -k 10 300 ./tools/call_bench 100 64 > gpurun_out/r05a_call64.json 2>&1 && cat gpurun_out/r05a_call64.json &&
timeout -k 10 600 python -u bench.py --cpu-seconds 3 > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err && tail -c 600 gpurun_out/r05a_bench.json &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_pytest.txt 2>&1; tail -5 gpurun_out/r05a_pytest.txt
