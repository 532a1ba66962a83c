set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full2.log 2>&1 || { tail -30 gpurun_out/full2.log; exit 1; }
tail -2 gpurun_out/full2.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || { cat gpurun_out/smoke2.log; exit 1; }
cat gpurun_out/smoke2.log
