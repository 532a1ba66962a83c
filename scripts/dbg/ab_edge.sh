set -o pipefail
# A/B: channel resident solve with a ghost-column-only sweep variant (new,
# libcfd_amd.so) against the ghost-row variant for every edge tile (old,
# libcfd_amd_old.so); parity first on the new build.
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py > gpurun_out/abe_tests.log 2>&1 || { tail -30 gpurun_out/abe_tests.log; exit 1; }
tail -2 gpurun_out/abe_tests.log
for o in lex rb; do
  for lib in new old new old; do
    if [ $lib = old ]; then L=libcfd_amd_old.so; else L=libcfd_amd.so; fi
    CFD_AMD_LIB=$L timeout -k 10 200 python -u bench.py --case channel --nx 4096 --ny 512 --ordering $o --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > gpurun_out/abe_$o$lib.json 2> gpurun_out/abe_$o$lib.err || { tail gpurun_out/abe_$o$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abe_$o$lib.json')); r=d['roofline']; print('$o $lib', d['value'], d['ms_per_step'], r.get('kernel'), r['avg_launch_us'], r['frac'])"
  done
done
