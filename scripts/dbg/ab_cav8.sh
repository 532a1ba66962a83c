set -o pipefail
# A/B: the cavity's reference-order resident groups of 8 sweeps (libcfd_amd_cav8.so) vs 6
D=gpurun_out/cav8; mkdir -p $D
CFD_AMD_LIB=libcfd_amd_cav8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py -k "lex" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for lib in cav8 ns6 cav8 ns6; do
  if [ $lib = ns6 ]; then L=libcfd_amd.so; else L=libcfd_amd_cav8.so; fi
  CFD_AMD_LIB=$L timeout -k 10 200 python -u bench.py --case cavity --nx 1024 --ny 1024 --ordering lex --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/$lib.json 2> $D/$lib.err || { tail $D/$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$lib.json')); r=d['roofline']; print('$lib', round(d['value']), d['ms_per_step'], r.get('us_per_sweep'), r.get('kernel'))"
done
