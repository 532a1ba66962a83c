set -o pipefail
# A/B: resident groups of 6 sweeps (12-cell halos; libcfd_amd_ns6.so) vs 4
D=gpurun_out/ns6; mkdir -p $D
CFD_AMD_LIB=libcfd_amd_ns6.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py > $D/tests.log 2>&1
tail -15 $D/tests.log | cut -c1-200
for c in "cavity --nx 1024 --ny 1024" "channel --nx 4096 --ny 512"; do
  n=${c%% *}
  for o in lex rb; do
    for lib in ns6 ns4 ns6 ns4; do
      if [ $lib = ns4 ]; then L=libcfd_amd.so; else L=libcfd_amd_ns6.so; fi
      CFD_AMD_LIB=$L timeout -k 10 200 python -u bench.py --case $c --ordering $o --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/$n$o$lib.json 2> $D/$n$o$lib.err || { tail $D/$n$o$lib.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/$n$o$lib.json')); r=d['roofline']; print('$n $o $lib', round(d['value']), d['ms_per_step'], r.get('kernel'), r.get('us_per_sweep'), d.get('proof_fallbacks'))"
    done
  done
done
