set -o pipefail
# A/B: resident hand-off by tagged granules (libcfd_amd.so) vs drained bands +
# flags (libcfd_amd_old.so); parity first on the new build.
D=gpurun_out/gran; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for c in "cavity --nx 1024" "channel --nx 4096 --ny 512"; do
  n=${c%% *}
  for o in rb lex; do
    for lib in new old new old; do
      if [ $lib = old ]; then L=libcfd_amd_old.so; else L=libcfd_amd.so; fi
      CFD_AMD_LIB=$L timeout -k 10 200 python -u bench.py --case $c --ordering $o --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/$n$o$lib.json 2> $D/$n$o$lib.err || { tail $D/$n$o$lib.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/$n$o$lib.json')); r=d['roofline']; print('$n $o $lib', round(d['value']), d['ms_per_step'], r.get('avg_launch_us'))"
    done
  done
done
CFD_AMD_LIB=libcfd_amd_rstamps.so timeout -k 10 200 python -u scripts/dbg/res_stamps.py 1024 1024 10000 cavity rb > $D/stamps_rb.json 2>&1 || { tail $D/stamps_rb.json; exit 1; }
python3 -c "import json; d=json.load(open('$D/stamps_rb.json')); print({k: v for k, v in d.items() if 'by_wave' in k or k.startswith('us_')})"
