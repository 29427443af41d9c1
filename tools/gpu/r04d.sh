#!/bin/bash
# r04: SLP (packed f32) A/B — halo stamps and the whole bench with the library built -fno-slp-vectorize
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
for v in slp noslp; do
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"build\": \"$v\", \"r\": " >> $O/halo_slp.jsonl
    timeout -k 5 60 tools/halo_stamps_$v $cfg >> $O/halo_slp.jsonl 2>> $O/halo_slp.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo_slp.jsonl
  done
done
cat $O/halo_slp.jsonl
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_halo_conv_gpu.py > $O/pytest.log 2>&1 || { echo "halo tests failed"; tail -30 $O/pytest.log; exit 4; }
for rep in 1 2; do
  for v in default noslp; do
    if [ $v = noslp ]; then export RDEIC_LIB=$PWD/rdeic_amd/lib_noslp/librdeic_hip.so; else unset RDEIC_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -20 $O/bench_${v}_$rep.err; exit 5; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));r=d['roofline'];print('$v', $rep, d['value'], d['ms_per_step'], r['achieved'], r['secondary'].get('attention',{}).get('achieved'))"
  done
done
