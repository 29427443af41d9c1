#!/bin/bash
# r06 first call: the GPU suite and smoke on the cleaned-up library, then a same-box A/B against the r05
# library (ab/r05: the r05 tree's package + its own build) — bench at the driver's counts, alternating, and
# layer_times once each.
# usage (repo root on the box): bash tools/gpu/r06a.sh TAG
set -o pipefail
TAG=${1:-r06a}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 6; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/new$i.json 2> $O/new$i.err || { echo "bench new$i failed"; tail -20 $O/new$i.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/new$i.json'));r=d['roofline'];print('new$i', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
  (cd ab/r05 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/r05_$i.json 2> $O/r05_$i.err) || { echo "bench r05_$i failed"; tail -20 $O/r05_$i.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/r05_$i.json'));r=d['roofline'];print('r05_$i', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done
timeout -k 10 300 python -u tools/layer_times.py > $O/layer_times_new.txt 2> $O/lt_new.err || { echo "layer_times new failed"; tail -20 $O/lt_new.err; exit 7; }
(cd ab/r05 && timeout -k 10 300 python -u tools/layer_times.py > $O/layer_times_r05.txt 2> $O/lt_r05.err) || { echo "layer_times r05 failed"; tail -20 $O/lt_r05.err; exit 7; }
head -12 $O/layer_times_new.txt
head -12 $O/layer_times_r05.txt
