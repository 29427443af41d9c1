#!/bin/bash
# r04: full GPU suite + smoke + bench on the current tree, then the sp3 A/B
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 6; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 5; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('algorithmic_bytes_per_launch'), r.get('traffic_over_algorithmic'), d['fp32_parity_mode'])"
bash tools/gpu/r04j.sh
