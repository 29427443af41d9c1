# One GPU call: the GPU tests (failures reported, not fatal), then the bench line, then optional
# per-layer conv profile. Stops at the first fault / abort / timeout (exit codes >= 124 or 134/139).
# usage (repo root on the box): bash tools/gpu_check.sh TAG [pytest-args...]
TAG=${1:-check}
shift || true
O=$PWD/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
cat $O/bench.json
if [ $rc -ne 0 ]; then tail -20 $O/bench.err; echo "bench exit $rc"; exit $rc; fi
