# bench throughput vs codec sessions in flight (same box)
O=$PWD/gpurun_out/${1:-streams}
mkdir -p $O
for s in ${STREAMS:-3 4 2 3 4}; do
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --fp32-steps 0 --no-roofline --streams $s > $O/s$s.json 2> $O/s$s.err || exit $?
  python -c "import json;a=json.load(open('$O/s$s.json'));print('streams',$s,a['value'],a['ms_per_step'])"
done
