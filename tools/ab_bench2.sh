# A/B of bench variants on one box (alternating), short runs: bash tools/ab_bench2.sh TAG "flagsA" "flagsB"
O=$PWD/gpurun_out/${1:-ab}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fp32-steps 0 $2 > $O/a$i.json 2> $O/a$i.err || exit $?
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fp32-steps 0 $3 > $O/b$i.json 2> $O/b$i.err || exit $?
  python -c "import json;a=json.load(open('$O/a$i.json'));b=json.load(open('$O/b$i.json'));print('A',a['value'],a['roofline']['ms_per_step'],'B',b['value'],b['roofline']['ms_per_step'])"
done
