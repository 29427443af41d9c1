# Config-3 line on the current tree, then the codec-session A/B (same box).
O=$PWD/gpurun_out/${1:-final_extra}
mkdir -p $O
timeout -k 10 600 python -u bench.py --size 1024 --ddim-steps 5 --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/config3.json 2> $O/config3.err || { echo "config3 failed"; tail -5 $O/config3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/config3.json').read().strip().splitlines()[-1]); print('config3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['secondary'].get('attention_d512'))"
STREAMS="4 6 8 4 6 8" bash tools/streams_ab.sh ${1:-final_extra}/streams
