set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python3 -u tools/halo256_ab.py 3 > $O/halo256_ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/halo256_ab.txt; exit 4; }
cat $O/halo256_ab.txt
timeout -k 10 300 python3 -u tools/layer_times.py --json $O/layer_times.json > $O/layer_times.txt 2>&1 || { echo "layer times failed"; tail -20 $O/layer_times.txt; exit 5; }
head -45 $O/layer_times.txt
for v in 1 0 1 0; do
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 --no-roofline --conv-option 10=$v > $O/bench_h256_$v.json 2>> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 6; }
python3 -c "import json;d=json.load(open('$O/bench_h256_$v.json'));print('halo256=$v', d['value'], d['ms_per_step'])"
done
