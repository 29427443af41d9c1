# Same-box A/B/C of three conv tile tables on the bench, alternating rounds.
# usage: bash tools/table_ab3.sh TAG TABLE_A TABLE_B TABLE_C [rounds]
O=$PWD/gpurun_out/${1:-table_ab3}
N=${5:-3}
mkdir -p $O
for i in $(seq 1 $N); do
  for T in A B C; do
    case $T in A) F=$2;; B) F=$3;; C) F=$4;; esac
    RDEIC_TILE_TABLE=$F timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/$T$i.json 2> $O/$T$i.err || { echo "bench $T$i failed"; tail -5 $O/$T$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$T$i.json').read().strip().splitlines()[-1]); print('$T$i', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'], d['roofline']['frac'])"
  done
done
