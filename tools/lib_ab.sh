# Same-box A/B/C of three builds of librdeic_hip.so (RDEIC_LIB): halo_diag per build, then the
# bench in alternating rounds.
# usage: bash tools/lib_ab.sh TAG LIB_A LIB_B LIB_C [rounds]
O=$PWD/gpurun_out/${1:-lib_ab}
N=${5:-2}
mkdir -p $O
for T in A B C; do
  case $T in A) F=$2;; B) F=$3;; C) F=$4;; esac
  RDEIC_LIB=$PWD/$F timeout -k 10 200 python -u tools/halo_diag.py > $O/diag_$T.log 2>&1 || { echo "diag $T failed"; tail -5 $O/diag_$T.log; exit 1; }
  echo "diag $T"; grep -v amdgpu.ids $O/diag_$T.log
done
for i in $(seq 1 $N); do
  for T in A B C; do
    case $T in A) F=$2;; B) F=$3;; C) F=$4;; esac
    RDEIC_LIB=$PWD/$F timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/$T$i.json 2> $O/$T$i.err || { echo "bench $T$i failed"; tail -5 $O/$T$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$T$i.json').read().strip().splitlines()[-1]); print('$T$i', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'], d['roofline']['frac'])"
  done
done
