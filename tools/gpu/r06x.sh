#!/bin/bash
# r06: runtime settings on the dispatch-bound config-5 step (captured hipGraph), alternating on one box
set -o pipefail
TAG=${1:-r06x}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for v in base kernarg pcap both; do
    case $v in
      base) E="";;
      kernarg) E="HIP_FORCE_DEV_KERNARG=1";;
      pcap) E="DEBUG_CLR_GRAPH_PACKET_CAPTURE=1";;
      both) E="HIP_FORCE_DEV_KERNARG=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1";;
    esac
    env $E timeout -k 10 300 python -u bench_train.py --dtype bf16 --no-roofline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "ft $v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$v $rep', d['value'], d['ms_per_step'])"
  done
done
