#!/bin/bash
# r04: every LDS-DMA tile on the UNet transformer linears (graph-replayed, per-launch us / TF / GB/s)
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 400 python -u tools/lin_bench.py > $O/lin.jsonl 2> $O/lin.err || { echo "lin_bench failed"; tail -20 $O/lin.err; exit 3; }
cat $O/lin.jsonl
