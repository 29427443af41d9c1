#!/bin/bash
# r06: edge-conv micro A/B, tests, then SQ counters of the edge kernels
set -o pipefail
TAG=${1:-r06i}
bash tools/gpu/r06e.sh $TAG && timeout -k 10 400 bash tools/pmc_edge.sh ${TAG}_pmc > gpurun_out/${TAG}_pmc.log 2>&1; rc=$?; tail -60 gpurun_out/${TAG}_pmc.log; exit $rc
