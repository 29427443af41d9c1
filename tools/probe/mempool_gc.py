"""Probe: does freeing a tensor after its torch MemPool was destroyed abort the process?
(Root cause check for the round-1 driver abort: a cyclic-GC pass destroyed a LaunchPlan's pool
before the plan's tensors.)  usage: python tools/probe/mempool_gc.py {pool_first|tensor_first}"""
import sys

import torch

order = sys.argv[1] if len(sys.argv) > 1 else "pool_first"
pool = torch.cuda.MemPool()
with torch.cuda.use_mem_pool(pool):
    t = torch.empty(1 << 20, device="cuda")
torch.cuda.synchronize()
if order == "pool_first":
    del pool
    print("pool destroyed with a live tensor", flush=True)
    del t
else:
    del t
    del pool
print("survived", order, flush=True)
