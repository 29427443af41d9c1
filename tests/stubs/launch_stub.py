"""Stub worker for tests/test_launch_cpu.py: the same `--gpus N` entry as bench.py (rdeic_amd.launch),
with a gloo all-gather in place of the GPU step. Rank 0 prints ONE JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--fail-rank", type=int, default=-1)
    args = ap.parse_args()
    from rdeic_amd.launch import maybe_launch
    maybe_launch(args.gpus, __file__, require_gpus=False)
    import torch
    import torch.distributed as dist
    from rdeic_amd import parallel
    rank, world, local = parallel.init_from_env(backend="gloo")
    if rank == args.fail_rank:
        raise SystemExit(3)
    rows = torch.tensor([[float(rank), float(local), float(os.environ["LOCAL_WORLD_SIZE"])]])
    allr = parallel.gather_metrics(rows, world)
    parallel.finish()
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": allr[:, 0].int().tolist(),
                          "local_ranks": allr[:, 1].int().tolist(), "lws": allr[:, 2].int().tolist()}), flush=True)


if __name__ == "__main__":
    main()
