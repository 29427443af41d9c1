"""Stub worker for tests/test_launch_cpu.py: bench.py's own argument parser, `--gpus N` launch, global-batch
sharding, sweep points and per-point result handling (bench.sweep_points / bench.run_sweep), with a gloo
all-gather of per-image rows in place of the GPU codec step. Rank 0 prints ONE JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench
    args = bench.parse()
    from rdeic_amd.launch import maybe_launch
    maybe_launch(args.gpus, __file__, require_gpus=False)
    import torch
    from rdeic_amd import parallel
    rank, world, local = parallel.init_from_env(backend="gloo")
    G = args.global_batch if args.global_batch is not None else args.batch * world
    g0, g1 = parallel.shard(G, rank, world)
    points, main_i = bench.sweep_points(args)

    def measure(i, target, rate_gain, headline):
        # one row per image of this rank's shard: (global image index, rank, point, target bpp)
        rows = torch.tensor([[float(g), float(rank), float(i), float(target or 0.0)] for g in range(g0, g1)])
        allr = parallel.gather_metrics(rows, G)
        return {"target_bpp": target, "rate_gain": rate_gain, "rows": allr, "out": torch.zeros(g1 - g0),
                "images": int(allr.shape[0])}

    results = bench.run_sweep(points, main_i, measure)
    parallel.finish()
    if rank == 0:
        head = results[main_i]["rows"]
        print(json.dumps({
            "n_gpus": world, "global_batch": G, "main_i": main_i,
            "targets": [p[0] for p in points], "rate_gains": [p[1] for p in points],
            "images_per_point": [r["images"] for r in results],
            "image_order": head[:, 0].int().tolist(), "rank_of_image": head[:, 1].int().tolist(),
            "out_kept": [r["out"] is not None for r in results]}), flush=True)


if __name__ == "__main__":
    main()
