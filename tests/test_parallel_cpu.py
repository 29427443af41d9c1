"""Data-parallel plumbing (rdeic_amd/parallel.py) on CPU with gloo, world_size 2: shards cover
the global batch exactly once, the metric all-gather returns every rank's rows in global image
order (unequal shards included),
and the timing reduction takes the max over ranks (bench.py's contract)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from rdeic_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, G):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, _ = parallel.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    s, e = parallel.shard(G, r, w)  # unequal shards when world does not divide G
    rows = torch.tensor([[float(i), float(r)] for i in range(s, e)], dtype=torch.float32)
    g = parallel.gather_metrics(rows, G)
    t = parallel.max_over_ranks(1.0 + r, torch.device("cpu"))
    parallel.barrier()
    q.put((r, g.tolist(), t))
    parallel.finish()


@pytest.mark.parametrize("world,G", [(2, 11), (3, 11), (3, 16)])
def test_gloo_gather_and_max(world, G):
    """G=16 on 3 ranks: config 4's uneven shards (6/5/5), the bench's --global-batch path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, G)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, g, t in res:
        assert t == float(world)
        ids = [row[0] for row in g]
        assert ids == list(range(G))  # global image order, padding dropped
        owners = [int(row[1]) for row in g]
        assert owners == [r for r in range(world) for _ in range(*parallel.shard(G, r, world))]


def test_shard_partition():
    for world in (1, 2, 3, 4, 8):
        for n in (1, 7, 16, 128):
            spans = [parallel.shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
