"""The sharded codec loop of bench.py / SURVEY.md §8e on the device: two ranks on ONE GPU (two
processes, gloo for the collective so they can share the card), a global batch of 3 images split
2 + 1 by parallel.shard. Each rank codes its contiguous shard end to end; ONE metric all-gather
returns the rows in global image order. Every rank's bodies must equal the single-process batch's
(the entropy model is batch-invariant), the reconstructions must agree, and
the gathered rows must match the bodies' sizes."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SIZE, G, WORLD = 128, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(g0, g1):
    from rdeic_amd.synthetic import relay_noise, synth_image
    imgs = torch.from_numpy(np.stack([synth_image(SIZE, SIZE, 231 + g) for g in range(g0, g1)]))
    noise = torch.cat([relay_noise((1, 4, SIZE // 8, SIZE // 8), 231 + g, 2)[0] for g in range(g0, g1)])
    return imgs, noise


def _rank(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                          LOCAL_RANK="0")  # both ranks on the one visible GPU
        from rdeic_amd import parallel
        from rdeic_amd.rdeic import RDEIC
        from rdeic_amd.synthetic import synth_context
        r, w, _ = parallel.init_from_env(backend="gloo")
        torch.cuda.set_device(0)
        g0, g1 = parallel.shard(G, r, w)
        imgs, noise = _inputs(g0, g1)
        m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
        out, bodies = m.codec_images(imgs.cuda(), synth_context().cuda(), noise, steps=2)
        rows = torch.tensor([[8.0 * len(b) / SIZE ** 2, float(len(b)), float(g), float(r)]
                             for g, b in zip(range(g0, g1), bodies)], dtype=torch.float32)
        gathered = parallel.gather_metrics(rows, G)
        q.put((r, bodies, out.cpu().numpy(), gathered.numpy()))
        parallel.finish()
    except Exception as e:  # surface the failure in the parent instead of a queue timeout
        q.put((rank, f"{type(e).__name__}: {e}", None, None))
        raise


def test_two_rank_sharded_codec_matches_single_process(gpu):
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, bodies, out, gathered = q.get(timeout=240)
        assert not isinstance(bodies, str), f"rank {r}: {bodies}"
        res[r] = (bodies, out, gathered)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, whole global batch
    imgs, noise = _inputs(0, G)
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    out_all, bodies_all = m.codec_images(imgs.cuda(), synth_context().cuda(), noise, steps=2)
    out_all = out_all.cpu().numpy()
    from rdeic_amd import parallel
    for r in range(WORLD):
        g0, g1 = parallel.shard(G, r, WORLD)
        bodies, out, gathered = res[r]
        assert bodies == bodies_all[g0:g1]
        # pixels: bit for bit — the split-K count is chosen per image (ops.SPLITK_NOMINAL_BATCH) and
        # every other kernel's reduction order is per image, so a shard decodes exactly as in the batch
        d = np.abs(out.astype(int) - out_all[g0:g1].astype(int))
        print(f"rank {r}: pixels identical to the single-process batch: {not d.any()} (max |d| {d.max()})")
        assert not d.any()
        assert gathered.shape == (G, 4)
        assert gathered[:, 2].tolist() == list(range(G))  # global image order
        assert gathered[:, 1].tolist() == [float(len(b)) for b in bodies_all]
        assert gathered[:, 3].tolist() == [float(o) for o in range(WORLD) for _ in range(*parallel.shard(G, o, WORLD))]


def _nccl_rank(port, q):
    try:
        import torch.distributed as dist
        from rdeic_amd import parallel
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        torch.cuda.set_device(0)
        dist.init_process_group(backend="nccl")  # RCCL on ROCm
        dev = torch.device("cuda", 0)
        rows = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
        out = torch.empty_like(rows)
        dist.all_gather_into_tensor(out, rows)  # the metric gather's collective, on RCCL
        t = torch.tensor([2.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
        g = torch.ones(1000, device=dev)
        h = dist.all_reduce(g, async_op=True)  # GradBuckets' async bucket all-reduce
        h.wait()
        parallel.barrier(dev)
        q.put((torch.equal(out, rows), float(t.item()), float(g.sum().item()), dist.get_backend()))
        dist.destroy_process_group()
    except Exception as e:
        q.put((False, f"{type(e).__name__}: {e}", 0.0, None))


def test_rccl_collectives_single_rank(gpu):
    """The RCCL ("nccl") process group the multi-GPU bench / fine-tune use, exercised on the one
    visible GPU (RCCL refuses two ranks on one device, so the two-rank tests above use gloo): the
    metric all_gather_into_tensor, the timing all_reduce(MAX), an async all_reduce and the device
    barrier run and return the identity results at world size 1."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_rank, args=(_free_port(), q))
    p.start()
    ok, t, s, backend = q.get(timeout=180)
    p.join(timeout=60)
    assert ok is True, t
    assert t == 2.5 and s == 1000.0 and backend == "nccl"
    assert p.exitcode == 0
