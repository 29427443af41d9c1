"""CPU pieces of the adapter fine-tune step (config 5): the AdamW restatement against torch and the
reference's golden step, the training draws, and the bucketed DDP gradient all-reduce on gloo."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

GOLD = os.path.join(os.path.dirname(__file__), "golden", "train_128.npz")


def test_adamw_restatement_matches_torch():
    from oracle import train_ref
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(1000, generator=g)
    grads = [torch.randn(1000, generator=g) * 10 ** torch.empty(1000).uniform_(-9, 1, generator=g) for _ in range(3)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=2e-5)
    ours, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    for step, gr in enumerate(grads, 1):
        ref.grad = gr.clone()
        opt.step()
        train_ref.adamw_step([ours], [gr], [m], [v], step, 2e-5)
        assert torch.equal(ours, ref.detach()), step


def test_golden_adamw_pinned_by_restatement():
    """The fixture's AdamW-updated tensors follow from its initial synthetic weights and its gradients
    through the restated update (bit for bit): the step the GPU test checks is the reference's."""
    from oracle import train_ref, weights_cpu
    from rdeic_amd import weights as W
    d = np.load(GOLD)
    checked = 0
    for k in d.files:
        if not k.startswith("grad:"):
            continue
        n = k[5:]
        shape = d[k].shape
        scale, offset = W.init_spec(n, shape)
        p = torch.from_numpy(weights_cpu.fill_uniform(int(np.prod(shape)), W.param_seed(n), scale, offset)).view(shape)
        g = torch.from_numpy(d[k])
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        train_ref.adamw_step([p], [g], [m], [v], 1, 2e-5)
        assert np.array_equal(p.numpy(), d["after_adamw:" + n]), n
        checked += 1
    assert checked >= 8


def test_training_draws_match_fixture():
    from rdeic_amd.config import CONFIG
    from rdeic_amd.synthetic import train_draws
    d = np.load(GOLD)
    dr = train_draws(1, 16, 16, CONFIG["compression"]["slice_ch"], 5, CONFIG["used_timesteps"])
    assert np.array_equal(dr["t"].numpy(), d["t"])
    assert np.array_equal(dr["post_eps"].numpy(), d["post_eps"])
    assert np.array_equal(dr["noise"].numpy(), d["noise"])
    for i, s in enumerate(dr["slice_noise"]):
        assert np.array_equal(s.numpy(), d[f"slice_noise{i}"])
        assert s.min() >= -0.5 and s.max() < 0.5


def test_golden_loss_is_the_sum_of_its_terms():
    d = np.load(GOLD)
    total = 3.0 * d["loss_l_simple"] + d["loss_l_bpp"] + d["loss_l_emb"] + 3.0 * d["loss_l_guide"]
    assert abs(total - d["loss_loss"]) < 1e-5 * abs(d["loss_loss"])
    assert len(d["grad_names"]) == 663 and np.all(np.isfinite(d["grad_proj"]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    try:
        import torch.distributed as dist
        from rdeic_amd.parallel import GradBuckets
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        shapes = [(7, 5), (300,), (64, 3, 3), (11,), (2000,), (3, 3)]
        total = sum(int(np.prod(s)) for s in shapes)
        flat, grad = torch.zeros(total), torch.zeros(total)
        params, off = [], 0
        g = torch.Generator().manual_seed(123)
        for s in shapes:
            k = int(np.prod(s))
            flat[off:off + k] = torch.randn(k, generator=g)
            p = flat[off:off + k].view(s)
            p.requires_grad_(True)
            p.grad = grad[off:off + k].view(s)
            params.append((p, off, k))
            off += k
        # ~1.2 KB buckets: several buckets, launched from the hooks while the backward runs
        gb = GradBuckets(grad, params, bucket_bytes=1200)
        coef = [torch.randn(p.shape, generator=g) for p, _, _ in params]
        for step in range(3):
            grad.zero_()
            gb.begin()
            if step < 2:
                loss = sum(((rank + 1 + step) * c * p * p).sum() for c, (p, _, _) in zip(coef, params))
                loss.backward()
            else:
                # step 2: every parameter gets its gradient from its own backward, in a rank-dependent
                # order, so the buckets complete in a different order on each rank; the collectives
                # must still be issued in bucket order on both (a mismatch would pair wrong buckets)
                order = list(range(len(params)))
                rng = np.random.default_rng(rank + 7)
                rng.shuffle(order)
                for i in order:
                    c, (p, _, _) = coef[i], params[i]
                    ((rank + 1 + step) * c * p * p).sum().backward()
            gb.finish()
            assert gb.launch_order == list(range(len(gb.buckets))), gb.launch_order
            expect = torch.cat([(sum(r + 1 + step for r in range(world)) / world * 2 * c * p.detach()).reshape(-1)
                                for c, (p, _, _) in zip(coef, params)])
            q.put((rank, step, float((grad - expect).abs().max()), len(gb.buckets)))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, -1, f"{type(e).__name__}: {e}", 0))
        raise


def test_bucketed_grad_allreduce_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(3 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, step, err, nb in res:
        assert step >= 0, err
        assert err < 1e-5, (rank, step, err)
        assert nb > 3


def test_precision_16_refused():
    """Lightning's precision 16 is fp16 autocast, which the step does not implement: refused rather
    than silently trained in bf16 (train.py)."""
    import train
    with pytest.raises(SystemExit):
        train.precision_dtype(16)
    assert train.precision_dtype("bf16") == torch.bfloat16 and train.precision_dtype(32) == torch.float32
