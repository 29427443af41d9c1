"""Adapter fine-tune step (config 5, §8f rank 1) against the reference's own autograd.

tests/golden/train_128.npz and train_512.npz (config 5's own size) hold one step of the REFERENCE modules (UNetModel frozen, NoiseEstimator,
Compression in training mode, VAE encoder; torch autograd, fp32, CPU; tests/golden/make_train_golden.py)
at 128x128 with the same synthetic weights and seeded draws. The HIP path runs the same step in fp32
parity mode through the C ABI (forward and backward kernels) and must reproduce:
  * the forward intermediates (x_start, h, c_latent, guide_hint, x_noisy, eps) and every loss term;
  * the gradient of every one of the 663 trainable tensors (76.7M parameters): norm and 4 seeded
    random projections within TOL_BY_SIZE of the reference gradient's norm, and within TOL64 of the
    float64 truth (train_{size}_f64.npz: the reference modules run in float64);
  * the VQ codebook re-initialisation (embed_prob, row sums of the updated codebook);
  * the AdamW update (full tensors of a few layers).
Tolerances are fp32 summation-order bounds (different reduction trees than torch's CPU kernels)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = "tests/golden/train_{}.npz"
GOLD64 = "tests/golden/train_{}_f64.npz"
TOL = 2e-3
# Gradients against the reference's fp32 result: an fp32 summation-order bound. At 512^2 it is not a
# tight check: the same step run through the reference modules in float64 (make_train_golden.py 512 f64,
# r05) shows that the reference's OWN fp32 gradients sit up to 1.8e-3 of the norm from the float64 truth
# on the hyperprior / encoder tensors (the bpp-gradient path; hyper_dec.0.subpel_conv.0.weight 1.8e-3,
# hyper_dec.0.upsample.0.weight 1.6e-3), so two independent fp32 results differ by up to ~2 x that
# (measured r04: 2.36e-3 on hyper_dec.0.upsample.0.weight). The 512^2 bar is therefore set against the
# float64 truth (TOL64), where ours measure 5.7e-5 (128^2) and 1.71e-3 (512^2) at worst (r05,
# tools/grad_dump.py): >= 3x margin, and our worst may not exceed the reference fp32's own worst by > 1.5x
# (512^2: 1.71e-3 against 1.81e-3).
TOL_BY_SIZE = {128: 2e-3, 512: 5e-3}    # vs the fp32 golden: two independent fp32 results (worst 2.36e-3, ~2.1x)
TOL64 = {128: 2e-4, 512: 5.5e-3}        # vs the float64 truth (worst 5.7e-5 / 1.71e-3)
REL_FLOOR = {128: 1e-4, 512: 0.0}       # ours-vs-reference accuracy bar floor (both ~1e-5 at 128^2)


# 128^2 (fast) and config 5's own 512^2 (train.py:10-28, configs/finetune_ood.yaml: out_size 512)
@pytest.fixture(scope="module", params=[128, 512])
def step(request):
    from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    size = request.param
    g = np.load(GOLD.format(size))
    m = RDEIC(compute_dtype=torch.float32).init_synthetic()
    ft = FineTuner(m)
    dr = train_draws(1, size // 8, size // 8, m.cfg["compression"]["slice_ch"], 5, m.used_timesteps)
    assert np.array_equal(dr["t"].numpy(), g["t"]) and np.array_equal(dr["noise"].numpy(), g["noise"])
    img = torch.from_numpy(synth_image(size, size, 231)).cuda()[None]
    ctx = synth_context().cuda()
    d = nchw_draws_to_nhwc(dr, "cuda")
    ft.zero_grad()
    x_start, h = ft.get_first_stage(img, d["post_eps"])
    loss, ld = ft.losses(x_start, h, ctx, d["t"], d["noise"], d["slice_noise"])
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: ft.grad[o:o + k].cpu() for n, (o, k) in ft.offsets.items()}
    E_after_fwd = ft.p("preprocess_model.quantize.embedding.weight").detach().double().cpu()
    ep = ft.embed_prob.cpu()
    ft.optimizer_step()
    torch.cuda.synchronize()
    params = {n: ft.flat[o:o + k].cpu() for n, (o, k) in ft.offsets.items()}
    fw = dict(x_start=x_start, h=h, **ft._last)
    sub = int(g["subsample"]) if "subsample" in g.files else 1  # train_512.npz: stride-4 pixel grid
    fw = {k: v.detach().permute(0, 3, 1, 2).float().cpu().numpy()[:, :, ::sub, ::sub] for k, v in fw.items()}
    return dict(size=size, g=g, ft=ft, ld={k: float(v.detach()) for k, v in ld.items()}, grads=grads, params=params, fw=fw,
                E_after_fwd=E_after_fwd, ep=ep)


def _close(a, b, rtol, name):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
    assert err < rtol, f"{name}: max rel err {err:.3e}"


def test_forward_intermediates(step):
    g, fw = step["g"], step["fw"]
    _close(fw["x_start"], g["x_start"], 1e-4, "x_start")
    _close(fw["h"], g["h"], 1e-4, "h")
    _close(fw["guide_hint"], g["guide_hint"], 1e-3, "guide_hint")
    _close(fw["c_latent"], g["c_latent"], 1e-3, "c_latent")
    _close(fw["x_noisy"], g["x_noisy"], 1e-3, "x_noisy")
    _close(fw["eps"], g["eps"], 1e-3, "eps")


def test_loss_terms(step):
    g, ld = step["g"], step["ld"]
    for ours, ref in (("T/loss", "loss_loss"), ("T/l_simple", "loss_l_simple"), ("T/l_bpp", "loss_l_bpp"),
                      ("T/q_bpp", "loss_q_bpp"), ("T/l_emb", "loss_l_emb"), ("T/l_guide", "loss_l_guide")):
        r = float(g[ref])
        assert abs(ld[ours] - r) <= 1e-4 * max(abs(r), 1e-3), (ours, ld[ours], r)


def test_vq_codebook_update(step):
    g = step["g"]
    _close(step["ep"].numpy(), g["vq_embed_prob"], 1e-5, "embed_prob")
    _close(step["E_after_fwd"].sum(1).numpy(), g["vq_E_after_fwd_rowsum"], 1e-4, "re-initialised codebook")


def test_gradients_of_every_trainable_tensor(step):
    from tests.golden.train_proj import projections
    g, grads = step["g"], step["grads"]
    names = [str(n) for n in g["grad_names"]]
    assert sorted(names) == sorted(grads), "trainable tensor set differs from the reference's"
    bad = []
    for i, n in enumerate(names):
        gr = grads[n]
        ref_norm = float(g["grad_norm"][i])
        norm = float(gr.double().norm())
        if ref_norm == 0.0:
            if norm != 0.0:
                bad.append((n, "nonzero", norm))
            continue
        pr = projections(n, gr)
        err = max(abs(norm - ref_norm), np.abs(pr - g["grad_proj"][i]).max()) / ref_norm
        if err > TOL_BY_SIZE[step["size"]]:
            bad.append((n, err, ref_norm))
    assert not bad, f"{len(bad)} / {len(names)} gradients off: {bad[:10]}"
    for k in g.files:
        if k.startswith("grad:"):
            n = k[5:]
            _close(grads[n].numpy().reshape(g[k].shape), g[k], TOL_BY_SIZE[step["size"]], k)


def _err(norm, proj, n64, p64):
    return max(abs(norm - n64), float(np.abs(proj - p64).max())) / n64


def test_gradients_against_float64_truth(step):
    """Every gradient against the same step computed by the reference's modules in float64: within TOL64 of the
    norm, and no less accurate overall than the reference's own fp32 gradients (worst error <= 1.5x theirs)."""
    from tests.golden.train_proj import projections
    g, grads = step["g"], step["grads"]
    g64 = np.load(GOLD64.format(step["size"]))
    names = [str(n) for n in g64["grad_names"]]
    assert names == [str(n) for n in g["grad_names"]]
    ours, ref = [], []
    for i, n in enumerate(names):
        n64 = float(g64["grad_norm"][i])
        if n64 == 0.0:
            continue
        gr = grads[n]
        ours.append((_err(float(gr.double().norm()), projections(n, gr), n64, g64["grad_proj"][i]), n))
        ref.append(_err(float(g["grad_norm"][i]), g["grad_proj"][i], n64, g64["grad_proj"][i]))
    worst = max(ours)
    print(f"[{step['size']}] worst gradient error vs float64: ours {worst[0]:.3e} ({worst[1]}), "
          f"reference fp32 {max(ref):.3e}")
    bad = [o for o in ours if o[0] > TOL64[step["size"]]]
    assert not bad, f"{len(bad)} gradients off the float64 truth: {sorted(bad)[-5:]}"
    assert worst[0] <= 1.5 * max(max(ref), REL_FLOOR[step["size"]]), (worst, max(ref))


def test_adamw_update(step):
    g, params = step["g"], step["params"]
    lr = 2e-5
    for k in g.files:
        if not k.startswith("after_adamw:"):
            continue
        n = k[len("after_adamw:"):]
        ours = params[n].numpy().reshape(g[k].shape)
        diff = np.abs(ours - g[k])
        # the first AdamW step moves each weight by ~lr * sign(grad): allow sign flips of tiny gradients
        assert (diff > 1e-6).mean() < 1e-3 and diff.max() <= 2.5 * lr, (n, diff.max(), (diff > 1e-6).mean())
    _close(params["preprocess_model.quantize.embedding.weight"].view(16384, -1).double().sum(1).numpy(),
           g["after_adamw_E_rowsum"], 1e-3, "codebook after AdamW")


def _run_step(dtype, seed_img=231, seed_draw=5, ddp=False, size=128):
    from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    m = RDEIC(compute_dtype=dtype).init_synthetic()
    ft = FineTuner(m)
    if ddp:
        ft.enable_ddp(bucket_bytes=8 << 20)
    dr = train_draws(1, size // 8, size // 8, m.cfg["compression"]["slice_ch"], seed_draw, m.used_timesteps)
    img = torch.from_numpy(synth_image(size, size, seed_img)).cuda()[None]
    d = ft.training_step(img, synth_context().cuda(), nchw_draws_to_nhwc(dr, "cuda"))
    torch.cuda.synchronize()
    return ft, {k: float(v.detach()) for k, v in d.items()}


@pytest.mark.parametrize("size", [128, 512])
def test_bf16_step_tracks_the_reference(gpu, size):
    """The bf16 training path (the throughput mode) against the fp32 reference step: loss terms within
    bf16 tolerance and the gradient directions of the large majority of tensors (bf16 activations
    through ~100 layers; the VQ / rounding decisions of the entropy model may flip). 512^2 is config 5's
    own size (bench_train.py's step)."""
    g = np.load(GOLD.format(size))
    ft, ld = _run_step(torch.bfloat16, size=size)
    assert all(np.isfinite(v) for v in ld.values())
    for ours, ref, tol in (("T/l_simple", "loss_l_simple", 0.1), ("T/l_guide", "loss_l_guide", 0.05),
                           ("T/l_bpp", "loss_l_bpp", 0.05), ("T/l_emb", "loss_l_emb", 0.1)):
        r = float(g[ref])
        assert abs(ld[ours] - r) <= tol * abs(r), (ours, ld[ours], r)
    # gradients were consumed by the AdamW step; recompute them with the bf16 model's updated state
    # would differ, so compare the update direction instead: sign(p_after - p_before) ~ -sign(grad)
    names = [str(n) for n in g["grad_names"]]
    agree, total = 0, 0
    from rdeic_amd import weights as W
    from oracle import weights_cpu
    for i, n in enumerate(names[:200]):
        o, k = ft.offsets[n]
        shape = tuple(g["grad:" + n].shape) if ("grad:" + n) in g.files else None
        if shape is None:
            continue
        scale, offset = W.init_spec(n, shape)
        p0 = torch.from_numpy(weights_cpu.fill_uniform(int(np.prod(shape)), W.param_seed(n), scale, offset))
        step = (ft.flat[o:o + k].cpu() - p0).numpy()
        ref_g = g["grad:" + n].reshape(-1)
        big = np.abs(ref_g) > 1e-3 * np.abs(ref_g).max()
        agree += int((np.sign(step[big]) == -np.sign(ref_g[big])).sum())
        total += int(big.sum())
    assert total > 0 and agree / total > 0.9, (agree, total)


def _ddp_rank(rank, port, q):
    import os
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                          LOCAL_RANK="0")
        from rdeic_amd import parallel
        parallel.init_from_env(backend="gloo")
        torch.cuda.set_device(0)
        ft, ld = _run_step(torch.float32, seed_img=231 + rank, seed_draw=5 + rank, ddp=True)
        q.put((rank, ft.flat.cpu().numpy(), ld))
        parallel.finish()
    except Exception as e:
        q.put((rank, f"{type(e).__name__}: {e}", None))
        raise


def test_two_rank_ddp_step_equals_averaged_gradients(gpu):
    """Two data-parallel ranks on one GPU (gloo for the collective): the bucketed all-reduce launched
    from the backward leaves both ranks with identical parameters, equal bit for bit to one process
    applying AdamW to the mean of the two single-image gradients."""
    import socket
    import torch.multiprocessing as mp
    from rdeic_amd import autograd as AG, ops
    from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, flat, ld = q.get(timeout=300)
        assert not isinstance(flat, str), f"rank {r}: {flat}"
        res[r] = flat
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0], res[1]), "ranks diverged"
    # single process: both images' gradients, averaged, one AdamW step
    m = RDEIC(compute_dtype=torch.float32).init_synthetic()
    ft = FineTuner(m)
    flat0 = ft.flat.clone()
    gsum = torch.zeros_like(ft.grad)
    for r in range(2):
        ft.flat.copy_(flat0)
        ft.embed_prob.zero_()
        ft.zero_grad()
        dr = train_draws(1, 16, 16, m.cfg["compression"]["slice_ch"], 5 + r, m.used_timesteps)
        d = nchw_draws_to_nhwc(dr, "cuda")
        img = torch.from_numpy(synth_image(128, 128, 231 + r)).cuda()[None]
        x_start, h = ft.get_first_stage(img, d["post_eps"])
        with ops.splitk_allowed(short_k=True):  # as FineTuner.training_step runs it
            loss, _ = ft.losses(x_start, h, synth_context().cuda(), d["t"], d["noise"], d["slice_noise"])
            loss.backward()
        gsum += ft.grad
        if r == 0:
            E_fwd0 = ft.p("preprocess_model.quantize.embedding.weight").detach().clone()
    # each rank re-initialised its own codebook copy from its own batch in the forward; the step ends by
    # broadcasting rank 0's (FineTuner.sync_codebook). Everything but the codebook is compared bit for bit.
    ft.flat.copy_(flat0)
    ft.grad.copy_(gsum / 2)
    ft.step_count = 0
    ft.optimizer_step()
    ours = ft.flat.cpu().numpy()
    o, k = ft.offsets["preprocess_model.quantize.embedding.weight"]
    mask = np.ones_like(ours, dtype=bool)
    mask[o:o + k] = False
    diff = np.abs(ours[mask] - res[0][mask]).max()
    assert diff <= 1e-7, diff


@pytest.mark.parametrize("dtype,size", [(torch.float32, 128), (torch.bfloat16, 512)])
def test_captured_step_replays_the_eager_steps(gpu, dtype, size):
    """CapturedStep (the whole step as one hipGraph) reproduces two eager steps bit for bit:
    parameters, AdamW moments, VQ usage EMA and the loss dict. bf16 at 512^2 is bench_train.py's
    step (config 5): its losses must also be finite."""
    from rdeic_amd.finetune import CapturedStep, FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    ctx = synth_context().cuda()
    imgs = [torch.from_numpy(synth_image(size, size, 300 + i)).cuda()[None] for i in range(2)]
    runs = []
    for captured in (False, True):
        m = RDEIC(compute_dtype=dtype).init_synthetic()
        ft = FineTuner(m)
        draws = [nchw_draws_to_nhwc(train_draws(1, size // 8, size // 8, m.cfg["compression"]["slice_ch"], 40 + i,
                                                m.used_timesteps), "cuda") for i in range(2)]
        cs = CapturedStep(ft, imgs[0], ctx, draws[0]) if captured else None
        losses = []
        for i in range(2):
            d = cs.step(imgs[i], draws[i]) if captured else ft.training_step(imgs[i], ctx, draws[i])
            losses.append({k: float(v.detach()) for k, v in d.items()})
        torch.cuda.synchronize()
        runs.append((ft.flat.cpu(), ft.exp_avg.cpu(), ft.exp_avg_sq.cpu(), ft.embed_prob.cpu(), losses))
    (p0, m0, v0, e0, l0), (p1, m1, v1, e1, l1) = runs
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1) and torch.equal(e0, e1)
    assert l0 == l1
    assert all(np.isfinite(v) for d in l0 for v in d.values())
