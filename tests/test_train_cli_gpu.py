"""Config 5's training loop (train.py, the reference's train.py:10-28 + configs/finetune_ood.yaml) and
its resume path, on the HIP kernels.

* VectorQuantiser with a non-zero usage EMA: tests/golden/vq_resume.npz holds the REFERENCE module's
  training forward/backward (compression_modules.py:228-307) from an embed_prob spread over the
  re-initialisation threshold (tests/golden/make_vq_golden.py). The HIP VQ step (AG.VQTrainFn) must
  reproduce the EMA, the partly re-initialised codebook, z_q, the loss and both gradients. A run
  resumed with embed_prob dropped (zeros) would re-initialise every code: the test checks that it
  is distinguishable.
* train.main for several steps at 128x128 (fp32, the reference's precision 32): the losses stay
  finite, safetensors checkpoints are written with the trainable weights, the codebook EMA, the
  AdamW moments and the global step; resuming from the step-2 checkpoint reproduces the
  uninterrupted run's step-4 checkpoint bit for bit.""" 
import os

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "vq_resume.npz")


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_vq_step_with_usage_ema_matches_reference(gpu):
    from rdeic_amd import autograd as AG
    from rdeic_amd import ops
    g = np.load(GOLD)
    ep0 = torch.from_numpy(g["embed_prob0"]).cuda()
    K = ep0.numel()
    z = torch.from_numpy(g["z"]).permute(0, 2, 3, 1).contiguous().cuda().requires_grad_(True)
    D = z.shape[3]
    E = ops.fill_uniform(torch.empty(K * D, dtype=torch.float32, device="cuda"), int(g["e_seed"]),
                         float(g["e_scale"]), 0.0).view(K, D).requires_grad_(True)
    E0 = E.detach().clone()
    ep = ep0.clone()
    zq, loss = AG.VQTrainFn.apply(z, E, ep, 0.25, 0.99, 0.07)
    r = torch.from_numpy(g["r"]).permute(0, 2, 3, 1).contiguous().cuda()
    (loss.sum() + (zq * r).sum()).backward()
    torch.cuda.synchronize()
    rows = torch.from_numpy(g["rows"])
    E_after = E.detach().double().cpu()
    checks = {
        "embed_prob": (_rel(ep.cpu(), g["embed_prob_after"]), 1e-5),
        "z_q": (_rel(zq.detach().permute(0, 3, 1, 2).cpu(), g["zq"]), 1e-6),
        "loss": (abs(float(loss) - float(g["loss"])) / abs(float(g["loss"])), 1e-5),
        "codebook rows": (_rel(E_after[rows], g["E_after_rows"]), 1e-5),
        "codebook row sums": (_rel(E_after.sum(1), g["E_after_rowsum"]), 1e-5),
        "dz": (_rel(z.grad.permute(0, 3, 1, 2).cpu(), g["dz"]), 1e-4),
        "dE rows": (_rel(E.grad[rows.cuda()].cpu(), g["dE_rows"]), 1e-4),
        "dE row norms": (_rel(E.grad.double().norm(dim=1).cpu(), g["dE_rownorm"]), 1e-4),
    }
    for name, (err, tol) in checks.items():
        print(f"{name}: rel err {err:.2e}")
        assert err < tol, (name, err)
    # the re-initialisation is partial: kept codes equal the old ones, replaced ones moved
    decay = torch.from_numpy(g["decay"])
    kept = decay < 1e-6
    assert kept.any() and (decay > 0.5).any()
    assert float((E.detach() - E0).abs().max(1).values.cpu()[kept].max()) < 1e-6
    # with the EMA dropped (a resume that loses embed_prob) every code would be replaced
    Ez = E0.clone().requires_grad_(True)
    zq0, _ = AG.VQTrainFn.apply(z.detach(), Ez, torch.zeros_like(ep0), 0.25, 0.99, 0.07)
    torch.cuda.synchronize()
    moved = (Ez.detach() - E0).abs().max(1).values.cpu()
    assert float(moved[kept].max()) > 1e-3, "a zero EMA must re-initialise the kept codes too"


def _cfg(tmp, name, max_steps, resume=None, precision=32):
    cfg = {"data": {"out_size": 128, "batch_size": 1, "n_images": 3},
           "model": {"learning_rate": 2e-5, "l_guide_weight": 3.0, "l_bpp_weight": 1.0, "used_timesteps": 300,
                     "sd_locked": True, "is_refine": False, "precision": precision, "resume": resume},
           "lightning": {"seed": 231, "trainer": {"max_steps": max_steps, "log_every_n_steps": 1},
                         "checkpoint": {"every_n_train_steps": 2, "dirpath": str(tmp / name)}}}
    p = tmp / f"{name}.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p)


def test_train_loop_checkpoint_and_bit_exact_resume(gpu, tmp_path):
    import train
    from safetensors import safe_open
    from safetensors.torch import load_file
    recs = train.main(["--config", _cfg(tmp_path, "full", 4)])
    assert [r["global_step"] for r in recs] == [1, 2, 3, 4]
    for r in recs:
        assert all(np.isfinite(v) for k, v in r.items() if k.startswith("T/")), r
    print("losses:", [round(r["T/loss"], 5) for r in recs])
    ck2 = tmp_path / "full" / "ood_finetune_step=2.safetensors"
    ck4 = tmp_path / "full" / "ood_finetune_step=4.safetensors"
    assert ck2.exists() and ck4.exists()
    with safe_open(str(ck2), "pt") as f:
        assert f.metadata()["global_step"] == "2"
    full4 = load_file(str(ck4))
    assert float(full4[train.EMBED_PROB].abs().sum()) > 0  # the usage EMA is saved
    for k in ("optimizer.exp_avg", "optimizer.exp_avg_sq", "control_model.middle_block_out.0.bias"):
        assert k in full4
    # resume from step 2, run to step 4: the same weights, EMA and AdamW moments, bit for bit
    recs2 = train.main(["--config", _cfg(tmp_path, "resumed", 4, resume=str(ck2))])
    assert [r["global_step"] for r in recs2] == [3, 4]
    for a, b in zip(recs[2:], recs2):
        assert a["T/loss"] == b["T/loss"], (a, b)
    res4 = load_file(str(tmp_path / "resumed" / "ood_finetune_step=4.safetensors"))
    assert set(res4) == set(full4)
    diff = [k for k in full4 if not torch.equal(full4[k], res4[k])]
    assert not diff, diff[:5]

