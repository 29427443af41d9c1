"""Benchmark: 512x512 images/s through the full RDEIC hot path on N MI355X GPUs.

One step = one batch of B synthetic 512x512 images per GPU through
  encode (VAE) -> entropy model + rANS/torchac to bytes -> bytes back through the entropy
  decoder -> relay DDIM (S steps, UNet + control) -> VAE decode -> uint8
plus the per-image metric rows (bpp, bytes, PSNR) and ONE all-gather of them across ranks.
Data: synthetic (seeded smooth images, random-init weights of the real architecture, a seeded
[1, 77, 1024] text context) — no datasets or checkpoints offline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 16] [--size 512] [--ddim-steps 2]
For N > 1 either run it as is (it starts N ranks itself: rdeic_amd/launch.py) or under
torch.distributed.run with --nproc-per-node N (WORLD_SIZE must equal --gpus); one process per GPU, RCCL.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def conv_traffic(workload: dict):
    """HBM bytes per conv launch, from the latest committed PMC run (tools/pmc_bench.sh ->
    profiles/conv_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md §HBM). Counters cannot be read inside this process, so the figure is the
    measured one with its source — attached only when that run's workload is this line's (size,
    relay steps, batch per GPU, dtype, sampler); otherwise None with the reason."""
    try:
        with open(os.path.join(ROOT, "profiles", "conv_traffic.json")) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return {"bytes_per_launch": None, "reason": "no committed PMC run (profiles/conv_traffic.json)"}
    if t.get("workload") != workload:
        return {"bytes_per_launch": None,
                "reason": f"the committed PMC run measured {t.get('workload')}, not this line's {workload}"}
    out = {"bytes_per_launch": t["bytes_per_launch"], "workload": workload,
           "source": t.get("source", "profiles/conv_traffic.json"), "head": t.get("head")}
    for k in ("bytes_per_step", "splitk_reduce_bytes_per_step", "splitk_reduce_launches", "launches_counted"):
        if k in t:
            out[k] = t[k]
    return out


def parse(argv=None):
    ap = argparse.ArgumentParser(epilog="environment: RDEIC_CODER_THREADS=N host rANS threads per rank (default: the "
                                        "CPU quota / affinity divided by LOCAL_WORLD_SIZE); RDEIC_RANK_BOUND=1 the "
                                        "launcher bound each rank to its own cores (the affinity set is not divided; "
                                        "detected when it is at most 1 / LOCAL_WORLD_SIZE of the machine)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); default: WORLD_SIZE under torch.distributed.run, else 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU per step (when --global-batch is unset)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="images per step over all ranks, sharded contiguously by parallel.shard "
                         "(config 4: 128 on 8 GPUs); default --batch x world")
    ap.add_argument("--bpp-sweep", default=None,
                    help="comma list of target bpp (config 4: 0.04,0.08,0.12); each point re-initialises the "
                         "synthetic rate layers with weights.rate_gain_for_bpp and is timed on its own; "
                         "value/roofline come from the point nearest 0.08")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--ddim-steps", type=int, default=2, help="relay sampler steps")
    ap.add_argument("--sampler", default="ddim", choices=["ddim", "ddpm"],
                    help="relay sampler (config 2 names 2-step relay DDIM; ddpm = the CLI's spaced sampler)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--streams", type=int, default=5,
                    help="codec sessions in flight per GPU (host thread + HIP stream each; RDEIC.session): one "
                         "batch's host rANS coding and small entropy-stage kernels overlap another batch's GPU work")
    ap.add_argument("--splitk-rule", default=None, metavar="BLOCKS,MAX",
                    help="inference split-K rule of the small-M convs (A/B only; ops.SPLITK_BLOCKS / SPLITK_MAX)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--prof-every", type=int, default=8,
                    help="roofline timing: every launch >= 50 GFLOP (64 MB for GroupNorm), and a hashed "
                         "1-in-N sample of the smaller ones (weighted estimate)")
    ap.add_argument("--coder-groups", type=int, default=None,
                    help="image groups interleaved in the entropy-stage loops (default: the library's)")
    ap.add_argument("--no-plans", action="store_true", help="eager launches (no launch-plan replay), A/B only")
    ap.add_argument("--no-geglu-fuse", action="store_true", help="unfused GEGLU (projection + geglu kernel), A/B only")
    ap.add_argument("--no-splitk-entropy", action="store_true", help="no split-K in the bf16 entropy nets, A/B only")
    ap.add_argument("--no-halo", action="store_true", help="materialised GroupNorm + im2col conv, A/B only")
    ap.add_argument("--conv-option", action="append", default=[], metavar="KEY=VALUE",
                    help="rdeic_set_conv_option(KEY, VALUE) before the run (include/rdeic_hip.h), A/B only")
    ap.add_argument("--rate-gain", type=float, default=None,
                    help="synthetic bpp knob (rdeic_amd/weights.py); default: the ~0.08 bpp gain of config 2")
    ap.add_argument("--fp32-steps", type=int, default=2,
                    help="one-GPU runs with --dtype bf16: also time this many steps of the fp32 parity mode (the "
                         "path whose bitstreams and pixels match the reference) on the same images, and report "
                         "its throughput and the bf16-vs-fp32 bpp / PSNR / MS-SSIM gap; 0 = skip")
    return ap.parse_args(argv)


def sweep_points(args):
    """[(target_bpp, rate_gain)] of the run and the headline index: config 4's sweep
    (--bpp-sweep) or the single config-2 point; the headline (and profiled) point is the one
    nearest 0.08 bpp."""
    from rdeic_amd import weights as W
    if args.bpp_sweep:
        points = [(float(v), W.rate_gain_for_bpp(float(v))) for v in args.bpp_sweep.split(",")]
    else:
        points = [(None, W.RATE_GAIN_BPP008 if args.rate_gain is None else args.rate_gain)]
    main_i = min(range(len(points)), key=lambda i: abs((points[i][0] or 0.08) - 0.08))
    return points, main_i


def run_sweep(points, main_i, measure):
    """measure(i, target_bpp, rate_gain, headline) -> result dict for each point, in order. Only the
    headline point keeps its output images ("out": the fp32 leg compares pixels against them)."""
    results = []
    for i, (target, rate_gain) in enumerate(points):
        r = measure(i, target, rate_gain, i == main_i)
        if i != main_i:
            r["out"] = None
        results.append(r)
    return results


def main():
    args = parse()
    # --gpus N > 1 without torch.distributed.run: this process only launches N ranks (never touches the GPU)
    from rdeic_amd.launch import maybe_launch
    maybe_launch(args.gpus, __file__)
    from rdeic_amd import metrics as quality, ops, parallel
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    rank, world, local = parallel.init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    S = args.size
    G = args.global_batch if args.global_batch is not None else args.batch * world
    g0, g1 = parallel.shard(G, rank, world)  # this rank's contiguous slice of the global batch
    B = g1 - g0
    if B < 1:
        raise SystemExit(f"global batch {G} leaves rank {rank} of {world} without images")
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    points, main_i = sweep_points(args)
    model = RDEIC(compute_dtype=dtype, device=dev)
    if args.coder_groups is not None:
        model.preprocess_model.coder_groups = args.coder_groups
    if args.no_plans:
        model.use_plans = False
    if args.no_geglu_fuse:
        ops.GEGLU_FUSED = False
    if args.no_splitk_entropy:
        ops.SPLITK_ENTROPY = False
    if args.no_halo:
        ops.set_halo_conv(0)
    for kv in args.conv_option:
        k, v = kv.split("=")
        ops.set_conv_option(int(k), int(v))
    if args.splitk_rule:
        ops.SPLITK_BLOCKS, ops.SPLITK_MAX = (int(v) for v in args.splitk_rule.split(","))

    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + g) for g in range(g0, g1)])).to(dev)
    draws = [relay_noise((1, 4, S // 8, S // 8), 231 + g, args.ddim_steps) for g in range(g0, g1)]
    noise = torch.cat([d[0] for d in draws])
    step_noise = torch.cat([d[1] for d in draws], 1) if args.sampler == "ddpm" else None
    ctx = synth_context().to(dev)
    nsess = max(1, args.streams)

    def run_batch(sess, mse):
        """One step's device work and host coding for one batch on the calling thread's stream;
        returns the per-image metric rows (host)."""
        out, bodies = sess.codec_images(imgs, ctx, noise, steps=args.ddim_steps, sampler=args.sampler,
                                        step_noise_nchw=step_noise)
        ops.call("rdeic_image_mse", imgs.data_ptr(), out.data_ptr(), B, S * S * 3, mse.data_ptr(), ops.stream_ptr())
        m = mse.cpu().numpy()
        _, ms = quality.ssim_ms_ssim(out, imgs)  # on the device (rdeic_image_ssim)
        sess._last_out = out  # the step's u8 images (bf16-vs-fp32 pixel PSNR of the fp32 leg)
        return torch.tensor([[len(b) * 8.0 / (S * S), float(len(b)),
                              10 * math.log10(255.0 ** 2 / max(float(v), 1e-10)), float(v), float(q), 1.0, float(rank)]
                             for b, v, q in zip(bodies, m, ms)], dtype=torch.float32)

    def log(msg):  # progress on stderr (the JSON line is the only stdout)
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    def measure(i, target, rate_gain, headline):
        log(f"point {i + 1}/{len(points)}: rate_gain {rate_gain}, {args.warmup} warm-up + {args.steps} timed steps, "
            f"{nsess} codec session(s) in flight")
        model.init_synthetic(rate_gain=rate_gain)
        model.preprocess_model.update(force=True)
        # codec sessions: each owns a host thread, a HIP stream and its launch plans; they share the
        # weights. Plans are recorded one session at a time (warm-up), then the sessions run
        # concurrently, so one batch's host entropy coding overlaps another batch's GPU work.
        sessions = [model] + [model.session() for _ in range(nsess - 1)]
        streams = [torch.cuda.Stream(device=dev) for _ in range(nsess)]
        mses = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(nsess)]
        for sess, st, mse in zip(sessions, streams, mses):
            with torch.cuda.stream(st):
                for _ in range(max(1, args.warmup)):
                    run_batch(sess, mse)
            torch.cuda.synchronize()
        rows_by_step = [None] * args.steps
        errors = []

        def worker(j):
            try:
                with torch.cuda.stream(streams[j]):
                    for kstep in range(j, args.steps, nsess):
                        rows_by_step[kstep] = run_batch(sessions[j], mses[j])
            except BaseException as e:  # surfaced after the join
                errors.append(e)

        parallel.barrier(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if nsess == 1:
            worker(0)
        else:
            threads = [threading.Thread(target=worker, args=(j,)) for j in range(nsess)]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
        if errors:
            raise errors[0]
        for kstep in range(args.steps):  # ONE metric all-gather per step, in step order
            metrics = parallel.gather_metrics(rows_by_step[kstep].to(dev), G)
        parallel.barrier(dev)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        prof = None
        if headline and not args.no_roofline:
            # Roofline pass (untimed): the same steps on ONE session with the native launch profiler
            # (HIP events on the launch stream; launches >= 50 GFLOP always, smaller ones 1 in
            # --prof-every), so each kernel's duration is its own and not shared with a concurrent
            # session's kernels.
            ops.prof_start(2048 * max(1, args.steps) + 1024, args.prof_every)
            torch.cuda.synchronize()
            tr0 = time.perf_counter()
            with torch.cuda.stream(streams[0]):
                for _ in range(args.steps):
                    run_batch(sessions[0], mses[0])
            torch.cuda.synchronize()
            rf_elapsed = time.perf_counter() - tr0
            ops.prof_stop()
            prof = ops.prof_read()
            prof = dict(prof, _wall_s=rf_elapsed,
                        _attn_shapes={k: ops.prof_read_keys(k) for k in ("attention", "attention_dh16", "attention_d512")})
        elapsed = parallel.max_over_ranks(elapsed, dev)
        mrows = metrics.cpu().numpy()
        last_out = sessions[(args.steps - 1) % nsess]._last_out
        del sessions
        return {"target_bpp": target, "rate_gain": rate_gain, "elapsed": elapsed, "prof": prof, "out": last_out,
                "mean_bpp": float(mrows[:, 0].mean()), "mean_psnr_db": float(mrows[:, 2].mean()),
                "mean_ms_ssim": float(mrows[:, 4].mean()),
                "images": int(mrows.shape[0]), "rows": rows_by_step[-1].numpy()}

    results = run_sweep(points, main_i, measure)
    fp32_leg = None
    if world == 1 and args.dtype == "bf16" and args.fp32_steps > 0 and not args.bpp_sweep:
        log(f"fp32 parity mode: 1 warm-up + {args.fp32_steps} timed steps on one session, same images")
        rg = results[main_i]["rate_gain"]
        del model
        torch.cuda.empty_cache()
        m32 = RDEIC(compute_dtype=torch.float32, device=dev).init_synthetic(rate_gain=rg)
        m32.preprocess_model.update(force=True)
        mse32 = torch.empty(B, dtype=torch.float32, device=dev)
        run_batch(m32, mse32)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.fp32_steps):
            rows32 = run_batch(m32, mse32)
        torch.cuda.synchronize()
        el32 = time.perf_counter() - t0
        r32 = rows32.numpy()
        r16 = results[main_i]["rows"]
        d = results[main_i]["out"].double() - m32._last_out.double()
        px_psnr = 10 * math.log10(255.0 ** 2 / max(float(d.pow(2).mean()), 1e-12))
        fp32_leg = {
            "dtype": "fp32", "path": "bitstream-parity (fp32 convs on v_mfma_f32_16x16x4f32; file bodies byte-equal "
                                     "to the oracle's, pixels within 1e-3 abs: tests/test_config2_gpu.py)",
            "images_per_s": round(B * args.fp32_steps / el32, 3), "ms_per_step": round(el32 / args.fp32_steps * 1e3, 2),
            "steps": args.fp32_steps, "codec_sessions": 1, "mean_bpp": round(float(r32[:, 0].mean()), 5),
            "mean_psnr_db": round(float(r32[:, 2].mean()), 3), "mean_ms_ssim": round(float(r32[:, 4].mean()), 5),
            "bf16_minus_fp32": {
                "mean_bpp_rel": round(float((r16[:, 0].mean() - r32[:, 0].mean()) / r32[:, 0].mean()), 5),
                "max_image_bpp_rel": round(float(np.abs((r16[:, 0] - r32[:, 0]) / r32[:, 0]).max()), 5),
                "mean_psnr_db": round(float(r16[:, 2].mean() - r32[:, 2].mean()), 4),
                "mean_ms_ssim": round(float(r16[:, 4].mean() - r32[:, 4].mean()), 5)},
            # the decoded u8 pixels of the two modes against each other (each codes its own bitstream)
            "bf16_vs_fp32_pixel_psnr_db": round(px_psnr, 2)}
        del m32
    parallel.finish()  # every rank leaves the group before rank 0's CPU-baseline leg
    if rank != 0:
        return
    r = results[main_i]
    elapsed, prof, rate_gain = r["elapsed"], r["prof"], r["rate_gain"]
    value = G * args.steps / elapsed
    roof = None
    if prof and "conv" in prof:
        n, flops, ms = prof["conv"]
        achieved = flops / (ms * 1e-3) / 1e12
        peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_FP32_TFLOPS
        roof = {"bound": "mfma", "kernel": "conv_dma_kernel / conv_kernel (implicit-GEMM conv + linear, rdeic_conv2d)",
                "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": conv_traffic({"size": S, "ddim_steps": args.ddim_steps, "batch": B, "dtype": args.dtype,
                                         "sampler": args.sampler}),
                "launches_per_step": round(n / args.steps, 1),
                "sampling": f"launches >= 50 GFLOP always timed, smaller ones 1 in {args.prof_every} (weighted); "
                            f"measured on one codec session over {args.steps} steps right after the timed region",
                "avg_launch_us": round(ms * 1e3 / max(1, n), 2), "ms_per_step": round(ms / args.steps, 3),
                "flops_per_step": round(flops / args.steps),
                "kernel_share_of_step": round(ms * 1e-3 / prof["_wall_s"], 4),
                "single_session_ms_per_step": round(prof["_wall_s"] / args.steps * 1e3, 2)}
        # secondary kernels the north star names: attention on MFMA, GroupNorm on HBM
        if "conv_bytes" in prof:  # algorithmic bytes of every conv launch (input once, weight, output, residual)
            nb, byts, _ = prof["conv_bytes"]
            roof["algorithmic_bytes_per_launch"] = round(byts / max(1, nb))
            roof["algorithmic_bytes_per_step"] = round(byts / args.steps)
            # PMC bytes of the step's conv launches (split-K reduces included) over the library's
            # algorithmic bytes of the same step: one launch set on both sides (per step, not per launch)
            tr = roof["traffic"] if isinstance(roof["traffic"], dict) else {}
            if tr.get("bytes_per_step"):
                roof["traffic_over_algorithmic"] = round(tr["bytes_per_step"] / (byts / args.steps), 3)
                roof["traffic_over_algorithmic_excl_splitk_reduce"] = round(
                    (tr["bytes_per_step"] - tr.get("splitk_reduce_bytes_per_step", 0)) / (byts / args.steps), 3)
        sec = {}
        for kind, v in prof.items():
            if kind in ("conv", "conv_bytes") or kind.startswith("_"):
                continue
            cnt, work, kms = v
            if kms <= 0:
                continue
            if kind.startswith("attention"):
                a = work / (kms * 1e-3) / 1e12
                sec[kind] = {"bound": "mfma", "achieved": round(a, 2), "peak": peak, "unit": "TFLOP/s",
                             "frac": round(a / peak, 4), "launches_per_step": round(cnt / args.steps, 1),
                             "ms_per_step": round(kms / args.steps, 3)}
            else:
                a = work / (kms * 1e-3) / 1e9
                sec[kind] = {"bound": "hbm", "achieved": round(a, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(a / PEAK_HBM_GBS, 4), "launches_per_step": round(cnt / args.steps, 1),
                             "ms_per_step": round(kms / args.steps, 3)}
        # per-shape attribution of the attention kinds (self vs cross: lk == 77 is the text context)
        shapes = []
        for kind, rows in prof.get("_attn_shapes", {}).items():
            for key, cnt, work, kms in rows:
                if kms <= 0:
                    continue
                a = work / (kms * 1e-3) / 1e12
                sh = ops.attention_key(key)
                shapes.append(dict(kind=kind, **sh, cross=sh["lk"] != sh["lq"], launches_per_step=round(cnt / args.steps, 2),
                                   ms_per_step=round(kms / args.steps, 4), achieved=round(a, 1), frac=round(a / peak, 4)))
        sec["attention_by_shape"] = sorted(shapes, key=lambda r: -r["ms_per_step"])
        roof["secondary"] = sec
    cpu = None
    if world > 1:
        cpu = {"value": None, "note": "reported on rank 0 of the one-GPU run only (bench.py --gpus 1)"}
    elif not args.no_cpu_baseline:
        log("cpu baseline (oracle restatement on the host cores)")
        try:
            from oracle.bench_cpu import run_cpu_baseline
            cpu = run_cpu_baseline(size=S, steps=args.ddim_steps, rate_gain=rate_gain)
        except Exception as e:  # the baseline is reported, never the target
            cpu = {"value": None, "error": f"{type(e).__name__}: {e}"}
    cfg_name = {(512, 2): "config 2", (1024, 5): "config 3"}.get((S, args.ddim_steps), "custom")
    line = {
        "metric": f"{S}x{S} images/sec encode+relay-decode @ fixed bpp; 1/2/4/8 GPU",
        "path": ("bf16: self-consistent bitstreams (the decoder decodes its own streams, batch-invariant coding); "
                 "bpp / quality gap to the fp32 bitstream-parity mode in fp32_parity_mode" if args.dtype == "bf16"
                 else "fp32: bitstream-parity mode (file bodies byte-equal to the oracle's)"),
        "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded images, random-init weights)",
        "config": {"workload": f"{cfg_name}: global batch {G} ({G // world}{'+' if G % world else ''}/GPU) {S}x{S}, "
                               f"{args.ddim_steps}-step relay "
                               f"{'DDIM' if args.sampler == 'ddim' else 'spaced DDPM'}, "
                               f"encode+entropy-code+decode+VAE-decode", "global_batch": G,
                   "image_size": S, "ddim_steps": args.ddim_steps, "sampler": args.sampler, "parallelism": f"dp{world}", "codec_sessions_per_gpu": nsess, "rate_gain": rate_gain,
                   "mean_bpp": round(r["mean_bpp"], 4), "mean_psnr_db": round(r["mean_psnr_db"], 2),
                   "mean_ms_ssim": round(r["mean_ms_ssim"], 4)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "fp32_parity_mode": fp32_leg,
    }
    if args.bpp_sweep:
        line["bpp_sweep"] = [{"target_bpp": p["target_bpp"], "rate_gain": p["rate_gain"],
                              "achieved_mean_bpp": round(p["mean_bpp"], 4), "mean_psnr_db": round(p["mean_psnr_db"], 2),
                              "images_per_s": round(G * args.steps / p["elapsed"], 3),
                              "ms_per_step": round(p["elapsed"] / args.steps * 1e3, 2), "images": p["images"]}
                             for p in results]
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
