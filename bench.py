#!/usr/bin/env python
"""Training-throughput benchmark of the MI355X hot path (BASELINE.json `metric`).

Workload (configs[1]): EnvNet-v2, bf16 compute (f32 master params / grads / Adam state),
batch 256 per GPU, synthetic 5 s @ 44.1 kHz clips resident in HBM.  One step = on-GPU BC
mixing -> EnvNet-v2 forward -> soft-label loss -> backward -> (N>1: RCCL gradient all-reduce)
-> global-norm clip 1.0 -> Adam(lr 1e-4, wd 1e-4).  `--model ast` times configs[2] instead
(waveform -> on-GPU log-mel -> AST fwd+bwd -> clip + Adam).

python bench.py [--gpus N --steps K --warmup W]; for N > 1 launch one process per GPU with
torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA
F32_PEAK_TF = 157.3

# Per-clip algorithmic work (measured with torch.utils.flop_counter)
ENVNET_FLOP_PER_CLIP = 32.74e9
AST_FLOP_PER_CLIP = 1139.7e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=["envnet", "ast"], default="envnet")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 256 for both models)")
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe", default=None, help="comma list of GEMM tags to time live (default: auto)")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def build_envnet(args, dev):
    from src.models.envnet_v2 import EnvNetV2
    from src.training.optim import FusedAdam
    torch.manual_seed(42)
    model = EnvNetV2(num_classes=50, dropout=0.5, compute_dtype=args.dtype).to(dev).train()
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    return model, opt


def make_batch(B, T, dev, rank, num_classes=50):
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    wav = 0.1 * torch.randn(B, T, generator=g, device=dev)
    wav = wav / wav.abs().amax(dim=1, keepdim=True)  # peak-normalised like prepare_esc50.py:98-101
    labels = torch.randint(0, num_classes, (B,), generator=g, device=dev)
    return wav, labels, g


def envnet_step_fn(model, opt, wav, labels, g, world, ddp):
    from src.datasets.augment import bc_mix
    from src.miaudio import kernels as K

    def step():
        x, y, _ = bc_mix(wav, labels, 50, gen=g)
        z = model(x.view(x.shape[0], 1, -1))
        loss, dz, _ = K.soft_ce(z, y, input_sigmoid=False)
        z.backward(dz)
        if ddp is not None:
            ddp.finish()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss
    return step


def frontend_summary(regions: dict, B: int):
    """The EnvNet-v2 1-D conv frontend (conv1 -> BN/ReLU -> conv2 -> BN/ReLU -> pool, fwd + bwd) as
    one HBM-bound path: its algorithmic bytes (SURVEY.md §8(d), 86.6 MB/clip in bf16) over the live
    HIP-event time of all its kernels, against the 8 TB/s HBM peak."""
    f, b = regions.get("frontend.fwd"), regions.get("frontend.bwd")
    if not f or not b:
        return None
    byts = f["bytes"] + b["bytes"]
    ms = f["ms"] + b["ms"]
    return {"bytes_per_clip": byts // B, "ms_fwd": round(f["ms"], 4), "ms_bwd": round(b["ms"], 4),
            "achieved_gbs": round(byts / (ms * 1e-3) / 1e9, 1), "peak_gbs": HBM_PEAK_GBS,
            "frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# probe tag -> substring of its kernel symbol (disambiguates launches with similar durations)
KERNEL_HINT = {
    "t0b.fwd": "conv8_kernel<true, true, 2>",
    "t0b.dgrad": "conv8_kernel<false, false, 2>",
    "t0b.wgrad": "wgrad8_kernel",
    "conv2.fwd": "feconv_kernel<32, 16, 2, true>",
    "conv2.dgrad": "feconv_kernel<64, 8, 1, false>",
    "conv2.wgrad": "fe_wgrad_kernel",
    "conv1.fwd": "fe_conv1_kernel",
    "attn.fwd": "attn_fwd_kernel",
}


def pmc_traffic(model: str, ks: dict, tag: str | None = None):
    """HBM bytes per launch of the probed kernel from the committed rocprofv3 PMC summary of the same
    bench command (profiles/<round>_pmc_<model>.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes).  The probed launch is matched to a kernel symbol by launches per
    step and by its rocprof average duration (must agree with the live HIP-event time within 10 %)."""
    files = sorted((REPO / "profiles").glob(f"r*_pmc_{model}.json"))
    if not files:
        return None, None
    table = json.loads(files[-1].read_text())["kernels"]
    hint = KERNEL_HINT.get(tag or "")
    if hint and any(hint in n for n in table):
        table = {n: e for n, e in table.items() if hint in n}
    best = None
    for name, e in table.items():
        if "hbm_bytes" not in e or e["launches_per_step"] != round(ks["launches_per_step"]):
            continue
        rel = abs(e["avg_ms"] - ks["ms"]) / ks["ms"]
        if rel < 0.10 and (best is None or rel < best[0]):
            best = (rel, name, e)
    if best is None:
        return None, {"file": files[-1].name, "match": None}
    rel, name, e = best
    return e["hbm_bytes"], {"file": files[-1].name, "kernel": name, "rocprof_avg_ms": e["avg_ms"],
                            "live_vs_rocprof": round(rel, 4)}


def cpu_baseline_envnet(threads: int, batch: int = 4, steps: int = 10):
    """Oracle (CPU restatement of the reference path) timed on this host: fwd+loss+bwd+clip+Adam."""
    sys.path.insert(0, str(REPO))
    from oracle import envnet as oenv
    from oracle import train as otrain
    torch.set_num_threads(threads)
    gen = torch.Generator().manual_seed(0)
    params = {}
    for name, shape in oenv.param_shapes().items():
        params[name] = (torch.randn(shape, generator=gen) * 0.02).requires_grad_(True)
    for name, shape in oenv.buffer_shapes().items():
        params[name] = torch.zeros(shape) if name.endswith("mean") else torch.ones(shape)
    names = oenv.trainable_names(params)
    opt = torch.optim.Adam([params[n] for n in names], lr=1e-4, weight_decay=1e-4)
    x = torch.randn(batch, 1, 220_500, generator=gen) * 0.1
    y = torch.zeros(batch, 50)
    y[torch.arange(batch), torch.randint(0, 50, (batch,), generator=gen)] = 1.0

    def one():
        z = oenv.forward(params, x, training=True)
        loss = otrain.soft_ce(z, y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_([params[n] for n in names], 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"oracle EnvNet-v2 f32 train step (fwd+loss+bwd+clip+Adam), batch {batch}, "
                      f"{steps} timed steps after 1 warm-up, {dt:.1f} s of CPU work on {threads} threads "
                      f"of {cpu_model()}"}


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from src.miaudio import kernels as K
    from src.training.ddp import GradAllReducer

    if args.model == "envnet":
        B = args.batch or 256
        model, opt = build_envnet(args, dev)
        wav, labels, g = make_batch(B, 220_500, dev, rank)
        ddp = GradAllReducer(model, world) if world > 1 else None
        step = envnet_step_fn(model, opt, wav, labels, g, world, ddp)
        flop_per_clip = ENVNET_FLOP_PER_CLIP
        probe_tags = (args.probe.split(",") if args.probe else ["t0b.fwd", "t0b.dgrad", "t0b.wgrad", "conv1.fwd", "conv1.wgrad", "conv2.fwd", "conv2.dgrad", "conv2.wgrad"])
        probe_tags += ["frontend.fwd", "frontend.bwd"]
        workload = "EnvNet-v2 train step (BC-mix, fwd, soft-CE, bwd, clip, Adam), ESC-50 shape"
    else:
        sys.path.insert(0, str(REPO))
        from bench_ast import build_ast_step  # noqa: E402
        B = args.batch or 256  # AST at batch 256 on one MI355X (~84 GB of activations)
        step, flop_per_clip, probe_tags, workload = build_ast_step(args, dev, rank, world, B)

    if world > 1:
        model_sync = getattr(step, "broadcast", None)
        if model_sync:
            model_sync()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    K.PROBE = {t: [] for t in probe_tags}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    probes = K.PROBE
    K.PROBE = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ms = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed

    # live per-kernel timing (HIP events on the launch stream) for the roofline
    kstats = {}
    for tag, recs in probes.items():
        if not recs:
            continue
        dur = sum(e0.elapsed_time(e1) for e0, e1, _, _ in recs) / len(recs)  # ms per launch
        flops, byts = recs[0][2], recs[0][3]
        kstats[tag] = {"ms": dur, "tflops": flops / (dur * 1e-3) / 1e12, "gbs": byts / (dur * 1e-3) / 1e9,
                       "launches_per_step": len(recs) / args.steps, "flop": flops, "bytes": byts}
    regions = {k: v for k, v in kstats.items() if k.startswith("frontend.")}
    kstats = {k: v for k, v in kstats.items() if k not in regions}
    dom = max(kstats, key=lambda k: kstats[k]["ms"] * kstats[k]["launches_per_step"]) if kstats else None
    peak_tf = BF16_MFMA_PEAK_TF if args.dtype == "bf16" else F32_PEAK_TF
    roof = None
    if dom:
        ks = kstats[dom]
        kname = {"attn.fwd": "attn_fwd_kernel", "attn.bwd": "attn_bwd_dkdv_kernel+attn_bwd_dq_kernel",
                 "t0b.fwd": "conv8_kernel<PRE,STATS>", "t0b.dgrad": "conv8_kernel"}.get(
            dom, KERNEL_HINT.get(dom, "igemm_kernel"))
        traffic, tsrc = pmc_traffic(args.model, ks, dom)
        if tsrc and tsrc.get("kernel"):
            kname = tsrc["kernel"].replace("_ZN12_GLOBAL__N_1", "").replace("(anonymous namespace)::", "").split("(")[0]
        roof = {"bound": "mfma", "kernel": f"{kname} [{dom}]", "achieved": round(ks["tflops"], 2),
                "peak": peak_tf, "unit": "TFLOP/s", "frac": round(ks["tflops"] / peak_tf, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "algorithmic_per_launch": {"flop": ks["flop"], "bytes": ks["bytes"]},
                "ms_per_launch": round(ks["ms"], 4)}
    step_tf = flop_per_clip * B / (ms * 1e-3) / 1e12
    out = {
        "metric": "training clips/sec (EnvNet-v2, ESC-50 shape)" if args.model == "envnet"
        else "training clips/sec (AST, ESC-50 shape)",
        "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (peak-normalised 0.1*N(0,1) clips, uniform labels)",
        "config": {"workload": workload, "model": "envnet_v2" if args.model == "envnet" else "ast",
                   "global_batch": B * world, "per_gpu_batch": B, "clip_samples": 220_500,
                   "parallelism": f"dp{world}"},
        "roofline": roof,
        "step_tflops": round(step_tf, 2),
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in kstats.items()},
        "frontend_path": frontend_summary(regions, B),
        "loss": float(loss),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "envnet":
        threads = min(16, len(os.sched_getaffinity(0)))
        out["cpu_baseline"] = cpu_baseline_envnet(threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
