#!/usr/bin/env python
"""Training-throughput benchmark of the MI355X hot path (BASELINE.json `metric`: training clips/sec
for EnvNet-v2 & AST).

Default invocation (what the driver runs) times BOTH configs on the same GPUs, one after the other:
  * configs[1] — EnvNet-v2, bf16 compute (f32 master params / grads / Adam state), batch 256 per GPU:
    on-GPU BC mixing -> forward -> soft-label loss -> backward -> (N>1: RCCL gradient all-reduce)
    -> global-norm clip 1.0 -> Adam(lr 1e-4, wd 1e-4).  This is the top-level JSON line.
  * configs[2] — AST, bf16, batch 256 per GPU: on-GPU log-mel -> SpecAugment + Mixup -> forward ->
    soft-label loss -> backward -> (all-reduce) -> clip + Adam.  Nested as the "ast" object with its
    own value / ms_per_step / roofline (attention forward, the north-star MFMA kernel) / cpu_baseline.
Synthetic 5 s @ 44.1 kHz clips resident in HBM.  `--model envnet|ast` times one leg only (profiling).

python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one process per GPU: under a launcher
(torch.distributed.run: RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in the env) WORLD_SIZE must equal N;
without one, this process starts ``torch.distributed.run --nproc-per-node N`` itself (before it
touches the GPU) and exits with its status.  Every rank checks dist.get_world_size() == N.  Rank 0
prints ONE line; for N > 1 it carries each rank's exposed gradient-exchange time ("comm").
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import subprocess
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

# probe tags whose roofline is HBM bandwidth (the rest are MFMA-bound contractions)
HBM_TAGS = {"optim.step", "logmel.fwd", "conv1.fwd", "conv1.wgrad"}


T_START = time.time()


def log(msg):
    """Progress on stderr (a long silent run looks hung to the GPU harness)."""
    print(f"[bench {time.time() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=["both", "envnet", "ast", "ast-fp8"], default="both",
                    help="both = EnvNet-v2 leg + AST bf16 leg + AST fp8-mixed leg (config 5's linears)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU EnvNet batch (default 256)")
    ap.add_argument("--ast-batch", type=int, default=None, help="per-GPU AST batch (default 256)")
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe", default=None, help="comma list of probe tags to time live (default: auto)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL, the product path); gloo only to rehearse N > 1 ranks on one GPU")
    ap.add_argument("--fc1-exchange", choices=["gather", "shard", "allreduce"], default="shard",
                    help="N > 1, EnvNet FC1 weight gradient: all-gather the bf16 operands and defer the averaged "
                         "gradient to the fused Adam GEMM (the N = 1 program), the same with each rank updating "
                         "its row slice only, or materialise + chunked all-reduce")
    return ap.parse_args()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, script: str, argv: list[str]) -> int:
    """One process per GPU through torch.distributed.run on this node (rendezvous on 127.0.0.1); the
    children inherit stdout, so rank 0's JSON line is this process's output.  Must run before anything
    in this process touches the GPU (it never does: the children do the work)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *argv]
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd)


def check_world(requested, world: int) -> None:
    """--gpus N and the process group must agree: a mismatch would time the wrong number of ranks."""
    if requested is not None and requested != world:
        raise SystemExit(f"bench.py: --gpus {requested} but the process group has {world} ranks")


def setup_dist(backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if backend == "gloo":  # rehearsal: ranks may share a device (RCCL refuses duplicate GPUs)
            local %= torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def make_batch(B, T, dev, rank, num_classes=50):
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    wav = 0.1 * torch.randn(B, T, generator=g, device=dev)
    wav = wav / wav.abs().amax(dim=1, keepdim=True)  # peak-normalised like prepare_esc50.py:98-101
    labels = torch.randint(0, num_classes, (B,), generator=g, device=dev)
    return wav, labels, g


def build_envnet_step(args, dev, rank, world, B):
    from src.datasets.augment import bc_mix
    from src.miaudio import kernels as K
    from src.models.envnet_v2 import EnvNetV2
    from src.training.ddp import GradAllReducer
    from src.training.optim import FusedAdam
    torch.manual_seed(42)
    model = EnvNetV2(num_classes=50, dropout=0.5, compute_dtype=args.dtype).to(dev).train()
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    wav, labels, g = make_batch(B, 220_500, dev, rank)
    ddp = GradAllReducer(model, world, fc1_exchange=args.fc1_exchange) if world > 1 else None

    def step():
        if ddp is not None:
            ddp.begin_step()
        x, y, _ = bc_mix(wav, labels, 50, gen=g)
        z = model(x.view(x.shape[0], 1, -1))
        loss, dz, _ = K.soft_ce(z, y, input_sigmoid=False)
        z.backward(dz)
        if ddp is not None:
            ddp.finish()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    step.ddp = ddp
    tags = ["t0b.fwd", "t0b.dgrad", "t0b.wgrad", "conv1.fwd", "conv1.wgrad", "conv2.fwd", "conv2.dgrad",
            "conv2.wgrad", "fc1.fwd", "fc1.wgrad", "fc1.dgrad", "optim.step", "frontend.fwd", "frontend.bwd"]
    workload = "EnvNet-v2 train step (BC-mix, fwd, soft-CE, bwd, clip, Adam), ESC-50 shape"
    return step, ENVNET_FLOP_PER_CLIP, tags, workload


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


def cpu_threads() -> tuple[int, str]:
    """Threads for the CPU baseline: every core this process may run on — the affinity set, capped by
    the cgroup CPU quota (a GPU box's share of a large host: affinity shows all 256 host threads while
    the quota grants 16, and 256 threads on 16 CPUs run 20x slower than 16)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    if quota is not None and quota < aff:
        return quota, f"cgroup cpu.max quota {quota} of {aff} affinity CPUs"
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) < aff:
        return int(env), f"OMP_NUM_THREADS={env} of {aff} affinity CPUs"
    return aff, f"all {aff} affinity CPUs"


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# probe tag -> substrings of its kernel symbols in the rocprof / PMC tables
KERNEL_HINT = {
    "t0b.fwd": ["conv8_kernel<true, true, 2>"],
    "t0b.dgrad": ["conv8_kernel<false, false, 2>"],
    "t0b.wgrad": ["wgrad8_kernel"],
    "conv2.fwd": ["feconv_kernel<32, 16, 2, true>"],
    "conv2.dgrad": ["feconv_kernel<64, 8, 1, false>"],
    "conv2.wgrad": ["fe_wgrad_kernel"],
    "conv1.fwd": ["fe_conv1_kernel"],
    "attn.fwd": ["attn_fwd_kernel"],
    "attn.bwd": ["attn_bwd_prep_kernel", "attn_bwd_fused_kernel", "attn_bwd_dkdv_kernel", "attn_bwd_dq_kernel"],
    "optim.step": ["sqnorm_kernel", "norm_final_kernel", "adam_kernel", "dgemm_kernel<1, 1, true>"],
    "logmel.fwd": ["fft_mel_db_kernel", "clip_stats_kernel", "clip_norm_kernel", "logmel"],
}


def pmc_traffic(model: str, ks: dict, tag: str | None = None):
    """HBM bytes per launch of the probed launch from the committed rocprofv3 PMC summary of the same
    bench command (profiles/<round>_pmc_<model>.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes).  A multi-kernel launch (optim.step, logmel.fwd) sums its kernels;
    a single-kernel tag is matched by its symbol, launches per step and the rocprof average duration
    (which must agree with the live HIP-event time within 10 %)."""
    files = sorted((REPO / "profiles").glob(f"r*_pmc_{model}.json"))
    if not files:
        return None, None
    table = json.loads(files[-1].read_text())["kernels"]
    hints = KERNEL_HINT.get(tag or "", [])
    if len(hints) > 1:
        sel = {n: e for n, e in table.items() if any(h in n for h in hints) and "hbm_bytes" in e}
        if not sel:
            return None, {"file": files[-1].name, "match": None}
        per = sum(e["hbm_bytes"] * e["launches_per_step"] for e in sel.values()) / max(ks["launches_per_step"], 1)
        avg = sum(e["avg_ms"] * e["launches_per_step"] for e in sel.values()) / max(ks["launches_per_step"], 1)
        rel = abs(avg - ks["ms"]) / ks["ms"]
        src = {"file": files[-1].name, "kernels": sorted(sel), "rocprof_ms_per_launch": round(avg, 4),
               "live_vs_rocprof": round(rel, 4)}
        if rel >= 0.10:  # the same 10 % agreement rule as a single-kernel tag: a disagreeing profile's bytes
            src["match"] = None  # describe some other run, so no traffic is attached
            return None, src
        return per, src
    if hints and any(hints[0] in n for n in table):
        table = {n: e for n, e in table.items() if hints[0] in n}
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


def roofline(model: str, tag: str, ks: dict, peak_tf: float):
    traffic, tsrc = pmc_traffic(model, ks, tag)
    kname = "+".join(KERNEL_HINT.get(tag, ["igemm_kernel/dgemm_kernel"]))
    if tsrc and tsrc.get("kernel"):
        kname = tsrc["kernel"].replace("_ZN12_GLOBAL__N_1", "").replace("(anonymous namespace)::", "").split("(")[0]
    if tag in HBM_TAGS:
        ach, peak, unit = ks["gbs"], HBM_PEAK_GBS, "GB/s"
    else:
        ach, peak, unit = ks["tflops"], peak_tf, "TFLOP/s"
    return {"bound": "hbm" if tag in HBM_TAGS else "mfma", "kernel": f"{kname} [{tag}]", "achieved": round(ach, 2),
            "peak": peak, "unit": unit, "frac": round(ach / peak, 4), "traffic": traffic,
            "live_vs_rocprof": (tsrc or {}).get("live_vs_rocprof"), "traffic_source": tsrc,
            "algorithmic_per_launch": {"flop": ks["flop"], "bytes": ks["bytes"]},
            "ms_per_launch": round(ks["ms"], 4), "launches_per_step": ks["launches_per_step"]}


def time_leg(step, probe_tags, args, world, dev, warmup, steps):
    """W untimed steps, then exactly K steps between barrier + synchronize; max over ranks."""
    from src.miaudio import kernels as K
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    log("warm-up done, timing")
    K.PROBE = {t: [] for t in probe_tags}
    ddp = getattr(step, "ddp", None)
    if ddp is not None:
        ddp.timing = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    probes, K.PROBE = K.PROBE, None
    comm = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
        if ddp is not None:
            mine = torch.tensor([ddp.exposed_ms() or 0.0, ddp.backward_ms() or 0.0], device=dev)
            every = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(every, mine)
            nbytes = sum(p.numel() * p.element_size() for p in ddp.params)
            comm = {"exposed_ms_per_step": [round(float(v[0]), 3) for v in every],
                    "exposed_from": "end of the backward's last compute kernel (compute-stream event)",
                    "fwd_bwd_ms_per_step": [round(float(v[1]), 3) for v in every],
                    "allreduce_bytes_per_step": nbytes - ddp.last_gathered_param_bytes,
                    "allgather_bytes_per_rank_per_step": ddp.last_gathered_bytes,
                    "chunks_per_step": ddp.last_chunks, "fc1_exchange": ddp.fc1_exchange,
                    "gathered_per_step": ddp.last_gathered, "backend": dist.get_backend()}
            ddp.timing = None
    kstats = {}
    for tag, recs in probes.items():
        if not recs:
            continue
        dur = sum(e0.elapsed_time(e1) for e0, e1, _, _ in recs) / len(recs)  # ms per launch
        flops, byts = recs[0][2], recs[0][3]
        kstats[tag] = {"ms": dur, "tflops": flops / (dur * 1e-3) / 1e12, "gbs": byts / (dur * 1e-3) / 1e9,
                       "launches_per_step": len(recs) / steps, "flop": flops, "bytes": byts}
    if comm is not None:
        kstats["_comm"] = comm
    return elapsed, float(loss), kstats


ATTN_KERNELS = ("attn_fwd_kernel", "attn_bwd_dkdv_kernel", "attn_bwd_dq_kernel")


def attention_summary(model: str, ks: dict, peak_tf: float):
    """The north-star attention figure two ways: the credited rate of forward + backward live (SURVEY.md §8(d):
    4 N^2 d H per clip forward, twice that backward, the backward's S / dP recompute not credited) against the
    bf16 MFMA peak, and the hardware MFMA utilisation of the three attention kernels from the committed
    rocprofv3 SQ pass of the same bench command (profiles/<round>_sq_<model>.json, tools/sq_summary.py:
    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x the run's own clock x duration)), time-weighted."""
    f, b = ks.get("attn.fwd"), ks.get("attn.bwd")
    res = {}
    if f and b:
        fl = f["flop"] * f["launches_per_step"] + b["flop"] * b["launches_per_step"]
        t = f["ms"] * f["launches_per_step"] + b["ms"] * b["launches_per_step"]
        res["credited_tflops"] = round(fl / (t * 1e-3) / 1e12, 1)
        res["credited_frac"] = round(fl / (t * 1e-3) / 1e12 / peak_tf, 4)
        res["ms_per_step"] = round(t, 3)
    files = sorted((REPO / "profiles").glob(f"r*_sq_{model}.json"))
    if files:
        table = json.loads(files[-1].read_text())["kernels"]
        per, wsum, tsum = {}, 0.0, 0.0
        for name, e in table.items():
            hit = next((k for k in ATTN_KERNELS if k in name), None)
            if hit and e.get("mfma_util") is not None:
                per[hit] = {"mfma_busy": e["mfma_util"], "clock_ghz": e.get("clock_ghz_pmc_run"),
                            "ms_per_step": e.get("ms_trace")}
                wsum += e["mfma_util"] * (e.get("ms_trace") or 0.0)
                tsum += e.get("ms_trace") or 0.0
        if per:
            res["mfma_busy"] = {"source": files[-1].name, "kernels": per,
                                "time_weighted": round(wsum / tsum, 4) if tsum else None}
    return res or None


def leg_result(model, B, world, steps, warmup, elapsed, loss, kstats, flop_per_clip, args, workload,
               roof_tag=None):
    ms = elapsed / steps * 1e3
    comm = kstats.pop("_comm", None)
    regions = {k: v for k, v in kstats.items() if k.startswith("frontend.")}
    ks = {k: v for k, v in kstats.items() if k not in regions}
    peak_tf = BF16_MFMA_PEAK_TF if args.dtype == "bf16" else F32_PEAK_TF
    dom = max(ks, key=lambda k: ks[k]["ms"] * ks[k]["launches_per_step"]) if ks else None
    name = {"envnet": "EnvNet-v2", "ast": "AST", "ast_fp8": "AST fp8-mixed"}[model]
    out = {
        "metric": f"training clips/sec ({name}, ESC-50 shape)",
        "value": round(B * world * steps / elapsed, 2), "unit": "clips/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (peak-normalised 0.1*N(0,1) clips, uniform labels)",
        "config": {"workload": workload, "global_batch": B * world, "per_gpu_batch": B, "clip_samples": 220_500,
                   "parallelism": f"dp{world}" + ("" if world == 1 or args.dist_backend == "nccl"
                                                  else f" ({args.dist_backend} rehearsal, not RCCL)")},
        "roofline": roofline(model, roof_tag or dom, ks[roof_tag or dom], peak_tf) if (roof_tag or dom) in ks else None,
        "dominant_kernel": roofline(model, dom, ks[dom], peak_tf) if dom and roof_tag else None,
        "step_tflops": round(flop_per_clip * B / (ms * 1e-3) / 1e12, 2),
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in ks.items()},
        "loss": loss,
    }
    if comm is not None:
        out["comm"] = comm
    if model == "envnet":
        out["frontend_path"] = frontend_summary(regions, B)
    if model.startswith("ast"):
        out["attention"] = attention_summary(model, ks, peak_tf)
    if out["dominant_kernel"] is None:
        out.pop("dominant_kernel")
    return out


CPU_WARMUP = 2  # BASELINE.md §3 / SURVEY.md §8(d): 2 warm-up and >= 5 timed steps


def cpu_baseline_envnet(threads: int, batch: int, steps: int):
    """Oracle (CPU restatement of the reference path) timed on this host: BC-mix + fwd + loss + bwd +
    clip + Adam (kind "port")."""
    sys.path.insert(0, str(REPO))
    import random

    from oracle import augment as oaug
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
    pool = [torch.randn(1, 220_500, generator=gen) * 0.1 for _ in range(2 * batch)]
    pool_labels = [int(v) for v in torch.randint(0, 50, (2 * batch,), generator=gen)]
    rng = random.Random(0)

    def one():
        xs, ys = [], []
        for b in range(batch):  # per-sample BC mixing as in the reference's DataLoader workers
            m, y, _, _, _ = oaug.apply_bc_mixing(pool[b], pool_labels[b], pool, pool_labels, 50, rng)
            xs.append(m)
            ys.append(y)
        z = oenv.forward(params, torch.stack(xs), training=True)
        loss = otrain.soft_ce(z, torch.stack(ys))
        loss.backward()
        torch.nn.utils.clip_grad_norm_([params[n] for n in names], 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(CPU_WARMUP):
        one()
    t0 = time.perf_counter()
    for i in range(steps):
        one()
        log(f"  cpu EnvNet B={batch} step {i + 1}/{steps}")
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"oracle EnvNet-v2 f32 train step (BC-mix, fwd, loss, bwd, clip, Adam), batch {batch}, "
                      f"{steps} timed steps after {CPU_WARMUP} warm-ups, {dt:.1f} s of CPU work on {threads} threads "
                      f"of {cpu_model()}", "warmup": CPU_WARMUP, "steps": steps}


def cpu_baseline_ast(threads: int, batch: int = 2, steps: int = 5):
    """Oracle AST train step on this host with the feature path included: log-mel of the waveform
    (ASTPreprocessor restatement), SpecAugment + Mixup per clip, fwd, loss, bwd, clip, Adam."""
    sys.path.insert(0, str(REPO))
    import random

    from oracle import ast as oast
    from oracle import augment as oaug
    from oracle import logmel as olog
    from oracle import train as otrain
    torch.set_num_threads(threads)
    hw, hb = oast.head_hash(900, 50)
    params = {k: v.clone().requires_grad_(True) for k, v in oast.model_params(oast.deit_hash_state(300), hw, hb).items()}
    opt = torch.optim.Adam(list(params.values()), lr=1e-4, weight_decay=1e-4)
    gen = torch.Generator().manual_seed(0)
    wav = (torch.randn(batch, 220_500, generator=gen) * 0.1).numpy()
    labels = [int(v) for v in torch.randint(0, 50, (batch,), generator=gen)]
    rng = random.Random(0)

    def one():
        spec = olog.logmel(wav)                                    # (B, 128, 1379)
        pool = [spec[b:b + 1] for b in range(batch)]
        xs, ys = [], []
        for b in range(batch):
            s, _ = oaug.specaugment(pool[b], 192, 48, rng)
            s, y, _, _ = oaug.apply_mixup(s, labels[b], pool, labels, 50, 0.5, rng)
            xs.append(s)
            ys.append(y)
        probs = oast.forward(params, torch.cat(xs))
        loss = otrain.soft_ce(probs, torch.stack(ys))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(params.values()), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(CPU_WARMUP):
        one()
    t0 = time.perf_counter()
    for i in range(steps):
        one()
        log(f"  cpu AST B={batch} step {i + 1}/{steps}")
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 4), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"oracle AST f32 train step (log-mel, SpecAugment+Mixup, fwd, loss, bwd, clip, Adam), "
                      f"batch {batch}, {steps} timed steps after {CPU_WARMUP} warm-ups, {dt:.1f} s of CPU work on "
                      f"{threads} threads of {cpu_model()}", "warmup": CPU_WARMUP, "steps": steps}


def hbm_calibration(dev, gib: int = 2, iters: int = 5):
    """This box's HBM streaming rate, measured in this process: a 2 GiB -> 2 GiB float4 copy
    (``mia_stream_copy``: 4 groups in flight per thread, non-temporal), read + write bytes over the HIP-event
    time on the launch stream.  Boxes differ (the fused FC1 Adam GEMM streamed the same bytes at 6.1 TB/s on
    one box and 5.0-5.3 on others), so HBM-bound kernels report ``frac_vs_box`` = achieved / this rate beside
    ``frac`` = achieved / the 8 TB/s spec."""
    from src.miaudio import lib as L
    n = gib << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    lib, s = L.load(), L.stream_ptr()
    for _ in range(2):
        L.check(lib.mia_stream_copy(src.data_ptr(), dst.data_ptr(), n, s), "stream_copy")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream())
    for _ in range(iters):
        L.check(lib.mia_stream_copy(src.data_ptr(), dst.data_ptr(), n, s), "stream_copy")
    e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    del src, dst
    torch.cuda.empty_cache()
    return {"kernel": "stream_copy_kernel (mia_stream_copy)", "copy_bytes": n, "traffic_bytes": 2 * n,
            "ms": round(ms, 4), "gbs": round(2 * n / (ms * 1e-3) / 1e9, 1),
            "frac_of_spec": round(2 * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def mfma_calibration(dev, iters: int = 16384, reps: int = 5):
    """This box's bf16 MFMA rate, measured in this process: every SIMD issuing back-to-back
    ``v_mfma_f32_16x16x32_bf16`` on pseudo-random operands (``mia_mfma_rate``: 2 waves per SIMD, 4 independent
    accumulators each), FLOPs over the HIP-event time on the launch stream.  The clock a box holds under an MFMA
    load differs box to box (whole AST legs moved 3-5 % between boxes with every MFMA kernel moving together),
    so MFMA-bound figures report ``frac_vs_box`` = achieved / this rate beside ``frac`` = achieved / the
    2.5 PF spec."""
    from src.miaudio import lib as L
    lib, s = L.load(), L.stream_ptr()
    wps = 2
    sink = torch.empty(int(lib.mia_mfma_rate_sink_floats(wps)), dtype=torch.float32, device=dev)
    L.check(lib.mia_mfma_rate(sink.data_ptr(), iters // 8, wps, s), "mfma_rate")  # warm-up (clock ramp)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        L.check(lib.mia_mfma_rate(sink.data_ptr(), iters, wps, s), "mfma_rate")
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    flop = sink.numel() / 64 * iters * 16 * 16384  # waves x iters x 16 MFMAs x 2*16*16*32
    del sink
    tf = flop / (best * 1e-3) / 1e12
    return {"kernel": "mfma_rate_kernel (mia_mfma_rate)", "instruction": "v_mfma_f32_16x16x32_bf16",
            "flop": flop, "ms": round(best, 4), "tflops": round(tf, 1),
            "frac_of_spec": round(tf / BF16_MFMA_PEAK_TF, 4)}


def add_box_fraction(leg: dict, box_gbs: float, box_tf: float = None):
    """frac_vs_box beside frac for every HBM-bound (copy rate) and MFMA-bound (MFMA rate) figure of a leg."""
    for key in ("roofline", "dominant_kernel"):
        r = leg.get(key)
        if r and r.get("unit") == "GB/s":
            r["frac_vs_box"] = round(r["achieved"] / box_gbs, 4)
        elif r and r.get("unit") == "TFLOP/s" and box_tf and leg.get("dtype", "bf16").startswith(("bf16", "mxfp8")):
            r["frac_vs_box"] = round(r["achieved"] / box_tf, 4)
    fp = leg.get("frontend_path")
    if fp:
        fp["frac_vs_box"] = round(fp["achieved_gbs"] / box_gbs, 4)


def free_leg():
    from src.miaudio import kernels as K
    K._WS.clear()
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, str(Path(__file__).resolve()), sys.argv[1:]))
    world, rank, local = setup_dist(args.dist_backend)
    check_world(args.gpus, dist.get_world_size() if world > 1 else 1)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    calib = hbm_calibration(dev)
    log(f"HBM calibration: {calib['gbs']} GB/s streaming copy on this box")
    mcal = mfma_calibration(dev)
    log(f"MFMA calibration: {mcal['tflops']} TFLOP/s bf16 on this box")
    results = {}
    if args.model in ("both", "envnet"):
        log("EnvNet-v2 leg: building")
        B = args.batch or 256
        step, fpc, tags, workload = build_envnet_step(args, dev, rank, world, B)
        tags = args.probe.split(",") if args.probe else tags
        el, loss, ks = time_leg(step, tags, args, world, dev, args.warmup, args.steps)
        results["envnet"] = leg_result("envnet", B, world, args.steps, args.warmup, el, loss, ks, fpc, args,
                                       workload)
        results["envnet"]["config"]["model"] = "envnet_v2"
        log(f"EnvNet-v2: {results['envnet']['value']} clips/s")
        del step
        free_leg()
    if args.model in ("both", "ast"):
        sys.path.insert(0, str(REPO))
        from bench_ast import build_ast_step
        log("AST leg: building")
        B = args.ast_batch or 256  # AST at batch 256 on one MI355X
        step, fpc, tags, workload = build_ast_step(args, dev, rank, world, B)
        tags = args.probe.split(",") if args.probe else tags
        el, loss, ks = time_leg(step, tags, args, world, dev, args.warmup, args.steps)
        results["ast"] = leg_result("ast", B, world, args.steps, args.warmup, el, loss, ks, fpc, args, workload,
                                    roof_tag="attn.fwd")
        results["ast"]["config"]["model"] = "ast"
        log(f"AST: {results['ast']['value']} clips/s")
        del step
        free_leg()
    if args.model in ("both", "ast-fp8"):
        sys.path.insert(0, str(REPO))
        from bench_ast import build_ast_step
        log("AST fp8-mixed leg: building")
        B = args.ast_batch or 256
        step, fpc, tags, workload = build_ast_step(args, dev, rank, world, B, compute="fp8")
        tags = args.probe.split(",") if args.probe else tags
        el, loss, ks = time_leg(step, tags, args, world, dev, args.warmup, args.steps)
        results["ast_fp8"] = leg_result("ast_fp8", B, world, args.steps, args.warmup, el, loss, ks, fpc, args,
                                        workload, roof_tag="attn.fwd")
        results["ast_fp8"]["config"]["model"] = "ast"
        results["ast_fp8"]["config"]["precision"] = "fp8-mixed"
        results["ast_fp8"]["dtype"] = "mxfp8-e4m3 (block linears fwd) + bf16"
        log(f"AST fp8-mixed: {results['ast_fp8']['value']} clips/s")
        del step
        free_leg()
    if "ast" in results or "ast_fp8" in results:
        from src.miaudio import kernels as K
        K.check_attention_errors()  # raises if a timed step's one-pass attention backward gave up a dQ hand-off
    for leg in results.values():
        add_box_fraction(leg, calib["gbs"], mcal["tflops"])
    out = results.get("envnet") or results.get("ast") or results["ast_fp8"]
    if "envnet" in results and "ast" in results:
        out = dict(results["envnet"])
        out["ast"] = results["ast"]
    if "ast_fp8" in results and out is not results["ast_fp8"]:
        out["ast_fp8"] = results["ast_fp8"]
    out["hbm_calibration"] = calib
    out["mfma_calibration"] = mcal
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads, why = cpu_threads()
        log(f"CPU baseline threads: {threads} ({why})")
        if "envnet" in results:
            log(f"CPU baseline EnvNet-v2 B=4 on {threads} threads")
            b4 = cpu_baseline_envnet(threads, batch=4, steps=8)
            log(f"CPU baseline EnvNet-v2 B=16: B=4 gave {b4['value']} clips/s")
            b16 = cpu_baseline_envnet(threads, batch=16, steps=5)
            out["cpu_baseline"] = dict(b4, samples=[b4, b16], threads_rule=why)
        if "ast" in results:
            target = out["ast"] if "envnet" in results else out
            log("CPU baseline AST B=2")
            target["cpu_baseline"] = dict(cpu_baseline_ast(threads), threads_rule=why)
        log("CPU baselines done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
