"""AST leg of bench.py (`python bench.py --model ast`): BASELINE.json configs[2].

Timed by bench.py (the nested "ast" object of the default run).  One step = on-GPU log-mel of 5 s @ 44.1 kHz clips (1379 frames x 128 mels) -> SpecAugment + Mixup
against the batch -> AST (DeiT-base/384 geometry, 12 blocks, 1645 tokens, random init: no
checkpoint offline) forward -> soft-label loss (softmax on the sigmoid outputs, as reference
engine.py:175-176 does with ast.py:64) -> backward -> (N>1: RCCL all-reduce) -> clip 1.0 + Adam.
"""
from __future__ import annotations

import os

import torch

AST_FLOP_PER_CLIP = 1139.7e9  # fwd+bwd at 1645 tokens (flop_counter)


def build_ast_step(args, dev, rank, world, B, compute=None):
    os.environ.setdefault("MIA_QUIET", "1")
    from src.datasets.augment import spec_augment_mixup
    from src.datasets.features import GpuLogMel
    from src.miaudio import kernels as K
    from src.models.ast import ASTModel
    from src.training.ddp import GradAllReducer
    from src.training.optim import FusedAdam

    torch.manual_seed(42)
    model = ASTModel(num_classes=50, compute_dtype=compute or args.dtype).to(dev).train()
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    ddp = GradAllReducer(model, world) if world > 1 else None
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    wav = 0.1 * torch.randn(B, 220_500, generator=g, device=dev)
    wav = wav / wav.abs().amax(dim=1, keepdim=True)
    labels = torch.randint(0, 50, (B,), generator=g, device=dev)
    logmel = GpuLogMel(44_100, 128, True, 0.0, 0.5)

    def step():
        if ddp is not None:
            ddp.begin_step()
        spec = logmel(wav)
        spec, y = spec_augment_mixup(spec, labels, 50, 192, 48, 0.5, 0.25, gen=g)
        probs = model(spec)
        loss, dprobs, _ = K.soft_ce(probs, y, input_sigmoid=False)
        probs.backward(dprobs)
        if ddp is not None:
            ddp.finish()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    step.ddp = ddp
    tags = ["attn.fwd", "attn.bwd", "qkv.fwd", "proj.fwd", "fc1.fwd", "fc2.fwd", "qkv.wgrad", "qkv.dgrad",
            "proj.wgrad", "proj.dgrad",
            "fc1.wgrad", "fc1.dgrad", "fc2.wgrad", "fc2.dgrad", "logmel.fwd", "optim.step"]
    workload = ("AST train step (log-mel, SpecAugment+Mixup, fwd, soft-CE, bwd, clip, Adam), "
                "5 s @ 44.1 kHz -> 128x1379 log-mel -> 1645 tokens, DeiT-base/384 geometry")
    if (compute or args.dtype) == "fp8":
        workload += ("; trainer.precision=fp8-mixed: block linears' forward GEMMs on MX-fp8 operands "
                     "(e4m3 + E8M0 per 32, v_mfma_scale_f32_16x16x128_f8f6f4), the rest bf16")
    return step, AST_FLOP_PER_CLIP, tags, workload
