"""GPU: config 5's data-parallel leg rehearsed on one GPU -- AST under GradAllReducer.

Two ranks share the one GPU (gloo carries the GPU tensors; RCCL refuses two ranks on one device, and the
8-GPU RCCL run is the driver's).  Each rank runs ASTModel(depth=2) in bf16 and in fp8-mixed (the block
linears' forward GEMMs on MX-fp8 operands) on its own clips, with its own on-GPU log-mel and
SpecAugment + Mixup (per-rank generator, as each Lightning DDP rank augments its own shard): a warm-up
step, a plain step whose gradients are the reference, then the same step (same generator state) under
GradAllReducer, whose buckets leave from inside the AST backward through ``_grad_ready`` on the side
stream and from ``finish()``.  The kernels are deterministic, so every averaged gradient must equal
(g_0 + g_1) * 0.5 of the two ranks' plain gradients bit for bit (Lightning DDP's mean over ranks,
reference configs/base_training.yaml:45-51), and after FusedAdam.step both ranks hold the same
parameters and Adam moments bit for bit."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_training_cpu import _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, compute, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MIA_QUIET="1")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle.synth import synth_waveform
        from src.datasets.augment import spec_augment_mixup
        from src.datasets.features import GpuLogMel
        from src.miaudio import kernels as K
        from src.models.ast import ASTModel
        from src.training.ddp import GradAllReducer
        from src.training.optim import FusedAdam
        dev = torch.device("cuda", 0)
        torch.manual_seed(42)  # identical initial weights on both ranks (the reducer re-broadcasts rank 0's)
        m = ASTModel(num_classes=10, depth=2, compute_dtype=compute).to(dev).train()
        B = 8
        wav = torch.from_numpy(synth_waveform(71 + rank, B, 220_500)).to(dev)
        labels = torch.tensor([(3 * i + rank) % 10 for i in range(B)], device=dev)
        logmel = GpuLogMel(44_100, 128, True, 0.0, 0.5)
        g = torch.Generator(device=dev)

        def step():
            g.manual_seed(1234 + rank)  # the same masks / partners / lambdas every time this rank steps
            spec = logmel(wav)
            spec, y = spec_augment_mixup(spec, labels, 10, 192, 48, 0.5, 0.25, gen=g)
            probs = m(spec)
            _, dprobs, _ = K.soft_ce(probs, y, input_sigmoid=False)
            probs.backward(dprobs)
            return spec.detach().clone(), probs.detach().clone()

        step()  # warm-up
        m.zero_grad(set_to_none=True)
        s1, o1 = step()
        plain = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        m.zero_grad(set_to_none=True)
        s2, o2 = step()  # the same step again: the plain gradients must be bit-reproducible (else nothing below can hold)
        nondet = [n for n, p in m.named_parameters() if not torch.equal(p.grad, plain[n])]
        if nondet:  # where it starts: the input spectrogram, the forward output, or the backward only
            nondet = [f"{len(nondet)} of {len(plain)} differ; spec equal {torch.equal(s1, s2)}, "
                      f"probs equal {torch.equal(o1, o2)}; last: {nondet[-3:]}"] + nondet
        m.zero_grad(set_to_none=True)
        same_init = []
        for n, p in m.named_parameters():  # identical initial weights on both ranks (the reducer broadcasts rank 0's)
            parts = [torch.empty_like(p.detach(), device="cpu") for _ in range(world)]
            dist.all_gather(parts, p.detach().cpu())
            same_init.append(torch.equal(parts[0], parts[1]))
        opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-4, clip=1.0)
        red = GradAllReducer(m, world)
        step()
        red.finish()
        torch.cuda.synchronize()
        mism, nz = [], 0
        for n, p in m.named_parameters():
            parts = [torch.empty_like(plain[n], device="cpu") for _ in range(world)]
            dist.all_gather(parts, plain[n].cpu())
            ref = (parts[0] + parts[1]) * (1.0 / world)
            nz += int(not torch.equal(parts[0], parts[1]))  # the ranks' own gradients really differ
            if p.grad is None or not torch.equal(p.grad.cpu(), ref):
                mism.append((n, None if p.grad is None else float((p.grad.cpu() - ref).abs().max())))
        opt.step()
        torch.cuda.synchronize()
        same = []
        for n, p in m.named_parameters():
            v = torch.cat([p.detach().flatten(), opt.state[p]["exp_avg"].flatten(),
                           opt.state[p]["exp_avg_sq"].flatten()]).cpu()
            parts = [torch.empty_like(v) for _ in range(world)]
            dist.all_gather(parts, v)
            same.append(torch.equal(parts[0], parts[1]))
        lm = K.logmel_error_counts().get(str(dev), (0, 0, None, None))  # the in-kernel FFT self-check
        q.put((rank, red.last_fired, len(plain), nz, mism, all(same), (nondet[:5], all(same_init), lm), None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, 0, 0, 0, [], False, None, traceback.format_exc()))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("compute", ["bf16", "fp8"])
def test_grad_allreducer_ast_two_ranks(compute):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, compute, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, *rest = q.get(timeout=500)
        res[r] = rest
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, (fired, nparam, nz, mism, same, diag, err) in res.items():
        assert err is None, (r, err)
        nondet, same_init, lm = diag
        print(f"rank {r}: log-mel self-check (failed, retried, first failed, first retried) = {lm}")
        assert lm[0] == 0, f"rank {r}: log-mel frames failed the FFT self-check on every try: {lm}"
        assert not nondet, f"rank {r}: plain AST {compute} gradients differ between two identical steps: {nondet}"
        assert same_init, f"rank {r}: the ranks built different initial weights"
        assert fired > 0, "no gradient left through _grad_ready inside the AST backward"
        assert nparam > 20 and nz > nparam // 2, (nparam, nz)
        assert not mism, (r, mism[:5])
        assert same, "ranks diverged after FusedAdam.step"
