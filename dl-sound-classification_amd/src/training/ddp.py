"""Data-parallel gradient exchange over RCCL (torch.distributed "nccl" backend = RCCL on ROCm).

Replaces what Lightning's DDPStrategy -> torch DistributedDataParallel does on the reference path
(configs/base_training.yaml:47-49, scripts/train.py:190-194): rank-0 parameter broadcast at wrap
time, per-step fp32 gradient all-reduce averaged over ranks, and ``broadcast_buffers`` of the
BatchNorm running statistics (BN itself stays per-rank: no SyncBN, as in the reference).

Gradients are exchanged in buckets on a dedicated communication stream.  Models whose backward
reports gradients as they become ready (the EnvNetV2 and AST autograd nodes do, through
``module._grad_ready``) get their buckets launched during the backward, so the transfer of the
FC-head gradients (1.4 GB for EnvNet) overlaps the convolution backward; everything else is flushed
in ``finish()``.  The hook is installed on the wrapped module AND every submodule, because the
drop-in path wraps the LitClassifier while the autograd nodes look for it on the inner model.
A gradient too large for one bucket can also be handed over in row chunks as its producer writes them
(``module._grad_chunk_ready``): EnvNet's FC1 weight gradient (4096 x 84480 f32, 1.38 GB) is computed
as 16 weight-gradient GEMMs of 256 rows (86.5 MB each) and every chunk's all-reduce is launched as
soon as its GEMM is enqueued, so the transfer of the largest gradient starts after 1/16 of its
GEMM instead of after all of it (64-128 MB chunks, FC head first).

``fc1_exchange`` chooses how a gradient that FusedAdam could take deferred (EnvNet's FC1: dW = dY^T X,
never written on one GPU; src/miaudio/kernels.py::defer_weight_grad) crosses the ranks:

* ``"gather"``: the backward hands the reducer its two bf16 operands instead of the product;
  the reducer all-gathers dY (B x 4096, pre-scaled by 1/world) and X (B x 84 480) on the comm stream --
  45 MB per rank instead of a 1.38 GB f32 ring all-reduce -- and ``finish()`` defers the AVERAGED gradient
  (dY_all / world)^T X_all, K = world * B, to FusedAdam exactly as one GPU does.  Every rank runs the same
  sums-only and Adam GEMMs on identical operands, so the parameters stay identical bit for bit, and the
  per-GPU program at N > 1 is the N = 1 program with K = world * B in those two GEMMs.  Above
  ``materialise_k`` gathered rows (world >= 8 at B = 256) the averaged gradient is instead written once by
  the same GEMM with its per-tile sums of squares (the deferred pair recomputes the product; at K = 2048
  that is 5.06 against 4.27 ms per step) -- the same sums, so the same parameters;
* ``"shard"`` (default): the same all-gather of the two bf16 operands, but rank r owns only rows
  [r M / world, (r + 1) M / world) of FC1 (whole 128-row GEMM tiles): its sums-only GEMM covers that row slice
  of the averaged gradient, the per-tile sums of squares of all slices are all-gathered (the slot array of
  the gather form, so the clip norm is the same bit for bit), and FusedAdam's Adam GEMM updates only the
  slice -- 1/world of the product and of the 9 GB of f32 parameter + moment traffic.  The updated bf16 operand
  copy of the slice (K.bf16_shadow) is then all-gathered on the comm stream, overlapping the next forward's
  convolutions; FC1's forward waits for it (K.wait_param).  The f32 master rows and Adam moments of the other
  ranks' slices go stale on purpose; ``sync_sharded()`` all-gathers them (lite.Trainer calls it at every
  epoch end, before validation and checkpointing, and FusedAdam before any step that does not shard).
  Every rank's slice is computed exactly as the gather form computes those rows, so parameters, moments
  and norm equal the gather form's bit for bit;
* ``"allreduce"``: FC1's gradient is materialised as 16 row chunks, each all-reduced as its GEMM is enqueued
  (above).

The per-step BatchNorm buffer broadcast (DDP ``broadcast_buffers``) is one coalesced collective per
dtype, issued after the gradient exchange.  torch DDP broadcasts rank 0's buffers at the start of
each forward; the values it sends there (rank 0's statistics after the previous step's forward) are
the ones sent here at the end of that previous step, so every forward sees the same buffers.

``timing`` (a list, or None): when set, ``begin_step()`` (called before the forward) records a step-start
HIP event and ``finish()`` appends one (step start, compute done, exchange done) triple per step.  "Compute
done" is an event recorded on the compute stream when ``finish()`` is entered, before it enqueues anything:
it completes when the backward's last compute kernel does.  ``exposed_ms()`` is then the time the exchange
ran past the end of the backward (what the backward did not hide), and ``backward_ms()`` the forward +
backward time of the step with the exchange running beside it -- compared with the same figure at N = 1 it
shows how much the concurrent collectives slowed the compute itself (bench.py reports both per rank).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20
# Gathered rows K above which the averaged FC1 gradient is materialised by one GEMM (with per-tile sums of
# squares) instead of deferred: the deferred form runs the product twice (sums-only GEMM in the backward,
# the Adam GEMM in the step), the materialised form once plus a 1.38 GB write and read.  Measured on one
# MI355X (tools/bench_fc1_update.py, EnvNet FC1 4096 x 84 480): K = 256 / 512 / 1024 / 2048 -> deferred
# 1.93 / 2.22 / 2.98 / 5.06 ms, materialised 2.32 / 2.52 / 3.26 / 4.27 ms per update.
MATERIALISE_K = 1536


class GradAllReducer:
    def __init__(self, model: torch.nn.Module, world: int | None = None, bucket_bytes: int = BUCKET_BYTES,
                 broadcast_buffers: bool = True, fc1_exchange: str = "shard",
                 materialise_k: int = MATERIALISE_K):
        if fc1_exchange not in ("gather", "shard", "allreduce"):
            raise ValueError(f"fc1_exchange must be 'gather', 'shard' or 'allreduce', not {fc1_exchange!r}")
        self.fc1_exchange = fc1_exchange
        self.materialise_k = materialise_k
        self.model = model
        self.world = world or dist.get_world_size()
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.sharded = {}  # id -> parameter whose f32 rows / moments outside this rank's slice are stale
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.bucket_bytes = bucket_bytes
        self.broadcast_buffers = broadcast_buffers
        self.cuda = self.params[0].is_cuda
        self.stream = torch.cuda.Stream(self.params[0].device) if self.cuda else None
        self.pending = []
        self.done = set()
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(p.data, 0)
                p._mia_bf16_ver = None  # a collective writes behind autograd's version counter: recast
            for b in model.buffers():
                dist.broadcast(b.data, 0)
        for m in model.modules():
            m._grad_ready = self.grad_ready
            m._grad_chunk_ready = self.grad_chunk_ready
            m._grad_gather = self.grad_gather if fc1_exchange in ("gather", "shard") else None
        self.gathers = []  # (param, dY_all, X_all, M, N, K) launched this step, deferred in finish()
        self.gathered = self.last_gathered = 0
        self.gathered_bytes = self.last_gathered_bytes = 0            # operand bytes each rank sends
        self.gathered_param_bytes = self.last_gathered_param_bytes = 0  # f32 gradient bytes not all-reduced
        self.fired = self.last_fired = 0  # gradients received through _grad_ready per step (tests)
        self.chunks = self.last_chunks = 0  # row chunks launched through _grad_chunk_ready per step
        self.timing = None

    # ------------------------------------------------------------------ async launches
    def _launch(self, tensors):
        if self.cuda:
            ev = torch.cuda.current_stream().record_event()
            self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                work = self._reduce(tensors)
            for t in tensors:
                t.record_stream(self.stream)
        else:
            work = self._reduce(tensors)
        self.pending.append(work)

    def _reduce(self, tensors):
        if len(tensors) == 1:
            flat = tensors[0]
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.mul_(1.0 / self.world)
            return (flat, tensors, False)
        flat = torch.cat([t.reshape(-1) for t in tensors])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.mul_(1.0 / self.world)
        return (flat, tensors, True)

    def grad_ready(self, params_and_grads):
        """Called from inside the backward with a list of (param, grad) that are final."""
        big, small = [], []
        for p, g in params_and_grads:
            if id(p) not in self.index or id(p) in self.done:
                continue
            p.grad = g
            p._mia_sqsum = None  # the averaged gradient is not what the GEMM's per-tile sums describe
            self.done.add(id(p))
            self.fired += 1
            (big if g.numel() * g.element_size() >= self.bucket_bytes // 4 else small).append(g)
        for g in big:
            self._launch([g])
        if small:
            self._launch(small)

    def grad_chunk_ready(self, param, full, rows, last: bool):
        """Called from inside the backward with ``rows``, a contiguous row block of ``full`` (the
        gradient of ``param``) that is final: its all-reduce is launched now, in place.  With ``last``
        the whole gradient is handed to ``param.grad`` (the caller then gives autograd None for it)."""
        if id(param) not in self.index or id(param) in self.done:
            return
        self._launch([rows])
        self.chunks += 1
        if last:
            param.grad = full
            param._mia_sqsum = None
            self.done.add(id(param))
            self.fired += 1

    def _all_gather(self, out, inp):
        """out (world * rows, cols) <- the ranks' inp (rows, cols) in rank order."""
        if dist.get_backend() == "nccl":
            dist.all_gather_into_tensor(out, inp)
        else:  # gloo (rehearsal / CPU tests): list form, then the rank-ordered copy
            parts = list(out.chunk(self.world, 0))
            tmp = [torch.empty_like(inp) for _ in range(self.world)]
            dist.all_gather(tmp, inp)
            for d, t in zip(parts, tmp):
                d.copy_(t)

    def grad_gather(self, param, dy, x) -> bool:
        """Called from inside the backward for a weight gradient dW = dy^T x (dy: (B, M), x: (B, N), bf16)
        that FusedAdam may take deferred.  Returns False (the caller materialises dW as usual) unless the
        parameter defers; otherwise the operands leave now on the comm stream and ``finish()`` defers the
        averaged gradient over all ranks' rows."""
        from ..miaudio import kernels as K
        if id(param) not in self.index or id(param) in self.done or not K.defers_to_fused_adam(param):
            return False
        if param.grad is not None:  # an accumulated gradient is there: materialise and add, as one GPU does
            return False
        if self.world & (self.world - 1):
            # dY / world is exact in bf16 only for a power-of-two world; otherwise the f32 all-reduce path
            # (no extra rounding) carries this gradient
            return False
        B, M = dy.shape
        N = x.shape[1]
        dy_all = torch.empty(self.world * B, M, dtype=dy.dtype, device=dy.device)
        x_all = torch.empty(self.world * B, N, dtype=x.dtype, device=x.device)

        def run():
            dys = dy * (1.0 / self.world)  # exact in bf16: the world is a power of two (checked above)
            self._all_gather(dy_all, dys)
            self._all_gather(x_all, x)
            return dys

        if self.cuda:
            ev = torch.cuda.current_stream().record_event()
            self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                keep = run()
            for t in (dy, x, dy_all, x_all, keep):
                t.record_stream(self.stream)
        else:
            run()
        self.gathers.append((param, dy_all, x_all, M, N, self.world * B))
        self.done.add(id(param))
        self.gathered += 1
        self.gathered_bytes += (dy.numel() + x.numel()) * dy.element_size()
        self.gathered_param_bytes += param.numel() * 4
        return True

    def begin_step(self):
        """Record the step-start event (timing on, CUDA only); call before the forward."""
        self._t_start = None
        if self.cuda and self.timing is not None:
            self._t_start = torch.cuda.Event(enable_timing=True)
            self._t_start.record(torch.cuda.current_stream())

    def exposed_ms(self):
        """Mean over the recorded steps of the time the exchange ran past the end of the backward's last
        compute kernel."""
        if not self.timing:
            return None
        ts = [max(0.0, e0.elapsed_time(e1)) for _, e0, e1 in self.timing]
        return sum(ts) / len(ts)

    def backward_ms(self):
        """Mean over the recorded steps of step start -> the backward's last compute kernel (None unless every
        step called begin_step)."""
        if not self.timing or any(s is None for s, _, _ in self.timing):
            return None
        ts = [s.elapsed_time(e0) for s, e0, _ in self.timing]
        return sum(ts) / len(ts)

    def finish(self):
        """Reduce every gradient not yet reduced, then wait for all buckets (on the compute stream)."""
        t0 = None
        if self.cuda and self.timing is not None:
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(torch.cuda.current_stream())
        rest = [p.grad for p in self.params if p.grad is not None and id(p) not in self.done]
        for p in self.params:
            p._mia_sqsum = None
        bucket, size = [], 0
        for g in rest:
            bucket.append(g)
            size += g.numel() * g.element_size()
            if size >= self.bucket_bytes:
                self._launch(bucket)
                bucket, size = [], 0
        if bucket:
            self._launch(bucket)
        if t0 is not None:
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record(self.stream)
            self.timing.append((getattr(self, "_t_start", None), t0, t1))
            self._t_start = None
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.stream)
        if self.gathers:
            from ..miaudio import kernels as K
            from ..miaudio import lib as L
            for param, dy_all, x_all, M, N, Kk in self.gathers:
                A, B = K.dense(dy_all, L.RC, Kk, M), K.dense(x_all, L.RC, Kk, N)
                if self.fc1_exchange == "shard" and M % (128 * self.world) == 0:
                    self._defer_shard(param, dy_all, x_all, M, N, Kk)
                elif Kk > self.materialise_k:
                    # one GEMM (same main loop and sum order as the deferred pair) writes the gradient and
                    # its per-tile sums of squares; FusedAdam then streams it like any other gradient
                    dW = torch.empty(M, N, dtype=torch.float32, device=dy_all.device)
                    sq = K.sqsum_slots(dW, M, N)
                    K.gemm(A, B, K.epilogue(dW, N, sqsum=sq), M, N, Kk, L.BF16, tag="fc1.wgrad")
                    param.grad = dW.view_as(param)
                    K.tag_sqsum(param, dW, sq)
                else:
                    K.defer_weight_grad(param, A, B, M, N, Kk, keep=(dy_all, x_all), tag="fc1.wgrad")
            self.gathers.clear()
        for flat, tensors, copied in self.pending:
            if copied:
                off = 0
                for t in tensors:
                    n = t.numel()
                    t.copy_(flat[off:off + n].view_as(t))
                    off += n
        self.pending.clear()
        self.done.clear()
        self.last_fired, self.fired = self.fired, 0
        self.last_chunks, self.chunks = self.chunks, 0
        self.last_gathered, self.gathered = self.gathered, 0
        self.last_gathered_bytes, self.gathered_bytes = self.gathered_bytes, 0
        self.last_gathered_param_bytes, self.gathered_param_bytes = self.gathered_param_bytes, 0
        if self.broadcast_buffers:
            self._broadcast_buffers()

    # ------------------------------------------------------------------ fc1_exchange="shard"
    def _defer_shard(self, param, dy_all, x_all, M, N, Kk):
        """Defer this rank's row slice of the averaged gradient (dY_all[:, slice])^T X_all to FusedAdam, with
        the per-tile sums of squares of ALL slices (one all-gather of f64 slots) for the clip norm."""
        from ..miaudio import kernels as K
        from ..miaudio import lib as L
        if getattr(param, "_mia_deferred", None) is not None:
            raise RuntimeError("a deferred weight gradient is still pending: call FusedAdam.step() between "
                               "backward passes")
        w, r = self.world, self.rank
        Ms = M // w
        r0 = r * Ms
        sq = torch.empty(int(L.load().mia_gemm_sqsum_slots(M, N)), dtype=torch.float64, device=dy_all.device)
        per = sq.numel() // w  # slots are row-block-major (128 x 128 tiles): a slice's slots are contiguous
        A = K.dense(dy_all[:, r0:], L.RC, Kk, Ms, ld=M)
        B = K.dense(x_all, L.RC, Kk, N)
        mine = sq[r * per:(r + 1) * per]
        K.gemm_sqsum_only(A, B, Ms, N, Kk, mine, tag="fc1.wgrad")
        self._all_gather(sq, mine.clone())
        param._mia_deferred = dict(A=A, B=B, M=Ms, N=N, K=Kk, sq=sq, keep=(dy_all, x_all), row0=r0, rows_total=M,
                                   shard=self)

    def after_shard_update(self, param, shadow, d):
        """FusedAdam has updated rows [row0, row0 + M) of ``param`` (and of its bf16 copy ``shadow``): all-gather
        the updated operand rows on the comm stream; FC1's next forward waits for them (K.wait_param)."""
        r0, Ms, M = d["row0"], d["M"], d["rows_total"]
        full = (shadow if shadow is not None else param.data).view(M, -1)

        def run():
            self._all_gather(full, full[r0:r0 + Ms].clone())

        if self.cuda:
            ev = torch.cuda.current_stream().record_event()
            self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                run()
                param._mia_ready = torch.cuda.current_stream().record_event()
            full.record_stream(self.stream)
        else:
            run()
        param._mia_shard = (self, r0, Ms, M)
        self.sharded[id(param)] = param

    @torch.no_grad()
    def sync_param(self, param):
        """All-gather the f32 master rows and Adam moments of a sharded parameter, so every rank holds all of
        them (a collective: every rank calls it at the same point)."""
        from ..miaudio import kernels as K
        info = getattr(param, "_mia_shard", None)
        if info is None:
            return
        _, r0, Ms, M = info
        K.wait_param(param)
        ref = getattr(param, "_mia_fused_adam", None)
        st = getattr(ref() if callable(ref) else None, "state", {}).get(param)  # FusedAdam's moments
        ts = [param.data]
        if st:
            ts += [st["exp_avg"], st["exp_avg_sq"]]
        for t in ts:
            t2 = t.view(M, -1)
            self._all_gather(t2, t2[r0:r0 + Ms].clone())
        param._mia_shard = None
        self.sharded.pop(id(param), None)

    def sync_sharded(self):
        """sync_param for every parameter this reducer sharded (epoch end: before validation / checkpoint)."""
        for p in list(self.sharded.values()):
            self.sync_param(p)

    @torch.no_grad()
    def _broadcast_buffers(self):
        """Rank 0's BatchNorm running statistics (+ counters) to every rank: one flat broadcast per
        dtype instead of one collective per buffer."""
        groups = {}
        for b in self.model.buffers():
            groups.setdefault((b.dtype, b.device), []).append(b)
        for bufs in groups.values():
            flat = torch.cat([b.reshape(-1) for b in bufs])
            dist.broadcast(flat, 0)
            off = 0
            for b in bufs:
                n = b.numel()
                b.copy_(flat[off:off + n].view_as(b))
                off += n
