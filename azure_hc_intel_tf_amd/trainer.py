"""One synchronous data-parallel training step, HIP-graph captured.

The step is the reference's tf_cnn_benchmarks ``train_op`` with
``--variable_update=horovod --optimizer=momentum`` (/root/reference/benchmark-scripts/
run-tf-sing-ucx-openmpi.sh:62-81):

    zero grads -> fp32 masters -> bf16 GEMM operands (1 launch)
    -> forward (conv/BN/ReLU/pool/affine) -> softmax cross-entropy (+dlogits)
    -> backward (weight grads written straight into the flat gradient buffer)
    -> gradient allreduce (average over workers)
    -> fused momentum update (+L2 weight decay, + L2 term of total_loss) in ONE launch.

On the GPU the whole sequence (≈500-1000 kernels for ResNet-50) is captured once in a HIP
graph (torch.cuda.CUDAGraph == hipGraph on ROCm) and replayed every step, so Python and
launch overhead vanish. With more than one worker the step is captured as one graph per
backward SEGMENT (``model.backward_segments``: one per ResNet stage, last stage first) plus
an optimizer graph; after each segment's replay the gradient ranges it finished are handed
to the communication engine (``parallel/``) asynchronously on its own stream, so the
allreduce of stage 4's gradients overlaps the backward of stages 3..1 and only the last
segment's (small) reduction is exposed. With the native RCCL engine (``graph_safe``) the
collectives are captured INTO the step graph: after each backward segment the engine forks
its comm stream off the capture stream, so the reductions are a parallel branch of one
graph and the step is a single launch. Other reducers (torch.distributed) replay one graph
per segment and issue their collectives from the host between the replays.

roctx ranges (``utils/tracing.py``) mark the step, forward, each backward segment, the
allreduce enqueue and the optimizer, so ``rocprofv3 --marker-trace`` timelines line up with
the kernels. ``comm_profile`` measures allreduce time, exposed communication and overlap.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Optional

import torch

from .nn import layers as L
from .nn.layers import Logits
from .ops import functional as Fn
from .ops import _ext
from .utils.tracing import range_


def resnet_lr_schedule(global_batch: int, num_examples_per_epoch: int = 1281167, base_lr: float = 0.128,
                       warmup_epochs: float = 5.0):
    """tf_cnn_benchmarks ResnetModel.get_learning_rate: linear warmup, then piecewise decay
    at epochs 30/60/80/90; base lr scaled by batch/256."""
    rescaled = base_lr * global_batch / 256.0
    per_epoch = num_examples_per_epoch / float(global_batch)
    bounds = [int(per_epoch * e) for e in (30, 60, 80, 90)]
    vals = [rescaled * v for v in (1, 0.1, 0.01, 0.001, 0.0001)]
    warm = int(per_epoch * warmup_epochs)

    def lr(step: int) -> float:
        if step < warm:
            return rescaled * step / max(warm, 1)
        for b, v in zip(bounds, vals):
            if step < b:
                return v
        return vals[-1]

    return lr


def constant_lr(v: float):
    return lambda step: v


class Trainer:
    def __init__(self, model, batch_size: int, lr_fn: Callable[[int], float], momentum: float = 0.9,
                 weight_decay: float = 4e-5, reducer=None, world_size: int = 1, use_graph: bool = True,
                 nesterov: bool = False, graph_warmup: int = 2, forward_only: bool = False,
                 loss_scale: Optional[float] = None, dynamic_loss_scale: bool = False,
                 loss_scale_interval: int = 1000, force_overlap: bool = False, comm_check: Optional[bool] = None,
                 label_smoothing: float = 0.0):
        self.model = model
        self.label_smoothing = float(label_smoothing)  # --label_smoothing (the loss kernel's targets)
        self.ps = model.ps
        self.B = batch_size
        self.dev = model.device
        self.lr_fn = lr_fn
        self.momentum = momentum
        self.wd = weight_decay
        self.reducer = reducer
        self.world = world_size
        self.nesterov = nesterov
        self.forward_only = forward_only
        if forward_only and hasattr(model, "set_training"):
            model.set_training(False)  # inference BN / no dropout (tf_cnn_benchmarks phase_train=False)
        # every model whose ops run on the HIP kernels (bf16, the IEEE-fp16 build, and fp32 on the
        # bf16-plane GEMMs) is graph-captured; models on the PyTorch path (CPU, or fp32 for a model
        # without the fp32 kernels) run eagerly (MIOpen's first-call searches are not capturable)
        # comm_check (HCB_COMM_CHECK=1 / --comm_check): the race detector of the overlapped
        # allreduce -- every async segment reduction is re-done by a blocking reference
        # allreduce of a snapshot taken before it was issued and the two must agree (a missing
        # stream dependency between backward and the comm stream shows up as a mismatch).
        # Eager steps only (host comparison).
        self.comm_check = (os.environ.get("HCB_COMM_CHECK", "0") == "1") if comm_check is None else comm_check
        self.comm_check_errs = []
        self._check = None
        self.use_graph = (use_graph and self.dev.type == "cuda" and getattr(model, "native", True)
                          and not self.comm_check)
        self.graph_warmup = graph_warmup
        ld = model.fc.ld if hasattr(model, "fc") else (model.num_classes + 7) // 8 * 8
        self.ld = ld
        # loss scaling (tf_cnn_benchmarks --use_fp16 --fp16_loss_scale /
        # --fp16_enable_auto_loss_scale): dlogits scaled by S on the device, gradients unscaled
        # in the optimizer, the step skipped on Inf/NaN; all state device-resident so the
        # captured graph needs no host round trip.
        self.loss_scaling = loss_scale is not None or dynamic_loss_scale
        self.dynamic_ls = dynamic_loss_scale
        S = float(loss_scale or (2.0 ** 15 if dynamic_loss_scale else 1.0))
        h = [0.0, momentum, weight_decay, 1.0 / (world_size * S if self.loss_scaling else world_size)]
        if self.loss_scaling:
            h += [0.0, S, 0.0, float(loss_scale_interval)]
        self.hyper = torch.tensor(h, dtype=torch.float32, device=self.dev)
        self._lr_dev = None  # the learning rate last written to hyper[0]
        self.row_loss = torch.zeros(batch_size, dtype=torch.float32, device=self.dev)
        self.dlogits = torch.zeros((batch_size, ld), dtype=model.act_dtype, device=self.dev)
        # 16-bit dlogits on the HIP path: the loss kernel also writes them unrounded, the
        # classifier's bias gradient source (nn/layers.py Logits.backward)
        self.dlogits32 = None
        fc = getattr(model, "fc", None)
        if (self.dev.type == "cuda" and getattr(model, "native", False) and model.act_dtype != torch.float32
                and isinstance(fc, Logits)):
            self.dlogits32 = torch.zeros((batch_size, ld), dtype=torch.float32, device=self.dev)
            fc.dl32 = self.dlogits32
            fc.dl32_src = self.dlogits
        # weight-gradient GEMMs on a side stream (nn/layers.py run_wgrad), HCB_WGRAD_STREAM=1
        self._wg_stream = (torch.cuda.Stream(device=self.dev) if self.dev.type == "cuda"
                           and os.environ.get("HCB_WGRAD_STREAM", "0") == "1" else None)
        # sum of w^2 of the decayed tensors (the reported loss's weight-decay term): on the GPU the
        # optimizer kernel's per-block partials (every slot written each step, no zeroing launch),
        # summed in a fixed order by loss_total -- deterministic; on the CPU one accumulator
        self.l2 = torch.zeros(4096 if self.dev.type == "cuda" else 1, dtype=torch.float32, device=self.dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.dev)
        self.steps_done = 0
        self._g_fb = None
        self._g_opt = None
        self._g_all = None
        self._segs = None
        self._seg_ranges = {}
        self._static = None
        self.logits = None
        self._skip_comm = False  # comm_profile: the same step with the collectives left out
        # overlap the allreduce with backward (segmented graphs + async reducer)
        # (force_overlap: take the segmented multi-GPU path on one rank -- tests / N=1 timing)
        self.overlap = (reducer is not None and (world_size > 1 or force_overlap) and not forward_only
                        and hasattr(reducer, "allreduce_ranges_async_")
                        and os.environ.get("HCB_OVERLAP", "1") != "0")

    # ---------------------------------------------------------------- pieces
    def _forward(self, images, labels):
        if hasattr(self.model, "activate"):
            self.model.activate()
        ps = self.ps
        if ps.statbuf.is_cuda and ps.statbuf.numel() % 4 == 0 and ps.grad.numel() % 4 == 0:
            # one HIP launch clears the gradient and the per-step statistics scratch
            Fn.zero_bufs([ps.statbuf] if self.forward_only else [ps.grad, ps.statbuf])
        else:
            if not self.forward_only:
                ps.zero_grad()
            ps.zero_stats()
        ps.repack()
        with range_("forward"):
            logits = self.model.forward(images)
        self.logits = logits
        Fn.softmax_xent(logits, labels, self.model.num_classes, self.row_loss, self.dlogits, 1.0 / self.B,
                        self.hyper[5:6] if self.loss_scaling else None, self.dlogits32,
                        label_smoothing=self.label_smoothing)

    def _forward_backward(self, images, labels):
        self._forward(images, labels)
        if self.forward_only:
            self.model.clear()
            return
        self.model.backward(self.dlogits)
        L.wgrad_join()

    def _ranges(self, i, layers):
        if i not in self._seg_ranges:
            self._seg_ranges[i] = ([(0, self.ps.grad.numel())] if layers is None
                                   else self.model.grad_ranges(layers))
        return self._seg_ranges[i]

    def _optimizer(self):
        with range_("optimizer"):
            self._optimizer_body()

    def _optimizer_body(self):
        if self.forward_only:
            Fn.loss_total(self.row_loss, self.B, None, 0.0, self.loss)
            return
        if self.l2.numel() == 1:
            self.l2.zero_()
        if self.loss_scaling:
            self.hyper[4:5].zero_()
            Fn.nonfinite(self.ps.grad, self.hyper[4:5])
        Fn.sgd_momentum(self.ps.master, self.ps.momentum, self.ps.grad, self.ps.n_decay, self.hyper, self.l2,
                        self.nesterov)
        if self.loss_scaling:
            Fn.loss_scale_update(self.hyper, self.world, self.dynamic_ls)
        Fn.loss_total(self.row_loss, self.B, self.l2, 0.5 * self.wd, self.loss)

    def _reduce(self):
        if self.reducer is not None and self.world > 1 and not self.forward_only and not self._skip_comm:
            with range_("allreduce"):
                self.reducer.allreduce_(self.ps.grad)

    def _segments_with_comm(self):
        """Backward segment by segment; each finished segment's gradient ranges go to the
        communication engine (asynchronously, on its comm stream) while the next runs."""
        gen = self.model.backward_segments(self.dlogits)
        i = 0
        while True:
            with range_(f"backward.segment{i}"):
                try:
                    layers, _ = next(gen)
                except StopIteration:
                    break
                L.wgrad_join()  # the segment's weight gradients are complete before they are reduced
            if not self._skip_comm:
                if self.comm_check:
                    self._check_snapshot(self._ranges(i, layers))
                with range_(f"allreduce.segment{i}"):
                    self.reducer.allreduce_ranges_async_(self.ps.grad, self._ranges(i, layers))
            else:
                self._ranges(i, layers)
            i += 1
        if not self._skip_comm:
            self.reducer.join()
            if self.comm_check:
                self._check_verify()

    def _check_snapshot(self, ranges):
        """comm_check: copy the segment's local gradient ranges (stream-ordered before the fork)."""
        if self._check is None:
            self._check = torch.zeros_like(self.ps.grad)
            self._check_ranges = []
        g = self.ps.grad
        for off, n in ranges:
            self._check[off:off + n].copy_(g[off:off + n])
            self._check_ranges.append((off, n))

    def _check_verify(self):
        """comm_check: blocking reference allreduce of the snapshots vs the engine's result.

        fp32 wire: every element within 1e-5 of its range's max |value| (summation order only).
        16-bit wire (bf16 / fp16 compression): each rank's input and each of RCCL's world - 1
        partial sums is rounded to the wire format, i.e. by at most ``ulp`` (bf16 2^-8, fp16 2^-11)
        of sum_r |g_r| -- and the engine (cut per segment) and the reference (whole buffer) may sum
        in different orders. So the bound is per ELEMENT: |engine - ref| <= 2 * ulp * world *
        S_i, S_i = sum over ranks of |g_r,i| (an exact fp32 allreduce of |snapshot|). A range whose
        reduction missed or doubled one rank's contribution is off by |g_r,i| ~ S_i / world for
        most elements, far above that bound."""
        ref = self._check
        wire = getattr(self.reducer, "compression", None) or {1: "bf16", 2: "fp16"}.get(
            getattr(self.reducer, "compress", 0))
        ulp = {"bf16": 2.0 ** -8, "fp16": 2.0 ** -11}.get(wire)
        mag = None
        if ulp is not None:
            mag = ref.abs()
            if self.world > 1:
                import torch.distributed as dist

                if not dist.is_initialized():
                    raise RuntimeError("comm check with a compressed wire needs torch.distributed for the "
                                       "per-element bound (sum over ranks of |g|)")
                dist.all_reduce(mag)
        self.reducer.allreduce_(ref)
        g = self.ps.grad
        worst = 0.0
        for off, n in self._check_ranges:
            if n == 0:
                continue
            a, b = g[off:off + n], ref[off:off + n]
            d = (a - b).abs()
            if mag is None:
                scale = float(b.abs().max())
                err = float(d.max())
                rel, bad = err / (scale + 1e-30), err > 1e-5 * scale + 1e-20
            else:
                # fp16 also flushes what underflows its range: 2^-24 per rank, absolute
                floor = self.world * 2.0 ** -24 if wire == "fp16" else 1e-30
                bound = 2.0 * ulp * max(self.world, 1) * mag[off:off + n] + floor
                ratio = d / bound
                i = int(ratio.argmax())
                rel, bad = float(ratio[i]) * 2.0 * ulp * max(self.world, 1), bool(ratio[i] > 1.0)
                err, scale = float(d[i]), float(mag[off + i])
            worst = max(worst, rel)
            if bad:
                raise RuntimeError(f"comm check: reduced gradient range [{off}, {off + n}) differs from the blocking "
                                   f"reference allreduce by {err:.3e} (reference magnitude {scale:.3e}): the "
                                   "overlapped reduction read the gradients before backward had finished writing "
                                   "them")
        self.comm_check_errs.append(worst)
        self._check_ranges = []

    def _eager_step(self, images, labels):
        if self.overlap:
            self._forward(images, labels)
            self._segments_with_comm()
            self._optimizer()
            return
        self._forward_backward(images, labels)
        self._reduce()
        self._optimizer()

    # ---------------------------------------------------------------- graphs
    def _capture(self, images, labels):
        torch.cuda.synchronize()
        single = self.reducer is None or self.world <= 1 or getattr(self.reducer, "graph_safe", False)
        pool = torch.cuda.graph_pool_handle()
        if self.overlap and getattr(self.reducer, "graph_safe", False):
            # ONE graph for the whole step with the collectives inside it: after each backward
            # segment the engine forks its comm stream off the capture stream (fork / join
            # events become graph edges), so the segment's gradient reductions run on a
            # parallel branch of the graph, overlapped with the rest of the backward, and
            # the step is a single launch. (Several graphs with event records between their
            # launches let a later graph start before the previous one had finished on
            # MI355X -- tools/dp_variants.sh.) thread_local capture: the comm watchdog
            # thread may touch its own events meanwhile.
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                    self._forward(images, labels)
                    self._segments_with_comm()
                    self._optimizer()
                self._g_all = g
                self._static = (images, labels)
                torch.cuda.synchronize()
                return
            except RuntimeError as e:  # collectives not capturable here: per-segment graphs
                print(f"[trainer] capturing the collectives failed ({e}); replaying one graph per "
                      "backward segment instead", flush=True)
                torch.cuda.synchronize()
                self.reducer.graph_safe = False
                pool = torch.cuda.graph_pool_handle()
        if self.overlap and not getattr(self.reducer, "graph_safe", False):
            # one graph per backward segment (the first also holds the forward), replayed in
            # capture order (they share one memory pool)
            segs = []
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                self._forward(images, labels)
                gen = self.model.backward_segments(self.dlogits)
                layers, last = next(gen)
                L.wgrad_join()
            segs.append((g, self._ranges(0, layers)))
            while not last:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    layers, last = next(gen)
                    L.wgrad_join()
                segs.append((g, self._ranges(len(segs), layers)))
            gen.close()
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool):
                self._optimizer()
            self._segs, self._g_opt = segs, g2
        elif single and not self.overlap:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                self._forward_backward(images, labels)
                if self.reducer is not None and self.world > 1:
                    self._reduce()
                self._optimizer()
            self._g_all = g
        else:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, pool=pool):
                self._forward_backward(images, labels)
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool):
                self._optimizer()
            self._g_fb, self._g_opt = g1, g2
        self._static = (images, labels)
        torch.cuda.synchronize()

    def step(self, images, labels):
        """One training step; returns the device tensor holding total_loss of this step."""
        with range_("step"):
            return self._step(images, labels)

    def _step(self, images, labels):
        L.WGRAD_SIDE["stream"] = self._wg_stream
        try:
            return self._step_body(images, labels)
        finally:
            L.WGRAD_SIDE["stream"] = None
            L.WGRAD_SIDE["keep"].clear()

    def _step_body(self, images, labels):
        lr = float(self.lr_fn(self.steps_done))
        if lr != self._lr_dev:  # host write outside the graph, only when the schedule moves
            self.hyper[0:1].fill_(lr)
            self._lr_dev = lr
        if not self.use_graph:
            self._eager_step(images, labels)
        else:
            if self._static is not None and (images is not self._static[0] or labels is not self._static[1]):
                raise ValueError("graph-captured trainer needs the same (static) input buffers every step")
            if self._g_all is None and self._g_fb is None and self._segs is None:
                if self.steps_done < self.graph_warmup:
                    self._eager_step(images, labels)
                    self.steps_done += 1
                    return self.loss
                self._capture(images, labels)
            if self._g_all is not None:
                self._g_all.replay()
                if self.reducer is not None and (self.world > 1 or self.overlap):
                    # the replayed graph's collectives make no host call: heartbeat for the
                    # native engine's stall watchdog (one watch cycle per step)
                    mark = getattr(self.reducer, "step_mark", None)
                    if mark is not None:
                        mark()
            elif self._segs is not None:
                for g, rng in self._segs:
                    g.replay()
                    self.reducer.allreduce_ranges_async_(self.ps.grad, rng)
                self.reducer.join()
                self._g_opt.replay()
            else:
                self._g_fb.replay()
                self._reduce()
                self._g_opt.replay()
        self.steps_done += 1
        return self.loss

    # ---------------------------------------------------------------- metrics
    def accuracy(self, labels):
        """(top-1, top-5) accuracy of the last step's logits on ``labels`` as device scalars
        (tf_cnn_benchmarks --print_training_accuracy; the logits of a graph replay live in the
        graph's static output buffer)."""
        if self.logits is None:
            return None
        lg = self.logits[:, :self.model.num_classes].float()
        top = lg.topk(min(5, lg.shape[1]), dim=1).indices
        lab = labels.view(-1, 1).to(top.device)
        top1 = (top[:, :1] == lab).any(dim=1).float().mean()
        top5 = (top == lab).any(dim=1).float().mean()
        return top1, top5

    def comm_profile(self, images, labels, iters: int = 10):
        """Allreduce time, exposed communication and overlap of the data-parallel step
        (SURVEY.md §5 metrics), measured after the timed loop on the same buffers:

        * ``step_ms``: the real step (as timed by the benchmark);
        * ``compute_ms``: the same step with the collectives left out (its own graph);
        * ``allreduce_ms``: the step's gradient reductions alone (all segment ranges, in the
          same bucket schedule, back to back on the comm stream);
        * ``exposed_comm_ms`` = step - compute; ``overlap_pct`` = share of the allreduce
          time hidden under backward.

        The profile runs real optimizer steps (and, for ``compute_ms``, steps whose gradients are
        NOT reduced), so the training state -- fp32 masters, momentum, BN moving statistics and
        shifts, the device hyper-parameters (loss-scale state), ``steps_done`` and the last
        loss / logits -- is snapshotted before and restored after: the model leaves the profile
        exactly as the timed run left it, identical on every rank."""
        if self.reducer is None or self.forward_only or not self.overlap or self.dev.type != "cuda":
            return None
        ps = self.ps
        torch.cuda.synchronize()
        snap = [(t, t.clone()) for t in (ps.master, ps.momentum, ps.buf, ps.persistbuf, self.hyper, self.loss,
                                          self.row_loss)]
        if self.logits is not None:
            snap.append((self.logits, self.logits.clone()))
        steps = self.steps_done
        try:
            return self._comm_profile(images, labels, iters)
        finally:
            torch.cuda.synchronize()
            for t, c in snap:
                t.copy_(c)
            self.steps_done = steps
            self._lr_dev = None  # hyper was restored: the next step rewrites hyper[0]
            ps.repack()
            torch.cuda.synchronize()

    def _comm_profile(self, images, labels, iters):

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / iters

        step_ms = timed(lambda: self.step(images, labels))
        self._skip_comm = True
        try:
            if self.use_graph:
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle()):
                    self._forward(images, labels)
                    self._segments_with_comm()
                    self._optimizer()
                compute_ms = timed(g.replay)
                del g
            else:
                compute_ms = timed(lambda: self._eager_step(images, labels))
        finally:
            self._skip_comm = False
        ranges = [self._seg_ranges[i] for i in sorted(self._seg_ranges)]

        def reduce_all():
            for rng in ranges:
                self.reducer.allreduce_ranges_async_(self.ps.grad, rng)
            self.reducer.join()

        comm = getattr(self.reducer, "comm", None)
        b0 = comm.buckets_issued() if hasattr(comm, "buckets_issued") else None
        allreduce_ms = timed(reduce_all)
        per_step = None
        if b0 is not None:
            per_step = (comm.buckets_issued() - b0) // (iters + 1)
        exposed = max(step_ms - compute_ms, 0.0)
        overlap = 100.0 * (1.0 - min(exposed / allreduce_ms, 1.0)) if allreduce_ms > 0 else None
        return {"step_ms": round(step_ms, 4), "compute_ms": round(compute_ms, 4),
                "allreduce_ms": round(allreduce_ms, 4), "exposed_comm_ms": round(exposed, 4),
                "overlap_pct": None if overlap is None else round(overlap, 1),
                "buckets_per_step": per_step,
                "fusion_threshold_bytes": getattr(self.reducer, "bucket_bytes", None)}


def synthetic_batch(model, batch_size: int, seed: int = 0):
    """tf_cnn_benchmarks synthetic ImageNet: truncated-normal images (mean 127, sd 60) and
    uniform labels in [0, num_classes-1), created once and reused every step."""
    shape = model.input_shape(batch_size)
    dev = model.device
    if dev.type == "cuda" and getattr(model, "native", True):
        img = torch.empty(shape, dtype=model.act_dtype, device=dev)  # (makes the model current)
        lab = torch.empty(batch_size, dtype=torch.int64, device=dev)
        hcb = _ext.ops()
        hcb.synth_images(img, 3, shape[3], 127.0, 60.0, seed + 1)
        hcb.synth_labels(lab, model.num_classes - 1, seed + 2)
        return img, lab
    g = torch.Generator().manual_seed(seed)
    img = torch.empty(shape, dtype=torch.float32)
    img.normal_(0, 1, generator=g)
    img.clamp_(-2, 2).mul_(60.0).add_(127.0)
    if shape[3] > 3:
        img[..., 3:] = 0
    lab = torch.randint(0, model.num_classes - 1, (batch_size,), generator=g, dtype=torch.int64)
    return img.to(dev, model.act_dtype), lab.to(dev)
