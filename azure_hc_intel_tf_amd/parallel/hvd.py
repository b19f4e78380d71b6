"""Horovod-compatible data-parallel API on RCCL (MI355X) / gloo (CPU).

The reference drives Horovod through tf_cnn_benchmarks ``--variable_update=horovod``
(/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:77-78, installed at
/root/reference/install-scripts/install_conda_tf_hvd.sh:24; SURVEY.md §2.2 "Horovod Python
API", §3.5). This module gives the same surface -- ``init / rank / size / local_rank /
local_size / cross_rank / allreduce / allgather / broadcast / broadcast_parameters /
broadcast_optimizer_state / broadcast_global_variables / DistributedOptimizer /
Compression`` -- on top of one process per GPU:

* rendezvous = the launcher's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT), not MPI;
* collectives = torch.distributed with backend "nccl" (== RCCL over xGMI on ROCm) for GPU
  tensors and gloo for CPU tensors (``--horovod_device=cpu`` semantics);
* the fused gradient allreduce of the training engine is the bucketed flat-buffer reducer
  (``parallel/reducer.py``) or the native C++ RCCL engine (``parallel/native.py``).

Horovod knobs honoured: HOROVOD_FUSION_THRESHOLD (bucket bytes), HOROVOD_TIMELINE (Chrome
trace of collectives), HOROVOD_STALL_CHECK_TIME_SECONDS (watchdog), HOROVOD_MPI_THREADS_DISABLE
(accepted, meaningless without MPI).
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, Iterable, List, Optional, Union

import torch
import torch.distributed as dist

from .compression import Compression  # noqa: F401  (re-export)
from .monitor import tracked
from .reducer import fusion_threshold_bytes, make_buckets

_state = {"initialized": False, "owns_pg": False, "cpu_group": None}


class Average:  # op tags, horovod.torch style
    pass


class Sum:
    pass


Adasum = None  # not supported (absent from the reference's Horovod era)


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init(backend: Optional[str] = None, timeout_s: float = 1800.0) -> None:
    """Initialise from the launcher environment. Single process if WORLD_SIZE is unset."""
    if _state["initialized"]:
        return
    world = _env_int("WORLD_SIZE", 1)
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            lr = _env_int("LOCAL_RANK", 0)
            torch.cuda.set_device(lr)
            kw["device_id"] = torch.device("cuda", lr)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
        _state["owns_pg"] = True
    if dist.is_initialized() and dist.get_backend() != "gloo":
        # host-side objects (allgather of python objects, cpu tensors) use a gloo side group
        _state["cpu_group"] = dist.new_group(backend="gloo")
    _state["initialized"] = True


def is_initialized() -> bool:
    return _state["initialized"]


def shutdown() -> None:
    from . import monitor as _monitor

    _monitor.reset()  # stop the stall inspector, write HOROVOD_TIMELINE
    if _state["owns_pg"] and dist.is_initialized():
        dist.destroy_process_group()
    _state.update(initialized=False, owns_pg=False, cpu_group=None)


def _dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def size() -> int:
    return dist.get_world_size() if _dist() else 1


def rank() -> int:
    return dist.get_rank() if _dist() else 0


def local_rank() -> int:
    return _env_int("LOCAL_RANK", rank())


def local_size() -> int:
    return _env_int("LOCAL_WORLD_SIZE", size())


def cross_rank() -> int:
    return _env_int("GROUP_RANK", rank() // max(local_size(), 1))


def cross_size() -> int:
    return max(size() // max(local_size(), 1), 1)


def mpi_threads_supported() -> bool:
    return False


def mpi_enabled() -> bool:
    return False


def nccl_built() -> bool:
    return torch.cuda.is_available()


def _group_for(t: torch.Tensor):
    if not t.is_cuda and _state["cpu_group"] is not None:
        return _state["cpu_group"]
    return None


# ---------------------------------------------------------------------- collectives
def allreduce_(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
               compression=Compression.none, op=None) -> torch.Tensor:
    if average is None:
        average = op is not Sum
    if not _dist() or size() == 1:
        return tensor
    c, ctx = compression.compress(tensor)
    with tracked(f"allreduce.{name or 'tensor'}", c.numel() * c.element_size()):
        dist.all_reduce(c, group=_group_for(c))
    out = compression.decompress(c, ctx)
    if average:
        out = out / size() if not out.is_floating_point() else out.mul_(1.0 / size())
    if out is not tensor:
        tensor.copy_(out)
    return tensor


def allreduce(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
              compression=Compression.none, op=None) -> torch.Tensor:
    return allreduce_(tensor.clone(), average=average, name=name, compression=compression, op=op)


def grouped_allreduce_(tensors: List[torch.Tensor], average=True, compression=Compression.none):
    """Fused allreduce of many tensors through one flat buffer per dtype (tensor fusion)."""
    if not _dist() or size() == 1 or not tensors:
        return tensors
    by_dtype: Dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (_, _), ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        bucket = max(fusion_threshold_bytes() // flat.element_size(), 64)
        for off, n in make_buckets(flat.numel(), bucket):
            allreduce_(flat[off:off + n], average=average, compression=compression)
        o = 0
        for t in ts:
            t.copy_(flat[o:o + t.numel()].view_as(t))
            o += t.numel()
    return tensors


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Concatenate along dim 0 across ranks; first dimensions may differ per rank."""
    if not _dist() or size() == 1:
        return tensor.clone()
    g = _group_for(tensor)
    n = torch.tensor([tensor.shape[0]], dtype=torch.int64, device=tensor.device)
    sizes = [torch.zeros_like(n) for _ in range(size())]
    dist.all_gather(sizes, n, group=g)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    pad[:tensor.shape[0]] = tensor
    outs = [torch.empty_like(pad) for _ in range(size())]
    dist.all_gather(outs, pad, group=g)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)], dim=0)


def allgather_object(obj):
    if not _dist() or size() == 1:
        return [obj]
    out = [None] * size()
    dist.all_gather_object(out, obj, group=_state["cpu_group"])
    return out


def broadcast_(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    if _dist() and size() > 1:
        dist.broadcast(tensor, src=root_rank, group=_group_for(tensor))
    return tensor


def broadcast(tensor: torch.Tensor, root_rank: int = 0, name: Optional[str] = None) -> torch.Tensor:
    return broadcast_(tensor.clone(), root_rank, name)


def broadcast_object(obj, root_rank: int = 0):
    if not _dist() or size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=root_rank, group=_state["cpu_group"])
    return lst[0]


def barrier():
    if _dist() and size() > 1:
        dist.barrier()


def broadcast_parameters(params: Union[Dict[str, torch.Tensor], Iterable], root_rank: int = 0) -> None:
    """horovod.torch.broadcast_parameters: dict (state_dict / named_parameters) or list of pairs."""
    if isinstance(params, dict):
        items = sorted(params.items())
    else:
        items = list(params)
        if items and not isinstance(items[0], tuple):
            items = [(str(i), p) for i, p in enumerate(items)]
    with torch.no_grad():
        for _, p in items:
            t = p.data if hasattr(p, "data") else p
            broadcast_(t, root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    """horovod.torch.broadcast_optimizer_state for torch.optim optimizers (tensors in state)."""
    state = optimizer.state_dict()
    for _, st in sorted(state["state"].items()):
        for k, v in sorted(st.items()):
            if torch.is_tensor(v):
                broadcast_(v, root_rank)
    optimizer.load_state_dict(state)


def broadcast_global_variables(model_or_store, root_rank: int = 0) -> None:
    """hvd.broadcast_global_variables(0) of tf_cnn_benchmarks: every variable of the model
    (flat fp32 masters, momentum slots and BN moving statistics) from ``root_rank``."""
    ps = getattr(model_or_store, "ps", model_or_store)
    broadcast_(ps.master, root_rank)
    broadcast_(ps.momentum, root_rank)
    broadcast_(ps.buf, root_rank)


class DistributedOptimizer(torch.optim.Optimizer):
    """horovod.torch.DistributedOptimizer for ordinary torch modules: gradients are averaged with
    fused, bucketed allreduces before the wrapped optimizer's step. Gradients of a bucket are
    launched from autograd hooks as soon as the whole bucket is ready (overlap with backward)."""

    def __init__(self, optimizer: torch.optim.Optimizer, named_parameters=None, compression=Compression.none,
                 backward_passes_per_step: int = 1, op=Average):
        self.__dict__["_opt"] = optimizer
        self._compression = compression
        self._average = op is not Sum
        self._bpps = backward_passes_per_step
        params = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
        self._params = params
        self._counter = 0
        self._handles = []
        self._bucket_of = {}
        self._buckets: List[List[torch.Tensor]] = []
        self._pending: Dict[int, int] = {}
        self._launched = set()
        self._next = 0  # next bucket to launch (buckets go out strictly in order)
        limit = fusion_threshold_bytes()
        cur, cur_bytes = [], 0
        for p in reversed(params):  # backward produces the last layers' grads first
            nb = p.numel() * p.element_size()
            if cur and cur_bytes + nb > limit:
                self._buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            self._buckets.append(cur)
        for bi, b in enumerate(self._buckets):
            for p in b:
                self._bucket_of[p] = bi
        if _dist() and size() > 1:
            for p in params:
                p.register_post_accumulate_grad_hook(self._hook)

    def __getattr__(self, k):
        return getattr(self.__dict__["_opt"], k)

    @property
    def param_groups(self):
        return self._opt.param_groups

    @property
    def state(self):
        return self._opt.state

    def _hook(self, p):
        if (self._counter + 1) % self._bpps != 0:
            return
        bi = self._bucket_of[p]
        self._pending[bi] = self._pending.get(bi, 0) + 1
        # launch strictly in bucket order: a ready bucket waits for every earlier one, so all
        # ranks issue their collectives in the same order even when a data-dependent branch
        # leaves a bucket incomplete on some ranks only (it is then launched by synchronize(),
        # together with everything behind it -- no negotiation round needed)
        while self._next < len(self._buckets) and self._pending.get(self._next, 0) == len(self._buckets[self._next]):
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        ps = self._buckets[bi]
        for q in ps:  # a parameter that got no gradient this step contributes zeros (Horovod)
            if q.grad is None:
                q.grad = torch.zeros_like(q)
        grads = [q.grad for q in ps]
        flat = torch.cat([g.reshape(-1) for g in grads])
        c, ctx = self._compression.compress(flat)
        work = dist.all_reduce(c, async_op=True, group=_group_for(c))
        self._handles.append((work, c, ctx, flat, grads))
        self._launched.add(bi)

    def synchronize(self):
        # buckets whose parameters did not all receive a gradient (unused branch, frozen layer),
        # and every bucket behind the first such one, were not launched from the hooks: reduce
        # them now, continuing the same bucket order -- identical on every rank
        while self._next < len(self._buckets):
            self._launch(self._next)
            self._next += 1
        for work, c, ctx, flat, grads in self._handles:
            work.wait()
            out = self._compression.decompress(c, ctx)
            if self._average:
                out = out / size()
            o = 0
            for g in grads:
                g.copy_(out[o:o + g.numel()].view_as(g))
                o += g.numel()
        self._handles.clear()
        self._pending.clear()
        self._launched.clear()
        self._next = 0

    def step(self, closure=None):
        self._counter += 1
        if _dist() and size() > 1:
            if self._counter % self._bpps != 0:
                return None
            self.synchronize()
            if self._bpps > 1:
                for p in self._params:
                    if p.grad is not None:
                        p.grad.div_(self._bpps)
        return self._opt.step(closure)

    def zero_grad(self, set_to_none: bool = True):
        if self._counter % self._bpps == 0:
            self._opt.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self._opt.state_dict()

    def load_state_dict(self, sd):
        return self._opt.load_state_dict(sd)


class BroadcastGlobalVariablesHook:
    """tf.train.SessionRunHook analogue: call once after model creation."""

    def __init__(self, root_rank: int = 0):
        self.root_rank = root_rank

    def __call__(self, model_or_store):
        broadcast_global_variables(model_or_store, self.root_rank)
