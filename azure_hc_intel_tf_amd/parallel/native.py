"""Python face of the native C++ RCCL engine (``csrc/comm/comm.cpp`` -> ``_hcb_comm.so``).

``NativeReducer`` owns one RCCL communicator (created from an ncclUniqueId exchanged through
the torch.distributed TCP store -- no MPI) and reduces the flat gradient buffer bucket by
bucket on a dedicated high-priority comm stream forked from / joined to the compute stream.
Every gradient range handed to it (a whole backward segment on the overlap path) is cut by
the C++ engine into buckets of at most ``HOROVOD_FUSION_THRESHOLD`` wire bytes
(csrc/comm/engine.h). Optional Horovod compression: bf16 or IEEE fp16 on the wire (pack
kernel -> 16-bit allreduce -> unpack kernel, all on the comm stream). ``HOROVOD_TIMELINE``
writes a Chrome trace of the bucket reductions; the watchdog honours
``HOROVOD_STALL_CHECK_TIME_SECONDS`` and ``HCB_STALL_ABORT_SECONDS``.
"""
from __future__ import annotations

import itertools
import os
import threading

import torch
import torch.distributed as dist

from .reducer import fusion_threshold_bytes, make_buckets

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMM_SO = os.path.join(_PKG, "_hcb_comm.so")
_loaded = False
_lock = threading.Lock()
_counter = itertools.count()


def load():
    global _loaded
    if _loaded:
        return torch.ops.hcb_comm
    with _lock:
        if not _loaded:
            from ..ops import _ext

            _ext.load(act="bf16")  # the comm library links against the (bf16) kernel library
            if not os.path.exists(COMM_SO):
                from .. import _build

                _build.build_comm()
            torch.ops.load_library(COMM_SO)
            _loaded = True
    return torch.ops.hcb_comm


def rccl_version() -> int:
    return int(load().version())


def _exchange_uid(rank: int, world: int, tag: str) -> torch.Tensor:
    cc = load()
    if world == 1:
        return cc.unique_id()
    store = dist.distributed_c10d._get_default_store()
    key = f"hcb_comm_uid/{tag}"
    if rank == 0:
        uid = cc.unique_id()
        store.set(key, bytes(uid.numpy().tobytes()))
        return uid
    raw = store.get(key)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).clone()


class Communicator:
    """One RCCL communicator over all ranks of the default process group (or a 1-rank one)."""

    def __init__(self, device=None):
        cc = load()
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.device = torch.cuda.current_device() if device is None else int(device)
        tag = str(next(_counter))
        uid = _exchange_uid(self.rank, self.world, tag)
        self.h = cc.create(uid, self.rank, self.world, self.device)
        self._cc = cc

    def allreduce_(self, t, average=False):
        self._cc.allreduce_(self.h, t, average)
        return t

    def broadcast_(self, t, root=0):
        self._cc.broadcast_(self.h, t, root)
        return t

    def allgather_(self, inp, out):
        self._cc.allgather_(self.h, inp, out)
        return out

    def reduce_scatter_(self, inp, out, average=False):
        self._cc.reduce_scatter_(self.h, inp, out, average)
        return out

    def bucket_allreduce_(self, flat, buckets, compress=0, scale=1.0, average=False):
        self._cc.bucket_allreduce_(self.h, flat, buckets, compress, scale, average)
        return flat

    def bucket_allreduce_async_(self, flat, buckets, compress=0, scale=1.0, average=False):
        self._cc.bucket_allreduce_async_(self.h, flat, buckets, compress, scale, average)
        return flat

    def set_fusion_threshold(self, nbytes: int):
        self._cc.set_fusion_threshold(self.h, int(nbytes))

    def buckets_issued(self) -> int:
        return int(self._cc.buckets_issued(self.h))

    def step_mark(self):
        """Stall-watchdog heartbeat after a replayed step graph (its collectives make no host call)."""
        self._cc.step_mark(self.h)

    def steps_marked(self) -> int:
        return int(self._cc.steps_marked(self.h))

    def join_(self):
        self._cc.join_(self.h)

    def barrier(self):
        self._cc.barrier(self.h)

    def size(self) -> int:
        """Rank count as reported by the RCCL communicator itself."""
        return int(self._cc.size(self.h))

    def close(self):
        if getattr(self, "h", None) is not None:
            self._cc.destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def xgmi_probe(n: int, rank: int) -> torch.Tensor:
    """Rank-dependent probe values whose fp32 sums are exact in any order (small integers / 2)."""
    i = torch.arange(n, dtype=torch.float32)
    return ((i % 97) + 7 * (rank + 1) + (i % 5) * rank) * 0.5


def validate_xgmi(one_shot, rccl, agree_min, n: int, rank: int, device=None) -> str:
    """Startup cross-check of the one-shot xGMI allreduce against RCCL (every rank, collectively):
    reduce the same probe with both; the sums are exact, so they must match bitwise. Returns
    "on", or "disabled(<reason>)" when ANY rank saw a mismatch, a peer time-out (the kernel's
    bounded wait poisons with NaN and raises the error flag) or an exception. ``one_shot(t)`` /
    ``rccl(t)`` reduce in place (and for one_shot: return nonzero on a device error);
    ``agree_min(int) -> int`` is the MIN over ranks, so every rank takes the same decision."""
    reason = ""
    a = xgmi_probe(n, rank)
    if device is not None:
        a = a.to(device)
    b = a.clone()
    try:
        if one_shot(a):
            reason = "peer timeout"
    except Exception as e:  # noqa: BLE001 -- any failure disables the path, never the job
        reason = f"{type(e).__name__}: {e}"[:120]
    rccl(b)  # every rank takes part in the RCCL reduction whatever its one-shot did
    if device is not None:
        torch.cuda.synchronize(device)
    if not reason and not torch.equal(a.cpu(), b.cpu()):
        bad = int((a.cpu() != b.cpu()).sum())
        reason = f"mismatch vs RCCL in {bad}/{n} probe elements"
    ok = agree_min(0 if reason else 1)
    if ok:
        return "on"
    return f"disabled({reason or 'failed on another rank'})"


class NativeReducer:
    """Flat-buffer gradient allreduce on the C++ RCCL engine."""

    def __init__(self, compression=None, bucket_bytes=None, average=False, force=False):
        """``force``: run the collectives even on a 1-rank communicator (where they are the
        identity), so the multi-GPU code path can be exercised and timed on one GPU."""
        if compression not in (None, "none", "bf16", "fp16"):
            raise ValueError(compression)
        # wire formats: 0 fp32, 1 bf16, 2 IEEE fp16 (Horovod Compression.fp16)
        self.compress = {None: 0, "none": 0, "bf16": 1, "fp16": 2}[compression]
        self.bucket_bytes = bucket_bytes or fusion_threshold_bytes()
        self.average = average
        self.comm = Communicator()
        self.comm.set_fusion_threshold(self.bucket_bytes)
        # collectives captured inside the training-step graph (default); HCB_GRAPH_COMM=0
        # replays one graph per backward segment and launches the reductions from the host
        self.graph_safe = os.environ.get("HCB_GRAPH_COMM", "1") == "1"
        self.force = force
        self._buckets = None
        # opt-in one-shot xGMI allreduce for small fp32 ranges (single node only), validated
        # against RCCL at startup; ``xgmi_status`` ("off" | "on" | "disabled(reason)") goes into
        # the bench JSON's comm block
        self.xgmi, self.xgmi_bytes = None, int(os.environ.get("HCB_XGMI_BYTES", "0"))
        self.xgmi_status = "off"
        local = int(os.environ.get("LOCAL_WORLD_SIZE", self.comm.world))
        if self.xgmi_bytes > 0:
            if self.compress:
                self.xgmi_status = "disabled(compressed wire: the one-shot sums fp32 only)"
            elif self.comm.world == 1:
                self.xgmi_status = "disabled(single rank)"
            elif self.comm.world != local:
                self.xgmi_status = "disabled(multi-node: xGMI peers are node-local)"
            else:
                self._enable_xgmi()

    def _enable_xgmi(self):
        from .xgmi import XgmiAllreduce

        def agree_min(v: int) -> int:
            t = torch.tensor([v], dtype=torch.int32, device=torch.cuda.current_device())
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t.item())

        xg = None
        try:
            xg = XgmiAllreduce(capacity_bytes=self.xgmi_bytes)
            one_shot = lambda t: (xg.allreduce_(t), xg.error())[1]  # noqa: E731
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:120]

            def one_shot(t):
                raise RuntimeError(err)
        n = max(64, min(self.xgmi_bytes // 4, 1 << 18))
        self.xgmi_status = validate_xgmi(one_shot, self.comm.allreduce_, agree_min, n, self.comm.rank,
                                         device=torch.cuda.current_device())
        if self.xgmi_status == "on":
            self.xgmi = xg
        else:
            if xg is not None:
                xg.close()
            if self.comm.rank == 0:
                import sys

                print(f"[hcb] HCB_XGMI_BYTES={self.xgmi_bytes}: one-shot xGMI allreduce {self.xgmi_status}; "
                      "all ranges go through RCCL", file=sys.stderr)

    def _bucket_table(self, numel):
        # whole-buffer form: buckets from the END of the buffer first (the engine cuts each
        # of them again only if it exceeds the threshold)
        if self._buckets is None or self._numel != numel:
            esz = 2 if self.compress else 4
            b = make_buckets(numel, max(self.bucket_bytes // esz, 64))
            self._buckets = torch.tensor(b, dtype=torch.int64)
            self._numel = numel
        return self._buckets

    def allreduce_(self, flat):
        if self.comm.world == 1 and not self.compress and not self.force:
            return flat
        self.comm.bucket_allreduce_(flat, self._bucket_table(flat.numel()), self.compress, 1.0, self.average)
        return flat

    # -- overlap interface: reduce finished gradient ranges while backward continues
    def allreduce_ranges_async_(self, flat, ranges):
        if self.comm.world == 1 and not self.compress and not self.force:
            return
        if self.xgmi is not None:  # small ranges: one hop over xGMI on the caller's stream
            small = [r for r in ranges if r[1] * 4 <= self.xgmi_bytes]
            for off, n in small:
                self.xgmi.allreduce_(flat[off:off + n], average=self.average)
            ranges = [r for r in ranges if r[1] * 4 > self.xgmi_bytes]
            if not ranges:
                return
        table = torch.tensor([list(r) for r in ranges], dtype=torch.int64).view(-1, 2)
        self.comm.bucket_allreduce_async_(flat, table, self.compress, 1.0, self.average)

    def join(self):
        self.comm.join_()

    def step_mark(self):
        """Per-step stall-watchdog heartbeat of the graph-replayed step (trainer.py calls it after
        every replay): the captured collectives make no host call the watchdog could see."""
        self.comm.step_mark()

    def check_errors(self):
        """Raise if the one-shot xGMI path timed out waiting for a peer (its output was
        poisoned with NaN on the device). Synchronises; call outside the timed loop."""
        if self.xgmi is not None and self.xgmi.error():
            raise RuntimeError("xGMI allreduce: a peer did not publish within the bounded wait; gradients of "
                               "that step were poisoned (NaN) instead of being reduced unsynchronised")

    def broadcast_(self, t, root=0):
        if self.comm.world > 1:
            self.comm.broadcast_(t, root)
        return t

    def close(self):
        if self.xgmi is not None:
            self.xgmi.close()
        self.comm.close()
