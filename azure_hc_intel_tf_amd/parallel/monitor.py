"""Collective monitoring for the torch.distributed paths (gloo on the CPU, RCCL through
torch): Horovod's timeline and stall inspector, re-built for this engine.

* ``HOROVOD_TIMELINE=<file>``: every collective issued through ``hvd`` / ``TorchDistReducer``
  becomes a Chrome-trace complete event (``ph: X``; name, bytes, rank) in ``<file>`` (rank 0)
  or ``<file>.rank<N>`` -- open in chrome://tracing or Perfetto. The native C++ RCCL engine
  writes its own timeline (``csrc/comm/comm.cpp``).
* ``HOROVOD_STALL_CHECK_TIME_SECONDS`` (default 60): a watchdog thread warns on stderr when a
  collective has been outstanding longer than this -- one or more ranks have not joined it
  (Horovod's stall inspector message). ``HCB_STALL_ABORT_SECONDS`` > 0 additionally aborts
  the process (exit code 75) so the launcher tears the job down instead of hanging forever.

The reference relies on Horovod's C++ implementation of both (SURVEY.md §5 "Tracing",
"Failure detection"); /root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:104-106
shows the HOROVOD_* environment it passes.
"""
from __future__ import annotations

import atexit
import itertools
import json
import os
import sys
import threading
import time
from typing import Dict, Optional

STALL_EXIT_CODE = 75


class CommMonitor:
    def __init__(self, rank: int = 0, timeline: Optional[str] = None, stall_warn_s: float = 60.0,
                 stall_abort_s: float = 0.0, poll_s: float = 0.25):
        self.rank = rank
        self.stall_warn_s = stall_warn_s
        self.stall_abort_s = stall_abort_s
        self._ids = itertools.count()
        self._open: Dict[int, tuple] = {}
        self._warned = set()
        self._lock = threading.Lock()
        self._t0 = time.perf_counter()
        self._events = []
        self.timeline = None
        if timeline:
            self.timeline = timeline if rank == 0 else f"{timeline}.rank{rank}"
            atexit.register(self.flush)
        self.stalls = 0
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._watch, args=(poll_s,), name="hcb-stall-inspector", daemon=True)
        self._thr.start()

    # ------------------------------------------------------------ collective bracketing
    def begin(self, name: str, nbytes: int = 0) -> int:
        i = next(self._ids)
        with self._lock:
            self._open[i] = (name, nbytes, time.perf_counter())
        return i

    def end(self, i: int) -> None:
        with self._lock:
            name, nbytes, t = self._open.pop(i, (None, 0, None))
            if name is not None and self.timeline:
                now = time.perf_counter()
                self._events.append({"name": name, "ph": "X", "pid": self.rank, "tid": 0, "ts": (t - self._t0) * 1e6,
                                     "dur": (now - t) * 1e6, "args": {"bytes": nbytes}})

    # ------------------------------------------------------------ watchdog
    def _watch(self, poll_s: float):
        while not self._stop.wait(poll_s):
            now = time.perf_counter()
            with self._lock:
                items = list(self._open.items())
            for i, (name, nbytes, t) in items:
                waited = now - t
                if waited > self.stall_warn_s and i not in self._warned:
                    self._warned.add(i)
                    self.stalls += 1
                    print(f"[hcb stall inspector] rank {self.rank}: {name} ({nbytes} bytes) outstanding for "
                          f"{waited:.1f} s: one or more ranks have not joined it "
                          f"(HOROVOD_STALL_CHECK_TIME_SECONDS={self.stall_warn_s:g})", file=sys.stderr, flush=True)
                if self.stall_abort_s > 0 and waited > self.stall_abort_s:
                    print(f"[hcb stall inspector] rank {self.rank}: {name} stalled {waited:.1f} s > "
                          f"HCB_STALL_ABORT_SECONDS; aborting", file=sys.stderr, flush=True)
                    self.flush()
                    os._exit(STALL_EXIT_CODE)

    def flush(self):
        if not self.timeline:
            return
        with self._lock:
            ev = list(self._events)
        d = os.path.dirname(os.path.abspath(self.timeline))
        os.makedirs(d, exist_ok=True)
        with open(self.timeline, "w") as f:
            json.dump(ev, f)

    def close(self):
        self._stop.set()
        self.flush()


_MON: Optional[CommMonitor] = None


def monitor() -> CommMonitor:
    """The process-wide monitor (created on first use from the HOROVOD_* environment)."""
    global _MON
    if _MON is None:
        rank = int(os.environ.get("RANK", "0") or 0)
        _MON = CommMonitor(rank, os.environ.get("HOROVOD_TIMELINE") or None,
                           float(os.environ.get("HOROVOD_STALL_CHECK_TIME_SECONDS", "60") or 60),
                           float(os.environ.get("HCB_STALL_ABORT_SECONDS", "0") or 0))
    return _MON


def reset():
    global _MON
    if _MON is not None:
        _MON.close()
    _MON = None


class tracked:
    """``with tracked("allreduce", nbytes): dist.all_reduce(...)``"""

    def __init__(self, name: str, nbytes: int = 0):
        self.name, self.nbytes = name, nbytes

    def __enter__(self):
        self.i = monitor().begin(self.name, self.nbytes)
        return self

    def __exit__(self, *exc):
        monitor().end(self.i)
        return False
