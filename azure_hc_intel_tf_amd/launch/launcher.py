"""Per-GPU process launcher (the mpirun / mpiexec.hydra role of the reference,
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:99-113,
run-tf-sing-libfabric-intelmpi.sh:94-105; SURVEY.md §2.3 last row, §2.5).

* one worker process per MI355X (``--nproc_per_node``), ranks ``node_rank*nproc + local``;
* rendezvous env for torch.distributed / RCCL: RANK, LOCAL_RANK, WORLD_SIZE,
  LOCAL_WORLD_SIZE, GROUP_RANK, MASTER_ADDR, MASTER_PORT (+ HSA_ENABLE_IPC_MODE_LEGACY=0,
  which the host driver needs for dmabuf IPC);
* CPU pinning: each worker gets a contiguous, equal share of the node's cores (the
  ``--map-by ppr:W:socket,pe=C`` role), applied in the child before exec;
* fabric selection: ``ib`` = RCCL peer-to-peer over xGMI (default transports), ``sock`` =
  RCCL's socket transport only (P2P / SHM / IB disabled), the reference's A/B fabric arm;
* failure propagation: if any worker exits non-zero, the others are terminated and the
  launcher exits with that worker's code (MPI_Abort semantics).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional


# RCCL collective tuning for the intra-node xGMI mesh (the reference's transport choice,
# run-tf-sing-ucx-openmpi.sh:85-92 `-mca coll_hcoll_enable 1`, `UCX_TLS=rc_x,sm,self`).
# An MI355X talks to each of its 7 peers over its own xGMI link, so a ring all-reduce is bound by
# ONE link per hop; RCCL spreads its channels (one ring each) over the links, and every channel is
# a workgroup that occupies a CU while backward still runs on the others. Values are only set
# when asked for (the CLI below); a value already in the environment always wins.
RCCL_KNOBS = {"channels": ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS"), "algo": ("NCCL_ALGO",),
              "proto": ("NCCL_PROTO",)}


def rccl_env(channels: Optional[int] = None, algo: Optional[str] = None, proto: Optional[str] = None,
             base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """NCCL_* variables for the requested RCCL channel count / algorithm (Ring, Tree) / protocol
    (Simple, LL, LL128); names already set in ``base`` (default: os.environ) are left alone."""
    base = os.environ if base is None else base
    out = {}
    for key, val in (("channels", channels), ("algo", algo), ("proto", proto)):
        if val is None or val == "":
            continue
        for name in RCCL_KNOBS[key]:
            if name not in base:
                out[name] = str(val)
    return out


def fabric_env(fabric: str) -> Dict[str, str]:
    if fabric in ("ib", "xgmi", "", None):
        return {}
    if fabric in ("sock", "socket", "tcp"):
        return {"NCCL_P2P_DISABLE": "1", "NCCL_SHM_DISABLE": "1", "NCCL_IB_DISABLE": "1",
                "NCCL_SOCKET_IFNAME": os.environ.get("NCCL_SOCKET_IFNAME", "lo")}
    raise ValueError(f"unknown fabric {fabric!r} (expected ib or sock)")


def _parse_cpulist(text: str) -> List[int]:
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def gpu_numa_nodes(sysfs: str = "/sys") -> List[int]:
    """NUMA node of every GPU in HIP device order (the KFD topology's GPU agents, in node
    order), from the agent's PCI location -> /sys/bus/pci/devices/<bdf>/numa_node. -1 where
    unknown; [] without a KFD topology (no GPU driver, e.g. CPU-only hosts)."""
    root = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        props = _read(os.path.join(root, str(n), "properties"))
        if props is None:
            out.append(-1)  # an agent we may not read: keep the device index aligned
            continue
        kv = dict(line.split()[:2] for line in props.splitlines() if len(line.split()) >= 2)
        if int(kv.get("simd_count", "0")) == 0:
            continue  # CPU agent
        loc, dom = int(kv.get("location_id", "0")), int(kv.get("domain", "0"))
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        numa = _read(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node"))
        out.append(int(numa) if numa is not None and numa.strip().lstrip("-").isdigit() else -1)
    return out


def visible_gpu_count(sysfs: str = "/sys") -> int:
    """GPUs this process would see, counted WITHOUT any GPU runtime: the KFD topology's GPU
    agents, filtered by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (set but
    empty = none). A launcher parent uses this so that neither torch nor HIP is ever loaded in the
    process that forks the workers (torch.cuda.device_count() falls back to hipGetDeviceCount,
    which initialises HIP, whenever its amdsmi query fails)."""
    n = len(gpu_numa_nodes(sysfs))
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        ids = [i.strip() for i in v.split(",") if i.strip() != ""]
        try:
            n = len([i for i in ids if 0 <= int(i) < n])
        except ValueError:  # UUID-style ids: trust their count
            n = min(n, len(ids))
    return n


def cpu_shares(n_workers: int, cpus: Optional[List[int]] = None, sysfs: str = "/sys") -> List[List[int]]:
    """CPU set per local worker: the cores of its GPU's NUMA node, split evenly between the
    workers whose GPUs share that node (the reference's ``--map-by ppr:W:socket,pe=C``,
    run-tf-sing-ucx-openmpi.sh:102, made GPU-affine); contiguous equal shares of the allowed
    CPUs when the topology is unknown."""
    cpus = sorted(cpus if cpus is not None else os.sched_getaffinity(0))
    if n_workers <= 0:
        return []
    per = max(len(cpus) // n_workers, 1)
    flat = [cpus[i * per:(i + 1) * per] or cpus for i in range(n_workers)]
    numa = gpu_numa_nodes(sysfs)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis and numa:
        try:
            numa = [numa[int(i)] for i in vis.split(",") if i.strip() != ""]
        except (ValueError, IndexError):
            return flat
    if len(numa) < n_workers or any(n < 0 for n in numa[:n_workers]):
        return flat
    allowed = set(cpus)
    by_node = {}
    for w in range(n_workers):
        by_node.setdefault(numa[w], []).append(w)
    shares: List[List[int]] = [[] for _ in range(n_workers)]
    for node, ws in by_node.items():
        text = _read(os.path.join(sysfs, "devices/system/node", f"node{node}", "cpulist"))
        node_cpus = [c for c in _parse_cpulist(text)] if text else []
        node_cpus = sorted(c for c in node_cpus if c in allowed)
        if len(node_cpus) < len(ws):
            return flat
        k = len(node_cpus) // len(ws)
        for j, w in enumerate(ws):
            shares[w] = node_cpus[j * k:(j + 1) * k]
    return shares


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker_env(base: Dict[str, str], rank: int, local_rank: int, world: int, nproc: int, node_rank: int,
               master_addr: str, master_port: int, fabric: str, omp_threads: Optional[int],
               rccl: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": str(node_rank), "NODE_RANK": str(node_rank),
                "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
                "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    # graph packet capture off unless the user chose (azure_hc_intel_tf_amd/__init__.py)
    env.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
    env.update(fabric_env(fabric))
    env.update(rccl or {})
    if omp_threads:
        env["OMP_NUM_THREADS"] = str(omp_threads)
    return env


def launch(cmd: List[str], nproc_per_node: int, nnodes: int = 1, node_rank: int = 0,
           master_addr: str = "127.0.0.1", master_port: Optional[int] = None, fabric: str = "ib",
           pin_cpus: bool = True, omp_threads: Optional[int] = None, env: Optional[Dict[str, str]] = None,
           poll_s: float = 0.2, rccl: Optional[Dict[str, str]] = None) -> int:
    world = nproc_per_node * nnodes
    port = master_port or int(os.environ.get("MASTER_PORT", 0)) or free_port()
    base = dict(os.environ if env is None else env)
    rccl = {k: v for k, v in (rccl or {}).items() if k not in base}
    shares = cpu_shares(nproc_per_node) if pin_cpus else [None] * nproc_per_node
    procs = []
    for lr in range(nproc_per_node):
        rank = node_rank * nproc_per_node + lr
        e = worker_env(base, rank, lr, world, nproc_per_node, node_rank, master_addr, port, fabric, omp_threads,
                       rccl)
        share = shares[lr]

        def pre(share=share):
            os.setsid()
            if share:
                try:
                    os.sched_setaffinity(0, share)
                except OSError:
                    pass

        procs.append(subprocess.Popen(cmd, env=e, preexec_fn=pre))
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                r = p.poll()
                if r is None:
                    alive += 1
                elif r != 0 and rc == 0:
                    rc = r
            if rc != 0:
                _terminate(procs)
                break
            if alive == 0:
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _terminate(procs)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
    return rc


def _terminate(procs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + 10
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.1)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="one process per MI355X launcher")
    ap.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node_rank", type=int, default=0)
    ap.add_argument("--master_addr", default="127.0.0.1")
    ap.add_argument("--master_port", type=int, default=0)
    ap.add_argument("--fabric", default="ib")
    ap.add_argument("--no_pin", action="store_true")
    ap.add_argument("--omp_threads", type=int, default=None)
    ap.add_argument("--rccl_channels", type=int, default=None, help="NCCL_MIN/MAX_NCHANNELS")
    ap.add_argument("--rccl_algo", default=None, help="NCCL_ALGO (Ring, Tree)")
    ap.add_argument("--rccl_proto", default=None, help="NCCL_PROTO (Simple, LL, LL128)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing worker command")
    return launch(cmd, a.nproc_per_node, a.nnodes, a.node_rank, a.master_addr, a.master_port or None, a.fabric,
                  pin_cpus=not a.no_pin, omp_threads=a.omp_threads,
                  rccl=rccl_env(a.rccl_channels, a.rccl_algo, a.rccl_proto))


if __name__ == "__main__":
    sys.exit(main())
