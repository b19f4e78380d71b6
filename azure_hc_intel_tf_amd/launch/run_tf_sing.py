"""Logic behind ``benchmark-scripts/run-tf-sing-*.sh <NUM_NODES> <WORKERS_PER_SOCKET> <batch_size> <fabric>``.

Reproduces the reference runners' behaviour (/root/reference/benchmark-scripts/
run-tf-sing-ucx-openmpi.sh:27-113, run-tf-sing-libfabric-intelmpi.sh:28-110):
the same positional CLI, the same topology derivation from ``lscpu`` (workers per node,
cores per worker, intra/inter threads), the same tf_cnn_benchmarks flag set, the config
echo and a ``tee``'d log -- but the workers are one process per MI355X started by the
local launcher (no mpirun / ssh / Singularity), the fabric argument selects RCCL's
transport, and the reference's quirks are fixed (``WORKERS_PER_SOCKET=0`` no longer yields
``ppr:0``, no undefined ``$args`` / ``$FABRIC_ARGS`` echo).

Env overrides: MODEL, NUM_BATCHES, NUM_WARMUP_BATCHES, DISPLAY_EVERY, DEVICE (gpu|cpu),
GPUS_PER_NODE, HOSTFILE (multi-node: one host per line; this node's rank = its line),
DRY_RUN=1 (print the plan, launch nothing), LOG_DIR, EXTRA_ARGS.

Multi-node from ONE shell (the reference's ``mpirun -hostfile``, run-tf-sing-ucx-openmpi.sh:99-103):
``FANOUT=1`` on the hostfile's first node starts the same runner on every other host of the
hostfile over ssh (``SSH``, default ``ssh -o BatchMode=yes``; the repo and the hostfile at the same
paths on every node, as the reference assumes for ~/nodeips.txt), forwarding the overrides above and
every ``HCB_*`` / ``NCCL_*`` / ``RCCL_*`` variable, runs its own node, and returns the worst exit
code. Each node derives its rank from its line of the hostfile.
"""
from __future__ import annotations

import argparse
import os
import shlex
import socket
import subprocess
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
INTER_T = 2  # run-tf-sing-ucx-openmpi.sh:35


def lscpu_topology() -> Dict[str, int]:
    sockets, cps = 1, os.cpu_count() or 1
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        vals = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                vals[k.strip()] = v.strip()
        sockets = int(vals.get("Socket(s)", sockets) or sockets)
        cps = int(vals.get("Core(s) per socket", cps) or cps)
    except Exception:
        pass
    return {"sockets": max(sockets, 1), "cores_per_socket": max(cps, 1)}


def gpus_per_node_default() -> int:
    v = os.environ.get("GPUS_PER_NODE")
    if v:
        return int(v)
    from .launcher import visible_gpu_count

    return visible_gpu_count()  # KFD topology: this launcher process never loads torch / HIP


@dataclass
class Plan:
    num_nodes: int
    workers_per_socket: int
    batch_size: int
    fabric: str
    sockets: int
    cores_per_socket: int
    workers_per_node: int
    cores_per_worker: int
    intra_t: int
    inter_t: int
    total_workers: int
    device: str


def worker_math(num_nodes: int, wps: int, sockets: int, cores_per_socket: int, device: str = "gpu",
                gpus_per_node: int = 8, batch_size: int = 64, fabric: str = "ib") -> Plan:
    """run-tf-sing-ucx-openmpi.sh:40-50, capped at one worker per GPU on the MI355X path."""
    if wps <= 0:
        wpn = 1
        cpw = sockets * cores_per_socket
    else:
        wpn = wps * sockets
        cpw = max(cores_per_socket // wps, 1)
    if device == "gpu":
        if gpus_per_node <= 0:
            raise ValueError("no GPUs visible; use DEVICE=cpu")
        wpn = min(wpn, gpus_per_node)
        cpw = max((sockets * cores_per_socket) // wpn, 1)
    intra = max(cpw // INTER_T, 1)
    return Plan(num_nodes, wps, batch_size, fabric, sockets, cores_per_socket, wpn, cpw, intra, INTER_T,
                num_nodes * wpn, device)


def tf_args(plan: Plan, env=os.environ) -> List[str]:
    """The reference's TF_ARGS (run-tf-sing-ucx-openmpi.sh:62-81), synthetic data."""
    a = [f"--batch_size={plan.batch_size}",
         f"--num_warmup_batches={env.get('NUM_WARMUP_BATCHES', '50')}",
         f"--num_batches={env.get('NUM_BATCHES', '100')}",
         f"--model={env.get('MODEL', 'resnet50')}",
         f"--num_intra_threads={plan.intra_t}",
         f"--num_inter_threads={plan.inter_t}",
         "--kmp_blocktime=1",
         "--kmp_affinity=granularity=fine,noverbose,compact,1,0",
         f"--display_every={env.get('DISPLAY_EVERY', '10')}",
         "--data_format=NCHW",
         "--optimizer=momentum",
         "--forward_only=False",
         f"--device={plan.device}",
         "--mkl=TRUE",
         "--variable_update=horovod",
         f"--horovod_device={'gpu' if plan.device == 'gpu' else 'cpu'}",
         "--local_parameter_device=cpu",
         "--data_name=imagenet"]
    extra = env.get("EXTRA_ARGS")
    if extra:
        a += shlex.split(extra)
    return a


def flavor_settings(flavor: str) -> Dict[str, object]:
    """What distinguishes the two reference runners, mapped onto the per-GPU launcher.

    * ucx-openmpi (run-tf-sing-ucx-openmpi.sh:99-106): ``--map-by ppr:W:socket,pe=C`` core
      pinning, ``-x HOROVOD_MPI_THREADS_DISABLE=1``, quiet transport.
    * libfabric-intelmpi (run-tf-sing-libfabric-intelmpi.sh:94-105): ``mpiexec.hydra -ppn W``
      with NO pinning, ``-genv I_MPI_DEBUG 5`` (transport selection printed at start-up; here
      ``NCCL_DEBUG=INFO`` with the INIT / NET / TUNING subsystems, RCCL's equivalent), and no
      HOROVOD_MPI_THREADS_DISABLE.
    """
    if flavor == "ucx-openmpi":
        return {"pin": True, "env": {"HOROVOD_MPI_THREADS_DISABLE": "1"}, "unset": []}
    if flavor == "libfabric-intelmpi":
        return {"pin": False, "env": {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,NET,TUNING"},
                "unset": ["HOROVOD_MPI_THREADS_DISABLE"]}
    raise ValueError(flavor)


def node_rank_from_hostfile(path: str) -> (List[str], int):
    hosts = [l.split()[0] for l in open(path) if l.strip() and not l.startswith("#")]
    me = {socket.gethostname(), socket.getfqdn(), "127.0.0.1", "localhost"}
    try:
        me.add(socket.gethostbyname(socket.gethostname()))
    except OSError:
        pass
    for i, h in enumerate(hosts):
        if h in me:
            return hosts, i
    return hosts, 0


FORWARD_ENV = ("MODEL", "NUM_BATCHES", "NUM_WARMUP_BATCHES", "DISPLAY_EVERY", "DEVICE", "GPUS_PER_NODE",
               "HOSTFILE", "LOG_DIR", "EXTRA_ARGS")
FORWARD_PREFIXES = ("HCB_", "NCCL_", "RCCL_")


def fanout_commands(hosts: List[str], node_rank: int, argv: List[str], env=os.environ,
                    repo: str = REPO) -> List[List[str]]:
    """ssh command lines that start this runner (same arguments) on every host but this one."""
    ssh = shlex.split(env.get("SSH", "ssh -o BatchMode=yes"))
    fwd = {k: v for k, v in env.items() if k in FORWARD_ENV or k.startswith(FORWARD_PREFIXES)}
    fwd["HCB_FANOUT_CHILD"] = "1"  # a child never fans out again
    exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in sorted(fwd.items()))
    out = []
    for i, h in enumerate(hosts):
        if i == node_rank:
            continue
        remote = (f"cd {shlex.quote(repo)} && env {exports} {shlex.quote(sys.executable)} -m "
                  f"azure_hc_intel_tf_amd.launch.run_tf_sing " + " ".join(shlex.quote(x) for x in argv))
        out.append(ssh + [h, remote])
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="run-tf-sing")
    ap.add_argument("--flavor", default="ucx-openmpi", choices=["ucx-openmpi", "libfabric-intelmpi"])
    ap.add_argument("num_nodes", type=int)
    ap.add_argument("workers_per_socket", type=int)
    ap.add_argument("batch_size", type=int)
    ap.add_argument("fabric", choices=["ib", "sock"])
    argv = list(sys.argv[1:] if argv is None else argv)
    a = ap.parse_args(argv)
    env = os.environ
    topo = lscpu_topology()
    device = env.get("DEVICE", "gpu")
    gpn = gpus_per_node_default() if device == "gpu" else 0
    plan = worker_math(a.num_nodes, a.workers_per_socket, topo["sockets"], topo["cores_per_socket"], device,
                       gpn, a.batch_size, a.fabric)
    targs = tf_args(plan)
    hosts, node_rank = (["127.0.0.1"], 0)
    if plan.num_nodes > 1:
        hf = env.get("HOSTFILE", os.path.expanduser("~/nodeips.txt"))
        if not os.path.exists(hf):
            print(f"NUM_NODES={plan.num_nodes} needs a hostfile ({hf}); this engine is single-node by design",
                  file=sys.stderr)
            if env.get("DRY_RUN") != "1":
                return 2
        else:
            hosts, node_rank = node_rank_from_hostfile(hf)
    fl = flavor_settings(a.flavor)
    launcher = [sys.executable, "-m", "azure_hc_intel_tf_amd.launch.launcher",
                f"--nproc_per_node={plan.workers_per_node}", f"--nnodes={plan.num_nodes}",
                f"--node_rank={node_rank}", f"--master_addr={hosts[0]}", f"--fabric={plan.fabric}",
                f"--omp_threads={plan.intra_t}"] + ([] if fl["pin"] else ["--no_pin"]) + [
                "--", sys.executable, os.path.join(REPO, "tf_cnn_benchmarks.py")] + targs
    # config echo (run-tf-sing-ucx-openmpi.sh:52-58,97,111)
    print(f"NUM_NODES: {plan.num_nodes}  WORKERS_PER_SOCKET: {plan.workers_per_socket}  "
          f"NUM_SOCKETS: {plan.sockets}  CORES_PER_SOCKET: {plan.cores_per_socket}")
    print(f"WORKERS_PER_NODE: {plan.workers_per_node}  CORES_PER_WORKER: {plan.cores_per_worker}  "
          f"INTRA_T: {plan.intra_t}  INTER_T: {plan.inter_t}  TOTAL_WORKERS: {plan.total_workers}")
    print(f"BATCH_SIZE: {plan.batch_size}  FABRIC: {plan.fabric} ({'RCCL P2P/xGMI' if plan.fabric == 'ib' else 'RCCL sockets'})"
          f"  DEVICE: {plan.device}  FLAVOR: {a.flavor}")
    from ..bench.flags import parse_flags, precision_label

    print(f"Precision: {precision_label(parse_flags(targs))}")
    print("ENV: " + " ".join(f"{k}={v}" for k, v in sorted(fl["env"].items())) +
          (f"  (unset {' '.join(fl['unset'])})" if fl["unset"] else "") +
          f"  PINNING: {'per-GPU NUMA cores' if fl['pin'] else 'none'}")
    print("COMMAND: " + " ".join(shlex.quote(c) for c in launcher), flush=True)
    fan = []
    if plan.num_nodes > 1 and env.get("FANOUT") == "1" and env.get("HCB_FANOUT_CHILD") != "1":
        if node_rank != 0:
            print("FANOUT=1 must be started on the hostfile's first node", file=sys.stderr)
            return 2
        fan = fanout_commands(hosts[:plan.num_nodes], node_rank, argv, env)
        for c in fan:
            print("FANOUT: " + " ".join(shlex.quote(x) for x in c), flush=True)
    if env.get("DRY_RUN") == "1":
        return 0
    remotes = [subprocess.Popen(c) for c in fan]
    log_dir = env.get("LOG_DIR", os.path.join(REPO, "gpurun_out", "logs"))
    os.makedirs(log_dir, exist_ok=True)
    log = os.path.join(log_dir, f"tfmn-{plan.num_nodes}n-{plan.batch_size}b-synthetic-{plan.fabric}-r1.log")
    child_env = dict(env, PYTHONPATH=REPO + os.pathsep + env.get("PYTHONPATH", ""))
    for k in fl["unset"]:
        child_env.pop(k, None)
    for k, v in fl["env"].items():
        child_env.setdefault(k, v)
    with open(log, "w") as lf:
        p = subprocess.Popen(launcher, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=child_env)
        for line in p.stdout:
            sys.stdout.write(line)
            lf.write(line)
        rc = p.wait()
    for r in remotes:  # the other nodes' runners (their output goes to their own logs and this terminal)
        rr = r.wait()
        if rc == 0 and rr != 0:
            rc = rr
    print(f"log: {log}")
    return rc


if __name__ == "__main__":
    sys.exit(main())
