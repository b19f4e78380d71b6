"""MI355X-native re-design of md-k-sarker/azure-hc-intel-tf (tf_cnn_benchmarks + Horovod on
Azure HC): hand-written HIP/CDNA4 kernels, HIP-graph captured training steps and RCCL over xGMI.

HIP graph packet capture (``DEBUG_CLR_GRAPH_PACKET_CAPTURE``, the runtime's default) is left as
the runtime sets it. Rounds 2-3 forced it off: with it on, the captured step replayed inexactly.
The round-4 buffer-level bisection (tools/pc_buffer_bisect.py: every buffer of the step hashed
after each replay, capture on vs off, in separate processes) found the first differing producer:
the fc-bias gradient's column sum, whose zeroing was a ``hipMemsetAsync`` node inside the graph
(every activation, statistic and other gradient equal; that one slice garbage, ~1e37-1e38, at the
third replay). Its zeroing is now part of the kernel (csrc/kernels/misc.hip launch_colsum2) and
the step graph contains no memset node: with capture on, single-graph and data-parallel replays
are bitwise equal to capture off (profiles/r4_packet_capture_root_cause.txt).

Packet capture nevertheless defaults to OFF in every process (``setdefault``: a user who exports
the variable keeps their choice). The evidence that the memset node was THE cause is where the bad
value appeared; no same-box A/B has yet shown the old memset path diverging and the fixed build not
(the legacy path no longer reproduced on a later box), and the failure it guards against is silent
inexact training. Capture on/off makes no measurable throughput difference on one GPU, so off costs
nothing.
"""
import os as _os

_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
