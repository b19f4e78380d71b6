"""MI355X-native re-design of md-k-sarker/azure-hc-intel-tf (tf_cnn_benchmarks + Horovod on
Azure HC): hand-written HIP/CDNA4 kernels, HIP-graph captured training steps and RCCL over xGMI.

Importing the package sets HIP runtime defaults that must be in place before the GPU is first
touched (the HIP runtime reads them once, at initialisation):

* ``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0``: with the runtime's default pre-recorded graph packets,
  training-step graphs that fork a communication stream (fork / join event edges, the
  multi-GPU overlap path) intermittently ran kernels ahead of their predecessors on MI355X
  (corrupted gradients within a few steps; reproduced with ``tools/dp_variants.sh`` even with
  the collective itself removed). With it off the same graphs are exact and the step time is
  unchanged (7.80 vs 7.81 ms/step, ResNet-50 bs=64). Set it explicitly to override.
  Investigation (profiles/r2f_graph_packet_capture.txt): only graphs with SEVERAL fork/join
  pairs between backward segments diverge (also with empty comm branches and with a distinct
  event per edge); no-fork and single-fork step graphs, and the standalone fork/join repro
  ``tools/graph_fork_repro.hip`` (same API sequence), are exact with packet capture on.
"""
import os as _os

_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
