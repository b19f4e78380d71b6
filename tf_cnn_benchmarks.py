#!/usr/bin/env python3
"""Drop-in entry point with the same name and flags as the script the reference runs
(/opt/tensorflow-benchmarks/scripts/tf_cnn_benchmarks/tf_cnn_benchmarks.py,
/root/reference/benchmark-scripts/run-tf-sing-ucx-openmpi.sh:23,108), backed by the
MI355X engine. Example:

    python tf_cnn_benchmarks.py --model=resnet50 --batch_size=64 --num_batches=100 \\
        --num_warmup_batches=50 --display_every=10 --optimizer=momentum \\
        --variable_update=horovod --device=gpu
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from azure_hc_intel_tf_amd.bench.benchmark_cnn import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
