"""Kernel-level view of CNN graph replays (for rocprofv3 --kernel-trace):
ResNet-50 and DenseNet-169, bf16, 1 image, 50 replays each; CNN_TUNE=1 runs
MIOpen's solver search first (the serving default), else immediate mode.
CNN_ARCH picks one network."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seldon_core_amd.models import cnn  # noqa: E402

TUNE = os.environ.get("CNN_TUNE") == "1"
for arch in os.environ.get("CNN_ARCH", "resnet50,densenet169").split(","):
    m = cnn.CompiledCnn(cnn.build(arch), device=0, max_batch=1, tune=TUNE)
    X = (np.random.default_rng(0).random((1, 3, 224, 224)) * 255).astype(np.float64)
    for _ in range(50):
        m(X)
    torch.cuda.synchronize()
    print(arch, "graphs", sorted(m.graphs), flush=True)
