"""GraphedModule vs eager PyTorch for a small served MLP (the MLflow pytorch
flavour's path): host-timed ms per call (numpy in, numpy out)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seldon_core_amd.models.graphed import GraphedModule  # noqa: E402

torch.manual_seed(0)
net = torch.nn.Sequential(torch.nn.Linear(32, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                          torch.nn.Linear(256, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10),
                          torch.nn.Softmax(dim=1)).cuda().eval()
gm = GraphedModule(net, device=0)


def eager(X):
    with torch.no_grad():
        return net(torch.as_tensor(X, device="cuda")).cpu().numpy()


for rows in (1, 16, 256):
    X = np.random.default_rng(rows).normal(size=(rows, 32)).astype(np.float32)
    res = {"rows": rows}
    for name, fn in (("eager", eager), ("graphed", gm)):
        for _ in range(5):
            fn(X)
        t = time.perf_counter()
        for _ in range(200):
            y = fn(X)
        res[f"{name}_ms"] = round((time.perf_counter() - t) / 200 * 1e3, 4)
    res["max_abs_diff"] = float(np.abs(gm(X) - eager(X)).max())
    print(json.dumps(res), flush=True)
