"""Does a CompiledCnn call hold the GIL while the GPU works?  A second Python
thread counts loop iterations; per phase of the call we report how far it
got (a phase that holds the GIL for t ms shows ~0 progress over t ms)."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seldon_core_amd.models import cnn  # noqa: E402

count = [0]
stop = [False]


def spin():
    while not stop[0]:
        count[0] += 1


m = cnn.CompiledCnn(cnn.build("densenet169"), device=0, max_batch=8)
X = (np.random.default_rng(0).random((1, 3, 224, 224)) * 255).astype(np.float64)
for _ in range(3):
    m(X)
th = threading.Thread(target=spin, daemon=True)
th.start()
time.sleep(0.2)
c0, t0 = count[0], time.perf_counter()
time.sleep(0.2)
base = (count[0] - c0) / (time.perf_counter() - t0)
res = {"spin_per_ms_idle": round(base / 1e3, 1)}
phases = {}
for _ in range(20):
    def ph(name, fn):
        c, t = count[0], time.perf_counter()
        out = fn()
        dt = time.perf_counter() - t
        p = phases.setdefault(name, [0.0, 0])
        p[0] += dt
        p[1] += count[0] - c
        return out
    t = ph("from_numpy+to", lambda: torch.from_numpy(X).reshape(-1, 3, 224, 224).to(m.device))
    y = ph("run", lambda: m.run(t))
    ph("synchronize", lambda: m.stream.synchronize())
    ph("cpu", lambda: y.double().cpu().numpy())
    ph("whole_call", lambda: m(X))
stop[0] = True
for k, (dt, c) in phases.items():
    res[k] = {"ms": round(dt / 20 * 1e3, 3), "spin_share": round(c / (base * dt), 3) if dt > 0 else None}
print(json.dumps(res), flush=True)
