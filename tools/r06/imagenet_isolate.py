"""Which node bounds the ImageNet ensemble's throughput: each node alone in a
one-node graph at concurrency 32 (in-process Deployment.predict)."""
import concurrent.futures as cf
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import seldon_core_amd as sca  # noqa: E402
from seldon_core_amd.components.examples import ImageNetModel, ImageNetTransformer  # noqa: E402
from imagenet_bench import jpeg  # noqa: E402


def run(name, graph, comps, reqs, conc=32, n=256):
    dep = sca.Deployment({"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}, device=0,
                         components=comps)
    try:
        for _ in range(3):
            dep.predict(reqs[0])
        t = time.perf_counter()
        with cf.ThreadPoolExecutor(conc) as ex:
            list(ex.map(lambda i: dep.predict(reqs[i % len(reqs)]), range(n)))
        wall = time.perf_counter() - t
        st = {k: u.native.stats() for k, u in dep.python_units.items() if getattr(u, "native", None) is not None}
        print(json.dumps({"case": name, "conc": conc, "req_per_s": round(n / wall, 1),
                          "calls": {k: (v["jobs"], v["calls"]) for k, v in st.items()}}), flush=True)
    finally:
        dep.close()


reqs = [{"binData": jpeg(i)} for i in range(32)]
tr = ImageNetTransformer(device=0)
treqs = [tr.transform_input_raw(r) for r in reqs]
run("transformer", {"name": "t", "type": "TRANSFORMER", "implementation": "IMAGENET_TRANSFORMER"}, {}, reqs)
for arch in ("resnet50", "densenet169"):
    run(arch, {"name": "m", "type": "MODEL", "implementation": "IMAGENET_MODEL"},
        {"m": ImageNetModel(arch, device=0, max_batch=32)}, treqs)
run("transformer->resnet50", {"name": "t", "type": "TRANSFORMER", "implementation": "IMAGENET_TRANSFORMER",
                              "children": [{"name": "m", "type": "MODEL", "implementation": "IMAGENET_MODEL"}]},
    {"m": ImageNetModel("resnet50", device=0, max_batch=32)}, reqs)
