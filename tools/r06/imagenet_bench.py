"""The reference's OpenVINO ImageNet ensemble graph (seldon_ov_predict_ensemble.json:
output transformer <- transformer <- combiner <- DenseNet-169 + ResNet-50) on
one MI355X, driven in-process through Deployment.predict with binData JPEG
requests.  Prints one JSON line per concurrency level: request latency
p50 / p99 and images/s.  Random-init weights (no checkpoints offline)."""
import base64
import concurrent.futures as cf
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

import seldon_core_amd as sca  # noqa: E402
from seldon_core_amd.components.examples import ImageNetModel  # noqa: E402


def jpeg(seed):
    img = (np.random.default_rng(seed).random((360, 480, 3)) * 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=90)
    return base64.b64encode(b.getvalue()).decode()


def stage_breakdown(comps, reqs):
    """Each node's own work for one request, called directly (ms, mean of 20)."""
    from seldon_core_amd.components.examples import (ImageNetCombiner, ImageNetOutputTransformer,
                                                      ImageNetTransformer)

    tr, comb, ot = ImageNetTransformer(device=0), ImageNetCombiner(device=0), ImageNetOutputTransformer(device=0)

    def t(fn, n=20):
        fn()
        t0 = time.perf_counter()
        for _ in range(n):
            out = fn()
        return out, round((time.perf_counter() - t0) / n * 1e3, 3)

    ti, ms_tr = t(lambda: tr.transform_input_raw(reqs[0]))
    from seldon_core_amd.serving.codec import dumps
    _, ms_tr_json = t(lambda: dumps(ti))  # what the reply would cost as JSON (not paid inside a graph)
    X = np.asarray(ti["data"]["tftensor"], dtype=np.float64)
    p1, ms_m1 = t(lambda: comps["prediction1"].predict(X, []))
    p2, ms_m2 = t(lambda: comps["prediction2"].predict(X, []))
    avg, ms_comb = t(lambda: comb.aggregate([p1, p2], []))
    _, ms_ot = t(lambda: ot.transform_output_raw({"data": {"ndarray": avg.tolist()}}))
    print(json.dumps({"stage_ms": {"transformer": ms_tr, "transformer_json_dump": ms_tr_json, "densenet169_b1": ms_m1,
                                   "resnet50_b1": ms_m2, "combiner": ms_comb, "output_transformer": ms_ot}}),
          flush=True)
    comps["prediction1"].calls = comps["prediction2"].calls = 0


def _heartbeat():
    import threading

    t0 = time.time()

    def beat():
        while True:
            time.sleep(20)
            print(f"# alive {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    _heartbeat()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
    from test_cnn import _ensemble

    t0 = time.perf_counter()
    comps = {"prediction1": ImageNetModel("densenet169", device=0, max_batch=32),
             "prediction2": ImageNetModel("resnet50", device=0, max_batch=32)}
    setup = time.perf_counter() - t0
    graph = _ensemble(0, 224)
    workers = int(os.environ.get("IMAGENET_TR_WORKERS", "0"))
    if workers:  # the transformer (JPEG decode + crop) in a pool of worker processes
        graph["children"][0]["workers"] = workers
    spec = {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=0, components=comps)
    reqs = [{"binData": jpeg(i)} for i in range(64)]
    try:
        for _ in range(4):
            dep.predict(reqs[0])
        stage_breakdown(comps, reqs)
        for conc, n in ((1, 64), (4, 128), (16, 256), (32, 512)):
            lat = []

            def one(i):
                t = time.perf_counter()
                o = dep.predict(reqs[i % len(reqs)])
                lat.append(time.perf_counter() - t)
                return o

            c0 = comps["prediction2"].calls
            t = time.perf_counter()
            with cf.ThreadPoolExecutor(conc) as ex:
                outs = list(ex.map(one, range(n)))
            wall = time.perf_counter() - t
            assert all(o.get("strData", "").isdigit() for o in outs), outs[:2]
            lat.sort()
            print(json.dumps({"graph": "imagenet-ensemble (densenet169 + resnet50, bf16, HIP graphs)",
                              "transformer_workers": workers,
                              "concurrency": conc, "requests": n, "images_per_s": round(n / wall, 1),
                              "p50_ms": round(lat[len(lat) // 2] * 1e3, 2),
                              "p99_ms": round(lat[min(len(lat) - 1, int(len(lat) * 0.99))] * 1e3, 2),
                              "model_calls": comps["prediction2"].calls - c0, "setup_s": round(setup, 1),
                              "units": {k: getattr(u, "native").stats() for k, u in dep.python_units.items()
                                        if getattr(u, "native", None) is not None}}),
                  flush=True)
    finally:
        dep.close()


if __name__ == "__main__":
    main()
