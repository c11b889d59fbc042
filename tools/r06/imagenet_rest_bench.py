"""The ImageNet ensemble served over REST by the native front end
(Deployment.serve), driven by closed-loop keep-alive HTTP clients posting
{"binData": <JPEG>} to /api/v0.1/predictions.  One JSON line per concurrency:
images/s, p50 / p99 latency.  Transformer in 4 worker processes, tuned CNNs."""
import concurrent.futures as cf
import http.client
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests"))

import seldon_core_amd as sca  # noqa: E402
from imagenet_bench import _heartbeat, jpeg  # noqa: E402
from seldon_core_amd.components.examples import ImageNetModel  # noqa: E402
from test_cnn import _ensemble  # noqa: E402


def main():
    _heartbeat()
    comps = {"prediction1": ImageNetModel("densenet169", device=0, max_batch=32),
             "prediction2": ImageNetModel("resnet50", device=0, max_batch=32)}
    graph = _ensemble(0, 224)
    graph["children"][0]["workers"] = 4
    dep = sca.Deployment({"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}, device=0,
                         components=comps)
    h = dep.serve(http_port=0, grpc_port=None, threads=8, host="127.0.0.1")
    bodies = [json.dumps({"binData": jpeg(i)}).encode() for i in range(64)]
    try:
        def client(n, lat, k0):
            c = http.client.HTTPConnection("127.0.0.1", h.http_port, timeout=60)
            for i in range(n):
                t = time.perf_counter()
                c.request("POST", "/api/v0.1/predictions", bodies[(k0 + i) % len(bodies)],
                          {"Content-Type": "application/json"})
                r = c.getresponse()
                body = r.read()
                assert r.status == 200, body[:200]
                assert json.loads(body)["strData"].isdigit()
                lat.append(time.perf_counter() - t)
            c.close()

        client(8, [], 0)  # warm every worker path
        for conc, per in ((1, 64), (16, 32), (32, 24)):
            lat = []
            t = time.perf_counter()
            with cf.ThreadPoolExecutor(conc) as ex:
                list(ex.map(lambda k: client(per, lat, k), range(conc)))
            wall = time.perf_counter() - t
            lat.sort()
            print(json.dumps({"graph": "imagenet-ensemble over REST (native front end)", "concurrency": conc,
                              "requests": len(lat), "images_per_s": round(len(lat) / wall, 1),
                              "p50_ms": round(lat[len(lat) // 2] * 1e3, 2),
                              "p99_ms": round(lat[min(len(lat) - 1, int(len(lat) * 0.99))] * 1e3, 2)}), flush=True)
    finally:
        h.stop()
        dep.close()


if __name__ == "__main__":
    main()
