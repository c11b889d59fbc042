"""ImageNet CNNs (models/cnn.py) on one MI355X: per-image latency at batch 1
and throughput at larger batches for fp32 NCHW eager, bf16 NHWC eager and
bf16 NHWC HIP graphs; numerics against the fp32 CPU network.  One JSON line
per measurement."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seldon_core_amd.models import cnn  # noqa: E402

ARCHS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["resnet50", "densenet169"]
T0 = time.time()


def _heartbeat():  # library kernel compiles can be silent for minutes
    while True:
        time.sleep(20)
        print(f"# alive {time.time() - T0:.0f} s", flush=True)


import threading  # noqa: E402

threading.Thread(target=_heartbeat, daemon=True).start()


def emit(**kw):
    print(json.dumps(kw), flush=True)


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for arch in ARCHS:
    net = cnn.build(arch, seed=1)
    x_cpu = torch.rand(4, 3, 224, 224, generator=torch.Generator().manual_seed(2)) * 255.0
    with torch.no_grad():
        ref_logits = net(x_cpu)
    ref = torch.softmax(ref_logits, 1).double().numpy()
    # (dtype, channels_last, graphs, tune)
    configs = [("fp32", False, False, False), ("bf16", True, False, False), ("bf16", True, True, False),
               ("bf16", None, True, True)]
    if os.environ.get("CNN_CONFIGS") == "layouts":  # dtype / layout A/B, graphs on, untuned
        configs = [("bf16", True, True, False), ("fp16", True, True, False), ("bf16", False, True, False),
                   ("fp16", False, True, False)]
    if os.environ.get("CNN_CONFIGS") == "default":  # the serving default (tuned NHWC) + untuned NCHW
        configs = [("bf16", None, True, True), ("bf16", False, True, False)]
    if os.environ.get("CNN_CONFIGS") == "tuned":  # both layouts with MIOpen's solver search
        configs = [("bf16", True, True, True), ("bf16", False, True, True)]
    for dtype, cl, graphs, tune in configs:
        t0 = time.perf_counter()
        m = cnn.CompiledCnn(cnn.build(arch, seed=1), device=0, dtype=dtype, max_batch=32, graphs=graphs,
                            channels_last=cl, tune=tune)
        setup_s = time.perf_counter() - t0
        got = m(x_cpu.numpy())
        err = float(np.abs(got - ref).max())
        top1 = float((got.argmax(1) == ref.argmax(1)).mean())
        res = {"arch": arch, "tune": tune, "dtype": dtype, "channels_last": m.channels_last, "graphs": bool(m.graphs), "setup_s": round(setup_s, 1),
               "graph_error": m.graph_error, "max_abs_prob_err": err, "top1_agree": top1}
        for bs in (1, 8, 32):
            xd = torch.rand(bs, 3, 224, 224, device="cuda")
            ms = timed(lambda: m.run(xd), 20 if bs > 1 else 50)
            res[f"b{bs}_ms"] = round(ms, 3)
            res[f"b{bs}_img_s"] = round(bs / ms * 1e3, 1)
        emit(**res)
        del m
        torch.cuda.empty_cache()
