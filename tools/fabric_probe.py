"""RCCL fabric end-to-end check (run with torchrun, one process per GPU).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port 29533 tools/fabric_probe.py [--same-device]

Rank 0 serves a graph whose MODEL children live on ranks 1..N-1 (plus one on
rank 0), sends batches through the engine and checks every answer against the
CPU reference of the same model; ranks > 0 run PeerServer loops.
``--same-device`` puts every rank on GPU 0: RCCL rejects two ranks on one
device (ncclCommInitRank -> invalid usage, seen on the 1-GPU box), so it only
checks the control-plane rendezvous; the CPU fabric tests (tests/test_fabric.py)
run the whole peer protocol without GPUs.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--requests", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    if torch.cuda.is_available():
        dev = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(dev)
    else:  # CPU fabric: the same peer protocol with the payloads on the control sockets
        dev = -1
    dist.init_process_group("gloo")
    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer

    lr = iris_logistic_regression()
    kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(world)]
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "ab", "type": "ROUTER", "implementation": "SIMPLE_ROUTER", "children": kids}
            if world == 1 else
            {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids}}
    comps = {f"m{r}": lr for r in range(world)}
    fabric = init_fabric(device=dev)
    if rank != 0:
        srv = serve_peer(spec, fabric, comps)
        srv.join()
        err = srv.error()
        print(json.dumps({"rank": rank, "batches": srv.batches, "rows": srv.rows, "error": err}), flush=True)
        fabric.close()
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(1 if err else 0)
    dep = sca.Deployment(spec, components=comps, device=dev, fabric=fabric)
    kinds = {n: dep.engine.unit_kind(n) for n in dep.engine.node_names()}
    rng = np.random.default_rng(0)
    worst = 0.0
    t0 = time.perf_counter()
    for i in range(args.requests):
        X = rng.normal(size=(1 + i % 7, 4))
        out = dep.predict({"data": {"ndarray": X.tolist()}})
        got = np.array(out["data"]["ndarray"])
        worst = max(worst, float(np.abs(got - lr.predict_proba(X)).max()))
    dt = time.perf_counter() - t0
    dep.close()  # stops the peers
    fabric.close()
    print(json.dumps({"rank": 0, "world": world, "device": dev, "data_plane": "rccl" if dev >= 0 else "sockets",
                      "units": kinds, "requests": args.requests, "max_abs_err": worst,
                      "req_per_s": args.requests / dt}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if worst < 1e-12 else 2)


if __name__ == "__main__":
    main()
