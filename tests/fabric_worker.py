"""Rank process for tests/test_fabric.py (gloo + CPU fabric, device -1).

Rank 0 serves a graph with nodes placed on other ranks (``rank: r``) through
the native PeerRowModel, workers run the native PeerServer loop; rank 0 checks
every answer against sklearn and prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer

    lr = iris_logistic_regression()
    mode = sys.argv[1]
    if mode == "concurrent":
        return concurrent(lr, rank, world)
    if mode == "orphan":
        return orphan(lr, rank, world)
    if mode == "large":
        return large(lr, rank, world)
    if mode == "combiner":  # K-way gather: one model per rank, averaged on rank 0
        kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(world)]
        graph = {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids}
        comps = {f"m{r}": lr for r in range(world)}
    else:  # a single remote MODEL node on the last rank behind a local router
        graph = {"name": "m", "type": "MODEL", "rank": world - 1}
        comps = {"m": lr}
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": graph}
    fabric = init_fabric(device=-1)
    assert not fabric.gpu
    if rank != 0:
        srv = serve_peer(spec, fabric, comps)
        srv.join()
        print(json.dumps({"rank": rank, "batches": srv.batches, "rows": srv.rows, "host_syncs": srv.host_syncs,
                          "error": srv.error()}), flush=True)
        fabric.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    low_cpu = os.environ.get("SCA_TEST_LOW_CPU") == "1"  # the batcher's low-CPU mode (bench setting)
    dep = sca.Deployment(spec, components=comps, device=-1, fabric=fabric,
                         batcher={"spin_wait": False} if low_cpu else None)
    rng = np.random.default_rng(0)
    worst = 0.0
    n = 0
    for i in range(40):
        X = rng.normal(loc=4.0, scale=1.5, size=(1 + i % 5, 4))
        out = dep.predict({"data": {"ndarray": X.tolist()}})
        got = np.asarray(out["data"]["ndarray"])
        worst = max(worst, float(np.abs(got - lr.predict_proba(X)).max()))
        n += len(X)
    kinds = {name: dep.engine.unit_kind(name) for name in dep.engine.node_names()}
    dep.close()  # stops the workers' loops
    fabric.close()
    print(json.dumps({"rank": 0, "worst": worst, "rows": n, "kinds": kinds}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def concurrent(lr, rank, world):
    """4 threads on rank 0 drive the native peer models at once -- one per
    worker and a fan-out over all of them -- so the workers see several
    batches in flight (K = SCA_FABRIC_SLOTS slots, slowed by
    SCA_FABRIC_WORKER_DELAY_US); every answer is checked against sklearn."""
    import threading

    import numpy as np
    import torch.distributed as dist

    import seldon_core_amd as sca
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer

    kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(1, world)]
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids}}
    fabric = init_fabric(device=-1)
    if rank != 0:
        srv = serve_peer(spec, fabric, {k["name"]: lr for k in kids})
        srv.join()
        print(json.dumps({"rank": rank, "batches": srv.batches, "rows": srv.rows, "max_inflight": srv.max_inflight,
                          "slots": srv.slots, "error": srv.error()}), flush=True)
        fabric.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    C = sca.native()
    models = [C.peer_row_model(fabric, [r], 0, 4, 3) for r in range(1, world)]
    models.append(C.peer_row_model(fabric, list(range(1, world)), 0, 4, 3))  # broadcast + gather + mean
    worst = [0.0]
    rows = [0]
    lock = threading.Lock()
    errors = []

    def client(t):
        rng = np.random.default_rng(t)
        try:
            for i in range(60):
                X = rng.normal(loc=4.0, scale=1.5, size=(1 + (i + t) % 6, 4))
                m = models[(i + t) % len(models)]
                got = m.run_cpu(X)
                err = float(np.abs(got - lr.predict_proba(X)).max())
                with lock:
                    worst[0] = max(worst[0], err)
                    rows[0] += len(X)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=client, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    fabric.stop_peers()
    fabric.close()
    print(json.dumps({"rank": 0, "worst": worst[0], "rows": rows[0], "errors": errors}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def large(lr, rank, world):
    """Replies far larger than a socket buffer (60k rows x 3 classes = 1.4 MB)
    arrive in pieces: the polling reader keeps its place in the reply across
    EAGAINs, both through the asynchronous path (two callers' replies queued
    back to back) and the synchronous one."""
    import threading

    import numpy as np
    import torch.distributed as dist

    import seldon_core_amd as sca
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer

    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "m", "type": "MODEL", "rank": 1}}
    fabric = init_fabric(device=-1)
    if rank != 0:
        srv = serve_peer(spec, fabric, {"m": lr})
        srv.join()
        print(json.dumps({"rank": rank, "batches": srv.batches, "rows": srv.rows, "error": srv.error()}), flush=True)
        fabric.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    C = sca.native()
    m = C.peer_row_model(fabric, [1], 0, 4, 3)
    rng = np.random.default_rng(3)
    worst = [0.0]
    errors = []

    def client(t):
        try:
            for _ in range(3):
                X = rng.normal(loc=4.0, scale=1.5, size=(60000 - 7 * t, 4))
                got = m.run_cpu(X)
                worst[0] = max(worst[0], float(np.abs(got - lr.predict_proba(X)).max()))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=client, args=(t,)) for t in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    # the batcher's asynchronous path (start_cpu + polling)
    dep = sca.Deployment(spec, components={"m": lr}, device=-1, fabric=fabric)
    X = rng.normal(loc=4.0, scale=1.5, size=(30000, 4))
    out = dep.predict({"data": {"ndarray": X.tolist()}})
    worst[0] = max(worst[0], float(np.abs(np.asarray(out["data"]["ndarray"]) - lr.predict_proba(X)).max()))
    dep.close()
    fabric.close()
    print(json.dumps({"rank": 0, "worst": worst[0], "errors": errors}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def orphan(lr, rank, world):
    """Rank 0 drops its fabric without a stop header (as a crashed front end
    would); the worker must leave its loop with an error."""
    import torch.distributed as dist

    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer

    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "m", "type": "MODEL", "rank": world - 1}}
    fabric = init_fabric(device=-1)
    if rank != 0:
        srv = serve_peer(spec, fabric, {"m": lr})
        srv.join()
        print(json.dumps({"rank": rank, "error": srv.error()}), flush=True)
        fabric.close()
    else:
        import time

        time.sleep(0.5)  # the worker is polling its ring by now
        fabric.close()
        print(json.dumps({"rank": 0}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
