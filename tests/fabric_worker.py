"""Rank process for the rank-placed graph tests (tests/test_fabric.py on CPU
gangs, tests/test_mesh_gpu.py with every rank on GPU 0).

Rank 0 serves a graph whose nodes are placed on other ranks (``rank: r``)
through the mesh (csrc/parallel/mesh.h); the workers run ``serve_peer``.
Rank 0 checks every answer against a CPU oracle and prints one JSON line;
workers print their mesh statistics.

    python tests/fabric_worker.py MODE      (RANK / WORLD_SIZE / MASTER_* set)

SCA_TEST_DEVICE: GPU for every rank (default: -1, a CPU gang).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _spec(graph):
    return {"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": graph}


def build(mode, world):
    """(graph, components, oracle, options) of a test mode."""
    import numpy as np

    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression

    C = sca.native()
    lr = iris_logistic_regression()
    proba = lr.predict_proba
    scale = 1.0 + 0.05 * np.arange(4)
    scale2 = 1.0 - 0.03 * np.arange(4)
    opts = {"requests": 40, "threads": 1, "max_rows": 6}
    if mode == "single":  # one remote MODEL node
        return {"name": "m", "type": "MODEL", "rank": world - 1}, {"m": lr}, proba, opts
    if mode == "combiner":  # K-way: one model per rank, averaged by the engine's combiner on rank 0
        kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(world)]
        return ({"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids},
                {f"m{r}": lr for r in range(world)}, proba, opts)
    if mode == "remote_combiner":  # every branch remote: ONE program, final mean on rank 0's host
        kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(1, world)]
        return ({"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids},
                {f"m{r}": lr for r in range(1, world)}, proba, opts)
    if mode == "pipeline":  # scaler@1 -> scaler@2 -> iris@3: stage-to-stage edges, 4 messages per batch
        s1 = C.linear_model(np.diag(scale), np.zeros(4), 0)
        s2 = C.linear_model(np.diag(scale2), np.zeros(4), 0)
        g = {"name": "s1", "type": "TRANSFORMER", "rank": 1, "children": [
            {"name": "s2", "type": "TRANSFORMER", "rank": 2, "children": [
                {"name": "m", "type": "MODEL", "rank": 3}]}]}
        return g, {"s1": s1, "s2": s2, "m": lr}, lambda X: proba(np.asarray(X) * scale * scale2), opts
    if mode == "dag":  # the bench pipeline: scaler@3 -> AVERAGE_COMBINER(rank 0) over a@1, b@2
        s = C.linear_model(np.diag(scale), np.zeros(4), 0)
        g = {"name": "scaler", "type": "TRANSFORMER", "rank": 3, "children": [
            {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
             "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}]}
        return g, {"scaler": s, "a": lr, "b": lr}, lambda X: proba(np.asarray(X) * scale), opts
    if mode == "nested_combiner":  # AVERAGE(AVERAGE(a@1, b@2), c@3), no ranks on the combiners
        W2 = np.random.default_rng(7).normal(size=(3, 4)) * 0.1
        s = C.linear_model(W2, np.zeros(3), 0)
        g = {"name": "outer", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
            {"name": "inner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
             "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]},
            {"name": "c", "type": "MODEL", "rank": 3}]}
        return (g, {"a": lr, "b": s, "c": lr},
                lambda X: 0.5 * (0.5 * (proba(X) + np.asarray(X) @ W2.T) + proba(X)), opts)
    if mode == "python":  # a Python TRANSFORMER on rank 1 feeding the iris MODEL on rank 2
        g = {"name": "double", "type": "TRANSFORMER", "rank": 1, "in_cols": 4,
             "children": [{"name": "m", "type": "MODEL", "rank": 2}]}
        return g, {"double": "mesh_components.Doubler", "m": lr}, lambda X: proba(2.0 * np.asarray(X)), opts
    if mode == "python_error":  # the Python stage raises for negative rows: those requests fail, others pass
        g = {"name": "picky", "type": "TRANSFORMER", "rank": 1, "in_cols": 4,
             "children": [{"name": "m", "type": "MODEL", "rank": 2}]}
        return g, {"picky": "mesh_components.Picky", "m": lr}, proba, dict(opts, errors=True)
    if mode == "concurrent":  # A/B router on rank 0 over two remote programs, 4 client threads
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}
        return g, {"a": lr, "b": lr}, proba, dict(opts, requests=60, threads=4)
    if mode == "large":  # requests far larger than a slot (chunked) and outputs wider than socket buffers
        W = np.random.default_rng(5).normal(size=(784, 4))
        wide = C.linear_model(W, np.zeros(784), 0)
        g = {"name": "w", "type": "MODEL", "rank": 1}
        return g, {"w": wide}, lambda X: np.asarray(X) @ W.T, dict(opts, requests=4, max_rows=3000, large=True)
    raise ValueError(mode)


def main():
    import threading

    import numpy as np
    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import seldon_core_amd as sca
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer
    from seldon_core_amd.serving.errors import EngineError

    mode = sys.argv[1]
    device = int(os.environ.get("SCA_TEST_DEVICE", "-1"))
    fabric = init_fabric(device=device)
    if mode == "orphan":
        return orphan(fabric, rank, world)
    graph, comps, oracle, opts = build(mode, world)
    spec = _spec(graph)
    if rank != 0:
        srv = serve_peer(spec, fabric, comps)
        srv.join()
        st = srv.stats()
        print(json.dumps(dict(st, rank=rank, error=srv.error(), slots=srv.slots, transport=fabric.transport)),
              flush=True)
        fabric.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    low_cpu = os.environ.get("SCA_TEST_LOW_CPU") == "1"  # the batcher's low-CPU mode (bench setting)
    batcher = {"max_batch": 64}
    if low_cpu:
        batcher["spin_wait"] = False
    dep = sca.Deployment(spec, components=comps, device=device, fabric=fabric, batcher=batcher)
    worst = [0.0]
    rows = [0]
    errors, failed = [], [0]
    lock = threading.Lock()

    def client(t):
        rng = np.random.default_rng(t)
        for i in range(opts["requests"]):
            n = (opts["max_rows"] - 7 * i) if opts.get("large") else 1 + (i + t) % opts["max_rows"]
            X = rng.normal(loc=4.0, scale=1.5, size=(n, 4))
            bad = opts.get("errors") and i % 5 == 3
            if opts.get("errors"):
                X[:, 0] = np.abs(X[:, 0])  # only the marked requests may carry a negative first feature
            if bad:
                X[0, 0] = -1.0
            try:
                out = dep.predict({"data": {"ndarray": X.tolist()}})
            except EngineError as e:
                with lock:
                    if bad:
                        failed[0] += 1
                    else:
                        errors.append(repr(e))
                continue
            except Exception as e:  # noqa: BLE001
                with lock:
                    errors.append(repr(e))
                continue
            got = np.asarray(out["data"]["ndarray"], dtype=np.float64)
            err = float(np.abs(got - oracle(X)).max())
            with lock:
                if bad:
                    errors.append("a failing request was answered")
                worst[0] = max(worst[0], err)
                rows[0] += len(X)

    th = [threading.Thread(target=client, args=(t,)) for t in range(opts["threads"])]
    for t in th:
        t.start()
    for t in th:
        t.join()
    kinds = {name: dep.engine.unit_kind(name) for name in dep.engine.node_names()}
    msgs = list(dep.mesh.messages) if dep.mesh is not None else []
    programs = [p.describe() for p in dep.mesh.programs] if dep.mesh is not None else []
    edges = list(dep.mesh.edges) if dep.mesh is not None else []
    peer = dict(dep.mesh.peer) if dep.mesh is not None else {}
    dep.close()  # stops the workers' loops
    fabric.close()
    print(json.dumps({"rank": 0, "worst": worst[0], "rows": rows[0], "errors": errors, "failed": failed[0],
                      "kinds": kinds, "messages": msgs, "programs": programs, "transport": fabric.transport,
                      "edges": edges, "peer": peer}),
          flush=True)
    dist.barrier()
    dist.destroy_process_group()


def orphan(fabric, rank, world):
    """Rank 0 drops the gang without a stop header (as a crashed front end
    would); the worker must leave its loop with an error."""
    import time

    import torch.distributed as dist

    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.parallel.fabric import serve_peer

    spec = _spec({"name": "m", "type": "MODEL", "rank": world - 1})
    if rank != 0:
        srv = serve_peer(spec, fabric, {"m": iris_logistic_regression()})
        srv.join()
        print(json.dumps({"rank": rank, "error": srv.error()}), flush=True)
        fabric.close()
        os._exit(0)  # rank 0 is gone: no barrier to meet
    else:
        import seldon_core_amd as sca

        dep = sca.Deployment(spec, components={"m": iris_logistic_regression()}, device=-1, fabric=fabric)
        time.sleep(0.5)  # the worker is polling its ring by now
        del dep
        print(json.dumps({"rank": 0}), flush=True)
        os._exit(0)  # no stop header, no clean close: the sockets just go away


if __name__ == "__main__":
    main()
