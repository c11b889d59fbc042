"""Latency / throughput probe of one rank-placed MODEL node over the CPU
fabric (2 ranks, REST load on rank 0), against the same node in-process
(PLACED=0).  Knobs: PLACED, SPIN (batcher spin_wait), SLOTS, THREADS, USERS.

    CUDA_VISIBLE_DEVICES= python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 tools/fabric_lat_probe.py
"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch.distributed as dist
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression
from seldon_core_amd.parallel.fabric import init_fabric, serve_peer
from seldon_core_amd.utils import benchkit as bk
lr = iris_logistic_regression()
placed = os.environ.get("PLACED", "1") == "1"
node = {"name": "m", "type": "MODEL"}
if placed: node["rank"] = 1
spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": node}
fabric = init_fabric(device=-1)
if rank != 0:
    srv = serve_peer(spec, fabric, {"m": lr}); srv.join(); print("worker", srv.batches, srv.rows, srv.max_inflight); fabric.close()
else:
    spin = os.environ.get("SPIN", "0") == "1"
    dep = sca.Deployment(spec, components={"m": lr}, device=-1, fabric=fabric, fuse=False,
                         batcher={"max_batch": 4096, "slots": int(os.environ.get("SLOTS", "4")), "spin_wait": spin})
    h = dep.serve(http_port=0, grpc_port=0, threads=int(os.environ.get("THREADS", "4")), host="127.0.0.1")
    wl = bk.Workload("iris")
    body = wl.rest_body()
    users = int(os.environ.get("USERS", "16"))
    bk.run_loadgen(h.http_port, 1, 0, "rest", body, users, 2, 5000, 60)
    for u in dep.batched.values(): u.reset_stats()
    t = time.perf_counter()
    lg = bk.run_loadgen(h.http_port, 2, 0, "rest", body, users, 2, 40000, 60)
    el = time.perf_counter() - t
    st = {k: u.stats() for k, u in dep.batched.items()}
    print(json.dumps({k: lg.get(k) for k in ("rps", "p50_ms", "p99_ms")}), json.dumps(st))
    h.stop(); dep.close(); fabric.close()
dist.barrier(); dist.destroy_process_group()
