#!/usr/bin/env python3
"""Rank-placed graphs over the mesh with every rank a separate process on
the SAME GPU (or CPU), against the same graphs in one process.

    python tools/mesh_bench.py --world 4 --device 0 [--kinds abtest,mab,pipeline]
                               [--users 64] [--threads 4] [--out FILE]

This is the "folded" rehearsal of BASELINE.json's multi-GPU configs on a
1-GPU box: rank processes, HIP contexts, IPC slabs and doorbells are real,
only the GPUs are one.  For each graph kind: rank 0 serves the rank-placed
graph (``bk.build_rank_graph``) over REST, the closed-loop native load
generator drives it (sampled reply bodies checked), a CPU-oracle self check
runs, then rank 0 serves the in-process graph (``bk.build_graph``, every node
on --device) under the same load.  One JSON line with both numbers per kind.
"""
import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--kinds", default="abtest,mab,pipeline")
    ap.add_argument("--model", default="iris")
    ap.add_argument("--users", type=int, default=64)
    ap.add_argument("--threads", type=int, default=4, help="front-end threads on rank 0")
    ap.add_argument("--client-threads", type=int, default=4)
    ap.add_argument("--window", type=float, default=2.0, help="seconds per measured window")
    ap.add_argument("--spin", action="store_true", help="batcher spin_wait (default: the bench's low-CPU mode)")
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def measure(port, wl, oracle, a, bk):
    body = wl.rest_body()
    expect = bk.rest_expect(port, body)
    rate = bk.probe_rate(port, "rest", body, a.users, a.client_threads, lambda: 60.0, min_s=0.5, expect=expect)
    n = bk.window_requests(rate, a.window)
    lg = bk.run_loadgen(port, 2, 0, "rest", body, a.users, a.client_threads, n, 120.0, expect=expect)
    chk = bk.self_check(port, wl, oracle, seed=7)
    return {"value": round(lg["rps"], 1), "p50_ms": lg["p50_ms"], "p99_ms": lg["p99_ms"],
            "window_s": round(lg["seconds"], 3), "sampled_replies_checked": lg.get("checked", 0), "self_check": chk}


def child(a):
    import torch.distributed as dist

    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer
    from seldon_core_amd.serving.deployment import Deployment
    from seldon_core_amd.utils import benchkit as bk

    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    rank, world = dist.get_rank(), dist.get_world_size()
    wl = bk.Workload(a.model)
    batcher = {"max_batch": 4096, "slots": 4, "spin_wait": bool(a.spin)}
    for kind in [k for k in a.kinds.split(",") if k]:
        if kind == "pipeline" and world < 4:
            continue
        g, comps, oracle, label = bk.build_rank_graph(wl, kind, world)
        fabric = init_fabric(device=a.device)
        if rank != 0:
            srv = serve_peer(bk.sdep(g), fabric, comps)
            srv.join()
            print(json.dumps({"kind": kind, "rank": rank, "stats": srv.stats(), "error": srv.error()}), flush=True)
            fabric.close()
            continue
        r = {"kind": kind, "graph": label, "world": world, "device": a.device, "transport": fabric.transport}
        dep = Deployment(bk.sdep(g), components=comps, device=a.device, fabric=fabric, fuse=False, batcher=batcher)
        h = dep.serve(http_port=0, grpc_port=0, threads=a.threads, host="127.0.0.1")
        try:
            r["ranks"] = measure(h.http_port, wl, oracle, a, bk)
            if dep.mesh is not None:
                r["programs"] = [{"root": p.root, "stages": p.describe(), "messages_per_batch": m}
                                 for p, m in zip(dep.mesh.programs, dep.mesh.messages)]
            r["unit_kinds"] = {n: dep.engine.unit_kind(n) for n in dep.engine.node_names()}
        finally:
            h.stop()
            dep.close()
            fabric.close()
        # the same graph in one process, every node on the device
        g2, comps2, oracle2, label2 = bk.build_graph(wl, kind, [a.device] * world)
        dep2 = Deployment(bk.sdep(g2), components=comps2, device=a.device, batcher=batcher)
        h2 = dep2.serve(http_port=0, grpc_port=0, threads=a.threads, host="127.0.0.1")
        try:
            r["in_process"] = measure(h2.http_port, wl, oracle2, a, bk)
            r["in_process"]["graph"] = label2
        finally:
            h2.stop()
            dep2.close()
        r["ratio_in_process_over_ranks"] = round(r["in_process"]["value"] / max(1e-9, r["ranks"]["value"]), 2)
        print(json.dumps(r), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(r) + "\n")
    dist.barrier()
    dist.destroy_process_group()


def main():
    a = parse()
    if a.child:
        child(a)
        return 0
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.pop("GPU_STREAMOPS_CP_WAIT", None)
        if a.device < 0:
            env["CUDA_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", *sys.argv[1:]], env=env))
    rc = 0
    t0 = time.time()
    for p in procs:
        try:
            rc = rc or p.wait(timeout=max(1.0, 900 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            rc = 124
    return rc


if __name__ == "__main__":
    sys.exit(main())
