"""Tree-ensemble kernel variants timed back-to-back on one stream (GPU only).

    python tools/tree_microbench.py [--trees 1000 --depth 8 --features 32]

For each batch size: two-pass (partial + reduce) vs fused last-workgroup
reduce, trees traversed from global memory vs staged in LDS, at the chunk
sizes the model's planner would pick.  Reports microseconds per batch from
HIP events over `iters` launches (includes launch gaps: the serving loop's
cost), and checks every variant against the two-pass global result.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=1000)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--rows", default="1,4,17,32,64,128,512,2048")
    ap.add_argument("--sweep", action="store_true", help="two-pass global at chunk = tpr x {1,2,4,8,16}")
    ap.add_argument("--sweep-rb", action="store_true", help="two-pass global, rows/block 1..64 at one tree/lane")
    ap.add_argument("--small", action="store_true",
                    help="small-batch plans: the whole-ensemble kernel at 1/2/4 trees per thread vs the fused "
                         "partial kernel (last-workgroup reduce) at 16-256 trees per workgroup")
    a = ap.parse_args()
    from seldon_core_amd import native

    K = native().kernels
    dev = "cuda"
    T, D, F = a.trees, a.depth, a.features
    ni = (1 << D) - 1
    g = torch.Generator().manual_seed(0)
    thr = torch.randn(T * ni, generator=g)
    feat = torch.randint(0, F, (T * ni,), generator=g, dtype=torch.int32)
    nodes = torch.stack([thr.view(torch.int32), feat], 1).contiguous().to(dev)  # {float thr, int feat}
    leaves = (torch.randn(T * (ni + 1), generator=g) * 0.01).to(dev)
    s = torch.cuda.current_stream().cuda_stream
    results = []
    for rows in [int(r) for r in a.rows.split(",")]:
        X = torch.randn(rows, F, dtype=torch.float64, generator=g).to(dev)
        rb = 1
        while rb < rows and rb < 64:
            rb <<= 1
        tpr = 256 // rb
        lds_cap = K.tree_lds_max_trees(D, rb, F)
        lds_chunk = 1
        while lds_chunk * 2 <= lds_cap:
            lds_chunk *= 2
        tiles = (rows + rb - 1) // rb
        want = max(1, 1024 // tiles)
        gchunk = max(tpr, -(-T // want))
        gchunk = 1 << (gchunk - 1).bit_length()
        out_ref = None
        row = {"rows": rows, "rb": rb}
        variants = [("2pass_global", gchunk, 0, False), ("2pass_lds", lds_chunk, lds_chunk, False),
                    ("fused_global", gchunk, 0, True), ("fused_lds", lds_chunk, lds_chunk, True)]
        if a.sweep:
            variants = [(f"2pass_c{c}", c, 0, False) for c in sorted({min(T, max(1, tpr * m)) for m in
                                                                    (1, 2, 4, 8, 16)} | {gchunk})]
        if a.sweep_rb:
            variants = []
            r = 1
            while r <= rb:
                variants.append((f"rb{r}", 256 // r, 0, False, r))
                r <<= 1
        if a.small:
            variants = []
            for tpt in (1, 2, 4):
                r = 1
                while r < 16 and r < rows and T * (r * 2) <= tpt * 1024:
                    r <<= 1
                variants.append((f"whole_tpt{tpt}", 0, 0, "whole", r, 0))
                if D == 8:
                    for la in (21, 22, 31, 32, 41, 42):
                        variants.append((f"whole_la{la}_tpt{tpt}", 0, 0, "whole", r, la))
            for r in sorted({1, 2, 4, min(rb, 16)}):
                for c in (16, 32, 64, 128, 256):
                    if c >= 256 // r:  # a chunk fills the block's tree lanes
                        variants.append((f"fused_rb{r}_c{c}", c, 0, True, r))
                cap = K.tree_lds_max_trees(D, r, F)  # trees copied whole into LDS: D LDS reads per walk
                for c in (4, 8, 16):
                    if c <= cap:
                        variants.append((f"fused_lds_rb{r}_c{c}", c, c, True, r))
        if a.small:  # whole ensemble split over `parts` workgroups per row tile (atomic fold)
            for parts in (4, 8, 16, 32):
                variants.append((f"split{parts}", parts, 0, "split"))
            variants.append(("tile", 0, 0, "tile"))
            for parts in (8, 16):
                variants.append((f"split{parts}_hostfold", parts, 0, "split_host"))
        for v in variants:
            name, chunk, lds, fused = v[:4]
            if fused == "split_host":  # part sums to out[r][part]; the host adds them (timed kernel only)
                out = torch.empty(rows * chunk, dtype=torch.float64, device=dev)

                def launch():
                    K.tree_perfect_split(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, T, chunk,
                                         0, 1.0, 0, out.data_ptr(), 1, 0, 0, s)

                for _ in range(20):
                    launch()
                torch.cuda.synchronize()
                folded = out.view(rows, chunk).sum(1)
                err = float((folded - out_ref).abs().max()) if out_ref is not None else None
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                row[name] = {"us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "max_err": err}
                continue
            if fused == "tile":
                out = torch.empty(rows, dtype=torch.float64, device=dev)
                acc = torch.zeros(rows, dtype=torch.float64, device=dev)
                cnt = torch.zeros(16, dtype=torch.int32, device=dev)

                def launch():
                    K.tree_perfect_tile(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, T, 0, 1.0,
                                        0, out.data_ptr(), 1, acc.data_ptr(), cnt.data_ptr(), s)

                for _ in range(20):
                    launch()
                torch.cuda.synchronize()
                err = float((out - out_ref).abs().max()) if out_ref is not None else None
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                row[name] = {"us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "max_err": err,
                             "acc_rezeroed": float(acc.abs().max()) == 0.0 and int(cnt.abs().max()) == 0}
                continue
            if fused == "split":
                out = torch.empty(rows, dtype=torch.float64, device=dev)
                acc = torch.zeros(rows, dtype=torch.float64, device=dev)
                cnt = torch.zeros(1024, dtype=torch.int32, device=dev)

                def launch():
                    K.tree_perfect_split(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, T, chunk,
                                         0, 1.0, 0, out.data_ptr(), 1, acc.data_ptr(), cnt.data_ptr(), s)

                for _ in range(20):
                    launch()
                torch.cuda.synchronize()
                if out_ref is None:
                    out_ref = out.clone()
                err = float((out - out_ref).abs().max())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                row[name] = {"us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "parts": chunk, "max_err": err,
                             "acc_rezeroed": float(acc.abs().max()) == 0.0 and int(cnt.abs().max()) == 0}
                continue
            rb_v = v[4] if len(v) > 4 else rb
            if fused == "whole":
                out = torch.empty(rows, dtype=torch.float64, device=dev)
                la = v[5]

                def launch():
                    K.tree_perfect_whole(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, T, rb_v,
                                         0, 1.0, 0, out.data_ptr(), 1, s, la)

                for _ in range(20):
                    launch()
                torch.cuda.synchronize()
                if out_ref is None:
                    out_ref = out.clone()
                err = float((out - out_ref).abs().max())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                row[name] = {"us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "rb": rb_v,
                             "workgroups": -(-rows // rb_v), "max_err": err}
                continue
            if lds and not lds_cap:
                continue
            begin = torch.arange(0, T + chunk, chunk, dtype=torch.int32).clamp_(max=T)
            begin = torch.unique_consecutive(begin).to(dev)
            nc = begin.numel() - 1
            if fused and rows * nc > 4096:
                continue
            group = torch.zeros(nc, dtype=torch.int32, device=dev)
            partial = torch.empty(nc * rows, dtype=torch.float64, device=dev)  # fp64 slab
            counter = torch.zeros(64, dtype=torch.int32, device=dev)
            out = torch.empty(rows, dtype=torch.float64, device=dev)

            def launch():
                if fused:
                    K.tree_perfect_fused(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0,
                                         begin.data_ptr(), nc, rb_v, partial.data_ptr(), counter.data_ptr(),
                                         group.data_ptr(), 1, 0, 1.0, 0, out.data_ptr(), 1, s, lds)
                else:
                    K.tree_perfect_partial(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0,
                                           begin.data_ptr(), nc, rb_v, partial.data_ptr(), s, lds)
                    K.tree_reduce(partial.data_ptr(), rows, nc, group.data_ptr(), 1, 0, 1.0, 0, out.data_ptr(), 1, s)

            for _ in range(20):
                launch()
            torch.cuda.synchronize()
            if out_ref is None:
                out_ref = out.clone()
            err = float((out - out_ref).abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                launch()
            e1.record()
            torch.cuda.synchronize()
            row[name] = {"us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "chunk": chunk, "chunks": nc,
                         "max_err": err}
        results.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
