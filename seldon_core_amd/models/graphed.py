"""Any PyTorch module served through captured HIP graphs.

A small served module (an MLflow ``pytorch`` flavour MLP, a TorchScript
classifier) spends most of a request in kernel launches: one per layer, op and
activation, a few microseconds of host time each.  :class:`GraphedModule`
captures the module once per (batch bucket, row shape) -- buckets 1, 2, 4, ...
``max_batch`` -- and serves a call as: copy the rows into the bucket's static
input, one graph replay, copy the rows back.  A batch is padded up to its
bucket; a larger one runs in ``max_batch`` pieces.  Capture is lazy (first
call of a shape) and every step runs on the module's own stream, never the
null stream (see :class:`~seldon_core_amd.models.cnn.CompiledCnn`).

The module must be row-wise (row i of the output depends only on row i of the
input) -- the contract batched serving already assumes -- and
capture-safe (no host synchronisation or data-dependent control flow inside
``forward``).  A module whose capture fails is served eagerly from then on,
with the reason kept in ``graph_error``.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


class GraphedModule:
    def __init__(self, module: "torch.nn.Module", device: int = 0, max_batch: int = 256,
                 in_dtype: "torch.dtype" = None, graphs: bool = True, max_graphs: int = 64):
        self.device = torch.device(f"cuda:{device}")
        self.module = module.eval().to(self.device)
        self.in_dtype = in_dtype or torch.float32
        self.max_batch = int(max_batch)
        self.use_graphs = graphs
        self.max_graphs = max_graphs
        self.stream = torch.cuda.Stream(self.device)
        self.graphs: Dict[Tuple, tuple] = {}
        self.graph_error: Optional[str] = None
        self.replays = 0
        self.eager_calls = 0

    def _bucket(self, n: int) -> int:
        b = 1
        while b < n:
            b *= 2
        return min(b, self.max_batch)

    def _capture(self, key: Tuple) -> Optional[tuple]:
        bs, row_shape = key[0], key[1:]
        x = torch.zeros((bs,) + row_shape, device=self.device, dtype=self.in_dtype)
        with torch.no_grad(), torch.cuda.stream(self.stream):
            for _ in range(2):  # library algorithm choice / workspaces before capture
                self.module(x)
        self.stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g, stream=self.stream):
            y = self.module(x)
        return g, x, y

    def _graph_for(self, key: Tuple) -> Optional[tuple]:
        if not self.use_graphs or self.graph_error is not None:
            return None
        got = self.graphs.get(key)
        if got is None and len(self.graphs) < self.max_graphs:
            try:
                got = self.graphs[key] = self._capture(key)
            except Exception as e:  # noqa: BLE001 -- not capture-safe: serve eagerly
                self.graph_error = f"{type(e).__name__}: {e}"
                self.graphs.clear()
                return None
        return got

    def run(self, x: "torch.Tensor") -> "torch.Tensor":
        """Device rows in (on this module's stream), device rows out."""
        outs = []
        with torch.no_grad():
            for i in range(0, x.shape[0], self.max_batch):
                part = x[i:i + self.max_batch]
                k = part.shape[0]
                entry = self._graph_for((self._bucket(k),) + tuple(part.shape[1:]))
                if entry is None:
                    self.eager_calls += 1
                    outs.append(self.module(part))
                    continue
                g, xs, ys = entry
                xs[:k].copy_(part)
                if k < xs.shape[0]:
                    xs[k:].zero_()
                g.replay()
                self.replays += 1
                outs.append(ys[:k].clone())
        return outs[0] if len(outs) == 1 else torch.cat(outs, 0)

    def __call__(self, X) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(X)) if isinstance(X, np.ndarray) else X
        with torch.cuda.stream(self.stream):
            td = t.to(self.device, dtype=self.in_dtype, non_blocking=False)
            y = self.run(td).float().cpu()
        return y.numpy()
