"""Multi-armed-bandit routers (reference components/routers/epsilon-greedy/
EpsilonGreedy.py and components/routers/thompson-sampling/ThompsonSampling.py).

Same constructor parameters and ``route`` / ``send_feedback`` API as the
reference classes, but the decision and state live in the native
``BanditModel`` (csrc/gpu/router.cc): inside a deployment the router node is a
native unit whose decisions for concurrent requests are micro-batched into one
``eg_route`` / ``ts_route`` kernel launch (csrc/kernels/bandit.hip); used
directly from Python it runs the same model on the CPU.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Optional

import numpy as np

from . import register

logger = logging.getLogger(__name__)

EPSILON_GREEDY, THOMPSON = 0, 1


def _n_success_failures(features, reward: float):
    n = int(np.asarray(features).shape[0]) if np.asarray(features).ndim > 0 else 0
    s = int(reward * n)
    return s, n - s


class _BanditRouter:
    kind = EPSILON_GREEDY

    def __init__(self, n_branches=None, epsilon: float = 0.1, best_branch: Optional[int] = None,
                 verbose: bool = False, seed: Optional[int] = None, history: bool = False,
                 branch_names: Optional[str] = None, device: Optional[int] = None, max_batch: int = 4096,
                 route_on: str = "auto"):
        from .._native import native

        try:
            n_branches = int(n_branches)
            assert n_branches > 0
        except (TypeError, ValueError, AssertionError):
            logger.exception("n_branches parameter must be given")
            raise
        self.n_branches = n_branches
        self.epsilon = float(epsilon)
        self.history = bool(history)
        self.branch_history = [] if self.history else None
        self.branch_names = branch_names.split(":") if branch_names else None
        self.device = device
        self.max_batch = max_batch
        # "auto": on a GPU deployment an epsilon-greedy decision is made on the
        # caller's thread from the bandit kernel's Philox stream (identical
        # decisions, one GPU round trip less per routed request); "device":
        # every decision through the micro-batched bandit kernel
        # (SCA_ROUTER_ON_DEVICE=1 makes that the default)
        if route_on not in ("auto", "device"):
            raise ValueError("route_on must be 'auto' or 'device'")
        self.route_on = "device" if os.environ.get("SCA_ROUTER_ON_DEVICE") == "1" else route_on
        self._C = native()
        self.model = self._C.BanditModel(self.kind, n_branches, float(epsilon),
                                         -1 if seed is None else int(seed),
                                         -1 if best_branch is None else int(best_branch))
        self._unit = None

    # -- native binding (Deployment) ---------------------------------------
    def share_state(self, name: str, worker: int = 0) -> None:
        """One router state across the engine processes of a host (``serve
        --gpus N``): counters in the shared mapping ``name``, so feedback sent
        to any worker trains the bandit every worker routes with (the
        reference has one router object per deployment,
        EpsilonGreedy.py:87-130)."""
        self.model.attach_shared(name, int(worker))

    def native_unit(self, device: int):
        dev = device if self.device is None else int(self.device)
        self._unit = self._C.BanditRouterUnit(self.model, dev, self.max_batch,
                                              device_route=self.route_on == "device")
        return self._unit

    # -- reference component API --------------------------------------------
    def route(self, features, feature_names) -> int:
        b = int(self.model.run_cpu(np.zeros((1, 1)))[0, 0])
        if self.history:
            self.branch_history.append(b)
        return b

    def send_feedback(self, features, feature_names, routing, reward, truth):
        s, f = _n_success_failures(features, reward)
        self.model.feedback(int(routing), s, f)

    @property
    def best_branch(self) -> int:
        return self.model.best_branch

    @property
    def branch_values(self):
        return list(self.model.values())

    def state(self) -> dict:
        return json.loads(self.model.snapshot())


@register("EPSILON_GREEDY")
class EpsilonGreedy(_BanditRouter):
    kind = EPSILON_GREEDY


@register("THOMPSON_SAMPLING")
class ThompsonSampling(_BanditRouter):
    kind = THOMPSON

    def __init__(self, n_branches=None, verbose: bool = False, seed: Optional[int] = None, history: bool = False,
                 branch_names: Optional[str] = None, device: Optional[int] = None, max_batch: int = 4096,
                 route_on: str = "auto"):
        super().__init__(n_branches, 0.0, None, verbose, seed, history, branch_names, device, max_batch, route_on)
