"""Cross-process graph placement (one engine process per MI355X).

Spec extension: a graph node may carry ``rank: r`` -- the torch.distributed
rank (= GPU) whose process hosts that node.  Rank 0 runs the front end
(REST/gRPC), the graph executor, routers and the micro-batchers; worker ranks
serve the nodes placed on them.

Transports (``SCA_FABRIC_TRANSPORT`` or ``init_fabric(transport=...)``):

* ``ipc`` (GPU default) / ``shm`` (CPU gangs): the mesh (csrc/parallel/mesh.h,
  ``parallel/mesh.py``).  Placed subtrees become programs with direct
  stage-to-stage edges: HIP IPC device slabs between workers (peer copies over
  xGMI across GPUs, plain copies when ranks share one GPU), shared-memory slabs
  and doorbells to and from rank 0.  Any MODEL / TRANSFORMER /
  OUTPUT_TRANSFORMER node -- a native row model or a Python component -- can
  sit on a worker.
* ``rccl`` / ``rccl1``: the star fabric (csrc/parallel/fabric.h): one
  ``PeerRowModel`` per placed row-model node, RCCL point-to-point per batch
  (two communicators and streams per link, or one of each with ``rccl1``).

Typical launch (one process per GPU)::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 my_server.py

    fabric = init_fabric()                      # control links + the data plane
    if fabric.rank == 0:
        dep = Deployment(spec, fabric=fabric)   # placed subtrees become remote units
        dep.serve(...)
    else:
        serve_peer(spec, fabric).join()         # until rank 0 calls dep.close()

Reference behaviour replaced: each graph hop is an HTTP/gRPC call to another
pod (InternalPredictionService.java:186-453) carrying JSON.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional

from .._native import gpu_count, native
from ..serving.spec import SpecError, iter_nodes, load_spec, select_predictor


def _control_links(rank: int, world: int, host: str = "127.0.0.1") -> List[int]:
    """Star of host sockets rank 0 <-> every worker (the fabric's control
    plane: batch headers).  Workers listen on an ephemeral port and publish it
    over the default process group; rank 0 connects.  fds[r] = socket to rank r
    (-1 where there is no link)."""
    import socket

    import torch.distributed as dist

    lst = None
    port = 0
    if rank != 0:
        lst = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        lst.bind((host, 0))
        lst.listen(1)
        port = lst.getsockname()[1]
    ports = [None] * world
    dist.all_gather_object(ports, port)
    fds = [-1] * world
    if rank == 0:
        for r in range(1, world):
            c = socket.create_connection((host, int(ports[r])))
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            fds[r] = c.detach()
    else:
        c, _ = lst.accept()
        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        fds[0] = c.detach()
        lst.close()
    return fds


TRANSPORTS = ("ipc", "shm", "rccl", "rccl1")


def fabric_transport(device: int, transport: Optional[str] = None) -> str:
    t = (transport or os.environ.get("SCA_FABRIC_TRANSPORT") or "").strip().lower()
    if not t:
        t = "ipc" if device >= 0 else "shm"
    if t not in TRANSPORTS:
        raise ValueError(f"unknown fabric transport {t!r} (one of {', '.join(TRANSPORTS)})")
    if device < 0 and t != "shm":
        raise ValueError(f"a CPU gang (device -1) uses the shm transport, not {t!r}")
    if device >= 0 and t == "shm":
        t = "ipc"  # GPU ranks: the same mesh, with device slabs
    return t


def gang_device(rank: int, world: int, requested: Optional[int] = None) -> int:
    """One placement for the whole gang: every rank on its own GPU when there
    are enough, all on ``requested`` when given (several ranks may share one
    GPU over the ipc transport), otherwise every rank on the CPU -- never a
    mix of GPU and CPU ranks."""
    if requested is not None:
        return int(requested)
    n = gpu_count()
    if n >= world:
        return int(os.environ.get("LOCAL_RANK", rank))
    return -1


def is_mesh(fabric) -> bool:
    return fabric is not None and isinstance(fabric, native().Mesh)


def init_fabric(device: Optional[int] = None, transport: Optional[str] = None, slots: Optional[int] = None):
    """Create the fabric for the current torch.distributed job: control
    sockets between rank 0 and every worker (liveness, ring names), then the
    data plane of the chosen transport (see the module doc).  ``device``
    defaults to ``gang_device``."""
    import torch.distributed as dist

    C = native()
    rank, world = dist.get_rank(), dist.get_world_size()
    if device is None:
        device = gang_device(rank, world)
    t = fabric_transport(int(device), transport)
    fds = _control_links(rank, world)
    if t in ("ipc", "shm"):
        k = int(slots or os.environ.get("SCA_FABRIC_SLOTS", "4") or 4)
        return C.Mesh(rank, world, int(device), fds, k)
    per_link = 1 if t == "rccl1" else 2
    box = [C.rccl_unique_ids(world, per_link) if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return C.Fabric(rank, world, box[0], int(device), fds, None, per_link)


def loopback_fabrics(world: int, device: int = 0) -> List[Any]:
    """Every rank of a ``world``-rank fabric in THIS process on ONE GPU (the
    loopback transport, csrc/parallel/fabric.h): the front end's and the
    workers' GPU code paths -- per-link streams, the worker's slot pipeline,
    the fan-out gather + combine -- run on a 1-GPU box.  The control plane is
    the real one (shared-memory header rings, socket pairs).  Returns the
    fabrics by rank; worker fabrics go to ``serve_peer`` like any other."""
    import socket
    import threading

    if world < 2:
        raise ValueError("loopback fabric needs world >= 2")
    C = native()
    hub = C.LoopbackHub(int(device))
    fds = [[-1] * world for _ in range(world)]
    for r in range(1, world):
        a, b = socket.socketpair()
        fds[0][r], fds[r][0] = a.detach(), b.detach()
    out: List[Any] = [None] * world
    errs: List[BaseException] = []

    def make(r: int) -> None:
        try:
            out[r] = C.Fabric(r, world, b"", int(device), fds[r], hub)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)

    # rank 0 hands each worker its header ring over the socket pair: the
    # constructors rendezvous, so they run concurrently (they drop the GIL)
    th = [threading.Thread(target=make, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return out


def node_rank(node: Dict) -> Optional[int]:
    r = node.get("rank")
    return None if r is None else int(r)


def rank_assignments(graph: Dict) -> Dict[int, List[str]]:
    """rank -> node names hosted there, in graph order (= PeerServer model ids)."""
    out: Dict[int, List[str]] = {}
    for n, _ in iter_nodes(graph):
        r = node_rank(n)
        if r is not None:
            out.setdefault(r, []).append(n["name"])
    return out


def peer_model_for(C, fabric, node: Dict, local_rm, model_id: int):
    """Front-end stand-in for a node hosted on another rank."""
    in_cols = int(local_rm.in_cols)
    if in_cols <= 0:
        raise SpecError([f"node '{node['name']}' on rank {node_rank(node)} needs a model with a fixed input width"])
    return C.peer_row_model(fabric, [node_rank(node)], model_id, in_cols, int(local_rm.out_cols(in_cols)),
                            list(local_rm.class_names()), bool(local_rm.flat_output))


class MeshServer:
    """A worker's side of the mesh: its program threads (serve_peer)."""

    def __init__(self, mesh, setup):
        self.mesh = mesh
        self.setup = setup

    def join(self) -> None:
        self.mesh.join()

    def error(self) -> str:
        return self.mesh.error()

    def stats(self) -> Dict[str, int]:
        return dict(self.mesh.stats())

    @property
    def batches(self) -> int:
        return int(self.mesh.stats()["batches"])

    @property
    def rows(self) -> int:
        return int(self.mesh.stats()["rows"])

    @property
    def max_inflight(self) -> int:
        return int(self.mesh.stats()["max_inflight"])

    @property
    def host_syncs(self) -> int:
        return 0  # the mesh never waits on a device from the host

    @property
    def slots(self) -> int:
        return int(self.mesh.slots)


def serve_peer(spec: Any, fabric, components: Optional[Dict[str, Any]] = None, predictor: Optional[str] = None):
    """Worker rank: build the nodes placed on this rank and serve them until
    rank 0 stops the fabric.  Returns the started server (``join()``,
    ``error()``, ``batches``, ``rows``, ``max_inflight``)."""
    from ..serving.deployment import Deployment

    sdep = load_spec(spec)
    pred = select_predictor(sdep, predictor)
    res = Deployment.resolver(sdep, components, pred)
    if is_mesh(fabric):
        from . import mesh as meshmod

        st = meshmod.setup(fabric, pred["graph"], lambda node: meshmod.stage_info(res, node),
                           bound=set(components or {}))
        return MeshServer(fabric, st)
    C = native()
    server = C.PeerServer(fabric)
    for name in rank_assignments(pred["graph"]).get(fabric.rank, []):
        node = next(n for n, _ in iter_nodes(pred["graph"]) if n["name"] == name)
        kind, obj = res._resolve(node)
        rm = res._row_model_of(res._instantiate(node, obj)) if kind == "object" else None
        if rm is None:
            raise SpecError([f"node '{name}' placed on rank {fabric.rank} is not a GPU row model"])
        server.add_model(rm)
    server.start()
    return server
