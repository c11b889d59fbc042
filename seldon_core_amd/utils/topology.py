"""GPU-local CPU placement for serving processes.

An MI355X node is two sockets of chiplet CPUs: each L3 is shared by one CCD
(8 cores + their SMT siblings on an EPYC 9575F), and the GPUs hang off the
sockets' PCIe roots (`/sys/bus/pci/devices/<bdf>/local_cpulist`).  A serving
process hands every request across threads -- front-end worker -> GPU device
thread -> hand-off thread -> worker -- so where those threads run matters as
much as how many there are: on one MI355X box the same 16-CPU share served
REST at ~770k req/s with its threads floating over the host, ~1.0M pinned to
16 CPUs of the GPU's socket, and 1.22M pinned to one CCD's 8 cores + SMT
siblings (`profiles/r02m_pinning`).

:func:`gpu_cpu_set` picks, for a GPU, whole L3 groups (CCDs) on that GPU's
NUMA node, offset by the GPU's ordinal among the node's GPUs so that processes
driving different GPUs of one host land on disjoint CCDs; :func:`pin` applies
it to the calling process (threads created afterwards inherit it, and so do
child processes such as the load generator).  Everything degrades to "no
pinning" when the topology cannot be read.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional


def _parse_cpulist(text: str) -> List[int]:
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def amd_gpus() -> List[Dict]:
    """AMD GPUs of the host (vendor 0x1002, display / processing-accelerator
    class), sorted by PCI address: [{"bdf", "numa", "cpus"}]."""
    gpus = []
    for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
        if _read(os.path.join(d, "vendor")) != "0x1002":
            continue
        cls = _read(os.path.join(d, "class")) or ""
        if not (cls.startswith("0x1200") or cls.startswith("0x0380") or cls.startswith("0x0300")):
            continue
        cpus = _read(os.path.join(d, "local_cpulist"))
        numa = _read(os.path.join(d, "numa_node"))
        if cpus is None:
            continue
        gpus.append({"bdf": os.path.basename(d), "numa": int(numa) if numa not in (None, "") else -1,
                     "cpus": _parse_cpulist(cpus)})
    return gpus


def l3_groups() -> List[List[int]]:
    """CPU sets that share an L3 cache (one per CCD), sorted by first CPU."""
    seen = set()
    groups = []
    for c in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/cache/index3/shared_cpu_list"):
        text = _read(c)
        if not text or text in seen:
            continue
        seen.add(text)
        groups.append(_parse_cpulist(text))
    return sorted(groups, key=lambda g: g[0])


def device_bdf(device: int) -> Optional[str]:
    """PCI address of torch / HIP device `device` (None if unknown)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        return "%04x:%02x:%02x.0" % (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    except Exception:  # noqa: BLE001 -- no GPU / old torch: no placement
        return None


def gpu_cpu_set(bdf: str, ncpus: int, allowed: Optional[List[int]] = None, gpus: Optional[List[Dict]] = None,
                groups: Optional[List[List[int]]] = None) -> List[int]:
    """Whole L3 groups on `bdf`'s NUMA node covering at least `ncpus` logical
    CPUs, starting at the group that matches the GPU's ordinal among the node's
    GPUs; [] if the topology is unavailable.  (`gpus` / `groups` default to
    the host's sysfs view.)"""
    gpus = amd_gpus() if gpus is None else gpus
    me = next((g for g in gpus if g["bdf"] == bdf), None)
    if me is None or ncpus <= 0:
        return []
    allowed_set = set(allowed if allowed is not None else os.sched_getaffinity(0))
    local = set(me["cpus"]) & allowed_set
    groups = [g for g in (l3_groups() if groups is None else groups) if set(g) <= local]
    if not groups:
        return []
    peers = [g["bdf"] for g in gpus if g["numa"] == me["numa"]]
    ordinal = peers.index(bdf) if bdf in peers else 0
    per_gpu = max(1, len(groups) // max(1, len(peers)))
    start = (ordinal * per_gpu) % len(groups)
    chosen: List[int] = []
    i = 0
    while len(chosen) < ncpus and i < len(groups):
        chosen.extend(groups[(start + i) % len(groups)])
        i += 1
    return sorted(chosen)


def pin(device: int, ncpus: int) -> List[int]:
    """Pin the calling process to `device`'s CPU set (see gpu_cpu_set);
    returns the CPUs, or [] when it left the affinity unchanged."""
    bdf = device_bdf(device)
    if bdf is None:
        return []
    cpus = gpu_cpu_set(bdf, ncpus)
    if not cpus:
        return []
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return []
    return cpus
