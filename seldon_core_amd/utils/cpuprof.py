"""Native sampling CPU profile of the serving process (csrc/core/cpuprof.cc).

    from seldon_core_amd.utils import cpuprof
    cpuprof.start()              # SIGPROF sampling of this process's CPU time
    ...                          # serve traffic
    table = cpuprof.stop()       # [{"function", "module", "samples", "frac"}], top first

Samples are program counters; they are symbolised here with llvm-symbolizer
(ROCm's LLVM) from each module's symbol table, so the extension's
hidden-visibility functions resolve too.  Leaf functions only (no stacks):
the table says where CPU time is spent, grouped by function.
"""
from __future__ import annotations

import collections
import os
import shutil
import subprocess
from typing import Dict, List

from .._native import native

_SYMBOLIZER = next((p for p in ("/opt/rocm/lib/llvm/bin/llvm-symbolizer", shutil.which("llvm-symbolizer") or "")
                    if p and os.path.exists(p)), None)


def start(hz: int = 997, depth: int = 1) -> bool:
    """depth > 1 also records depth - 1 callers per sample (DWARF unwinder)."""
    return bool(native().cpu_profile_start(int(hz), int(depth)))


def _symbolize(module: str, offsets: List[int]) -> Dict[int, str]:
    if not _SYMBOLIZER or not module or not os.path.exists(module):
        return {}
    inp = "\n".join(hex(o) for o in offsets) + "\n"
    try:
        res = subprocess.run([_SYMBOLIZER, "--obj", module, "--functions=linkage", "--demangle", "--no-inlines",
                              "--output-style=LLVM"], input=inp, capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.TimeoutExpired):
        return {}
    # LLVM style: "<function>\n<file:line:col>\n\n" per address
    blocks = [b.split("\n") for b in res.stdout.strip("\n").split("\n\n")]
    return {o: (b[0] if b and b[0] and b[0] != "??" else f"{os.path.basename(module)}+{hex(o)}")
            for o, b in zip(offsets, blocks)}


def _short(fn: str) -> str:
    """Drop argument lists: 'ns::f(int, std::string)' -> 'ns::f'."""
    depth, out = 0, []
    for ch in fn:
        if ch == "(":
            depth += 1
        if depth == 0:
            out.append(ch)
        if ch == ")":
            depth -= 1
    return "".join(out).strip() or fn


def stop(top: int = 40) -> Dict:
    """Leaf-function table (``functions``), module shares, and with depth > 1
    the hottest call paths (``paths``: leaf <- caller <- ...)."""
    samples = native().cpu_profile_stop()
    pcs: Dict[str, set] = collections.defaultdict(set)
    for frames, _ in samples:
        for mod, off in frames:
            pcs[mod].add(off)
    names: Dict[tuple, str] = {}
    for mod, offs in pcs.items():
        offs = sorted(offs)
        sym = _symbolize(mod, offs)
        for o in offs:
            names[(mod, o)] = sym.get(o) or (f"{os.path.basename(mod)}+{hex(o)}" if mod else "[unknown]")
    total = sum(n for _, n in samples) or 1
    funcs: Dict[tuple, int] = collections.Counter()
    paths: Dict[tuple, int] = collections.Counter()
    for frames, n in samples:
        mod, off = frames[0]
        funcs[(names[(mod, off)], os.path.basename(mod) if mod else "?")] += n
        if len(frames) > 1:
            st = [_short(names[f])[:90] for f in frames if f[0] or f[1]]
            st = [x for i, x in enumerate(st) if i == 0 or x != st[i - 1]]  # the unwinder repeats the leaf
            paths[tuple(st)] += n
    rows = [{"function": fn[:160], "module": mod, "samples": n, "frac": round(n / total, 4)}
            for (fn, mod), n in funcs.most_common(top)]
    mods: Dict[str, int] = collections.Counter()
    for (fn, mod), n in funcs.items():
        mods[mod] += n
    out = {"total_samples": total, "functions": rows,
           "modules": [{"module": m, "frac": round(n / total, 4)} for m, n in mods.most_common(12)]}
    if paths:
        out["paths"] = [{"stack": list(p), "samples": n, "frac": round(n / total, 4)} for p, n in paths.most_common(top)]
    return out
