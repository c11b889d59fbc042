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


def start(hz: int = 997) -> bool:
    return bool(native().cpu_profile_start(int(hz)))


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


def stop(top: int = 40) -> List[Dict]:
    samples = native().cpu_profile_stop()
    by_mod: Dict[str, List] = collections.defaultdict(list)
    for mod, off, n in samples:
        by_mod[mod].append((off, n))
    total = sum(n for _, _, n in samples) or 1
    funcs: Dict[tuple, int] = collections.Counter()
    for mod, items in by_mod.items():
        names = _symbolize(mod, [o for o, _ in items])
        for off, n in items:
            fn = names.get(off) or (f"{os.path.basename(mod)}+{hex(off)}" if mod else "[unknown]")
            funcs[(fn, os.path.basename(mod) if mod else "?")] += n
    rows = [{"function": fn[:160], "module": mod, "samples": n, "frac": round(n / total, 4)}
            for (fn, mod), n in funcs.most_common(top)]
    mods = collections.Counter()
    for (fn, mod), n in funcs.items():
        mods[mod] += n
    return {"total_samples": total, "functions": rows,
            "modules": [{"module": m, "frac": round(n / total, 4)} for m, n in mods.most_common(12)]}
