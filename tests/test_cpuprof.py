"""Native sampling CPU profiler (csrc/core/cpuprof.cc, utils/cpuprof.py)."""
import hashlib
import time

from seldon_core_amd.utils import cpuprof


def _burn(seconds: float) -> int:
    n, t0 = 0, time.perf_counter()
    h = hashlib.sha256()
    while time.perf_counter() - t0 < seconds:
        h.update(b"x" * 4096)
        n += 1
    return n


def test_profile_attributes_cpu_to_functions():
    assert cpuprof.start(997)
    assert not cpuprof.start(997)  # one session at a time
    _burn(0.6)
    prof = cpuprof.stop()
    assert prof["total_samples"] >= 40  # >= ~100 Hz per busy thread (kernel tick bound)
    fr = sum(r["frac"] for r in prof["functions"])
    assert 0.5 < fr <= 1.0001
    mods = {m["module"] for m in prof["modules"]}
    assert any("crypto" in m or "python" in m or "libc" in m for m in mods), mods
    assert cpuprof.stop()["total_samples"] <= 1  # stopped: nothing collected
