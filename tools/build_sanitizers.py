#!/usr/bin/env python3
"""Sanitizer builds of the native host core.

Builds ``build/san/<kind>/core_stress`` from the host sources of the engine --
codecs, graph executor, built-in units, metrics, message logger, HTTP/1.1 and
gRPC front ends -- plus ``csrc/tests/core_stress.cc``, with

* ``asan``: ``-fsanitize=address,undefined`` (heap/stack misuse, leaks, UB)
* ``tsan``: ``-fsanitize=thread`` (data races in continuations, executors,
  front-end workers, metrics registry, traffic split, the micro-batcher's
  submission shards / device thread / hand-off thread / response parcels on
  its CPU path)

GPU code is not part of these builds: GPU AddressSanitizer / XNACK runs are
not available on the MI355X pool, so device kernels are checked by numerics
tests against fp32/fp64 references instead.

Usage: ``python tools/build_sanitizers.py [asan|tsan ...] [--run]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "san"
SOURCES = [
    "core/json.cc", "core/message.cc", "core/pbwire.cc", "core/spec.cc", "core/metrics.cc",
    "core/engine.cc", "core/units.cc", "core/msglog.cc", "core/roctx.cc",
    "server/http_server.cc", "server/grpc_server.cc", "server/remote_unit.cc",
    "gpu/batcher.cc",  # host machinery only: the stress driver runs it on its CPU path
    "gpu/driver.cc",
    "parallel/mesh.cc",  # CPU gangs (shared memory); the GPU path is not exercised here
    "tests/core_stress.cc",
]
FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


def _nghttp2():
    sys.path.insert(0, str(ROOT / "tools"))
    import build_native  # noqa: WPS433

    return build_native._private_include(), build_native._vendor_nghttp2()


def _compile(kind: str, src_rel: str, inc: Path) -> Path:
    src = CSRC / src_rel
    obj = BUILD / kind / "obj" / (src_rel.replace("/", "__") + ".o")
    obj.parent.mkdir(parents=True, exist_ok=True)
    dep = obj.with_suffix(".d")
    fresh = obj.exists() and dep.exists() and all(
        Path(t).stat().st_mtime <= obj.stat().st_mtime
        for t in dep.read_text().replace("\\\n", " ").split(":", 1)[-1].split() if Path(t).exists())
    if fresh:
        return obj
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Wall", "-Wno-unused-function",
           *FLAGS[kind], f"-I{CSRC}", f"-I{inc}", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-MMD", "-MF", str(dep), "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"[{kind}] compile failed: {src_rel}\n{res.stderr}")
    return obj


def build(kind: str, jobs: int = 8) -> Path:
    """Compile + link under an exclusive file lock (pytest-xdist workers build
    the same tree concurrently); the executable is linked to a temporary name
    and renamed into place so a running copy is never overwritten."""
    import fcntl

    (BUILD / kind).mkdir(parents=True, exist_ok=True)
    with open(BUILD / kind / ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        inc, ng = _nghttp2()
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            objs = list(ex.map(lambda s: _compile(kind, s, inc), SOURCES))
        out = BUILD / kind / "core_stress"
        if not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
            tmp = out.with_name(f"core_stress.{os.getpid()}.tmp")
            cmd = ["g++", *FLAGS[kind], *map(str, objs), str(ng), f"-Wl,-rpath,{ng.parent}",
                   "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-lamdhip64", "-lpthread",
                   "-o", str(tmp)]
            res = subprocess.run(cmd, capture_output=True, text=True)
            if res.returncode != 0:
                raise RuntimeError(f"[{kind}] link failed\n{res.stderr}")
            os.replace(tmp, out)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kinds", nargs="*", default=["asan", "tsan"], choices=["asan", "tsan"])
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--run", action="store_true", help="run the fuzz and engine stress modes")
    args = ap.parse_args()
    rc = 0
    for kind in args.kinds:
        exe = build(kind, args.j)
        print(f"built {exe.relative_to(ROOT)}")
        if args.run:
            for mode, n in (("fuzz", "3000"), ("engine", "4000")):
                r = subprocess.run([str(exe), mode, n], capture_output=True, text=True)
                print(f"  {mode}: rc={r.returncode} {r.stdout.strip()[-200:]}")
                if r.returncode:
                    print(r.stderr[-4000:], file=sys.stderr)
                    rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(main())
