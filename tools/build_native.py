#!/usr/bin/env python3
"""Build the native core in-tree: ``seldon_core_amd/_C*.so`` and the C++ load
generator ``seldon_core_amd/bin/sca_loadgen``.

* ``.hip`` files -> ``hipcc --offload-arch=gfx950`` (device code for CDNA4 only)
* ``.cc`` files  -> ``g++`` (host code; HIP runtime API headers only)
* incremental: objects are rebuilt when the source or any header it includes
  (``-MMD`` depfiles) is newer than the object.

Usage: ``python tools/build_native.py [-j N] [--clean] [--verbose]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
OBJ = BUILD / "obj"
PKG = ROOT / "seldon_core_amd"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("SCA_OFFLOAD_ARCH", "gfx950")
NGHTTP2_INC = Path("/opt/conda/include/nghttp2")
NGHTTP2_LIB = Path("/opt/conda/lib/libnghttp2.so.14")

LIB_SOURCES = [
    "core/json.cc", "core/message.cc", "core/pbwire.cc", "core/spec.cc", "core/metrics.cc",
    "core/engine.cc", "core/units.cc", "core/msglog.cc", "core/roctx.cc", "core/cpuprof.cc",
    "server/http_server.cc", "server/grpc_server.cc", "server/remote_unit.cc",
    "gpu/models.cc", "gpu/batcher.cc", "gpu/driver.cc", "gpu/router.cc", "gpu/graph.cc", "gpu/replica.cc", "gpu/mlp_model.cc", "gpu/lstm_model.cc", "gpu/maha_device.cc", "parallel/fabric.cc", "parallel/mesh.cc",
    "kernels/linear.hip", "kernels/linear_graph.hip", "kernels/tree.hip", "kernels/combine.hip", "kernels/bandit.hip", "kernels/image.hip", "kernels/mlp.hip", "kernels/mahalanobis.hip", "kernels/lstm.hip", "kernels/lstm_valu.hip", "kernels/gemm.hip",
    "bindings/module.cc",
]
LOADGEN_SOURCES = ["tools/loadgen.cc", "core/json.cc"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_include() -> str:
    import pybind11  # noqa: WPS433

    return pybind11.get_include()


def _private_include() -> Path:
    """Expose only nghttp2's headers (not all of /opt/conda/include)."""
    inc = BUILD / "include"
    inc.mkdir(parents=True, exist_ok=True)
    link = inc / "nghttp2"
    if not link.exists() and NGHTTP2_INC.exists():
        try:  # the compile pool's threads race here on a fresh tree
            link.symlink_to(NGHTTP2_INC)
        except FileExistsError:
            pass
    return inc


def _common_flags() -> list[str]:
    return [
        "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
        f"-I{CSRC}", f"-I{_private_include()}", f"-I{ROCM / 'include'}",
        "-D__HIP_PLATFORM_AMD__",
    ]


def _needs_build(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    mtime = obj.stat().st_mtime
    if src.stat().st_mtime > mtime:
        return True
    dep = obj.with_suffix(".d")
    if not dep.exists():
        return True
    text = dep.read_text().replace("\\\n", " ")
    for tok in text.split(":", 1)[-1].split():
        p = Path(tok)
        if p.exists() and p.stat().st_mtime > mtime:
            return True
    return False


def _compile(src_rel: str, verbose: bool) -> Path:
    src = CSRC / src_rel
    obj = OBJ / (src_rel.replace("/", "__") + ".o")
    if not _needs_build(src, obj):
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    flags = _common_flags() + ["-MMD", "-MF", str(obj.with_suffix(".d"))]
    if src.suffix == ".hip":
        cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-x", "hip", *flags,
               "-munsafe-fp-atomics", "-c", str(src), "-o", str(obj)]
    else:
        py_inc = sysconfig.get_paths()["include"]
        cmd = ["g++", *flags, "-fvisibility=hidden", f"-I{_pybind_include()}", f"-I{py_inc}",
               "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src_rel}\n{res.stdout}\n{res.stderr}")
    if res.stderr.strip() and verbose:
        print(res.stderr, file=sys.stderr)
    return obj


def _vendor_nghttp2() -> Path:
    libdir = PKG / "lib"
    libdir.mkdir(exist_ok=True)
    dst = libdir / NGHTTP2_LIB.name
    if NGHTTP2_LIB.exists() and (not dst.exists() or dst.stat().st_mtime < NGHTTP2_LIB.stat().st_mtime):
        shutil.copy2(NGHTTP2_LIB, dst)
    return dst


def build(jobs: int = 8, verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), LIB_SOURCES))
        lg_objs = list(ex.map(lambda s: _compile(s, verbose), LOADGEN_SOURCES))
    ng = _vendor_nghttp2()
    out = PKG / ("_C" + _ext_suffix())
    newest = max(o.stat().st_mtime for o in objs)
    if not out.exists() or out.stat().st_mtime < newest:
        cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
               "-o", str(out), f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", str(ng),
               "-Wl,-rpath,$ORIGIN/lib", f"-Wl,-rpath,{ROCM / 'lib'}", "-lpthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed\n{res.stdout}\n{res.stderr}")
    bindir = PKG / "bin"
    bindir.mkdir(exist_ok=True)
    lg = bindir / "sca_loadgen"
    if not lg.exists() or lg.stat().st_mtime < max(o.stat().st_mtime for o in lg_objs):
        cmd = ["g++", "-O3", *map(str, lg_objs), "-o", str(lg), str(ng), "-Wl,-rpath,$ORIGIN/../lib", "-lpthread"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"loadgen link failed\n{res.stdout}\n{res.stderr}")
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    if a.clean and BUILD.exists():
        shutil.rmtree(BUILD)
    out = build(a.jobs, a.verbose)
    print(f"built {out.relative_to(ROOT)}")


if __name__ == "__main__":
    main()
