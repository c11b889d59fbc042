"""Sanitizer runs of the native host core: ASan+UBSan and TSan
builds of the codecs, graph executor, HTTP/gRPC front ends and the micro-batcher host machinery
(tools/build_sanitizers.py, csrc/tests/core_stress.cc).  Device kernels are
not sanitizer-built: GPU ASan is unavailable on the MI355X pool."""
import json
import os
import subprocess
import sys
import urllib.error
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import build_sanitizers  # noqa: E402

LOADGEN = os.path.join(ROOT, "seldon_core_amd", "bin", "sca_loadgen")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=0")


@pytest.fixture(scope="module", params=["asan", "tsan"])
def stress_exe(request):
    return str(build_sanitizers.build(request.param, jobs=min(8, os.cpu_count() or 4))), request.param


def _clean(stderr: str) -> bool:
    return ("ERROR: AddressSanitizer" not in stderr and "runtime error:" not in stderr
            and "WARNING: ThreadSanitizer" not in stderr and "ERROR: LeakSanitizer" not in stderr)


@pytest.mark.parametrize("mode,n", [("fuzz", "2000"), ("engine", "3000"), ("batcher", "2000"), ("mesh", "600")])
def test_core_stress(stress_exe, mode, n):
    exe, kind = stress_exe
    r = subprocess.run([exe, mode, n], capture_output=True, text=True, timeout=600, env=SAN_ENV)
    assert r.returncode == 0 and _clean(r.stderr), f"[{kind}] {mode}\n{r.stderr[-6000:]}"
    assert f"ok {mode}" in r.stdout


def _loadgen(port, mode, body_args):
    cmd = [LOADGEN, "--host", "127.0.0.1", "--port", str(port), "--users", "16", "--threads", "2", "--steps", "1",
           "--warmup", "0", "--step-requests", "1500", "--mode", mode, *body_args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_front_ends_under_sanitizer(stress_exe, tmp_path):
    import seldon_core_amd as sca

    exe, kind = stress_exe
    p = subprocess.Popen([exe, "serve"], stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=SAN_ENV)
    try:
        _, hp, gp = p.stdout.readline().split()
        rest = _loadgen(hp, "rest", ["--path", "/api/v0.1/predictions", "--body",
                                     json.dumps({"data": {"names": ["a", "b"], "ndarray": [[1.0, 2.0]]}})])
        assert rest["ok"] == 1500 and rest["errors"] == 0
        codes = []
        for path in ("/ping", "/pause", "/ready", "/unpause", "/ready", "/prometheus"):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{hp}{path}", timeout=30) as f:
                    codes.append(f.status)
            except urllib.error.HTTPError as e:
                codes.append(e.code)
        assert codes == [200, 200, 503, 200, 200, 200]
        pb = tmp_path / "req.pb"
        pb.write_bytes(sca.native().json_to_pb(json.dumps({"data": {"tensor": {"shape": [3, 2],
                                                                               "values": [1, 2, 3, 4, 5, 6]}}})))
        grpc = _loadgen(gp, "grpc", ["--path", "/seldon.protos.Seldon/Predict", "--body-file", str(pb),
                                     "--streams-per-conn", "8"])
        assert grpc["ok"] == 1500 and grpc["errors"] == 0
        out, err = p.communicate("", timeout=120)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == 0 and _clean(err), f"[{kind}] serve\n{err[-6000:]}"
    assert "ok serve" in out
