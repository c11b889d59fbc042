"""Source-to-image builder (reference wrappers/s2i/python/s2i/bin/
{assemble,run}): environment checks with the reference messages, the build
context, and the image's run command serving a user component."""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

from seldon_core_amd import builder

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MODEL = '''
class MyModel:
    def predict(self, X, names):
        return [[sum(r)] for r in X]
'''


def _src(tmp_path, env="MODEL_NAME=MyModel\nAPI_TYPE=REST\nSERVICE_TYPE=MODEL\nPERSISTENCE=0\n"):
    src = tmp_path / "src"
    (src / ".s2i").mkdir(parents=True)
    (src / "MyModel.py").write_text(MODEL)
    (src / "requirements.txt").write_text("")
    (src / ".s2i" / "environment").write_text("# s2i env\n" + env)
    return src


@pytest.mark.parametrize("env,msg", [
    ({}, "MODEL_NAME"),
    ({"MODEL_NAME": "M"}, "API_TYPE, should be either REST or GRPC"),
    ({"MODEL_NAME": "M", "API_TYPE": "REST"}, "SERVICE_TYPE, should be one of"),
    ({"MODEL_NAME": "M", "API_TYPE": "REST", "SERVICE_TYPE": "MODEL", "PERSISTENCE": "2"}, "PERSISTENCE"),
])
def test_environment_checks(env, msg):
    with pytest.raises(builder.BuildError, match=msg):
        builder.check_environment(env)


def test_build_context(tmp_path):
    src = _src(tmp_path)
    ctx = builder.build(str(src), "me/model:0.1", {"SERVICE_TYPE": "TRANSFORMER"}, base="base:1",
                        context=str(tmp_path / "ctx"), docker=False)
    df = open(os.path.join(ctx, "Dockerfile")).read()
    assert df.splitlines()[1] == "FROM base:1"
    assert 'ENV SERVICE_TYPE="TRANSFORMER"' in df and 'ENV MODEL_NAME="MyModel"' in df  # override wins
    assert 'CMD ["python", "-m", "seldon_core_amd.builder", "run"]' in df
    assert os.path.exists(os.path.join(ctx, "microservice", "MyModel.py"))
    assert builder.run_argv({"MODEL_NAME": "M", "API_TYPE": "GRPC", "SERVICE_TYPE": "ROUTER",
                             "PERSISTENCE": "1"}) == ["M", "GRPC", "--service-type", "ROUTER", "--persistence"]
    assert builder.main(["build", str(tmp_path / "nope"), "x", "--no-docker"]) == 1


def test_packaging_scripts_present():
    for f in ("assemble", "run", "usage"):
        p = os.path.join(ROOT, "packaging", "s2i", "bin", f)
        assert os.access(p, os.X_OK), p
    df = open(os.path.join(ROOT, "packaging", "engine", "Dockerfile")).read()
    assert "tools/build_native.py" in df and "PYTORCH_ROCM_ARCH=gfx950" in df


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_run_serves_the_component(tmp_path):
    src = _src(tmp_path)
    ctx = builder.build(str(src), "me/model:0.1", context=str(tmp_path / "ctx"), docker=False)
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT, GUNICORN_WORKERS="1", PREDICTIVE_UNIT_SERVICE_PORT=str(port),
               **builder.read_environment(str(src)))
    proc = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.builder", "run"],
                            cwd=os.path.join(ctx, "microservice"), env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        body = json.dumps({"data": {"ndarray": [[1.0, 2.0, 3.5]]}}).encode()
        deadline = time.time() + 60
        while True:
            try:
                req = urllib.request.Request(f"http://127.0.0.1:{port}/predict", data=body,
                                             headers={"Content-Type": "application/json"})
                out = json.loads(urllib.request.urlopen(req, timeout=5).read())
                break
            except OSError:
                if time.time() > deadline or proc.poll() is not None:
                    raise AssertionError(proc.stdout.read().decode() if proc.poll() is not None else "timeout")
                time.sleep(0.2)
        assert out["data"]["ndarray"] == [[6.5]]
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=20)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
