"""`serve --gpus N` as a multi-process deployment.

* Shared router state: an epsilon-greedy MAB over N replica workers learns
  from feedback that SO_REUSEPORT hands to ANY worker, as fast as one process
  (the reference keeps one router object per deployment,
  components/routers/epsilon-greedy/EpsilonGreedy.py:87-130).
* Rank placement from the spec: a graph with ``rank:`` nodes runs as ONE
  graph over the N processes (rank 0 front end, rank 1.. serve_peer), the
  operator-built multi-component deployment
  (operator/controllers/seldondeployment_controller.go:253-392).

The CPU tests use device -1 (the mesh over shared memory); the gang test
marked gpu runs every rank on GPU 0 (the mesh over HIP IPC)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    from portutil import free_port

    return free_port()


def _post(port, path, body, timeout=10):
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json", "Connection": "close"})
    return json.loads(urllib.request.urlopen(req, timeout=timeout).read())


def _start(tmp_path, spec, n, extra=(), env_extra=None, device=-1):
    sp = tmp_path / "spec.json"
    sp.write_text(json.dumps(spec))
    hp, gp = _free_port(), _free_port()
    log = open(tmp_path / "serve.log", "w")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, str(tmp_path)]), **(env_extra or {}))
    if device < 0:
        env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--spec", str(sp), "--gpus", str(n),
                          "--device", str(device), "--http-port", str(hp), "--grpc-port", str(gp), "--admin-port", "0",
                          "--threads", "2", "--log-level", "INFO", *extra],
                         env=env, cwd=ROOT, start_new_session=True, stdout=log, stderr=subprocess.STDOUT)
    return p, hp, tmp_path / "serve.log"


def _wait_log(path, needle, count, timeout=120):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if path.read_text().count(needle) >= count:
            return True
        time.sleep(0.2)
    return False


def _stop(p):
    try:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
            return p.wait(timeout=90)
        return p.returncode
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


def test_mab_feedback_to_any_worker_trains_every_worker(tmp_path):
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "mab", "type": "ROUTER", "implementation": "EPSILON_GREEDY",
                      "parameters": [{"name": "n_branches", "value": "2", "type": "INT"},
                                     {"name": "epsilon", "value": "0.1", "type": "FLOAT"},
                                     {"name": "best_branch", "value": "0", "type": "INT"}],
                      "children": [{"name": "b0", "type": "MODEL", "implementation": "SIMPLE_MODEL"},
                                   {"name": "b1", "type": "MODEL", "implementation": "SIMPLE_MODEL"}]}}
    p, hp, log = _start(tmp_path, spec, 4)
    try:
        assert _wait_log(log, "serving p:", 4), log.read_text()[-3000:]
        req = {"data": {"ndarray": [[1.0, 2.0]]}}

        def share_of_branch1(k):
            return np.mean([_post(hp, "/api/v0.1/predictions", req)["meta"]["routing"]["mab"] == 1 for _ in range(k)])

        assert share_of_branch1(80) < 0.3  # every worker starts on branch 0
        # ONE feedback, on one connection: whichever worker takes it
        _post(hp, "/api/v0.1/feedback", {"request": req, "response": {"meta": {"routing": {"mab": 1}},
                                                                        "data": {"ndarray": [[0.0]]}},
                                          "reward": 1.0})
        # ... and every worker now routes to branch 1 (90% = 1 - epsilon)
        share = share_of_branch1(200)
        assert share > 0.8, share
        assert _stop(p) == 0
    finally:
        _stop(p)
    assert not [n for n in os.listdir("/dev/shm") if n.startswith(f"sca_state_{p.pid}_")]


def test_rank_placed_spec_serves_through_the_cli(tmp_path):
    (tmp_path / "mymodels.py").write_text(
        "from seldon_core_amd.models import iris_logistic_regression\n"
        "from seldon_core_amd.servers import SKLearnServer\n\n\n"
        "class Iris(SKLearnServer):\n"
        "    def __init__(self):\n"
        "        super().__init__(model=iris_logistic_regression())\n")
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
                      "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
                      "children": [{"name": "a", "type": "MODEL", "rank": 1},
                                   {"name": "b", "type": "MODEL", "rank": 2}]}}
    p, hp, log = _start(tmp_path, spec, 3, extra=("--component", "a=mymodels.Iris", "--component", "b=mymodels.Iris"))
    try:
        assert _wait_log(log, "serving p:", 1), log.read_text()[-3000:]
        text = log.read_text()
        assert "mesh_program" in text, text[-2000:]  # rank 0 reaches a and b through the mesh
        from seldon_core_amd.models import iris_logistic_regression

        lr = iris_logistic_regression()
        rng = np.random.default_rng(0)
        seen = set()
        for i in range(40):
            X = rng.normal(loc=4.0, scale=1.5, size=(1 + i % 4, 4))
            out = _post(hp, "/api/v0.1/predictions", {"data": {"ndarray": X.tolist()}})
            np.testing.assert_allclose(np.asarray(out["data"]["ndarray"]), lr.predict_proba(X), rtol=0, atol=1e-12)
            seen.add(out["meta"]["routing"]["ab"])
        assert seen == {0, 1}
        assert _stop(p) == 0
    finally:
        _stop(p)
    text = log.read_text()
    assert text.count("done:") == 2, text[-3000:]  # both peer ranks left their loops on rank 0's stop


def test_python_transformer_and_model_on_worker_ranks_through_the_cli(tmp_path):
    """Any node on any rank: a Python TRANSFORMER on rank
    1 feeds the iris MODEL on rank 2; rank 0 only runs the front end."""
    (tmp_path / "mymodels.py").write_text(
        "import numpy as np\n"
        "from seldon_core_amd.models import iris_logistic_regression\n"
        "from seldon_core_amd.servers import SKLearnServer\n\n\n"
        "class Iris(SKLearnServer):\n"
        "    def __init__(self):\n"
        "        super().__init__(model=iris_logistic_regression())\n\n\n"
        "class Shift:\n"
        "    def transform_input(self, X, names):\n"
        "        return np.asarray(X, dtype=np.float64) * 0.5 + 1.0\n")
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "t", "type": "TRANSFORMER", "rank": 1, "in_cols": 4,
                      "children": [{"name": "m", "type": "MODEL", "rank": 2}]}}
    p, hp, log = _start(tmp_path, spec, 3, extra=("--component", "t=mymodels.Shift", "--component", "m=mymodels.Iris"))
    try:
        assert _wait_log(log, "serving p:", 1), log.read_text()[-3000:]
        text = log.read_text()
        assert "mesh program" in text and "node:t@rank1" in text, text[-2000:]
        from seldon_core_amd.models import iris_logistic_regression

        lr = iris_logistic_regression()
        rng = np.random.default_rng(1)
        for i in range(30):
            X = rng.normal(loc=4.0, scale=1.5, size=(1 + i % 5, 4))
            out = _post(hp, "/api/v0.1/predictions", {"data": {"ndarray": X.tolist()}})
            np.testing.assert_allclose(np.asarray(out["data"]["ndarray"]), lr.predict_proba(X * 0.5 + 1.0),
                                       rtol=0, atol=1e-12)
        assert _stop(p) == 0
    finally:
        _stop(p)
    text = log.read_text()
    assert text.count("done:") == 2, text[-3000:]


def test_rank_placement_needs_enough_gpus(tmp_path):
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "m", "type": "MODEL", "rank": 3}}
    p, _, log = _start(tmp_path, spec, 2)
    assert p.wait(timeout=60) == 2
    assert "places nodes on 4 ranks" in log.read_text()


MYMODELS = (
    "import numpy as np\n"
    "from seldon_core_amd.models import iris_logistic_regression\n"
    "from seldon_core_amd.servers import SKLearnServer\n\n"
    "SCALE = 1.0 + 0.05 * np.arange(4)\n\n\n"
    "class Iris(SKLearnServer):\n"
    "    def __init__(self):\n"
    "        super().__init__(model=iris_logistic_regression())\n\n\n"
    "class Scaler:\n"
    "    def row_model(self):\n"
    "        import seldon_core_amd as sca\n"
    "        return sca.native().linear_model(np.diag(SCALE), np.zeros(4), 0)\n")


def _gang_spec(kind):
    if kind == "abtest":
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}
        return g, 3, ("a=mymodels.Iris", "b=mymodels.Iris"), 1.0
    if kind == "mab":
        g = {"name": "mab", "type": "ROUTER", "implementation": "EPSILON_GREEDY",
             "parameters": [{"name": "n_branches", "value": "2", "type": "INT"},
                            {"name": "epsilon", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "m1", "type": "MODEL", "rank": 1}, {"name": "m2", "type": "MODEL", "rank": 2}]}
        return g, 3, ("m1=mymodels.Iris", "m2=mymodels.Iris"), 1.0
    g = {"name": "scaler", "type": "TRANSFORMER", "rank": 3, "children": [
        {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
         "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}]}
    return g, 4, ("scaler=mymodels.Scaler", "a=mymodels.Iris", "b=mymodels.Iris"), 1.0 + 0.05 * np.arange(4)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["abtest", "mab", "pipeline"])
def test_rank_placed_gang_on_one_gpu_over_ipc(tmp_path, kind):
    """serve --gpus N --device 0: N rank processes, each with its own HIP
    context on GPU 0, serve one rank-placed graph over the ipc mesh; answers
    match sklearn to 1e-12 and the workers keep several batches in flight."""
    from seldon_core_amd._native import gpu_count

    if gpu_count() < 1:
        pytest.skip("needs a GPU")
    import threading

    from seldon_core_amd.models import iris_logistic_regression

    (tmp_path / "mymodels.py").write_text(MYMODELS)
    graph, n, comps, scale = _gang_spec(kind)
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": graph}
    extra = []
    for c in comps:
        extra += ["--component", c]
    p, hp, log = _start(tmp_path, spec, n, extra=extra, device=0,
                        env_extra={"SCA_FABRIC_WORKER_DELAY_US": "1500", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    lr = iris_logistic_regression()
    errs, worst = [], [0.0]
    try:
        assert _wait_log(log, "serving p:", 1, timeout=150), log.read_text()[-3000:]
        text = log.read_text()
        assert "mesh program" in text and "(ipc," in text, text[-3000:]

        def client(t):
            rng = np.random.default_rng(t)
            for i in range(25):
                X = rng.normal(loc=4.0, scale=1.5, size=(1 + (i + t) % 4, 4))
                try:
                    out = _post(hp, "/api/v0.1/predictions", {"data": {"ndarray": X.tolist()}}, timeout=30)
                    err = float(np.abs(np.asarray(out["data"]["ndarray"]) - lr.predict_proba(X * scale)).max())
                    worst[0] = max(worst[0], err)
                except Exception as e:  # noqa: BLE001
                    errs.append(repr(e))

        th = [threading.Thread(target=client, args=(t,)) for t in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert errs == [] and worst[0] < 1e-12, (errs[:3], worst[0])
        assert _stop(p) == 0
    finally:
        _stop(p)
    text = log.read_text()
    done = [ln for ln in text.splitlines() if " done: " in ln and "max in flight" in ln]
    assert len(done) == n - 1, text[-3000:]
    assert max(int(ln.rsplit("max in flight ", 1)[1].split()[0]) for ln in done) >= 2, done
