"""Bounded, deadlock-free shutdown under repeated signals.

The reference engine pauses its connector and force-stops after a <= 20 s
drain (``engine/src/main/java/io/seldon/engine/App.java:89-92``).  Here a
double SIGTERM (a ``killpg`` plus the supervisor's forwarded SIGTERM) or a
Ctrl-C followed by SIGTERM used to re-enter a handler blocked inside
``threading.Event.set()`` and hang the worker forever.  The handlers now only
flip a flag (``seldon_core_amd/utils/shutdown.py``); these tests drive the
double signal through real ``serve`` process trees, many times over, and
require every exit to be fast and complete (each worker files its stats)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from seldon_core_amd.utils.shutdown import StopSignal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUNDS = int(os.environ.get("SCA_SHUTDOWN_ROUNDS", "20"))
PAR = 4  # process trees in flight at once (8 CPUs here; each tree is 3 processes)


def _free_port():
    from portutil import free_port

    return free_port()


def test_stop_signal_reentrant_handler_never_blocks():
    """The handler re-entered from itself (what a second signal landing inside
    it does) completes; ``wait`` returns once it ran."""
    st = StopSignal()
    assert not st.wait(0.01)

    def nested(depth):
        st.handler(signal.SIGTERM)
        if depth:
            nested(depth - 1)

    nested(50)
    assert st.wait(0.0) and st.first_signal == signal.SIGTERM and st.signals == 51
    for _ in range(10000):  # a full self-pipe never blocks the handler
        st.handler(signal.SIGINT)
    assert st.wait(None)
    st.close()


def test_stop_signal_real_signals_in_one_process():
    st = StopSignal().install()
    old = (signal.getsignal(signal.SIGTERM), signal.getsignal(signal.SIGINT))
    try:
        os.kill(os.getpid(), signal.SIGINT)
        os.kill(os.getpid(), signal.SIGTERM)
        os.kill(os.getpid(), signal.SIGTERM)
        t0 = time.monotonic()
        assert st.wait(5.0)
        assert time.monotonic() - t0 < 1.0
        assert st.first_signal == signal.SIGINT
    finally:
        signal.signal(signal.SIGTERM, old[0])
        signal.signal(signal.SIGINT, old[1])
        st.close()


MYMODELS = (
    "from seldon_core_amd.models import iris_logistic_regression\n"
    "from seldon_core_amd.servers import SKLearnServer\n\n\n"
    "class Iris(SKLearnServer):\n"
    "    def __init__(self):\n"
    "        super().__init__(model=iris_logistic_regression())\n")


class _Tree:
    def __init__(self, tmp, gang: bool, idx: int):
        self.dir = tmp / f"t{idx}"
        self.dir.mkdir()
        (self.dir / "mymodels.py").write_text(MYMODELS)
        self.stats = self.dir / "stats"
        self.stats.mkdir()
        if gang:
            graph = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
                     "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
                     "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL"}]}
            comps = ["--component", "a=mymodels.Iris", "--component", "b=mymodels.Iris"]
        else:
            graph = {"name": "m", "type": "MODEL"}
            comps = ["--component", "m=mymodels.Iris"]
        sp = self.dir / "spec.json"
        sp.write_text(json.dumps({"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": graph}))
        self.gang = gang
        self.log_path = self.dir / "serve.log"
        self.log = open(self.log_path, "w")
        env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, str(self.dir)]), CUDA_VISIBLE_DEVICES="",
                   SCA_WORKER_STATS_DIR=str(self.stats))
        self.p = subprocess.Popen(
            [sys.executable, "-m", "seldon_core_amd.serve", "--spec", str(sp), "--gpus", "2", "--device", "-1",
             "--http-port", str(_free_port()), "--grpc-port", str(_free_port()), "--admin-port", "0",
             "--threads", "1", "--log-level", "INFO", *comps],
            env=env, cwd=ROOT, start_new_session=True, stdout=self.log, stderr=subprocess.STDOUT)

    def ready(self) -> bool:
        text = self.log_path.read_text()
        if self.gang:
            return "serving p:" in text and "serving its placed nodes" in text
        return text.count("serving p:") >= 2

    def kill(self):
        if self.p.poll() is None:
            try:
                os.killpg(self.p.pid, signal.SIGKILL)
            except OSError:
                pass
            self.p.wait()
        self.log.close()


def _children(pid):
    out = []
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                with open(f"/proc/{d}/stat") as f:
                    if int(f.read().rsplit(")", 1)[1].split()[1]) == pid:
                        out.append(int(d))
            except (OSError, ValueError, IndexError):
                pass
    return out


def _cycle(tmp_path, gang: bool, sigs):
    """Start ROUNDS process trees (PAR at a time), deliver ``sigs`` back to
    back to each whole process group once it serves, and check the exits."""
    results, i = [], 0
    while i < ROUNDS:
        batch = [_Tree(tmp_path, gang, i + k) for k in range(min(PAR, ROUNDS - i))]
        i += len(batch)
        try:
            deadline = time.time() + 120
            while not all(t.ready() for t in batch):
                assert time.time() < deadline, [t.log_path.read_text()[-2000:] for t in batch if not t.ready()]
                for t in batch:
                    assert t.p.poll() is None, t.log_path.read_text()[-3000:]
                time.sleep(0.1)
            for t in batch:
                t0 = time.monotonic()
                for s in sigs:
                    os.killpg(t.p.pid, s)
                try:
                    rc = t.p.wait(timeout=8)
                except subprocess.TimeoutExpired:  # hang triage: every worker dumps its stacks
                    for pid in _children(t.p.pid):
                        try:
                            os.kill(pid, signal.SIGUSR1)
                        except OSError:
                            pass
                    time.sleep(1.0)
                    rc = None
                results.append((rc, time.monotonic() - t0, sorted(os.listdir(t.stats)), t))
        finally:
            for t in batch:
                t.kill()
    bad = [(rc, round(dt, 2), files, t.log_path.read_text()[-6000:]) for rc, dt, files, t in results
           if rc is None or dt >= 5.0 or (files != ["worker-0.json", "worker-1.json"] if not gang else
                                          files != ["worker-0.json"])]
    assert not bad, bad[:2]
    if gang:  # the peer rank left its loop on rank 0's stop every time
        for _, _, _, t in results:
            assert " done: " in t.log_path.read_text(), t.log_path.read_text()[-2000:]
    return max(dt for _, dt, _, _ in results)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sigs", [(signal.SIGTERM, signal.SIGTERM), (signal.SIGINT, signal.SIGTERM)],
                         ids=["term-term", "int-term"])
def test_replica_workers_exit_fast_on_double_signal(tmp_path, sigs):
    _cycle(tmp_path, False, sigs)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sigs", [(signal.SIGTERM, signal.SIGTERM), (signal.SIGINT, signal.SIGTERM)],
                         ids=["term-term", "int-term"])
def test_rank_gang_exits_fast_on_double_signal(tmp_path, sigs):
    _cycle(tmp_path, True, sigs)


def test_supervisor_sigkills_a_worker_that_ignores_sigterm(tmp_path):
    """Escalation: a worker that never drains is SIGKILLed ``--kill-after``
    seconds after the forwarded SIGTERM; the supervisor still exits."""
    from seldon_core_amd.serve import Supervisor

    stub = tmp_path / "stub.py"
    stub.write_text("import signal, time\nsignal.signal(signal.SIGTERM, signal.SIG_IGN)\n"
                    "print('up', flush=True)\nwhile True:\n    time.sleep(0.1)\n")
    sup = Supervisor(2, [], kill_after=1.0)
    sup._start = lambda rank, ready_file=None: subprocess.Popen([sys.executable, str(stub)])  # noqa: ARG005
    import threading

    rc = []
    sup.spawn(0)
    sup.spawn(1)
    th = threading.Thread(target=lambda: rc.append(sup._loop()), daemon=True)
    th.start()
    time.sleep(1.5)
    sup.request_stop(signal.SIGTERM)
    sup.request_stop(signal.SIGTERM)  # idempotent
    th.join(10)
    assert not th.is_alive() and rc == [0]
    assert len(sup.killed_pids) == 2
