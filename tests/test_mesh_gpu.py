"""The mesh's GPU transport ("ipc") with every rank of the gang on GPU 0.

Each rank is a separate process with its own HIP context (the cross-process
paths: HIP IPC device slabs between workers, hipHostRegister'ed shared-memory
slabs and doorbells written by stream operations, zero-copy kernels reading
rank 0's input slab and writing its output slab).  Same modes and oracles as
the CPU gang tests (tests/fabric_worker.py); tools/micro/ipc_probe.hip showed
same-device IPC works on this image (profiles/r05a_ipc_probe)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from seldon_core_amd._native import gpu_count

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    from portutil import free_port

    return free_port()


def _run_gpu_ranks(world, mode, timeout=150, **extra_env):
    if gpu_count() < 1:
        pytest.skip("needs a GPU")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SCA_TEST_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0", **extra_env)
        env.pop("GPU_STREAMOPS_CP_WAIT", None)  # breaks IPC event waits (profiles/r05a_ipc_probe)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "fabric_worker.py"), mode],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads([line for line in o.splitlines() if line.startswith("{")][-1]))
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
                q.wait()
    return outs


def _check(outs, messages=None, split=False):
    front = outs[0]
    assert front["transport"] == "ipc", front
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    if messages is not None:
        assert front["messages"] == messages, front
    for w in outs[1:]:
        assert w["error"] == "" and w["transport"] == "ipc", w
        assert split or w["rows"] == front["rows"], w
    if split:  # a router on rank 0 sends each request to one branch
        assert sum(w["rows"] for w in outs[1:]) == front["rows"], outs
    return front


def test_ipc_single_remote_model():
    _check(_run_gpu_ranks(2, "single"), [2])


def test_ipc_remote_combiner_mean_on_rank0():
    _check(_run_gpu_ranks(3, "remote_combiner"), [4])


def test_ipc_pipeline_device_to_device_stage_edges():
    """scaler@1 -> scaler@2 -> iris@3, every rank a process on GPU 0: the
    stage-to-stage edges are D2D copies into the next rank's IPC-mapped slab."""
    _check(_run_gpu_ranks(4, "pipeline"), [4])


def test_ipc_bench_pipeline_dag():
    _check(_run_gpu_ranks(4, "dag"), [5])


def test_ipc_python_transformer_on_gpu_worker():
    _check(_run_gpu_ranks(3, "python"), [3])


def test_ipc_failing_python_stage():
    outs = _run_gpu_ranks(3, "python_error")
    assert outs[0]["errors"] == [] and outs[0]["failed"] == 8 and outs[0]["worst"] < 1e-12, outs[0]
    assert outs[1]["stage_errors"] >= 1, outs[1]


def test_ipc_concurrent_keeps_batches_in_flight():
    outs = _run_gpu_ranks(3, "concurrent", SCA_FABRIC_SLOTS="4", SCA_FABRIC_WORKER_DELAY_US="3000")
    _check(outs, split=True)
    for w in outs[1:]:
        assert w["batches"] > 0 and w["max_inflight"] >= 2, w


def test_ipc_large_chunked_wide():
    outs = _run_gpu_ranks(2, "large")
    assert outs[0]["errors"] == [] and outs[0]["worst"] < 1e-9, outs[0]
    assert outs[1]["error"] == "" and outs[1]["rows"] == outs[0]["rows"], outs[1]


def test_ipc_pipeline_edges_are_device_slabs_after_a_clean_probe():
    front = _check(_run_gpu_ranks(4, "pipeline"), [4])
    (edges,) = front["edges"]
    kinds = {(e["from"], e["to_rank"]): e["transport"] for e in edges}
    assert kinds == {("s1@1", 2): "ipc", ("s2@2", 3): "ipc", ("m@3", 0): "host"}, kinds
    assert front["peer"]["failed_edges"] == [] and front["peer"]["devices"] == [0, 0, 0, 0], front["peer"]


@pytest.mark.parametrize("fault", ["peer", "canary"])
def test_ipc_probe_failure_falls_back_to_host_staged_edges(fault):
    """an injected hipIpcOpenMemHandle failure (or canary
    mismatch) on every worker -> worker edge: the gang still serves, those
    edges become host-staged slabs ("ipc-host"), answers stay at 1e-12."""
    front = _check(_run_gpu_ranks(4, "pipeline", SCA_MESH_FAULT=fault), [4])
    (edges,) = front["edges"]
    kinds = {(e["from"], e["to_rank"]): e["transport"] for e in edges}
    assert kinds == {("s1@1", 2): "ipc-host", ("s2@2", 3): "ipc-host", ("m@3", 0): "host"}, kinds
    assert {"1->2", "2->3", "3->1"} <= set(front["peer"]["failed_edges"]), front["peer"]
    assert any(fault in e for e in front["peer"]["errors"]), front["peer"]
