"""bench.py driver contract: one JSON line from rank 0, whole-job value,
max-over-ranks timing; multi-rank via torch.distributed.run (gloo on CPU)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_bench_two_ranks_cpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--step-requests", "1000", "--users", "16", "--extra-steps", "1"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = _json_lines(res.stdout)
    assert len(lines) == 1, res.stdout  # rank 0 only
    line = lines[0]
    assert KEYS <= set(line)
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["warmup"] == 1
    assert line["config"]["parallelism"] == "dp2" and line["scaling"] == "weak"
    # value = both ranks' predictions over the slowest rank's window
    assert abs(line["value"] - 2 * 2 * 1000 / (line["ms_per_step"] * 2 / 1000.0)) / line["value"] < 0.01
    assert line["vs_baseline"] > 0 and line["higher_is_better"] is True
    # the driver's launch path (torch.distributed.run): the isolated variant
    # runner and the fabric probe form their own process groups from the ranks
    assert line["variants"]["abtest"]["self_check"]["ok"] and line["variants"]["mab"]["self_check"]["ok"]
    assert line["rccl_fabric"]["ok"], line["rccl_fabric"]


def test_bench_direct_launch_spawns_ranks_and_runs_variants():
    """`python bench.py --gpus 2` without torchrun spawns two fresh ranks; the
    multi-GPU graph configs run after the timed region and are self-checked."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--step-requests", "1000",
           "--users", "16"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = _json_lines(res.stdout)
    assert len(lines) == 1, res.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert [r["rank"] for r in line["config"]["per_rank"]] == [0, 1]
    assert all(r["cpu_budget"] > 0 and r["gpu_batches"] > 0 for r in line["config"]["per_rank"])
    assert line["self_check"]["ok"] and line["self_check"]["max_abs_err"] < 1e-9
    assert line["grpc"]["value"] > 0
    v = line["variants"]
    assert set(v) == {"abtest", "mab"}  # pipeline needs 4 GPUs
    assert v["abtest"]["gpus_per_graph"] == 2 and v["mab"]["gpus_per_graph"] == 2
    assert all(x["self_check"]["ok"] for x in v.values())
    assert v["mab"]["feedback_rps"] > 0
    # rank-placed graph over the p2p fabric (child processes, sockets data plane on CPU)
    fab = line["rccl_fabric"]
    assert fab["ok"] and fab["world"] == 2 and fab["data_plane"] == "sockets", fab
    assert fab["max_abs_err"] < 1e-12 and [r["status"] for r in fab["ranks"]] == ["ok", "ok"]


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True, text=True,
                         timeout=120, env=env)
    assert res.returncode == 2 and "WORLD_SIZE" in res.stderr


def test_group_devices_places_variant_nodes_on_distinct_gpus():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.group_devices(0, 2, 8) == [0, 1] and bench.group_devices(1, 2, 8) == [1, 0]
    assert bench.group_devices(5, 4, 8) == [5, 6, 7, 4]
    for r in range(8):
        devs = bench.group_devices(r, 8, 8)
        assert devs[0] == r and sorted(devs) == list(range(8))
    assert bench.group_devices(3, 2, 1) == [0, 0]  # one visible GPU: fold


def test_variant_failure_on_one_rank_is_reported_not_fatal():
    """A variant that fails on one rank (SCA_BENCH_FAULT=abtest:1) is skipped by
    every rank together -- no rank waits alone in a collective -- and shows up
    as an error in the line; the headline and the other variants stand."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--step-requests", "1000",
           "--users", "16", "--fabric-probe", "none"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", SCA_BENCH_FAULT="abtest:1")
    env.pop("WORLD_SIZE", None)
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    line = _json_lines(res.stdout)[0]
    assert line["value"] > 0 and line["self_check"]["ok"]
    ab = line["variants"]["abtest"]
    assert "injected abtest setup fault" in ab["error"] and ab["ranks_failed"] == 2, ab
    assert line["variants"]["mab"]["self_check"]["ok"]
