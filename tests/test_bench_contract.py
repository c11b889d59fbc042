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
           "--steps", "2", "--warmup", "1", "--step-requests", "1000", "--users", "16"]
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
