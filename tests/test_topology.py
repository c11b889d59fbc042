"""GPU-local CPU placement (seldon_core_amd/utils/topology.py) on a synthetic
MI355X host: 2 sockets x 8 CCDs (8 cores + SMT siblings), 4 GPUs per socket."""
from seldon_core_amd.utils import topology


def _host():
    ccds = [sorted(list(range(8 * i, 8 * i + 8)) + list(range(128 + 8 * i, 128 + 8 * i + 8))) for i in range(16)]
    node0 = [c for g in ccds[:8] for c in g]
    node1 = [c for g in ccds[8:] for c in g]
    gpus = [{"bdf": f"0000:{b}:00.0", "numa": 0 if i < 4 else 1, "cpus": node0 if i < 4 else node1}
            for i, b in enumerate(["0d", "26", "5d", "75", "8e", "a7", "dc", "f4"])]
    return gpus, ccds


def test_each_gpu_gets_its_own_ccds_on_its_socket():
    gpus, ccds = _host()
    allowed = list(range(256))
    sets = [topology.gpu_cpu_set(g["bdf"], 16, allowed, gpus, ccds) for g in gpus]
    assert all(len(s) == 16 for s in sets)
    assert sets[1] == ccds[2]  # second GPU of socket 0 -> third CCD (2 CCDs per GPU)
    assert sets[4] == ccds[8]  # first GPU of socket 1 -> first CCD of socket 1
    for s, g in zip(sets, gpus):  # always on the GPU's own socket
        assert set(s) <= set(g["cpus"])
    flat = [c for s in sets for c in s]
    assert len(flat) == len(set(flat))  # disjoint across GPUs


def test_budget_larger_than_a_ccd_takes_whole_neighbouring_ccds():
    gpus, ccds = _host()
    s = topology.gpu_cpu_set(gpus[0]["bdf"], 24, list(range(256)), gpus, ccds)
    assert s == sorted(ccds[0] + ccds[1])


def test_unknown_gpu_or_disallowed_cpus_mean_no_pinning():
    gpus, ccds = _host()
    assert topology.gpu_cpu_set("0000:ff:00.0", 16, list(range(256)), gpus, ccds) == []
    assert topology.gpu_cpu_set(gpus[0]["bdf"], 16, [0, 1, 2], gpus, ccds) == []


def test_cpulist_parser():
    assert topology._parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
