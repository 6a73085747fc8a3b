"""NUMA-local core -> GPU mapping (SURVEY.md §8e "its own host thread (NUMA-local)"),
checked on a fake sysfs tree: 2 nodes x 4 GPUs, 16 cores.

mOS binds each mTCP thread and its memory to its core's node (core/src/cpu.c:
56-87) and DPDK puts a port's queues on the port's socket (dpdk_module.c:679,
:726-743).  gpu_module_func maps core c to a GPU on c's node, round robin over
that node's GPUs by c's rank among the node's cores (csrc/topology.c), and
bench.py binds each rank to its GPU's node before its first GPU call
(mosrx.bind_to_gpu_node).  No GPU needed: everything is read from sysfs.
"""
import ctypes as C
import os

import pytest

import mosrx

# 8 GPUs: 4 on node 0, 4 on node 1 (MI355X nodes put 4 OAMs behind each socket)
BDFS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
        "0000:85:00.0", "0000:95:00.0", "0000:e5:00.0", "0000:f5:00.0"]
GPU_NODE = [0, 0, 0, 0, 1, 1, 1, 1]


def fake_tree(root, cpulists=("0-7", "8-15"), gpu_node=GPU_NODE, kfd=True):
    """sysfs as the code reads it: PCI numa_node per GPU, cpu<c>/node<n>, node cpulists,
    and (kfd) the KFD topology nodes HIP enumerates (a CPU node first, then the GPUs)."""
    for bdf, node in zip(BDFS, gpu_node):
        d = root / "sys" / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for n, cl in enumerate(cpulists):
        nd = root / "sys" / "devices" / "system" / "node" / f"node{n}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(cl + "\n")
        for c in mosrx._parse_cpulist(cl):
            (root / "sys" / "devices" / "system" / "cpu" / f"cpu{c}" / f"node{n}").mkdir(parents=True)
    if kfd:
        base = root / "sys" / "class" / "kfd" / "kfd" / "topology" / "nodes"
        (base / "0").mkdir(parents=True)
        (base / "0" / "properties").write_text("cpu_cores_count 16\nsimd_count 0\n")
        for i, bdf in enumerate(BDFS):
            dom, bus, df = bdf.split(":")
            dev, fn = df.split(".")
            loc = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn)
            (base / str(i + 1)).mkdir()
            (base / str(i + 1) / "properties").write_text(
                f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {loc}\ndomain {int(dom, 16)}\n")


@pytest.fixture
def topo(tmp_path):
    L = mosrx.lib()
    yield L, tmp_path
    L.mosrx_topology_set_root(None)


def pick(L, cpu, nodes):
    arr = (C.c_int * len(nodes))(*nodes)
    return L.mosrx_numa_pick(cpu, arr, len(nodes))


def test_sysfs_reads(topo):
    L, root = topo
    fake_tree(root)
    assert L.mosrx_topology_set_root(str(root).encode()) == 0
    assert [L.mosrx_pci_numa_node(b.encode()) for b in BDFS] == GPU_NODE
    assert L.mosrx_pci_numa_node(b"0000:05:00.0".upper()) == 0          # hipDeviceGetPCIBusId may use capitals
    assert L.mosrx_pci_numa_node(b"0000:aa:00.0") == -1
    assert [L.mosrx_cpu_numa_node(c) for c in range(16)] == [0] * 8 + [1] * 8
    assert L.mosrx_cpu_numa_node(16) == -1


def test_two_nodes_four_gpus_each(topo):
    """16 cores in two blocks: node 0's cores drive GPUs 0-3, node 1's 4-7, each
    GPU two cores, round robin by rank within the node."""
    L, root = topo
    fake_tree(root)
    L.mosrx_topology_set_root(str(root).encode())
    nodes = [L.mosrx_pci_numa_node(b.encode()) for b in BDFS]
    got = [pick(L, c, nodes) for c in range(16)]
    assert got == [0, 1, 2, 3, 0, 1, 2, 3, 4, 5, 6, 7, 4, 5, 6, 7]
    assert all(nodes[g] == L.mosrx_cpu_numa_node(c) for c, g in enumerate(got))


def test_interleaved_cores(topo):
    """Nodes whose cores interleave (even / odd): the rank within the node, not the
    core number, spreads them (c % 4 would put node 0's even cores on 2 GPUs only)."""
    L, root = topo
    fake_tree(root, cpulists=("0,2,4,6,8,10,12,14", "1,3,5,7,9,11,13,15"))
    L.mosrx_topology_set_root(str(root).encode())
    got = [pick(L, c, GPU_NODE) for c in range(16)]
    assert got == [0, 4, 1, 5, 2, 6, 3, 7, 0, 4, 1, 5, 2, 6, 3, 7]
    for g in range(8):
        assert got.count(g) == 2


def test_unknown_topology_falls_back(topo):
    """A GPU of unknown node, a node without GPUs, or no sysfs at all: -1, and the
    module takes gpu_base + c % ngpu (the round-3 map)."""
    L, root = topo
    fake_tree(root)
    L.mosrx_topology_set_root(str(root).encode())
    assert pick(L, 3, [0, 0, -1, 1]) == -1
    assert pick(L, 9, [0, 0, 0, 0]) == -1            # core 9 is on node 1: no GPU there
    assert pick(L, 99, GPU_NODE) == -1               # no such core
    L.mosrx_topology_set_root(str(root / "nowhere").encode())
    assert pick(L, 0, GPU_NODE) == -1


def test_module_uses_the_map_or_the_fallback():
    """gpu_module_func's device_of: cfg.numa on by default; with the GPUs' nodes
    unknown (no GPU here) it is gpu_base + c % ngpu."""
    L = mosrx.lib()
    cfg = mosrx.ModuleCfg()
    L.mosrx_gpu_module_cfg_default(C.byref(cfg))
    assert cfg.numa == 1
    cfg.num_ifs = 1
    assert L.mosrx_gpu_module_configure(C.byref(cfg)) == 0
    assert [L.mosrx_gpu_module_device_of(c, 8) for c in range(10)] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]


def test_bench_rank_binding(tmp_path, monkeypatch):
    """bench.py's rank binding reads device -> PCI address from the KFD topology (HIP's
    order, no HIP call), its node, and that node's cores; visible-device lists
    re-number the GPUs as HIP does."""
    fake_tree(tmp_path)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert mosrx.gpu_numa_cpus(0, str(tmp_path)) == (BDFS[0], 0, list(range(8)))
    assert mosrx.gpu_numa_cpus(5, str(tmp_path)) == (BDFS[5], 1, list(range(8, 16)))
    assert mosrx.gpu_numa_cpus(8, str(tmp_path)) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "6,1")
    assert mosrx.gpu_numa_cpus(0, str(tmp_path))[:2] == (BDFS[6], 1)
    assert mosrx.gpu_numa_cpus(1, str(tmp_path))[:2] == (BDFS[1], 0)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    allowed = os.sched_getaffinity(0)
    try:
        r = mosrx.bind_to_gpu_node(0, str(tmp_path))
        want = set(range(8)) & allowed
        if want:
            assert r["bound"] and os.sched_getaffinity(0) == want and r["node"] == 0
        else:
            assert not r["bound"]
    finally:
        os.sched_setaffinity(0, allowed)
    assert mosrx.gpu_numa_cpus(0, str(tmp_path / "none")) is None
