"""parallel/: rank environment, KFD link topology parsing (fake sysfs tree), exchange
settings agreement across ranks, launcher command lines."""
import os

import pytest

from quorum_amd.parallel import exchange, launcher, topology


def test_rank_env_precedence():
    assert topology.RankEnv.from_env({}) == topology.RankEnv(0, 1, 0)
    e = {"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3"}
    r = topology.RankEnv.from_env(e)
    assert (r.rank, r.world, r.local_rank, r.distributed) == (3, 8, 3, True)
    e.update(QMX_RANK="1", QMX_WORLD="2")  # qmx's launcher wins
    assert topology.RankEnv.from_env(e).rank == 1
    assert topology.RankEnv(5, 8, 5).device(8) == 5 and topology.RankEnv(5, 8, 5).device(1) == 0
    with pytest.raises(ValueError):
        topology.RankEnv.from_env({"RANK": "2", "WORLD_SIZE": "2"})


def _fake_kfd(root, n_gpus, kind=11):
    # node 0 = CPU, nodes 1..n = GPUs; each GPU: 1 link to the CPU + links to every peer
    (root / "0").mkdir(parents=True)
    (root / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for g in range(1, n_gpus + 1):
        d = root / str(g)
        (d / "io_links").mkdir(parents=True)
        (d / "properties").write_text("simd_count 1024\ngpu_id 1234\n")
        links = [(0, 2)] + [(p, kind) for p in range(1, n_gpus + 1) if p != g]
        for i, (to, t) in enumerate(links):
            (d / "io_links" / str(i)).mkdir()
            (d / "io_links" / str(i) / "properties").write_text(
                f"type {t}\nnode_from {g}\nnode_to {to}\nweight 15\nmax_bandwidth 153000\n")


def test_kfd_full_xgmi_mesh(tmp_path):
    _fake_kfd(tmp_path, 8)
    links = topology.gpu_links(tmp_path)
    assert len(links) == 8 * 7 and {x.kind for x in links} == {"xgmi"}
    assert topology.gpu_count(tmp_path) == 8
    s = topology.summary(root=tmp_path)
    assert s["gpus"] == 8 and s["full_xgmi_mesh"] and s["links_per_gpu"][0] == {"xgmi": 7}


def test_kfd_pcie_only_and_missing(tmp_path):
    _fake_kfd(tmp_path / "two", 2, kind=2)
    assert not topology.summary(root=tmp_path / "two")["full_xgmi_mesh"]
    _fake_kfd(tmp_path / "one", 1)
    assert topology.summary(root=tmp_path / "one") == {"gpus": 1, "links_per_gpu": {0: {}}, "full_xgmi_mesh": True}
    assert topology.gpu_links(tmp_path / "nope") == []
    assert topology.summary(root=tmp_path / "nope") == {"gpus": 0, "links_per_gpu": {}, "full_xgmi_mesh": False}


def _fake_numa(root, nodes, smt=2):
    """nodes: {node: n_physical_cores}; logical cpu numbering as on a 2-socket EPYC box:
    physical cores first (node by node), SMT siblings after them."""
    total = sum(nodes.values())
    first = 0
    for node, n in sorted(nodes.items()):
        cpus = []
        for i in range(n):
            for t in range(smt):
                cpu = first + i + t * total
                cpus.append(cpu)
                topo = root / "cpu" / f"cpu{cpu}" / "topology"
                topo.mkdir(parents=True)
                (topo / "physical_package_id").write_text(f"{node}\n")
                (topo / "core_id").write_text(f"{i}\n")
        d = root / "node" / f"node{node}"
        d.mkdir(parents=True)
        cpus.sort()
        # kernel format: ranges
        runs, start = [], cpus[0]
        for a, b in zip(cpus, cpus[1:] + [None]):
            if b != a + 1:
                runs.append(f"{start}-{a}" if a != start else str(a))
                start = b
        (d / "cpulist").write_text(",".join(runs) + "\n")
        first += n


def test_cpulist_and_pci_numa(tmp_path):
    assert topology.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    dev = tmp_path / "pci" / "0000:75:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    assert topology.pci_numa_node(0, 0x75, 0, root=tmp_path / "pci") == 1
    assert topology.pci_numa_node(0, 0x76, 0, root=tmp_path / "pci") == -1


def test_rank_cpus_split_by_numa_node(tmp_path):
    _fake_numa(tmp_path, {0: 8, 1: 8})  # 2 sockets x 8 cores x 2 threads = cpus 0-31
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]  # GPUs 0-3 on socket 0, 4-7 on socket 1
    kw = dict(node_root=tmp_path / "node", cpu_root=tmp_path / "cpu")
    sets = [topology.rank_cpus(nodes, r, **kw) for r in range(8)]
    assert sets[0] == [0, 1, 16, 17] and sets[3] == [6, 7, 22, 23] and sets[4] == [8, 9, 24, 25]
    flat = [c for s in sets for c in s]
    assert sorted(flat) == list(range(32))  # disjoint, covering every cpu
    # restricted affinity set; unknown node; more ranks than cores
    assert topology.rank_cpus(nodes, 0, allowed=[0, 1, 2, 3, 16], **kw) == [0, 16]
    assert topology.rank_cpus([-1, -1], 0, **kw) is None
    assert topology.rank_cpus([0] * 9, 0, **kw) is None
    # the plan refuses to strand a socket (every GPU reported on node 0)
    allowed = list(range(32))
    assert topology.plan_rank_cpus(nodes, allowed, **kw) == sets
    assert topology.plan_rank_cpus([0] * 8, allowed, **kw) is None
    assert topology.plan_rank_cpus([0, -1], allowed, **kw) is None


def test_compact_cpus_pack_last_level_caches(tmp_path):
    """compact_cpus (bench.py pin_single): N CPUs of the GPU's node on the fewest L3s — both
    SMT siblings per core (smt) or one thread per core — cores in L3 order."""
    _fake_numa(tmp_path, {0: 8, 1: 8})  # cpus 0-31: node 0 cores 0-7 (+16-23), node 1 8-15 (+24-31)
    for c in range(32):  # two 4-core L3s per node: cores {0-3}, {4-7}, {8-11}, {12-15}
        core = c % 16
        lo = core - core % 4
        cache = tmp_path / "cpu" / f"cpu{c}" / "cache" / "index3"
        cache.mkdir(parents=True)
        cache.joinpath("shared_cpu_list").write_text(f"{lo}-{lo + 3},{lo + 16}-{lo + 19}\n")
    kw = dict(node_root=tmp_path / "node", cpu_root=tmp_path / "cpu")
    assert topology.llc_cpus(1, **kw) == 8
    assert topology.compact_cpus(8, 1, smt=True, **kw) == [8, 9, 10, 11, 24, 25, 26, 27]  # one L3
    assert topology.compact_cpus(4, 0, **kw) == [0, 1, 2, 3]
    assert topology.compact_cpus(6, 0, **kw) == [0, 1, 2, 3, 4, 5]
    assert topology.compact_cpus(16, 0, smt=True, **kw) == list(range(8)) + list(range(16, 24))
    assert topology.compact_cpus(17, 0, smt=True, **kw) is None  # more than the node holds
    assert topology.compact_cpus(4, 0, allowed=[2, 3, 18, 19, 5], smt=True, **kw) == [2, 3, 18, 19]
    # another tenant keeps the first L3 busy: the next one is taken
    busy = {c: 0.9 for c in (0, 1, 2, 3, 16, 17, 18, 19)}
    assert topology.compact_cpus(8, 0, smt=True, busy=busy, **kw) == [4, 5, 6, 7, 20, 21, 22, 23]
    stat = tmp_path / "stat"
    stat.write_text("cpu  1 2 3 4\ncpu0 10 0 10 80 0\ncpu1 0 0 0 100 0\n")
    b = topology.cpu_busy(0.0, stat)
    assert set(b) == {0, 1}  # (no time passed between the samples: 0 busy)


def test_rank_llc_cpus_disjoint_compact_sets(tmp_path):
    """rank_llc_cpus (bench.py pin_rank): every rank whole L3s of its GPU's node, ranks of one
    node on consecutive, disjoint L3s; too many ranks for the node's L3s -> None."""
    _fake_numa(tmp_path, {0: 8, 1: 8})
    for c in range(32):  # 4-core L3s: {0-3,16-19}, {4-7,20-23}, {8-11,24-27}, {12-15,28-31}
        core = c % 16
        lo = core - core % 4
        cache = tmp_path / "cpu" / f"cpu{c}" / "cache" / "index3"
        cache.mkdir(parents=True)
        cache.joinpath("shared_cpu_list").write_text(f"{lo}-{lo + 3},{lo + 16}-{lo + 19}\n")
    kw = dict(node_root=tmp_path / "node", cpu_root=tmp_path / "cpu")
    nodes = [0, 0, 1, 1]
    sets = [topology.rank_llc_cpus(nodes, r, 8, **kw) for r in range(4)]
    assert sets[0] == [0, 1, 2, 3, 16, 17, 18, 19] and sets[1] == [4, 5, 6, 7, 20, 21, 22, 23]
    assert sets[2] == [8, 9, 10, 11, 24, 25, 26, 27] and sets[3] == [12, 13, 14, 15, 28, 29, 30, 31]
    assert topology.rank_llc_cpus([0, 0], 1, 9, **kw) is None  # 2 L3s each: node 0 holds 2
    assert topology.rank_llc_cpus([0], 0, 9, **kw) == list(range(8)) + list(range(16, 24))
    assert topology.rank_llc_cpus([-1], 0, 8, **kw) is None


def test_gpu_numa_nodes_from_kfd(tmp_path):
    _fake_kfd(tmp_path / "kfd", 2)
    for g, (bus, node) in enumerate([(0x05, 0), (0xE5, 1)], start=1):
        pp = tmp_path / "kfd" / str(g) / "properties"
        pp.write_text(pp.read_text() + f"domain 0\nlocation_id {bus << 8}\n")
        dev = tmp_path / "pci" / f"0000:{bus:02x}:00.0"
        dev.mkdir(parents=True)
        (dev / "numa_node").write_text(f"{node}\n")
    assert topology.gpu_numa_nodes(tmp_path / "kfd", tmp_path / "pci") == [0, 1]
    assert topology.gpu_numa_nodes(tmp_path / "none", tmp_path / "pci") == []


def test_exchange_settings_agree_across_ranks():
    cfgs = []
    for r in range(4):
        env = exchange.exchange_env(r, 4, 18000, nonce="42")
        cfgs.append(exchange.cluster_config("spread", "auto", 200, 30.0, 18000, "hip", env=env))
    assert [c["rank"] for c in cfgs] == [0, 1, 2, 3]
    for c in cfgs:  # one rendezvous for the whole node
        assert (c["world"], c["xchg"], c["xchg_port"], c["xchg_id_file"]) == \
            (4, "rccl", 18007, cfgs[0]["xchg_id_file"])
    assert exchange.cluster_config("local", "auto", 200, 30.0, 18000, "cpu", env={})["xchg"] == "tcp"
    with pytest.raises(ValueError):
        exchange.cluster_config("everywhere", "auto", 200, 30.0, 18000, "cpu", env={})


def test_launcher_rank_commands(monkeypatch):
    monkeypatch.delenv("QMX_XCHG_PORT", raising=False)
    cmds = launcher.rank_commands(["--impl", "native", "--gpus", "4"], 4, True, 9000, "7")
    assert len(cmds) == 4
    for r, (cmd, env) in enumerate(cmds):
        assert cmd[-2:] == ["--device", str(r)]
        assert env["QMX_RANK"] == str(r) and env["LOCAL_RANK"] == str(r) and env["QMX_WORLD"] == "4"
        assert env["QMX_XCHG_NONCE"] == "7" and env["QMX_XCHG_PORT"] == "9007"
    monkeypatch.setenv("QMX_XCHG_PORT", "1234")
    assert launcher.rank_commands([], 2, False, 9000, "7")[1][1]["QMX_XCHG_PORT"] == "1234"
