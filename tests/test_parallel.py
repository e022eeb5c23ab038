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
