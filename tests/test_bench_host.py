"""Host-side pieces of bench.py (no GPU): the roofline's PMC traffic lookup must parse every
committed profiles/*_pmc_summary.json (a crash there would cost the round's bench line) and prefer
a summary profiled on the same build and the same matrix image; `--gpus N` must start N ranks
(the launcher command), refuse a line that does not show N ranks, and never pick an allreduce
transport whose Lanczos coefficients differ from the RCCL run's."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_committed_traffic_parses_all_profiles():
    import bench
    import eigmi
    for img in bench.IMAGES:
        tr = bench.committed_traffic("k_lanczos_fused_march", 256, 1, eigmi.build_id(), img)
        assert tr is None or (tr[0] > 0 and tr[1].startswith("profiles/") and tr[2] in (True, False))
    assert bench.committed_traffic("no_such_kernel", 256, 1, None, "arrays") is None


def test_committed_traffic_prefers_same_build(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    k = "eigmi::k_lanczos_fused_march<unsigned char, true, 10>"
    for tag, build, stamp, b, img in (("old", "aaa", 1.0, 111, "arrays"), ("new", "bbb", 2.0, 222, "arrays"),
                                      ("newest", "bbb", 3.0, 333, "uniform")):
        line = {"config": {"N": 64, "image": img}, "n_gpus": 1}
        (prof / f"{tag}_pmc_summary.json").write_text(json.dumps(
            {"tag": tag, "build": build, "collected": stamp, "bench_line_under_trace": line,
             "kernels": {k: {"hbm_bytes": b}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    kk = "k_lanczos_fused_march<unsigned char, true, 10>"
    assert bench.committed_traffic(kk, 64, 1, "aaa", "arrays") == (111, "profiles/old_pmc_summary.json", True)
    assert bench.committed_traffic(kk, 64, 1, "ccc", "arrays") == (222, "profiles/new_pmc_summary.json", False)
    assert bench.committed_traffic("k_lanczos_fused_march", 64, 1, "ccc", "uniform")[0] == 333
    # another template instance of the same kernel is not this image's kernel
    assert bench.committed_traffic("k_lanczos_fused_march<unsigned char, true, 7>", 64, 1, "ccc", "arrays") is None


def test_launcher_command_runs_n_ranks():
    import bench
    argv = ["--gpus", "8", "--steps", "50", "--warmup", "5"]
    cmd = bench.launcher_command(8, argv, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    assert cmd[-len(argv) - 1] == os.path.abspath(bench.__file__) and cmd[-len(argv):] == argv
    assert 1024 <= bench.free_port() < 65536


def test_child_line_checks_rank_count():
    import bench
    good = {"metric": "m", "value": 1.0, "n_gpus": 2, "comm": {"nranks": 2, "allreduce": "rccl"}}
    d, err = bench.child_line("RCCL banner\n" + json.dumps(good) + "\n", 2)
    assert err is None and d["value"] == 1.0
    # a launcher that silently ran one GPU
    d, err = bench.child_line(json.dumps(dict(good, n_gpus=1)), 2)
    assert err and "n_gpus" in err
    # RCCL saw fewer ranks than the line claims
    d, err = bench.child_line(json.dumps(dict(good, comm={"nranks": 1})), 2)
    assert err and "communicator" in err
    assert bench.child_line("", 2)[1] and bench.child_line(json.dumps(good) * 2 + "\n" + json.dumps(good), 2)[1]


def test_world_size_must_match_gpus(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench.world_from_env(4) == (4, 3, 3)
    assert bench.world_from_env(None) == (4, 3, 3)
    with pytest.raises(SystemExit):
        bench.world_from_env(8)


def test_ab_mismatch_disqualifies_a_wrong_transport():
    import bench
    a = np.linspace(1.0, 2.0, 45)
    b = np.linspace(0.5, 0.7, 46)
    assert bench.ab_mismatch(a, b, a, b) == 0.0
    assert bench.ab_mismatch(a * (1 + 1e-15), b, a, b) <= bench.AB_RTOL
    assert bench.ab_mismatch(a * (1 + 1e-9), b, a, b) > bench.AB_RTOL
    bad = a.copy()
    bad[7] = np.nan
    assert bench.ab_mismatch(bad, b, a, b) == float("inf")


def test_gpus_2_launches_a_child_and_fails_on_mismatch(tmp_path):
    """End to end on the CPU: `bench.py --gpus 2` without WORLD_SIZE must start the launcher (here a
    stand-in torch.distributed module on PYTHONPATH that prints a one-rank line) and exit 4 because
    the line shows one GPU -- the check that stops a silent single-GPU run."""
    fake = tmp_path / "torch" / "distributed"
    fake.mkdir(parents=True)
    (tmp_path / "torch" / "__init__.py").write_text("")
    (fake / "__init__.py").write_text("")
    (fake / "run.py").write_text(
        "import json, sys\n"
        "assert '--nproc-per-node=2' in sys.argv\n"
        "print(json.dumps({'metric': 'm', 'value': 1.0, 'n_gpus': 1, 'comm': {'nranks': 1}}))\n")
    env = dict(os.environ, PYTHONPATH=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       env=env, timeout=120)
    assert p.returncode == 4, p.stderr.decode()[-2000:]
    assert b"n_gpus" in p.stderr and p.stdout.strip() == b""
