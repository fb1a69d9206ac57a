"""bench.py's rank launcher (`--gpus N` without torchrun, bench.py
launch_ranks): it refuses more ranks than visible GPUs unless
--allow-shared-gpu, and the rehearsal with ranks sharing one GPU reports every
rank in its line (ranks, oversubscribed, distinct n_gpus).  The multi-rank
protocol itself is tests/test_dist.py's (gloo, world 2)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--sites", "200000", "--steps", "1", "--warmup", "0", "--device-steps", "1", "--no-extras"]


def run_bench(args, timeout):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)   # the launcher path: no torchrun around it
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=env, capture_output=True, timeout=timeout)


def visible_gpus():
    import torch
    return torch.cuda.device_count()   # (counting does not initialise a device on this image)


def test_launcher_needs_a_device():
    if visible_gpus() > 0:
        pytest.skip("a GPU is visible: the refusal without one is the CPU container's case")
    r = run_bench(["--gpus", "2"] + SMALL, 120)
    assert r.returncode != 0
    assert b"no HIP device visible" in r.stderr


@pytest.mark.gpu
def test_launcher_refuses_more_ranks_than_gpus():
    n = visible_gpus()
    r = run_bench(["--gpus", str(n + 1)] + SMALL, 120)
    assert r.returncode != 0
    assert b"--allow-shared-gpu" in r.stderr
    assert b'{"metric"' not in r.stdout


@pytest.mark.gpu
def test_shared_gpu_rehearsal_reports_every_rank():
    if visible_gpus() != 1:
        pytest.skip("the rehearsal case: one visible GPU")
    r = run_bench(["--gpus", "2", "--allow-shared-gpu"] + SMALL, 300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1   # rank 0's line only
    d = json.loads(lines[0])
    assert d["config"]["ranks"] == 2
    assert d["config"]["oversubscribed"] is True
    assert d["n_gpus"] == 1
    assert d["config"]["sites_total"] == 2 * 200000
    assert d["value"] > 0
    assert_self_checked(d, 2)


def assert_self_checked(d, ranks):
    """What every line carries at any N: each rank's spot
    check of its first chunk of records against the oracle, and each rank's
    placement with the NUMA node of its pinned text's pages."""
    sc = d["spot_check"]
    assert sc["ranks_equal"] is True and [r["rank"] for r in sc["ranks"]] == list(range(ranks))
    assert all(r["equal"] is True and r["records"] > 0 for r in sc["ranks"])
    numa = d["config"]["numa"]
    assert [p["rank"] for p in numa] == list(range(ranks))
    for p in numa:
        assert p["text_numa_nodes"] and all(isinstance(x, int) and x >= 0 for x in p["text_numa_nodes"]), p
        assert "gpu_numa_node" in p and p["pci"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_two_rank_lynch_exchange_equals_one_process(sid, oracle, gpu, tmp_path):
    """C3's one collective (bench.py Rank.lynch_step_exchange): two ranks, each
    with 2M sites of seed 3, all-gather their unique-profile tables as device
    tensors, rank 0 runs the one Nelder-Mead estimate and broadcasts (pi, eps).
    The rank-ordered concatenation of both ranks' records (the timed PCIe
    leg's, from the engines' host arenas) must be the one-process oracle's CSV
    over the same 4M sites (call.cpp:62-143: the estimate is global), and both
    ranks' (pi, eps, iterations) the oracle's, bit for bit.  On one GPU the
    ranks share it over gloo (RCCL takes one rank per GPU); the exchange code
    and its device tensors are the same for either backend (sid_amd/dist.py)."""
    n = 2_000_000
    dump = tmp_path / "dump"
    r = run_bench(["--gpus", "2", "--allow-shared-gpu", "--config", "C3", "--sites", str(n), "--steps", "1",
                   "--warmup", "0", "--device-steps", "1", "--no-extras", "--dump-records", str(dump)], 600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith('{"metric"')][0])
    assert d["config"]["ranks"] == 2 and d["config"]["sites_total"] == 2 * n
    text, ln = gpu.synth_text_hbm(3, 30.0, 0, 2 * n)
    host = text[:ln].cpu().numpy().tobytes()
    del text
    p = tmp_path / "c3_4m.plp"
    p.write_bytes(host)
    ref = oracle.run_cli(["-R", "-m", "likelihood_ratio", str(p)])
    assert ref.returncode == 0
    got = sid.HEADER + b"".join((dump / f"rank{k}.csv").read_bytes() for k in range(2))
    if got != ref.stdout:
        import numpy as np
        m = min(len(got), len(ref.stdout))
        i = int(np.argmax(np.frombuffer(got[:m], np.uint8) != np.frombuffer(ref.stdout[:m], np.uint8)))
        raise AssertionError(f"first difference at byte {i}: {got[i - 80:i + 80]!r} vs {ref.stdout[i - 80:i + 80]!r}")
    s = sid.parse_text(host)
    rc, _, _, _, est, u = oracle.call_method(s.counts, "likelihood_ratio", estimate_prior=True)
    assert rc == 0
    for k in range(2):
        j = json.loads((dump / f"rank{k}.json").read_text())
        assert j["first_site"] == k * n and j["sites"] == n
        assert (j["pi"], j["eps"], j["iterations"]) == (est.heterozygosity, est.error_rate, est.iterations)
        assert j["n_unique"] == u
    assert d["estimate"]["pi"] == est.heterozygosity and d["estimate"]["eps"] == est.error_rate
    # each rank's first chunk checked by the bench itself, the oracle given the
    # gathered profile table (u rows before the coverage filter)
    assert_self_checked(d, 2)
    assert all(r["profile_table_rows"] >= u for r in d["spot_check"]["ranks"])


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("config", ["C2", "C3"])
def test_shared_gpu_rehearsal_runs_the_node_cli(config):
    """N > 1 (bench.py bench_cli_node): after the timed legs the ranks write
    their texts into one file and free their GPUs; rank 0 runs build/sid
    --devices N over it (the whole node's drop-in) and the line carries it,
    with the node's CPU baseline, every rank's spot check and placement."""
    if visible_gpus() != 1:
        pytest.skip("the rehearsal case: one visible GPU")
    args = ["--gpus", "2", "--allow-shared-gpu", "--config", config, "--sites", "300000", "--steps", "1",
            "--warmup", "0", "--device-steps", "1"]
    r = run_bench(args, 500)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith('{"metric"')][0])
    cli = d["cli"]
    assert "error" not in cli and "skipped" not in cli, cli
    assert cli["devices"] == 2 and cli["sites"] == 600_000
    assert cli["cli_stats"]["sites"] == 600_000
    assert cli["sites_per_s_wall"] > 0
    # per device: its GPU's PCI id and NUMA node, the CPUs its threads were
    # bound to (none when the GPU's local CPUs are all this job has), and the
    # NUMA node of its pinned host pages (run.cpp find_placement / on_node)
    pl = cli["placement"]
    assert len(pl) == 2 and all(p["pci"] and p["device"] == 0 for p in pl)
    assert all(p["cpus"] == 0 or p["first_cpu"] >= 0 for p in pl)
    # the same run through the runtime's pageable path (SID_UPLOAD_REGISTER=0)
    assert cli["upload_pageable"]["cli_stats"]["chunks_registered"] == 0
    assert cli["cli_stats"]["chunks_registered"] > 0
    assert_self_checked(d, 2)
    # the whole node's CPU path beside it: -m local, the oracle over the same
    # file, one shard process per CPU the job may use; the Lynch path (a
    # global estimate), one oracle process on a stated sample
    import bench
    cpu = d["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["kind"] == "port" and cpu["sample"]
    if config == "C2":
        assert cpu["cores"] == bench.cpu_share(os.sched_getaffinity(0))[0]
    else:
        assert cpu["cores"] == 1 and "global" in cpu["sample"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_strong_config_value_leg():
    """C5 (bench.py bench_strong) at a small total: the rank's eighth as
    pinned host text through the value leg's engine, device_path beside it."""
    r = run_bench(["--config", "C5", "--sites", "1600000", "--steps", "2", "--warmup", "1", "--device-steps", "2",
                   "--no-extras"], 500)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith('{"metric"')][0])
    assert d["config"]["sites_per_gpu"] == 200_000 and d["config"]["sites_all_ranks"] == 200_000
    assert d["scaling"] == "weak" and d["value"] > 0
    assert d["pcie"]["text_bytes"] == d["config"]["text_bytes_rank0"] and d["pcie"]["csv_bytes"] > 0
    assert d["device_path"]["sites_per_s"] > 0 and d["roofline"]["achieved"] > 0
