"""bench.py's CPU-side legs on the CPU (no GPU): the per-rank spot check of the
value leg's records against the oracle (spot_check_ranks) and the CPU
baseline (bench_cpu: the oracle port and the reference-sources harness), with
the rank's text as a CPU tensor -- so a broken CPU leg fails here, not in the
round's GPU run."""
import os
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class OneRank:
    rank, world, dist = 0, 1, None

    def gather(self, obj):
        return [obj]


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


@pytest.fixture(scope="module")
def text_c3(sid):
    import torch
    n = 30_000
    text = sid.synth_text(3, n, 30.0)
    return n, text, torch.from_numpy(np.frombuffer(text, np.uint8).copy())


def records_of(oracle, tmp_path, flags, text, env=None):
    p = tmp_path / "t.plp"
    p.write_bytes(text)
    r = oracle.run_cli(flags + [str(p)], env=env)
    assert r.returncode == 0
    return r.stdout


@pytest.mark.parametrize("config", ["C2", "C3", "C3B"])
def test_spot_check_ranks(bench, sid, oracle, tmp_path, text_c3, config):
    """The records of a prefix of the rank's text (as the engine's first chunk
    holds them) pass; the Lynch paths with the whole text's profile table
    (the records of the whole run, cut at a site); a changed byte fails."""
    n, text, t = text_c3
    cfg = bench.CONFIGS[config]
    flags = bench.method_flags(cfg)
    whole = records_of(oracle, tmp_path, flags, text)
    rows = whole.split(b"\n")[1:-1]
    spot = b"".join(r + b"\n" for r in rows[: len(rows) // 3])
    table = None
    if config != "C2":
        keys, cnt = np.unique(sid.profile_key(sid.synth_counts_host(3, n, 30.0)), return_counts=True)
        table = (keys, cnt.astype(np.uint64))
    a = types.SimpleNamespace(pcie_chunk_mib=0)
    res = bench.spot_check_ranks(OneRank(), a, cfg, t, len(text), spot, table)
    assert res["ranks_equal"] is True and res["ranks"][0]["records"] == len(rows) // 3
    bad = bytearray(spot)
    bad[len(bad) // 2] ^= 1
    with pytest.raises(SystemExit):
        bench.spot_check_ranks(OneRank(), a, cfg, t, len(text), bytes(bad), table)


@pytest.mark.parametrize("config", ["C2", "C3"])
def test_bench_cpu(bench, oracle, text_c3, config):
    """The CPU baseline leg on a small text: the port's value (16-shard -m
    local, one process for the Lynch path) and, for -m local, the
    reference-sources figures with the port/reference ratios."""
    n, text, t = text_c3
    cfg = bench.CONFIGS[config]
    cpus = os.sched_getaffinity(0)
    res = bench.bench_cpu(cfg, t, len(text), n, cpus, sample_sites=20_000)
    assert res["value"] > 0 and res["kind"] == "port"
    if config == "C2":
        assert res["cores"] == bench.cpu_share(cpus)[0] and res["single_core"]["value"] > 0
        if oracle.ref_pileup_available():
            rs = res["reference_sources"]
            assert rs["value"] > 0 and rs["single_core"]["value"] > 0
            assert rs["port_over_reference"]["single_core"] > 0
    else:
        assert res["cores"] == 1 and "global" in res["sample"]
