"""The exact paths bench.py times, at the configs' full sizes, byte for byte
against the oracle CLI (the reference's sid.cpp + call.cpp restated in C).

C2 (BASELINE.json configs[1]): seed 2, 50M sites, -m local.  C3 (configs[2]):
seed 3, 50M sites, -R -m likelihood_ratio.  For each, the text is made by the
device generator exactly as bench.py makes it, then run through
  - the device path (bench.py `device_path`): text resident in HBM, the
    engine's defaults for it (4000 MiB chunks, the HBM hold arena; C3: the
    pass-1 parse kept for pass 2), the records copied back and written;
  - the PCIe path (bench.py `value`): the text in pinned host memory,
    128 MiB chunks, records copied into the engine's pinned host arena
    during the ingest (C2) or the emit (C3), read from there.
The oracle is call.cpp:213-289 / 62-143 and sid.cpp:84-105 restated: -m local
is per site, so its 16 line-aligned shards run in parallel and their outputs
concatenate to the one-process output; the Lynch path is global
and runs as one process (π̂, ε̂ and the iteration count are in its stderr,
compared line for line with the engine's)."""
import concurrent.futures as cf
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 50_000_000


def first_diff(a: bytes, b: bytes) -> str:
    m = min(len(a), len(b))
    x = np.frombuffer(a, np.uint8, m) != np.frombuffer(b, np.uint8, m)
    i = int(np.argmax(x)) if x.any() else m
    return f"first difference at byte {i} of {len(a)} / {len(b)}: {a[max(0, i - 80):i + 80]!r} vs " \
           f"{b[max(0, i - 80):i + 80]!r}"


def assert_same(got: bytes, want: bytes, what: str):
    if got != want:
        raise AssertionError(f"{what}: {first_diff(got, want)}")


def write_text(text, ln, path):
    step = 256 << 20
    with open(path, "wb") as f:
        for lo in range(0, ln, step):
            f.write(text[lo:min(ln, lo + step)].cpu().numpy().tobytes())


def oracle_local_sharded(oracle, host: np.ndarray, tmp, P=16):
    """The oracle CLI over P line-aligned shards in parallel; the shards'
    outputs concatenated (one header)."""
    ln = len(host)
    cuts = [0]
    for k in range(1, P):
        c = ln * k // P
        cuts.append(c + host[c:c + (1 << 20)].tobytes().find(b"\n") + 1)
    cuts.append(ln)
    paths = []
    for k in range(P):
        p = os.path.join(tmp, f"shard{k}.plp")
        host[cuts[k]:cuts[k + 1]].tofile(p)
        paths.append(p)

    def one(p):
        r = subprocess.run([oracle.CLI, p], capture_output=True, timeout=900)
        assert r.returncode == 0, r.stderr
        return r.stdout
    with cf.ThreadPoolExecutor(P) as ex:
        outs = list(ex.map(one, paths))
    hdr = outs[0][:outs[0].index(b"\n") + 1]
    return hdr + b"".join(o[len(hdr):] for o in outs)


@pytest.fixture(scope="module")
def c2(sid, gpu, oracle, tmp_path_factory):
    text, ln = gpu.synth_text_hbm(2, 30.0, 0, N)
    host = text[:ln].cpu().numpy()
    ref = oracle_local_sharded(oracle, host, str(tmp_path_factory.mktemp("c2")))
    return text, ln, ref


@pytest.mark.timeout(900)
def test_c2_device_path_equals_oracle(sid, c2):
    text, ln, ref = c2
    eng = sid.Engine(method="local", devices=1)          # bench.py device_path: engine defaults
    eng.source_device_text(text.data_ptr(), ln, keep=text)
    out, st = eng.run()
    eng.close()
    assert st.sites == N and st.chunks == 1 and st.chunks_held == 1   # (4.07 GB: one 4000 MiB chunk)
    assert_same(out, ref, "C2 device path (text in HBM, the default chunks, hold arena)")


@pytest.mark.timeout(900)
def test_c2_pcie_path_equals_oracle(sid, c2):
    import torch
    text, ln, ref = c2
    host = text[:ln].cpu().pin_memory()
    eng = sid.Engine(method="local", devices=1, device_sink=2, host_hold_bytes=int(ln * 0.6))
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    st = eng.ingest()
    eng.estimate()
    _, st2 = eng.emit()
    got = eng.records_bytes(st.chunks)
    eng.close()
    assert st.sites == N and st.chunks_held == st.chunks > 20
    assert st2.bytes_out == len(got)
    assert_same(sid.HEADER + got, ref, "C2 PCIe path (pinned host text, host arena)")


# The C3 text (seed 3, 50M sites) through the Lynch path's three callers:
# bench.py C3 (-R -m likelihood_ratio, call.cpp:62-143), C3B (-m bayes,
# call.cpp:145-211) and -R -m local (call.cpp:213-289 with the estimate,
# :223-234); the oracle runs each as one process (a global estimate), the
# three at once.
C3_METHODS = {"lr_R": (dict(method="likelihood_ratio", estimate_prior=True), ["-R", "-m", "likelihood_ratio"]),
              "bayes": (dict(method="bayes"), ["-m", "bayes"]),
              "local_R": (dict(method="local", estimate_prior=True), ["-R", "-m", "local"])}


@pytest.fixture(scope="module")
def c3(sid, gpu, oracle, tmp_path_factory):
    text, ln = gpu.synth_text_hbm(3, 30.0, 0, N)
    path = str(tmp_path_factory.mktemp("c3") / "c3.plp")
    write_text(text, ln, path)

    def one(flags):
        r = subprocess.run([oracle.CLI] + flags + [path], capture_output=True, timeout=1500)
        assert r.returncode == 0, r.stderr
        return r
    with cf.ThreadPoolExecutor(len(C3_METHODS)) as ex:
        refs = dict(zip(C3_METHODS, ex.map(one, [f for _, f in C3_METHODS.values()])))
    os.unlink(path)
    return text, ln, refs


@pytest.mark.timeout(1800)
@pytest.mark.parametrize("kind", list(C3_METHODS))
def test_c3_device_path_equals_oracle(sid, c3, capfd, kind):
    text, ln, refs = c3
    ref = refs[kind]
    eng = sid.Engine(devices=1, lanes=1, verbose=True, **C3_METHODS[kind][0])
    eng.source_device_text(text.data_ptr(), ln, keep=text)
    capfd.readouterr()
    out, st = eng.run()
    err = capfd.readouterr().err.encode()
    eng.close()
    assert st.sites == N
    assert err == ref.stderr, (err, ref.stderr)   # unique profiles, pi-hat, eps-hat, iterations
    assert_same(out, ref.stdout, f"C3 text {kind}: device path (text in HBM, kept parse for pass 2)")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", list(C3_METHODS))
def test_c3_pcie_path_equals_oracle(sid, c3, kind):
    """bench.py pcie_engine's setup: 128 MiB host chunks, records into the
    pinned host arena (pass 2)."""
    import bench
    text, ln, refs = c3
    cfg = dict(bench.CONFIGS["C3"], method=C3_METHODS[kind][0]["method"],
               R=C3_METHODS[kind][0].get("estimate_prior", False))
    host = text[:ln].cpu().pin_memory()
    eng = bench.pcie_engine(cfg, 0, N, ln)
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    st = eng.ingest()
    eng.estimate()
    _, st2 = eng.emit()
    got = eng.records_bytes(st.chunks)
    eng.close()
    assert st.chunks > 20 and st2.bytes_out == len(got)
    assert_same(sid.HEADER + got, refs[kind].stdout, f"C3 text {kind}: PCIe path (pinned host text, host arena)")


# ---- C4 / C5 (configs[3], configs[4]): the strong-scaling device path ----
# bench.py bench_strong: the rank's shard generated into HBM by
# generate_resident, then device_path's engine (device_engine) with 4000 MiB
# chunks (STRONG_RESIDENT_CHUNK_MIB).  Here the same engine with device_sink
# 0, so the records come back, at sizes that span several chunks.

@pytest.fixture(scope="module")
def bench_mod():
    import bench
    return bench


def resident_shard(bench_mod, sid, cfg, first, n):
    import torch
    return bench_mod.generate_resident(torch, sid, torch.device("cuda", 0), 0, cfg, first, n)


@pytest.fixture(scope="module")
def c5(sid, gpu, oracle, bench_mod, tmp_path_factory):
    """15M sites of C5 (seed 5, 200x, 125M-site chromosomes): ~6.3 GB of text,
    6 chunks of 1 GiB, 3 of 2 GiB or 2 of 4000 MiB; lines of ~420 B, so the
    tile parse takes its quad shape after the first chunk."""
    cfg = bench_mod.CONFIGS["C5"]
    n = 15_000_000
    text, ln = resident_shard(bench_mod, sid, cfg, 0, n)
    assert ln / n > 256
    ref = oracle_local_sharded(oracle, text[:ln].cpu().numpy(), str(tmp_path_factory.mktemp("c5")))
    return cfg, text, ln, n, ref


@pytest.mark.timeout(900)
@pytest.mark.parametrize("chunk_mib", [4000, 2048, 1024], ids=["bench-4000MiB", "2GiB", "1GiB"])
def test_c5_device_path_equals_oracle(sid, bench_mod, c5, chunk_mib):
    cfg, text, ln, n, ref = c5
    if chunk_mib == 4000:
        assert bench_mod.STRONG_RESIDENT_CHUNK_MIB == 4000   # the chunking bench_strong uses
    eng = bench_mod.device_engine(cfg, 0, chunk_mib, device_sink=0)
    eng.source_device_text(text.data_ptr(), ln, keep=text)
    out, st = eng.run()
    eng.close()
    assert st.sites == n
    assert st.chunks >= max(2, ln // (chunk_mib << 20))
    assert_same(out, ref, f"C5 device path ({chunk_mib} MiB chunks)")


@pytest.fixture(scope="module")
def c4(sid, gpu, oracle, bench_mod, tmp_path_factory):
    """60M sites of C4 (seed 4, 30x, 24 x 125M-site chromosomes) from site
    100M: the slice crosses the chr1/chr2 boundary; ~4.9 GB of text, three
    2 GiB chunks."""
    cfg = bench_mod.CONFIGS["C4"]
    first, n = 100_000_000, 60_000_000
    text, ln = resident_shard(bench_mod, sid, cfg, first, n)
    ref = oracle_local_sharded(oracle, text[:ln].cpu().numpy(), str(tmp_path_factory.mktemp("c4")))
    assert b"\nchr1,125000000," in ref and b"\nchr2,1," in ref
    return cfg, text, ln, n, ref


@pytest.mark.timeout(900)
@pytest.mark.parametrize("hold", [0, 4 << 30], ids=["held", "hold-budget-spent"])
def test_c4_device_path_equals_oracle(sid, bench_mod, c4, hold):
    """hold-budget-spent: as at C4's full size on one GPU (131 GB of records
    against a hold budget of 40% of the HBM the text leaves), the chunks past
    the budget are formatted in pass 2 from the resident text."""
    cfg, text, ln, n, ref = c4
    eng = bench_mod.device_engine(cfg, 0, 2048, device_sink=0, hold_bytes=hold)   # (three chunks: some held, some not)
    eng.source_device_text(text.data_ptr(), ln, keep=text)
    out, st = eng.run()
    eng.close()
    assert st.sites == n and st.chunks >= 3
    if hold:
        assert 0 < st.chunks_held < st.chunks
    else:
        assert st.chunks_held == st.chunks
    assert_same(out, ref, f"C4 device path (2 GiB chunks, hold {hold})")


# ---- C4 / C5 value leg (bench.py bench_strong -> pcie_leg): the shard's text
# in pinned host memory, the engine pcie_engine builds (128 MiB host chunks,
# records copied into the pinned host arena during the ingest), the records
# read back from the arena.

def pcie_records(bench_mod, sid, cfg, text, ln, n):
    host = text[:ln].cpu().pin_memory()
    eng = bench_mod.pcie_engine(cfg, 0, n, ln)
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    st = eng.ingest()
    eng.estimate()
    _, st2 = eng.emit()
    got = eng.records_bytes(st.chunks)
    eng.close()
    assert st.sites == n and st.chunks_held == st.chunks
    assert st2.bytes_out == len(got)
    return st, sid.HEADER + got


@pytest.mark.timeout(900)
def test_c5_pcie_path_equals_oracle(sid, bench_mod, c5):
    """15M sites of 200x text (6.3 GB, ~50 host chunks of 128 MiB: the quad
    parse over long lines cut by the host chunking) through the value leg's
    engine, byte for byte against the 16-shard oracle CLI."""
    cfg, text, ln, n, ref = c5
    st, got = pcie_records(bench_mod, sid, cfg, text, ln, n)
    assert st.chunks >= 10
    assert_same(got, ref, "C5 PCIe path (pinned host text, 128 MiB chunks, host arena)")


@pytest.mark.timeout(900)
def test_c4_pcie_path_equals_oracle(sid, bench_mod, c4):
    """The C4 slice across chr1/chr2 (60M sites, 4.9 GB) through the value
    leg's engine."""
    cfg, text, ln, n, ref = c4
    st, got = pcie_records(bench_mod, sid, cfg, text, ln, n)
    assert st.chunks >= 10
    assert_same(got, ref, "C4 PCIe path (pinned host text, 128 MiB chunks, host arena)")
