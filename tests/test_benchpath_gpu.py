"""The exact paths bench.py times, at the configs' full sizes, byte for byte
against the oracle CLI (the reference's sid.cpp + call.cpp restated in C).

C2 (BASELINE.json configs[1]): seed 2, 50M sites, -m local.  C3 (configs[2]):
seed 3, 50M sites, -R -m likelihood_ratio.  For each, the text is made by the
device generator exactly as bench.py makes it, then run through
  - the device path (bench.py `device_path`): text resident in HBM, the
    engine's defaults for it (2 GiB chunks, the HBM hold arena; C3: the
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
    assert st.sites == N and st.chunks == 2 and st.chunks_held == 2
    assert_same(out, ref, "C2 device path (text in HBM, 2 GiB chunks, hold arena)")


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


@pytest.fixture(scope="module")
def c3(sid, gpu, oracle, tmp_path_factory):
    text, ln = gpu.synth_text_hbm(3, 30.0, 0, N)
    path = str(tmp_path_factory.mktemp("c3") / "c3.plp")
    write_text(text, ln, path)
    r = subprocess.run([oracle.CLI, "-R", "-m", "likelihood_ratio", path], capture_output=True, timeout=1200)
    assert r.returncode == 0, r.stderr
    os.unlink(path)
    return text, ln, r


@pytest.mark.timeout(1200)
def test_c3_device_path_equals_oracle(sid, c3, capfd):
    text, ln, ref = c3
    eng = sid.Engine(method="likelihood_ratio", estimate_prior=True, devices=1, lanes=1, verbose=True)
    eng.source_device_text(text.data_ptr(), ln, keep=text)
    capfd.readouterr()
    out, st = eng.run()
    err = capfd.readouterr().err.encode()
    eng.close()
    assert st.sites == N
    assert err == ref.stderr, (err, ref.stderr)   # unique profiles, pi-hat, eps-hat, iterations
    assert_same(out, ref.stdout, "C3 device path (text in HBM, kept parse for pass 2)")


@pytest.mark.timeout(900)
def test_c3_pcie_path_equals_oracle(sid, c3):
    text, ln, ref = c3
    host = text[:ln].cpu().pin_memory()
    eng = sid.Engine(method="likelihood_ratio", estimate_prior=True, devices=1, device_sink=2,
                     host_hold_bytes=int(ln * 0.6))
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    st = eng.ingest()
    eng.estimate()
    eng.emit()
    got = eng.records_bytes(st.chunks)
    eng.close()
    assert_same(sid.HEADER + got, ref.stdout, "C3 PCIe path (pinned host text, host arena in pass 2)")
