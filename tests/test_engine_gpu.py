"""The streaming engine (run.cpp, sid_engine_*) against the oracle CLI (the
reference's sid.cpp/call.cpp restated): many small chunks over several
devices, the hold / retain fallbacks of the two-pass flow, first-error
semantics across chunks, every kind of source, and a slice of the C4 layout
(seed 4, 24 x 125M-site chromosomes) spanning a chromosome boundary."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def run(exe, args, **kw):
    return subprocess.run([exe] + list(args), capture_output=True, timeout=600, **kw)


@pytest.fixture(scope="module")
def inputs(sid, tmp_path_factory):
    d = tmp_path_factory.mktemp("engine")
    paths = {"c1": os.path.join(GOLD, "c1_10k.plp"), "edge": os.path.join(GOLD, "edge.plp")}
    p = d / "deep.plp"
    p.write_bytes(sid.synth_text(5, 3000, 200.0, sites_per_chrom=1000))
    paths["deep"] = str(p)
    q = d / "q30.plp"
    q.write_bytes(sid.synth_text(7, 20_000, 30.0, sites_per_chrom=7000, mapq=True))
    paths["quality"] = str(q)
    return paths


FLAGS = [[], ["-R", "-m", "likelihood_ratio"], ["-m", "bayes"], ["-R", "-m", "local"],
         ["-E", "0.05", "-p", "0.01", "-r", "0.001"]]


@pytest.mark.parametrize("extra", [["--chunk-bytes", "4096"], ["--chunk-bytes", "65536", "--devices", "3"],
                                   ["--chunk-bytes", "3000", "--devices", "2"]], ids=lambda e: " ".join(e))
@pytest.mark.parametrize("flags", FLAGS, ids=lambda f: " ".join(f) or "default")
@pytest.mark.parametrize("name", ["c1", "edge", "deep"])
def test_chunked_cli_matches_oracle(sid, oracle, inputs, name, flags, extra):
    a = run(sid.CLI_PATH, extra + flags + [inputs[name]])
    b = oracle.run_cli(flags + [inputs[name]])
    assert a.returncode == b.returncode == 0, a.stderr
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


@pytest.mark.parametrize("extra", [["--chunk-bytes", "300000"], ["--chunk-bytes", "1000000", "--devices", "2"]],
                         ids=["300k", "1m-2dev"])
def test_tile_parse_quad_shape(sid, oracle, tmp_path, extra):
    """The quad shape (lines over 256 B on average: a quad of lanes per line,
    24 KiB tiles, at most 256 slots a tile) and its way out
    (run.cpp Dev::tile_set): 200x text, then depth-0 lines (~1200 a tile:
    past the quad list, so the next chunks take the lane shape), 200x text
    again (back to quads), 30x text, and 200x lines with reads over the halo.
    Every run's CSV is the oracle's."""
    deep = sid.synth_text(62, 6_000, 200.0, sites_per_chrom=10 ** 6)
    normal = sid.synth_text(63, 6_000, 30.0, sites_per_chrom=10 ** 6)
    zero = b"".join(b"chr2\t%d\tA\t0\t*\t*\n" % i for i in range(1, 30_000))
    rng = np.random.default_rng(62)
    alphabet = np.frombuffer(b"ACGTacgt.,$", np.uint8)
    longl = b"".join(b"chr3\t%d\tG\t600\t%s\t%s\n" % (i, rng.choice(alphabet, 600 + 3 * i).tobytes(),
                                                        b"I" * (600 + 3 * i)) for i in range(1, 400))
    text = deep + zero + deep + normal + longl + deep
    p = tmp_path / "quad.plp"
    p.write_bytes(text)
    b = oracle.run_cli([str(p)])
    a = run(sid.CLI_PATH, extra + [str(p)])
    assert b.returncode == 0
    assert a.returncode == 0, a.stderr[-400:]
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


@pytest.mark.parametrize("extra", [["--chunk-bytes", "200000"], ["--chunk-bytes", "1000000", "--devices", "2"]],
                         ids=["200k", "1m-2dev"])
def test_tile_fixups_and_general_routine(sid, oracle, tmp_path, extra):
    """Sites no class table covers (four alleles in numbers: the fix-up,
    textpath.hip fix_site) in both tile shapes, from the fast path (the tile
    parse lists them) and from the general routine (a '+'/'-' indel in the
    read bases: sid_tile_serial_kernel fixes them up itself), mixed with
    covered sites and lines of every other kind; the CSV is the oracle's."""
    rng = np.random.default_rng(64)

    def lines(chrom, n, depth, indel_every):
        out = []
        for i in range(1, n + 1):
            k = rng.integers(0, 4, 4) * (depth // 8) + rng.integers(0, 3, 4)
            bases = bytearray(b"A" * int(k[0]) + b"c" * int(k[1]) + b"G" * int(k[2]) + b"t" * int(k[3]) +
                              b"." * int(rng.integers(0, depth // 2)))
            rng.shuffle(bases)
            if indel_every and i % indel_every == 0:
                bases[len(bases) // 2:len(bases) // 2] = b"+2AC"
            if i % 7 == 0:
                bases[0:0] = b"^I"
            b = bytes(bases) or b"*"
            out.append(b"%s\t%d\tA\t%d\t%s\t%s\n" % (chrom, i, len(b), b, b"I" * len(b)))
        return b"".join(out)

    text = (lines(b"chr1", 3000, 40, 5) + sid.synth_text(65, 3000, 30.0, sites_per_chrom=10 ** 6) +
            lines(b"chr2", 1500, 1200, 4) + sid.synth_text(66, 2000, 200.0, sites_per_chrom=10 ** 6) +
            lines(b"chr3", 2000, 40, 0))
    p = tmp_path / "fixups.plp"
    p.write_bytes(text)
    b = oracle.run_cli([str(p)])
    a = run(sid.CLI_PATH, extra + [str(p)])
    assert b.returncode == 0
    assert a.returncode == 0, a.stderr[-400:]
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


@pytest.mark.parametrize("extra", [["--hold-bytes", "1"], ["--hold-bytes", "1", "--retain-bytes", "1"],
                                   ["--hold-bytes", "200000", "--retain-bytes", "150000"]],
                         ids=["all-in-pass-2-kept", "all-reloaded", "mixed"])
@pytest.mark.parametrize("flags", [[], ["-R", "-m", "likelihood_ratio"], ["-m", "quality"],
                                   ["-R", "-m", "quality"]], ids=lambda f: " ".join(f) or "default")
def test_hold_and_retain_fallbacks(sid, oracle, inputs, flags, extra):
    """Records that do not fit the hold budget are formatted in the second
    pass, from text kept in HBM or read again from the file."""
    name = "quality" if "quality" in flags else "c1"
    args = ["--chunk-bytes", "32768", "--devices", "2"] + extra + flags + [inputs[name]]
    a = run(sid.CLI_PATH, ["--stats"] + args)
    b = oracle.run_cli(flags + [inputs[name]])
    assert a.returncode == b.returncode == 0, a.stderr
    assert a.stdout == b.stdout
    lines = a.stderr.splitlines(keepends=True)   # --stats: the last stderr line
    assert b"".join(lines[:-1]) == b.stderr
    st = json.loads(lines[-1])
    assert st["chunks"] > 4
    lynch = "-R" in flags or "likelihood_ratio" in flags
    if lynch or extra[1] == "1":
        assert st["chunks_held"] == 0
    if extra == ["--hold-bytes", "1", "--retain-bytes", "1"]:
        assert st["chunks_retained"] == 0 and st["chunks_reloaded"] == st["chunks"]
    if extra == ["--hold-bytes", "1"]:
        # text is kept once the hold budget is seen to be spent; the chunks
        # already uploaded by then are read again
        assert st["chunks_retained"] > 0
        assert st["chunks_retained"] + st["chunks_reloaded"] == st["chunks"]


def test_quality_chunked(sid, oracle, inputs):
    for extra in (["--chunk-bytes", "8192"], ["--chunk-bytes", "50000", "--devices", "3"]):
        for flags in ([ "-m", "quality"], ["-m", "quality", "-r", "0.01", "-p", "0.2"]):
            a = run(sid.CLI_PATH, extra + flags + [inputs["quality"]])
            b = oracle.run_cli(flags + [inputs["quality"]])
            assert a.returncode == b.returncode == 0, a.stderr
            assert a.stdout == b.stdout, (extra, flags)


def test_first_error_in_a_late_chunk(sid, oracle, tmp_path):
    good = b"".join(b"chr1\t%d\tA\t3\t.,.\tIII\n" % i for i in range(1, 3000))
    cases = {
        "malformed_late": good * 3 + b"chr1\t1\tAC\t3\t...\tIII\n" + good + b" \t\n" + good,
        "blank_first": good + b" \t\n" + good * 2 + b"chr1\t1\tAC\t3\t...\tIII\n" + good,
        "last_line": good * 4 + b"chr1\t9\tA",
    }
    for tag, text in cases.items():
        p = tmp_path / f"{tag}.plp"
        p.write_bytes(text)
        b = oracle.run_cli([str(p)])
        for extra, flags in ((["--chunk-bytes", "4096"], []), (["--chunk-bytes", "10000", "--devices", "4"], []),
                             (["--chunk-bytes", "4096"], ["-R", "-m", "likelihood_ratio"]),
                             (["--chunk-bytes", "4096", "--devices", "3"], ["-m", "quality"])):
            bb = oracle.run_cli(flags + [str(p)]) if flags else b
            a = run(sid.CLI_PATH, extra + flags + [str(p)])
            assert a.returncode == bb.returncode, (tag, extra, a.returncode, bb.returncode)
            assert a.stdout == bb.stdout, (tag, extra)
            assert a.stderr == bb.stderr, (tag, extra)


def test_dense_short_lines(sid, oracle, tmp_path):
    """More than 2048 line starts in a 16 KiB index tile (lines of a few bytes,
    all malformed): the offset emit stores them directly instead of through
    its LDS buffer (textpath.hip EMIT_CAP), and the first malformed line is
    still the first of them."""
    good = b"".join(b"chr1\t%d\tA\t3\t.,.\tIII\n" % i for i in range(1, 2000))
    cases = {"x": good * 2 + b"x\n" * 9000 + good, "tabs": good + b"1\t2\n" * 5000 + good * 2,
             "short_first": b"ab\n" * 6000 + good}
    for tag, text in cases.items():
        p = tmp_path / f"{tag}.plp"
        p.write_bytes(text)
        for extra, flags in (([], []), (["--chunk-bytes", "20000", "--devices", "2"], []),
                             (["--chunk-bytes", "20000"], ["-R", "-m", "likelihood_ratio"])):
            b = oracle.run_cli(flags + [str(p)])
            a = run(sid.CLI_PATH, extra + flags + [str(p)])
            assert a.returncode == b.returncode != 0, (tag, extra, a.returncode, b.returncode)
            assert a.stdout == b.stdout, (tag, extra)
            assert a.stderr == b.stderr, (tag, extra)


def test_bayes_without_coverage_prints_the_header(sid, oracle, tmp_path):
    """callBayes on a file where no profile reaches coverage 4: the estimate
    runs on an empty table, no record survives, exit 0 (call.cpp:145-211)."""
    p = tmp_path / "low.plp"
    p.write_bytes(b"chr1\t1\tA\t2\t..\tII\nchr1\t2\tC\t3\t,,G\tIII\n")
    for extra in ([], ["--devices", "2"], ["--host-parse"]):
        a = run(sid.CLI_PATH, extra + ["-m", "bayes", str(p)])
        b = oracle.run_cli(["-m", "bayes", str(p)])
        assert b.returncode == 0, b.stderr
        assert a.returncode == 0, (extra, a.stderr)
        assert a.stdout == b.stdout == b"chrom,pos,label,gt,hom_conf,het_conf,conf_type\n"
        assert a.stderr == b.stderr


def test_stdin_pipe(sid, oracle, inputs):
    data = open(inputs["c1"], "rb").read()
    a = subprocess.run([sid.CLI_PATH, "--chunk-bytes", "5000", "/dev/stdin"], input=data, capture_output=True,
                       timeout=120)
    b = oracle.run_cli([inputs["c1"]])
    assert a.returncode == 0, a.stderr
    assert a.stdout == b.stdout


def engine_csv(sid, method, source, text, n=None, seed=None, depth=30.0, first=0, spc=0, **kw):
    eng = sid.Engine(method=method, **kw)
    if source == "text":
        eng.source_text(text)
    elif source == "device":
        import torch
        buf = torch.zeros(len(text) + 512, dtype=torch.uint8, device="cuda")
        buf[: len(text)] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        eng.source_device_text(buf.data_ptr(), len(text), keep=buf)
    elif source in ("synth_host", "synth_device"):
        eng.source_synth(seed, n, depth, first=first, sites_per_chrom=spc, sites_per_chunk=kw.get("per", 0),
                         on_device=source == "synth_device")
    out, st = eng.run()
    eng.close()
    return out, st


@pytest.mark.parametrize("source", ["text", "device", "synth_host", "synth_device"])
@pytest.mark.parametrize("method", ["local", "likelihood_ratio"])
def test_engine_sources_agree_with_oracle(sid, oracle, tmp_path, source, method):
    n, seed, depth, spc = 60_000, 11, 30.0, 25_000
    text = sid.synth_text(seed, n, depth, first=5, sites_per_chrom=spc)
    p = tmp_path / "s.plp"
    p.write_bytes(text)
    flags = [] if method == "local" else ["-R", "-m", method]
    ref = oracle.run_cli(flags + [str(p)])
    assert ref.returncode == 0
    out, st = engine_csv(sid, method, source, text, n=n, seed=seed, depth=depth, first=5, spc=spc,
                         chunk_bytes=1 << 20, estimate_prior=method != "local")
    assert st.sites == n
    assert st.chunks >= 4
    assert out == ref.stdout


def test_engine_file_source_and_reuse(sid, oracle, tmp_path):
    text = sid.synth_text(12, 40_000, 30.0, sites_per_chrom=15_000)
    p = tmp_path / "f.plp"
    p.write_bytes(text)
    ref = oracle.run_cli([str(p)]).stdout
    eng = sid.Engine(chunk_bytes=300_000)
    with open(p, "rb") as f:
        for _ in range(2):   # an engine is reusable
            eng.source_file(f.fileno())
            out, st = eng.run()
            assert out == ref
            assert st.chunks > 5
    eng.source_text(text)
    assert eng.run()[0] == ref
    eng.close()


def test_engine_device_sink_counts_the_same_records(sid, oracle):
    text = sid.synth_text(13, 30_000, 30.0)
    eng = sid.Engine(chunk_bytes=1 << 18, device_sink=True)
    eng.source_text(text)
    st = eng.ingest()
    eng.estimate()
    out, st2 = eng.emit()
    assert out == b"" and st.sites == 30_000 and st.chunks_held == st.chunks
    eng.close()


@pytest.mark.parametrize("depth,n", [(200.0, 4000), (30.0, 1)])
def test_device_generator_equals_host_text(sid, depth, n):
    """The device text generator writes the bytes of sid_synth_text."""
    import torch
    text = sid.synth_text(5, n, depth, first=777, sites_per_chrom=1000)
    eng = sid.Engine(device_sink=False, chunk_bytes=1 << 20)
    eng.source_synth(5, n, depth, first=777, sites_per_chrom=1000, on_device=True)
    out_dev, _ = eng.run()
    eng.source_text(text)
    out_txt, _ = eng.run()
    assert out_dev == out_txt
    eng.close()


def test_c4_layout_slice_across_devices(sid, oracle, tmp_path):
    """C4 (seed 4, 24 chromosomes x 125,000,000 sites): a 2M-site slice that
    spans the chr1/chr2 boundary, through the CLI on 8 (logical) devices in
    4 MiB chunks, byte for byte against the oracle CLI."""
    spc = 125_000_000
    first, n = spc - 1_000_000, 2_000_000
    p = tmp_path / "c4_slice.plp"
    with open(p, "wb") as f:
        for lo in range(0, n, 500_000):
            f.write(sid.synth_text(4, min(500_000, n - lo), 30.0, first=first + lo, sites_per_chrom=spc))
    ref = oracle.run_cli([str(p)])
    assert ref.returncode == 0
    assert b"\nchr1,125000000," in ref.stdout and b"\nchr2,1," in ref.stdout
    a = run(sid.CLI_PATH, ["--devices", "8", "--chunk-bytes", str(4 << 20), str(p)])
    assert a.returncode == 0, a.stderr
    assert a.stdout == ref.stdout


@pytest.mark.parametrize("lanes,source", [(2, "text"), (3, "device"), (2, "synth_device")])
@pytest.mark.parametrize("method", ["local", "likelihood_ratio"])
def test_engine_lanes_agree_with_oracle(sid, oracle, tmp_path, lanes, source, method):
    """Several pipelines per GPU (own streams, contexts, workspaces; chunks
    dealt over all of them; the Lynch histograms of the lanes merged) write the
    oracle's CSV, in file order."""
    n, seed, depth, spc = 50_000, 21, 30.0, 20_000
    text = sid.synth_text(seed, n, depth, first=3, sites_per_chrom=spc)
    p = tmp_path / "l.plp"
    p.write_bytes(text)
    flags = [] if method == "local" else ["-R", "-m", method]
    ref = oracle.run_cli(flags + [str(p)])
    assert ref.returncode == 0
    out, st = engine_csv(sid, method, source, text, n=n, seed=seed, depth=depth, first=3, spc=spc,
                         chunk_bytes=256 << 10, estimate_prior=method != "local", lanes=lanes)
    assert st.sites == n and st.chunks >= 2 * lanes
    assert out == ref.stdout


@pytest.mark.parametrize("namelen", [12, 40, 70])
def test_engine_long_chrom_names(sid, oracle, tmp_path, namelen):
    """Chrom names past the parse's 8 kept bytes (the formatter reads them from
    the text), records past a formatter tile's 32 KiB LDS buffer (512 sites of
    >64 B: stored straight to global memory), and headers past the parse's 48
    staged bytes (70: the general routine) -- byte for byte against the oracle."""
    n = 30_000
    text = sid.synth_text(31, n, 30.0, sites_per_chrom=7_000)
    lines = text.split(b"\n")
    out = []
    for ln in lines:
        if not ln:
            out.append(ln)
            continue
        chrom, rest = ln.split(b"\t", 1)
        name = (b"scaffold_" + chrom + b"_" + b"x" * namelen)[:namelen]
        out.append(name + b"\t" + rest)
    text = b"\n".join(out)
    p = tmp_path / "long.plp"
    p.write_bytes(text)
    for flags in ([], ["-R", "-m", "likelihood_ratio"]):
        ref = oracle.run_cli(flags + [str(p)])
        assert ref.returncode == 0
        got, st = engine_csv(sid, "local" if not flags else "likelihood_ratio", "text", text,
                             chunk_bytes=1 << 20, estimate_prior=bool(flags))
        assert st.sites == n
        assert got == ref.stdout


@pytest.mark.parametrize("hh", ["67108864", "150000", "1"], ids=["fits", "fills-midway", "too-small"])
@pytest.mark.parametrize("flags", [[], ["-R", "-m", "likelihood_ratio"], ["-m", "quality"], ["-m", "bayes"]],
                         ids=lambda f: " ".join(f) or "default")
def test_host_hold_cli_matches_oracle(sid, oracle, inputs, flags, hh):
    """--host-hold (sid_engine_cfg.host_hold_bytes): -m local / quality copy
    every chunk's records into pinned host memory during the ingest (the
    Lynch paths in the emit, instead of the pinned ring); chunks beyond the
    arena fall back to the HBM hold.  Byte for byte the oracle's output."""
    name = "quality" if "quality" in flags else "c1"
    for extra in (["--chunk-bytes", "32768"], ["--chunk-bytes", "50000", "--devices", "3"],
                  ["--chunk-bytes", "40000", "--hold-bytes", "1"]):
        a = run(sid.CLI_PATH, ["--stats", "--host-hold", hh] + extra + flags + [inputs[name]])
        b = oracle.run_cli(flags + [inputs[name]])
        assert a.returncode == b.returncode == 0, a.stderr
        assert a.stdout == b.stdout, (extra, hh)
        lines = a.stderr.splitlines(keepends=True)
        assert b"".join(lines[:-1]) == b.stderr
        st = json.loads(lines[-1])
        local = not ("-R" in flags or "likelihood_ratio" in flags or "bayes" in flags)
        if local and hh != "1":
            assert st["chunks_held"] > 0


def test_host_hold_first_error(sid, oracle, tmp_path):
    good = b"".join(b"chr1\t%d\tA\t3\t.,.\tIII\n" % i for i in range(1, 3000))
    p = tmp_path / "bad.plp"
    p.write_bytes(good * 3 + b"chr1\t1\tAC\t3\t...\tIII\n" + good)
    b = oracle.run_cli([str(p)])
    for extra in (["--chunk-bytes", "4096"], ["--chunk-bytes", "10000", "--devices", "2"]):
        a = run(sid.CLI_PATH, ["--host-hold", str(1 << 24)] + extra + [str(p)])
        assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)


@pytest.mark.parametrize("method", ["local", "likelihood_ratio"])
def test_engine_host_arena_records(sid, oracle, tmp_path, method):
    """device_sink 2 + host_hold_bytes (bench.py's PCIe-inclusive step): the
    records land in the engine's pinned host arena, in file order, equal to
    the oracle's CSV; an engine run twice reuses the arena."""
    import torch
    n, seed, spc = 80_000, 17, 30_000
    text = sid.synth_text(seed, n, 30.0, sites_per_chrom=spc)
    p = tmp_path / "h.plp"
    p.write_bytes(text)
    flags = [] if method == "local" else ["-R", "-m", method]
    ref = oracle.run_cli(flags + [str(p)])
    assert ref.returncode == 0
    host = torch.frombuffer(bytearray(text), dtype=torch.uint8).pin_memory()
    eng = sid.Engine(method=method, estimate_prior=method != "local", device_sink=2, chunk_bytes=1 << 20,
                     host_hold_bytes=len(text))
    eng.source_host_ptr(host.data_ptr(), len(text), keep=host)
    for _ in range(2):
        st = eng.ingest()
        eng.estimate()
        _, st2 = eng.emit()
        assert st.sites == n and st.chunks >= 4
        got = eng.records_bytes(st.chunks)
        assert st2.bytes_out == len(got)
        assert sid.HEADER + got == ref.stdout
    eng.close()


def test_engine_profile_exchange_api(sid, oracle, tmp_path):
    """sid_engine_profile_table / _load: the multi-rank Lynch exchange with
    several pipelines per rank -- two engines over the two halves of a text,
    each exporting its merged table, each loading the sum; the estimate is
    not merged again (a second estimate() gives the same answer)."""
    n = 60_000
    text = sid.synth_text(23, n, 30.0)
    cut = text.index(b"\n", len(text) // 2) + 1
    p = tmp_path / "x.plp"
    p.write_bytes(text)
    ref = oracle.run_cli(["-R", "-m", "likelihood_ratio", str(p)])
    engs = []
    for part in (text[:cut], text[cut:]):
        e = sid.Engine(method="likelihood_ratio", estimate_prior=True, devices=2, chunk_bytes=1 << 18)
        e.source_text(part)
        e.ingest()
        engs.append(e)
    tabs = [e.profile_table() for e in engs]
    keys = np.concatenate([t[0] for t in tabs])
    cnts = np.concatenate([t[1] for t in tabs])
    outs = []
    for e in engs:
        e.profile_load(keys, cnts)
        est = e.estimate()
        est2 = e.estimate()
        assert (est.heterozygosity, est.error_rate, est.n_unique) == \
            (est2.heterozygosity, est2.error_rate, est2.n_unique)
        outs.append(e.emit(header=None)[0])
        e.close()
    assert sid.HEADER + b"".join(outs) == ref.stdout


def test_source_file_range_past_eof(sid, tmp_path):
    p = tmp_path / "short.plp"
    p.write_bytes(b"chr1\t1\tA\t1\t.\tI\n")
    eng = sid.Engine()
    with open(p, "rb") as f:
        with pytest.raises(sid.SidError):
            eng.source_file(f.fileno(), 0, 1 << 20)
    eng.close()


@pytest.mark.parametrize("method", ["local", "quality"])
def test_stale_ring_slot_behind_a_last_line_without_newline(sid, oracle, tmp_path, method):
    """One ring slot (every chunk uploads into the same device buffer): the
    short last chunk, whose last line has no trailing newline, sits in front
    of the previous, longer chunk's stale lines.  Every kernel bounds its reads
    by the chunk's end (sid_internal.h), so no stale line is indexed or parsed
    and no stale byte joins the last line's fields (call.cpp:11-20 reads the
    last line without its newline)."""
    n = 40_000
    text = sid.synth_text(41, n, 30.0, sites_per_chrom=15_000, mapq=method == "quality")
    C = len(text) * 10 // 43   # 4.3 chunks: the last one ~0.3 of the others
    text = text.rstrip(b"\n")
    p = tmp_path / "nonl.plp"
    p.write_bytes(text)
    flags = ["-m", method] if method != "local" else []
    ref = oracle.run_cli(flags + [str(p)])
    assert ref.returncode == 0
    eng = sid.Engine(method=method, slots=1, chunk_bytes=C)
    eng.source_text(text)
    for _ in range(2):
        out, st = eng.run()
        assert st.sites == n and st.chunks == 5
        assert out == ref.stdout
    eng.close()


def test_arena_allocation_failure_falls_back(sid, oracle, tmp_path):
    """The hold arena's allocation failing (HBM taken by another allocation,
    a hold budget the GPU cannot meet) is not an error: the chunks are
    formatted in pass 2.  The failed hipMalloc must not leave the runtime's
    sticky last error behind for the next launch check on the compute thread
    (run.cpp DevPool::get / Dev::arena_reserve); the CSV equals the oracle's."""
    import torch
    n = 300_000
    text = sid.synth_text(43, n, 30.0, sites_per_chrom=100_000)
    p = tmp_path / "oom.plp"
    p.write_bytes(text)
    ref = oracle.run_cli([str(p)])
    assert ref.returncode == 0
    eng = sid.Engine(method="local", chunk_bytes=1 << 20, hold_bytes=64 << 30)
    eng.source_text(text)
    free, _ = torch.cuda.mem_get_info()
    leave = 2 << 30   # the arena asks for a 4 GiB segment: it cannot get one
    filler = torch.empty(max(0, free - leave), dtype=torch.uint8, device="cuda")
    try:
        out, st = eng.run()
    finally:
        del filler
        torch.cuda.empty_cache()
    eng.close()
    assert st.sites == n and st.chunks > 10
    assert st.chunks_held == 0   # every chunk formatted in pass 2
    assert out == ref.stdout


@pytest.mark.parametrize("source", ["text", "device", "synth_device"])
def test_device_sink_formats_past_the_hold_budget_once(sid, source):
    """The device sink (records formatted into HBM and dropped) formats every
    -m local chunk in pass 1: past the hold budget into a scratch buffer,
    counted and dropped (run.cpp sink_all_pass1), so no chunk is indexed and
    parsed a second time.  Its byte count equals the CSV the same engine
    writes with a real sink, whose chunks past the budget take pass 2."""
    import torch
    n = 200_000
    text = sid.synth_text(47, n, 30.0, sites_per_chrom=70_000)
    kw = dict(chunk_bytes=1 << 20, hold_bytes=3 << 20)
    ref, st_ref = engine_csv(sid, "local", source, text, n=n, seed=47, spc=70_000, **kw)
    assert 0 < st_ref.chunks_held < st_ref.chunks   # the written run: chunks past the budget in pass 2
    eng = sid.Engine(device_sink=True, **kw)
    if source == "text":
        eng.source_text(text)
    elif source == "device":
        buf = torch.zeros(len(text) + 512, dtype=torch.uint8, device="cuda")
        buf[: len(text)] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
        eng.source_device_text(buf.data_ptr(), len(text), keep=buf)
    else:
        eng.source_synth(47, n, 30.0, sites_per_chrom=70_000, on_device=True)
    eng.profile(True)
    for _ in range(2):
        st = eng.ingest()
        eng.estimate()
        out, st2 = eng.emit()
        assert out == b"" and st.sites == n
        assert st.chunks_held == st.chunks and st2.chunks_reloaded == 0
        assert st2.bytes_out == len(ref) - len(sid.HEADER)
    prof = eng.profile_read()
    assert prof["chunks"] == 2 * st.chunks   # one index + parse per chunk and run
    eng.close()


@pytest.fixture(scope="module")
def pageable_30mb(sid, oracle, tmp_path_factory):
    """~30 MB of 30x text as a file, and the oracle's CSV of it."""
    d = tmp_path_factory.mktemp("reg")
    text = sid.synth_text(51, 370_000, 30.0, sites_per_chrom=150_000)
    p = d / "reg.plp"
    p.write_bytes(text)
    ref = oracle.run_cli([str(p)])
    assert ref.returncode == 0
    return text, str(p), ref.stdout


@pytest.mark.parametrize("register", ["1", "0"])
@pytest.mark.parametrize("devices", ["1", "2"])
@pytest.mark.parametrize("chunk", [3 << 20, (8 << 20) - 12345])
def test_registered_uploads_cli(sid, pageable_30mb, register, devices, chunk):
    """The CLI over a regular file uploads each chunk from its page-aligned
    body registered for DMA, its partial first and last pages through the
    runtime's pageable path (run.cpp UploadReg), chunks dealt over the
    devices; SID_UPLOAD_REGISTER=0 is the pageable path for everything.  Both
    write the oracle's CSV, and --stats says which path ran."""
    text, path, ref = pageable_30mb
    a = run(sid.CLI_PATH, ["--stats", "--chunk-bytes", str(chunk), "--devices", devices, path],
            env=dict(os.environ, SID_UPLOAD_REGISTER=register))
    assert a.returncode == 0, a.stderr[-400:]
    assert a.stdout == ref
    st = json.loads(a.stderr.splitlines()[-1])
    assert st["chunks"] >= 4
    if register == "1":
        # every chunk whose page-aligned body is at least 1 MiB (all but
        # perhaps a short last one)
        assert st["chunks_registered"] >= st["chunks"] - 1
        assert st["register_s"] > 0
    else:
        assert st["chunks_registered"] == 0
    assert st["h2d_bytes"] == len(text) and st["h2d_s"] > 0


def test_registered_uploads_engine_bytes(sid, pageable_30mb):
    """The same through the engine from host bytes the caller did not pin
    (not page-aligned: chunk 0 has a pageable head too)."""
    text, _, ref = pageable_30mb
    for devices in (1, 2):
        eng = sid.Engine(chunk_bytes=(5 << 20) + 7, devices=devices)
        eng.source_text(text)
        out, st = eng.run()
        eng.close()
        assert out == ref
        assert st.chunks >= 5 and st.chunks_registered >= st.chunks - 1
        assert st.h2d_bytes == len(text)


def test_line_past_the_chunk_limit_is_refused(sid):
    """Line offsets on the device are 32-bit: a line that carries a chunk past
    4 GiB is refused with SID_ELINE (its own message), not mis-parsed."""
    import torch
    n = (4 << 30) + (2 << 20)
    buf = torch.full((n + 512,), ord("A"), dtype=torch.uint8, device="cuda")
    buf[n - 1] = ord("\n")
    buf[n:] = 0
    torch.cuda.synchronize()
    eng = sid.Engine(chunk_bytes=64 << 20)
    eng.source_device_text(buf.data_ptr(), n, keep=buf)
    with pytest.raises(sid.SidError) as ei:
        eng.ingest()
    assert ei.value.status == 13
    assert b"too long" in sid.lib().sid_strerror(13)
    eng.close()
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("extra", [[], ["--chunk-bytes", "100000", "--devices", "2"], ["--chunk-bytes", "33333"],
                                   ["--host-hold", "1000000000", "--chunk-bytes", "250000"]],
                         ids=["one-chunk", "100k-2dev", "33k", "host-arena"])
def test_tile_parse_slot_caps(sid, oracle, tmp_path, extra):
    """-m local's tile parse (textpath.hip sid_tile_parse_kernel) lays its
    sites out in slots per 20 KiB tile, as many as the device's last chunk
    needed (run.cpp Dev::tile_next / tile_over): runs of depth-0 lines (~20
    B, ~1000 lines a tile: past the 288 slots 30x text takes, so a chunk runs
    again through the two-pass path and the next ones get more slots), runs of 10-B lines
    (more lines than the most slots a tile has: the two-pass path), lines of
    3-5 KiB (past the tile's LDS halo: read from HBM), and 30x text between
    them.  Every run's CSV is the oracle's.

    Over several chunks (--stats): tiles overflowed, at least once with the
    device's next chunk already popped behind the overflowing one (the
    run-ahead parse dropped and that chunk kept: round 5 lost such a chunk),
    and the tile parse came back after the 10-B lines turned it off
    (run.cpp Dev::tile_retry): the 30x and long-line text after them, three
    quarters of the file, is tiled."""
    normal = sid.synth_text(61, 20_000, 30.0, sites_per_chrom=10 ** 6)
    zero = b"".join(b"chr2\t%d\tA\t0\t*\t*\n" % i for i in range(1, 20_000))
    tiny = b"".join(b"c\t%d\tA\t0\t*\n" % (i % 10) for i in range(1, 20_000))
    rng = np.random.default_rng(61)
    alphabet = np.frombuffer(b"ACGTacgt.,$", np.uint8)
    longl = b"".join(b"chr3\t%d\tG\t900\t%s\t*\n" % (i, rng.choice(alphabet, 3000 + 7 * i).tobytes())
                     for i in range(1, 300))
    text = normal + zero + normal + tiny + normal + longl + normal
    p = tmp_path / "caps.plp"
    p.write_bytes(text)
    b = oracle.run_cli([str(p)])
    a = run(sid.CLI_PATH, extra + [str(p)])
    assert b.returncode == 0
    assert a.returncode == 0, a.stderr[-400:]
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr
    if not extra:
        return
    s = run(sid.CLI_PATH, ["--stats"] + extra + [str(p)])
    assert s.returncode == 0 and s.stdout == b.stdout
    st = json.loads(s.stderr.splitlines()[-1])
    assert st["chunks"] > 8, st
    assert st["tile_overflows"] > 0, st
    assert st["tile_overflows_queued"] > 0, st
    assert st["chunks_tiled"] >= 0.7 * st["chunks"], st


def test_tile_parse_recovers_on_a_reused_engine(sid, oracle, tmp_path):
    """A run of 10-B lines (more lines a tile than any slot list) turns the
    tile parse off for the device (run.cpp Dev::tile_over); the engine's next
    run starts with it on again (Dev::tile_reset) and tiles every chunk of 30x
    text, and within one run a chunk of 30x text after the tiny lines turns it
    back on (Dev::tile_retry).  Outputs are the oracle's throughout."""
    tiny = b"".join(b"c\t%d\tA\t0\t*\n" % (i % 10) for i in range(1, 60_000))
    normal = sid.synth_text(62, 30_000, 30.0, sites_per_chrom=10 ** 6)
    eng = sid.Engine(chunk_bytes=200_000)
    try:
        for text, tag in ((tiny, "tiny"), (normal, "normal"), (tiny + normal, "both")):
            p = tmp_path / f"{tag}.plp"
            p.write_bytes(text)
            ref = oracle.run_cli([str(p)])
            assert ref.returncode == 0
            eng.source_text(text)
            out, st = eng.run()
            assert out == ref.stdout, tag
            if tag == "tiny":
                assert st.tile_overflows >= 1 and st.chunks_tiled == 0, (st.chunks, st.chunks_tiled)
            elif tag == "normal":
                assert st.chunks > 8 and st.chunks_tiled >= st.chunks - 1, (st.chunks, st.chunks_tiled)
            else:
                tail = len(normal) // 200_000 - 2
                assert st.chunks_tiled >= tail, (st.chunks, st.chunks_tiled, tail)
    finally:
        eng.close()


@pytest.mark.parametrize("extra", [[], ["--chunk-bytes", "150000", "--devices", "2"]], ids=["one-chunk", "150k-2dev"])
def test_tile_compact_words_edges(sid, oracle, tmp_path, extra):
    """The lane-shape tile parse's compact class words (textpath.hip
    tile_wave_store: a site of its wave's reference chrom within 127
    positions after the reference line stores 4 B, the chrom and position
    coming from the wave's entry): position steps of 1, 126, 127, 128 and
    10^5 inside a wave, positions going backwards, 10-digit positions and
    zero-padded ones (no valid header pair: tokenised), chroms changing every few lines with names of 1, 7, 8
    and 9 bytes (8: the longest a header pair holds), and indel lines (the
    general routine) as a wave's first lines, so its reference is a later
    lane.  Every run's CSV is the oracle's."""
    rng = np.random.default_rng(67)
    alphabet = np.frombuffer(b"ACGTacgt.,", np.uint8)
    names = [b"c", b"chr12ab", b"chrom_08", b"chrom_009", b"chr1"]
    steps = [1, 1, 1, 126, 127, 128, 1, 1, 10 ** 5, -5, 1, -300, 2]
    out, pos, chrom = [], 1, names[0]
    for i in range(24_000):
        if i % 37 == 0 or (i % 4096 < 128 and i % 11 == 0):
            chrom = names[int(rng.integers(0, len(names)))]
        pos = max(1, pos + steps[int(rng.integers(0, len(steps)))])
        p = b"%d" % (pos if i % 97 else 10 ** 9 + i)   # (10 digits: the writer tokenises the line)
        if i % 53 == 0:
            p = b"%07d" % pos   # (leading zeros: printed without them, tokenised too)
        d = int(rng.integers(20, 40))
        b = bytearray(rng.choice(alphabet, d).tobytes())
        if i % 64 < 2 and i % 3 == 0:
            b[d // 2:d // 2] = b"-1A"   # a wave's first lines through the general routine
        out.append(b"%s\t%s\tA\t%d\t%s\t%s\n" % (chrom, p, d, bytes(b), b"I" * len(b)))
    text = b"".join(out)
    f = tmp_path / "compact.plp"
    f.write_bytes(text)
    b = oracle.run_cli([str(f)])
    a = run(sid.CLI_PATH, ["--stats"] + extra + [str(f)])
    assert b.returncode == 0
    assert a.returncode == 0, a.stderr[-400:]
    assert a.stdout == b.stdout
    st = json.loads(a.stderr.splitlines()[-1])
    assert st["chunks_tiled"] >= max(1, st["chunks"] - 1), st   # (through the tile parse)
