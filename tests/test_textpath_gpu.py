"""Device text path (textpath.hip): pileup text
parsed on the GPU must give the host parser's counts and first-error status
(the host parser is itself pinned to the reference's pileup.cpp by
tests/test_parser.py), and the device CSV must be byte-identical to the host
emitter (pinned to printf by tests/test_emit.py) for the same records."""
import gzip
import os

import numpy as np
import pytest

from test_emit import sample_doubles
from test_fmt import boundary_values, tie_values
from test_parser import blank, fuzz_lines

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def dparse(gpu, sid, text, chunk=0):
    ctx = sid.Context(0)
    t = sid.DText(ctx, text, chunk=chunk)
    n = len(t)
    counts = np.zeros((n, 4), np.uint16)
    if n:
        counts = gpu.device_view(t.counts_ptr, (n, 4)).cpu().numpy().view(np.uint16)
    return ctx, t, counts


def test_format_g6_device_equals_host(gpu, sid):
    import torch
    vals = np.concatenate([sample_doubles(50_000, seed=9), tie_values(), boundary_values()])
    vals = vals[~(np.isfinite(vals) & (np.abs(vals) >= 2.0 ** 63))]
    ctx = sid.Context(0)
    d = torch.from_numpy(vals.copy()).cuda()
    out = torch.zeros(len(vals) * 16, dtype=torch.uint8, device="cuda")
    sid.check(sid.lib().sid_format_g6_device(ctx.h, d.data_ptr(), len(vals), out.data_ptr(), None), "fmt")
    torch.cuda.synchronize()
    raw = out.cpu().numpy().tobytes()
    bad = []
    for i, v in enumerate(vals):
        got = raw[16 * i:16 * i + 16].split(b"\0")[0].decode()
        want = sid.format_g6(float(v))
        if got != want:
            bad.append((float(v), got, want))
            if len(bad) > 5:
                break
    assert not bad, bad


@pytest.mark.parametrize("depth,n,chunk", [(30.0, 200_000, 0), (30.0, 50_000, 4096), (200.0, 20_000, 1 << 16)])
def test_parse_synthetic_equals_host(gpu, sid, depth, n, chunk):
    text = sid.synth_text(21, n, depth, sites_per_chrom=n // 3 + 1)
    _, t, counts = dparse(gpu, sid, text, chunk)
    s = sid.parse_text(text)
    assert len(t) == len(s) == n
    assert np.array_equal(counts, s.counts)


@pytest.mark.parametrize("seed", [4, 5, 6])
def test_parse_fuzz_valid_lines_equal_host(gpu, sid, seed):
    lines = [l for l in fuzz_lines(seed, 4000) if not blank(l)]
    ok = []
    for l in lines:
        try:
            sid.parse_text(l + b"\n")
            ok.append(l)
        except sid.SidError:
            pass
    # empty lines, CR endings, NULs inside lines, no final newline
    text = b"\n".join(ok[:1000]) + b"\n\n\n" + b"\n".join(ok[1000:])
    s = sid.parse_text(text)
    for chunk in (0, 4096, 100_003):
        _, t, counts = dparse(gpu, sid, text, chunk)
        assert len(t) == len(s)
        assert np.array_equal(counts, s.counts)


@pytest.mark.parametrize("seed", [7, 8])
def test_parse_first_error_equals_host(gpu, sid, seed):
    lines = fuzz_lines(seed, 3000)
    rng = np.random.default_rng(seed)
    ctx = sid.Context(0)
    for trial in range(20):
        k = int(rng.integers(0, len(lines)))
        text = b"\n".join(lines[:k]) + b"\n"
        try:
            want = ("OK", len(sid.parse_text(text)))
        except sid.SidError as e:
            want = ("ERR", e.status, e.line)
        try:
            got = ("OK", len(sid.DText(ctx, text, chunk=int(rng.choice([0, 4096, 65536])))))
        except sid.SidError as e:
            # the device reports the byte offset, the host the 0-based line
            got = ("ERR", e.status, text[:e.offset].count(b"\n"))
        assert got == want, (trial, k)


def test_blank_and_edge_texts(gpu, sid):
    ctx = sid.Context(0)
    assert len(sid.DText(ctx, b"")) == 0
    assert len(sid.DText(ctx, b"\n\n\n")) == 0
    t = sid.DText(ctx, b"c1 1 A 0 * *")          # no final newline
    assert len(t) == 1
    with pytest.raises(sid.SidError) as e:
        sid.DText(ctx, b"c1 1 A 3 .,. III\n \t \nc1 2 A 1 . I\n")
    assert e.value.status == 6                      # ENULLCHROM: the reference's SIGSEGV
    with pytest.raises(sid.SidError) as e:
        sid.DText(ctx, b"c1 1 A 3 .,. III\nc1 2 AC 1 . I\n \t \n")
    assert e.value.status == 4                      # the earlier malformed line wins


def test_format_equals_host_emitter(gpu, sid):
    """Random records (codes incl. dropped sites, confs incl. nan/inf/denormals)
    over a fuzzed text: device CSV == host CSV."""
    import torch
    lines = [l for l in fuzz_lines(11, 6000) if not blank(l)]
    ok = []
    for l in lines:
        try:
            sid.parse_text(l + b"\n")
            ok.append(l)
        except sid.SidError:
            pass
    text = b"\n".join(ok) + b"\n"
    s = sid.parse_text(text)
    n = len(s)
    rng = np.random.default_rng(3)
    code = rng.integers(0, 256, n).astype(np.uint8) & 0xCF
    code[rng.random(n) < 0.9] &= 0xBF           # ~10% dropped
    pool = np.concatenate([sample_doubles(20_000, seed=4), tie_values()])
    pool = pool[~(np.isfinite(pool) & (np.abs(pool) >= 2.0 ** 63))]
    hom = pool[rng.integers(0, len(pool), n)]
    het = pool[rng.integers(0, len(pool), n)]
    want = sid.format_csv(s, code, hom, het, "p_value")
    ctx, t, _ = dparse(gpu, sid, text, 65536)
    dc = torch.from_numpy(code).cuda()
    dh = torch.from_numpy(hom.copy()).cuda()
    dt = torch.from_numpy(het.copy()).cuda()
    got = t.format(dc.data_ptr(), dh.data_ptr(), dt.data_ptr(), "p_value")
    assert got == want
    got = t.format(dc.data_ptr(), dh.data_ptr(), dt.data_ptr(), "probability", begin=17, end=n - 5)
    assert got == sid.format_csv(s, code, hom, het, "probability", 17, n - 5)


def test_c1_golden_end_to_end_on_device(gpu, sid):
    """C1 text -> device parse -> -m local -> device CSV == committed golden."""
    import torch
    text = open(os.path.join(GOLD, "c1_10k.plp"), "rb").read()
    want = gzip.open(os.path.join(GOLD, "c1_10k.local.csv.gz")).read()
    ctx, t, _ = dparse(gpu, sid, text)
    n = len(t)
    code = torch.empty(n, dtype=torch.uint8, device="cuda")
    hom = torch.empty(n, dtype=torch.float64, device="cuda")
    het = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.call_local(t.counts_ptr, n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), None)
    torch.cuda.synchronize()
    body = t.format(code.data_ptr(), hom.data_ptr(), het.data_ptr(), "p_value")
    assert b"chrom,pos,label,gt,hom_conf,het_conf,conf_type\n" + body == want


@pytest.mark.parametrize("n,threads,offset_lines", [(2_500, 1, 0), (2_200_000, 8, 0), (300_000, 3, 1234)])
def test_parse_fd_equals_host(gpu, sid, tmp_path, n, threads, offset_lines):
    """sid_dtext_parse_fd: pread into pinned staging (more chunks than readers
    for the large case), from a line-aligned offset into the file."""
    text = sid.synth_text(23, n, 30.0, sites_per_chrom=n // 2 + 1)
    p = tmp_path / "in.plp"
    p.write_bytes(text)
    off = 0
    for _ in range(offset_lines):
        off = text.index(b"\n", off) + 1
    ctx = sid.Context(0)
    fd = os.open(str(p), os.O_RDONLY)
    try:
        t = sid.DText(ctx, fd=fd, offset=off, length=len(text) - off, threads=threads)
    finally:
        os.close(fd)
    s = sid.parse_text(text[off:])
    assert len(t) == len(s)
    counts = gpu.device_view(t.counts_ptr, (len(t), 4)).cpu().numpy().view(np.uint16)
    assert np.array_equal(counts, s.counts)


def test_large_text_multi_block_scans(gpu, sid):
    """1.2M sites: the line-index scan (4 KiB tiles) and the record-offset scan
    (256 records per block) both span several 4096-element scan blocks."""
    import torch
    n = 1_200_000
    text = sid.synth_text(29, n, 30.0, sites_per_chrom=400_000)
    ctx, t, counts = dparse(gpu, sid, text)
    s = sid.parse_text(text)
    assert len(t) == len(s) == n
    assert np.array_equal(counts, s.counts)
    rng = np.random.default_rng(8)
    code = (rng.integers(0, 256, n).astype(np.uint8) & 0x8F)
    hom = rng.random(n) ** 8
    het = np.where(rng.random(n) < 0.5, 1.0, rng.random(n) * 1e-7)
    dc = torch.from_numpy(code).cuda()
    dh = torch.from_numpy(hom).cuda()
    dt = torch.from_numpy(het).cuda()
    got = t.format(dc.data_ptr(), dh.data_ptr(), dt.data_ptr(), "p_value")
    assert got == sid.format_csv(s, code, hom, het, "p_value")
