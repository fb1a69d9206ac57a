"""build/sid against the oracle CLI (sid.cpp restated): stdout and stderr byte
for byte, exit codes, on the golden inputs and on the reference's error
paths."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def run(exe, args, **kw):
    return subprocess.run([exe] + list(args), capture_output=True, timeout=600, **kw)


@pytest.fixture(scope="module")
def inputs(sid, tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    paths = {}
    paths["c1"] = os.path.join(GOLD, "c1_10k.plp")
    paths["edge"] = os.path.join(GOLD, "edge.plp")
    p = d / "deep.plp"
    p.write_bytes(sid.synth_text(5, 3000, 200.0, sites_per_chrom=1000))
    paths["deep"] = str(p)
    return paths


FLAGS = [[], ["-R", "-m", "likelihood_ratio"], ["-m", "likelihood_ratio"], ["-m", "bayes"],
         ["-R", "-m", "local"], ["-E", "0.05", "-p", "0.01", "-r", "0.001"], ["-m", "lynch"],
         ["-p", "0.2", "-m", "likelihood_ratio", "-R"]]


@pytest.mark.parametrize("flags", FLAGS, ids=lambda f: " ".join(f) or "default")
@pytest.mark.parametrize("name", ["c1", "edge", "deep"])
def test_cli_matches_oracle(sid, oracle, inputs, name, flags):
    a = run(sid.CLI_PATH, flags + [inputs[name]])
    b = oracle.run_cli(flags + [inputs[name]])
    assert a.returncode == b.returncode == 0, a.stderr
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


GOLDEN = {"local": [], "lr_R": ["-R", "-m", "likelihood_ratio"], "lr": ["-m", "likelihood_ratio"],
          "bayes": ["-m", "bayes"], "local_R": ["-R", "-m", "local"]}


@pytest.mark.parametrize("tag", sorted(GOLDEN))
def test_cli_matches_golden_files(sid, inputs, tag):
    import gzip
    a = run(sid.CLI_PATH, GOLDEN[tag] + [inputs["c1"]])
    assert a.returncode == 0
    assert a.stdout == gzip.open(os.path.join(GOLD, f"c1_10k.{tag}.csv.gz")).read()
    assert a.stderr == open(os.path.join(GOLD, f"c1_10k.{tag}.stderr"), "rb").read()


def test_cli_error_paths(sid, oracle, tmp_path):
    bad = tmp_path / "bad.plp"
    bad.write_bytes(b"chr1\t1\tA\t3\t...\tIII\nchr1\t2\tAC\t3\t...\tIII\n")
    blank = tmp_path / "blank.plp"
    blank.write_bytes(b"chr1\t1\tA\t3\t...\tIII\n \t\n")
    cases = [[], [str(tmp_path / "missing.plp")], ["-m", "nosuch", str(tmp_path / "missing.plp")],
             ["-h"], ["-h", str(bad)], [str(bad)], [str(blank)], ["-m", "nosuch", str(bad)],
             ["-x", str(bad)], ["-m"]]
    for args in cases:
        a = run(sid.CLI_PATH, args)
        b = oracle.run_cli(args)
        assert a.returncode == b.returncode, (args, a.returncode, b.returncode)
        assert a.stdout == b.stdout, args
        # getopt prefixes its messages with argv[0]
        assert a.stderr.replace(sid.CLI_PATH.encode(), b"P") == b.stderr.replace(oracle.CLI.encode(), b"P"), args


@pytest.mark.parametrize("extra", [["--devices", "3"], ["--host-parse"], ["--host-parse", "--devices", "2"]],
                         ids=lambda e: " ".join(e))
@pytest.mark.parametrize("flags", [[], ["-R", "-m", "likelihood_ratio"], ["-m", "bayes"], ["-R", "-m", "local"]],
                         ids=lambda f: " ".join(f) or "default")
@pytest.mark.parametrize("name", ["c1", "deep"])
def test_cli_shards_and_host_path_match_oracle(sid, oracle, inputs, name, flags, extra):
    """More shards than GPUs (shard d on device d % n: the multi-device split,
    histogram merge and ordered output) and the host parse/emit path."""
    a = run(sid.CLI_PATH, extra + flags + [inputs[name]])
    b = oracle.run_cli(flags + [inputs[name]])
    assert a.returncode == b.returncode == 0, a.stderr
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


def test_cli_first_error_across_shards(sid, oracle, tmp_path):
    good = b"".join(b"chr1\t%d\tA\t3\t.,.\tIII\n" % i for i in range(1, 4000))
    cases = {
        # malformed line in a late shard, blank (SIGSEGV) line even later
        "late": good + b"chr1\t1\tAC\t3\t...\tIII\n" + good + b" \t\n" + good,
        # blank line first, malformed later: the reference dies with SIGSEGV
        "blank_first": good + b" \t\n" + good + b"chr1\t1\tAC\t3\t...\tIII\n",
    }
    for tag, text in cases.items():
        p = tmp_path / f"{tag}.plp"
        p.write_bytes(text)
        b = oracle.run_cli([str(p)])
        for extra in ([], ["--devices", "4"], ["--host-parse", "--devices", "3"]):
            a = run(sid.CLI_PATH, extra + [str(p)])
            assert a.returncode == b.returncode, (tag, extra, a.returncode, b.returncode)
            assert a.stdout == b.stdout == b"", (tag, extra)
            assert a.stderr == b.stderr, (tag, extra)
