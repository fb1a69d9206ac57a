"""The ctypes mirrors of include/sid.h's structs (sid_amd/__init__.py) against
the header itself: gcc compiles a probe that prints every struct's size and
every field's offset, and each must equal ctypes' view.  A field added to the
C ABI (round 5: sid_run_stats.chunks_tiled / tile_overflows, sid_placement)
without its mirror, or in another order, fails here on the CPU, before a
GPU run reads garbage through the binding."""
import ctypes as C
import os
import subprocess

import pytest

import sid_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {
    "sid_opts": sid_amd.Opts,
    "sid_estimate": sid_amd.Estimate,
    "sid_engine_cfg": sid_amd.EngineCfg,
    "sid_run_stats": sid_amd.RunStats,
    "sid_placement": sid_amd.Placement,
    "sid_engine_prof": sid_amd.EngineProf,
}


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "sid.h"', "int main(void) {"]
    for name, cls in STRUCTS.items():
        lines.append(f'  printf("{name} size %zu\\n", sizeof({name}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    lines += ["  return 0;", "}"]
    src = d / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = d / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = {}
    for line in out.splitlines():
        name, field, val = line.split()
        got[(name, field)] = int(val)
    return got


@pytest.mark.parametrize("name", sorted(STRUCTS))
def test_ctypes_mirror_matches_header(c_layout, name):
    cls = STRUCTS[name]
    assert C.sizeof(cls) == c_layout[(name, "size")], name
    for f, _ in cls._fields_:
        assert getattr(cls, f).offset == c_layout[(name, f)], (name, f)
