"""The C ABI: libsid.so loads without a GPU and exports every function that
include/sid.h declares (no compute calls here).  CPU."""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(HERE), "include", "sid.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(sid_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("sid_create", "sid_destroy", "sid_call_local", "sid_profile_accumulate",
                 "sid_lynch_prepare", "sid_lynch_objective", "sid_lookup_sites", "sid_parse_text",
                 "sid_format_csv"):
        assert must in names


def test_every_declared_symbol_is_exported(sid):
    L = sid.lib()
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_python_signatures_cover_the_header(sid):
    bound = {name for name, _, _ in sid.SIGNATURES}
    assert set(declared()) <= bound, set(declared()) - bound


def test_status_strings_and_defaults(sid):
    L = sid.lib()
    assert L.sid_strerror(0) == b"ok"
    assert L.sid_strerror(4) == b"Malformed pileup line"
    o = sid.make_opts()
    assert (o.method, o.estimate_prior, o.snp_prior, o.significance_level, o.site_error_threshold) == \
        (0, 0, -1.0, 0.05, 0.1)   # sid.cpp:11-17


def test_context_without_gpu_fails_cleanly(sid):
    if sid.device_count() > 0:
        return
    import pytest
    with pytest.raises(sid.SidError):
        sid.Context(0)
