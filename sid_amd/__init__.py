"""sid_amd — Python bindings of libsid.so, the MI355X-native sid hot path.

The product is the C ABI in ``include/sid.h`` (``build/libsid.so``) and the
``build/sid`` command line that mirrors the reference's ``sid`` binary
(sid.cpp:1-110).  This module is a thin ctypes layer over that ABI for the
tests and ``bench.py``; it adds no computation of its own.

Device memory and streams come from PyTorch (plumbing only): when torch is
importable it is imported *before* libsid.so is loaded, so the process holds a
single HIP runtime.  There is no CPU fallback: if ``build/libsid.so`` is
missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SID_LIB_PATH: another build of the same sources (A/B measurements only)
LIB_PATH = os.environ.get("SID_LIB_PATH") or os.path.join(ROOT, "build", "libsid.so")
CLI_PATH = os.path.join(ROOT, "build", "sid")

METHOD_LOCAL, METHOD_LIKELIHOOD_RATIO, METHOD_BAYES, METHOD_QUALITY = 0, 1, 2, 3
METHODS = {"local": METHOD_LOCAL, "likelihood_ratio": METHOD_LIKELIHOOD_RATIO,
           "bayes": METHOD_BAYES, "quality": METHOD_QUALITY}

SID_OK = 0
STATUS = {0: "SID_OK", 1: "SID_EINVAL", 2: "SID_EHIP", 3: "SID_ENOMEM", 4: "SID_EMALFORMED",
          5: "SID_EMISSING_MQ", 6: "SID_ENULLCHROM", 7: "SID_ESTATE", 8: "SID_EBADFUNC",
          9: "SID_EEMPTY", 10: "SID_EIO", 11: "SID_ERANGE", 12: "SID_ENOBQ", 13: "SID_ELINE"}

CODE_HET = 0x80
CODE_DROPPED = 0x40


class SidError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = f"{what}: {STATUS.get(status, status)}" if what else STATUS.get(status, str(status))
        if status == 2 and _LIB is not None:
            msg += f" (hip error {_LIB.sid_last_hip_error()})"
        super().__init__(msg)


class Opts(C.Structure):
    """sid_opts = GlobalOptions (sid.cpp:11-17)."""
    _fields_ = [("method", C.c_int), ("estimate_prior", C.c_int), ("snp_prior", C.c_double),
                ("significance_level", C.c_double), ("site_error_threshold", C.c_double)]


class Estimate(C.Structure):
    _fields_ = [("heterozygosity", C.c_double), ("error_rate", C.c_double), ("fval", C.c_double),
                ("dist", C.c_double * 4), ("iterations", C.c_int), ("converged", C.c_int),
                ("evaluations", C.c_uint64), ("n_unique", C.c_uint64)]


class EngineCfg(C.Structure):
    """sid_engine_cfg (include/sid.h, streaming engine)."""
    _fields_ = [("devices", C.c_int), ("first_device", C.c_int), ("chunk_bytes", C.c_uint64),
                ("slots", C.c_int), ("hold_bytes", C.c_uint64), ("retain_bytes", C.c_uint64),
                ("host_threads", C.c_int), ("verbose", C.c_int), ("device_sink", C.c_int), ("lanes", C.c_int),
                ("host_hold_bytes", C.c_uint64)]


class RunStats(C.Structure):
    _fields_ = [("sites", C.c_uint64), ("chunks", C.c_uint64), ("bytes_in", C.c_uint64),
                ("bytes_out", C.c_uint64), ("chunks_held", C.c_uint64), ("chunks_retained", C.c_uint64),
                ("chunks_reloaded", C.c_uint64), ("devices", C.c_int), ("status_kind", C.c_int),
                ("err_offset", C.c_uint64), ("ingest_s", C.c_double), ("estimate_s", C.c_double),
                ("emit_s", C.c_double), ("estimate", Estimate), ("chunks_registered", C.c_uint64),
                ("register_s", C.c_double), ("h2d_s", C.c_double), ("h2d_bytes", C.c_uint64),
                ("chunks_tiled", C.c_uint64), ("tile_overflows", C.c_uint64),
                ("tile_overflows_queued", C.c_uint64)]


class Placement(C.Structure):
    """sid_placement (include/sid.h): a pipeline's host placement."""
    _fields_ = [("device", C.c_int), ("gpu_numa_node", C.c_int), ("cpus", C.c_int), ("first_cpu", C.c_int),
                ("arena_numa_node", C.c_int), ("ring_numa_node", C.c_int), ("pci", C.c_char * 16)]


class EngineProf(C.Structure):
    _fields_ = [("chunks", C.c_uint64), ("index_ms", C.c_double), ("parse_ms", C.c_double), ("call_ms", C.c_double),
                ("hist_ms", C.c_double), ("fmt_len_ms", C.c_double), ("fmt_write_ms", C.c_double)]


_LIB = None

# (name, restype, argtypes) for every entry point of include/sid.h
_P, _SZ, _U64, _I, _D = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_double
WRITE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_char), C.c_size_t)   # sid_write_fn
SIGNATURES = [
    ("sid_strerror", C.c_char_p, [_I]),
    ("sid_last_hip_error", _I, []),
    ("sid_version", C.c_char_p, []),
    ("sid_opts_default", None, [C.POINTER(Opts)]),
    ("sid_device_count", _I, [C.POINTER(C.c_int)]),
    ("sid_create", _I, [_I, C.POINTER(Opts), C.POINTER(_P)]),
    ("sid_destroy", _I, [_P]),
    ("sid_set_prior", _I, [_P, _D]),
    ("sid_call_local", _I, [_P, _P, _SZ, _P, _P, _P, _P]),
    ("sid_timing_enable", _I, [_P, _I]),
    ("sid_timing_read", _I, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("sid_profile_reset", _I, [_P, _P]),
    ("sid_profile_accumulate", _I, [_P, _P, _SZ, _P]),
    ("sid_profile_table", _I, [_P, _P, _P, _SZ, C.POINTER(C.c_size_t)]),
    ("sid_profile_load", _I, [_P, _P, _P, _SZ]),
    ("sid_lynch_setup", _I, [_P, C.POINTER(Estimate)]),
    ("sid_lynch_objective", _I, [_P, _D, _D, C.POINTER(C.c_double)]),
    ("sid_lynch_prepare", _I, [_P, _I, C.POINTER(Estimate)]),
    ("sid_lynch_prepare_given", _I, [_P, _I, C.POINTER(Estimate), C.POINTER(Estimate)]),
    ("sid_lookup_sites", _I, [_P, _P, _SZ, _P, _P, _P, _P]),
    ("sid_synth_counts", _I, [_P, _U64, _D, _U64, _SZ, _P, _P]),
    ("sid_synth_text", _I, [_U64, _D, _U64, _SZ, _U64, _P, _SZ, C.POINTER(C.c_size_t)]),
    ("sid_synth_counts_host", _I, [_U64, _D, _U64, _SZ, _P]),
    ("sid_synth_text_device", _I, [_P, _U64, _D, _U64, _SZ, _U64, _P, _SZ, C.POINTER(C.c_size_t), _P]),
    ("sid_synth_text_mq", _I, [_U64, _D, _U64, _SZ, _U64, _P, _SZ, C.POINTER(C.c_size_t)]),
    ("sid_parse_text", _I, [C.c_char_p, _SZ, _I, C.POINTER(_P), C.POINTER(C.c_uint64)]),
    ("sid_sites_free", None, [_P]),
    ("sid_sites_count", _SZ, [_P]),
    ("sid_sites_counts", _P, [_P]),
    ("sid_sites_positions", _P, [_P]),
    ("sid_sites_chrom_segments", _SZ, [_P]),
    ("sid_sites_chrom_name", C.c_char_p, [_P, _SZ, C.POINTER(C.c_uint64)]),
    ("sid_format_csv", _I, [_P, _SZ, _SZ, _P, _P, _P, C.c_char_p, _P, _SZ, C.POINTER(C.c_size_t)]),
    ("sid_format_double", _I, [_D, C.c_char_p, _SZ]),
    ("sid_dtext_parse", _I, [_P, _P, _SZ, _SZ, C.POINTER(_P), C.POINTER(C.c_uint64), _P]),
    ("sid_dtext_parse_fd", _I, [_P, _I, _U64, _U64, _I, C.POINTER(_P), C.POINTER(C.c_uint64), _P]),
    ("sid_dtext_count", _SZ, [_P]),
    ("sid_dtext_counts", _P, [_P]),
    ("sid_dtext_format", _I, [_P, _P, _SZ, _SZ, _P, _P, _P, C.c_char_p, WRITE_FN, _P, _P]),
    ("sid_dtext_free", _I, [_P]),
    ("sid_call_quality", _I, [_P, _P, _P, _P, _P, _P]),
    ("sid_format_g6", _I, [_D, C.c_char_p, _SZ]),
    ("sid_format_g6_device", _I, [_P, _P, _SZ, _P, _P]),
    ("sid_engine_cfg_default", None, [C.POINTER(EngineCfg)]),
    ("sid_engine_create", _I, [C.POINTER(Opts), C.POINTER(EngineCfg), C.POINTER(_P)]),
    ("sid_engine_destroy", _I, [_P]),
    ("sid_engine_devices", _I, [_P]),
    ("sid_engine_context", _P, [_P, _I]),
    ("sid_engine_placement", _I, [_P, _I, C.POINTER(Placement)]),
    ("sid_engine_source_text", _I, [_P, _P, _U64]),
    ("sid_engine_source_file", _I, [_P, _I, _U64, _U64]),
    ("sid_engine_source_device_text", _I, [_P, _P, _U64]),
    ("sid_engine_source_synth", _I, [_P, _U64, _D, _U64, _U64, _U64, _U64, _I]),
    ("sid_engine_ingest", _I, [_P, C.POINTER(RunStats)]),
    ("sid_engine_estimate", _I, [_P, C.POINTER(Estimate), C.POINTER(Estimate)]),
    ("sid_engine_emit", _I, [_P, C.c_char_p, WRITE_FN, _P, C.POINTER(RunStats)]),
    ("sid_engine_run", _I, [_P, C.c_char_p, WRITE_FN, _P, C.POINTER(RunStats)]),
    ("sid_engine_profile_table", _I, [_P, _P, _P, _SZ, C.POINTER(C.c_size_t)]),
    ("sid_engine_profile_load", _I, [_P, _P, _P, _SZ]),
    ("sid_engine_records", _I, [_P, _U64, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    ("sid_engine_profile", _I, [_P, _I]),
    ("sid_engine_profile_read", _I, [_P, C.POINTER(EngineProf)]),
]


def lib():
    """Load build/libsid.so (torch first, if importable: one HIP runtime)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()); "
                           "sid_amd has no CPU fallback")
    try:  # plumbing: device memory / streams / distributed come from torch
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def check(status: int, what: str = ""):
    if status != SID_OK:
        raise SidError(status, what)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def make_opts(method="local", estimate_prior=False, snp_prior=-1.0, significance_level=0.05,
              site_error_threshold=0.1) -> Opts:
    o = Opts()
    lib().sid_opts_default(C.byref(o))
    o.method = METHODS[method] if isinstance(method, str) else int(method)
    o.estimate_prior = int(bool(estimate_prior))
    o.snp_prior = float(snp_prior)
    o.significance_level = float(significance_level)
    o.site_error_threshold = float(site_error_threshold)
    return o


def device_count() -> int:
    n = C.c_int(0)
    st = lib().sid_device_count(C.byref(n))
    return n.value if st == SID_OK else 0


# --------------------------------------------------------------- host side --
@dataclass
class Sites:
    counts: np.ndarray          # (n, 4) uint16, A C G T
    positions: np.ndarray       # (n,) int32
    chroms: list                # [(start_site, name)]
    handle: object = None       # sid_sites* kept for format_csv

    def __len__(self):
        return len(self.positions)

    def __del__(self):
        if self.handle is not None and _LIB is not None:
            _LIB.sid_sites_free(self.handle)
            self.handle = None


def parse_text(text: bytes, threads: int = 0) -> Sites:
    """sid_parse_text: pileup text -> SoA (pileup.cpp:13-153 semantics)."""
    L = lib()
    h = C.c_void_p()
    bad = C.c_uint64(0)
    st = L.sid_parse_text(text, len(text), threads, C.byref(h), C.byref(bad))
    if st != SID_OK:
        err = SidError(st, "parse")
        err.line = bad.value
        raise err
    n = L.sid_sites_count(h)
    counts = np.ctypeslib.as_array(C.cast(L.sid_sites_counts(h), C.POINTER(C.c_uint16)),
                                   shape=(n * 4,)).reshape(n, 4).copy() if n else np.zeros((0, 4), np.uint16)
    pos = np.ctypeslib.as_array(C.cast(L.sid_sites_positions(h), C.POINTER(C.c_int32)),
                                shape=(n,)).copy() if n else np.zeros(0, np.int32)
    chroms = []
    for k in range(L.sid_sites_chrom_segments(h)):
        start = C.c_uint64(0)
        name = L.sid_sites_chrom_name(h, k, C.byref(start))
        chroms.append((start.value, name))
    return Sites(counts, pos, chroms, h)


def format_csv(sites: Sites, code: np.ndarray, hom: np.ndarray, het: np.ndarray,
               conf_type: str = "p_value", begin: int = 0, end: int = None) -> bytes:
    L = lib()
    code = np.ascontiguousarray(code, np.uint8)
    hom = np.ascontiguousarray(hom, np.float64)
    het = np.ascontiguousarray(het, np.float64)
    need = C.c_size_t(0)
    n = len(sites) if end is None else end
    L.sid_format_csv(sites.handle, begin, n, _ptr(code), _ptr(hom), _ptr(het), conf_type.encode(),
                     None, 0, C.byref(need))
    buf = C.create_string_buffer(max(need.value, 1))
    ln = C.c_size_t(0)
    check(L.sid_format_csv(sites.handle, begin, n, _ptr(code), _ptr(hom), _ptr(het), conf_type.encode(),
                           buf, need.value, C.byref(ln)), "format")
    return buf.raw[: ln.value]


def format_double(v: float) -> str:
    buf = C.create_string_buffer(48)
    k = lib().sid_format_double(float(v), buf, 48)
    return buf.value.decode()


def format_g6(v: float) -> str:
    """The device formatter's %g (fmt.h), host build."""
    buf = C.create_string_buffer(48)
    k = lib().sid_format_g6(float(v), buf, 48)
    if k < 0:
        raise SidError(-k, "format_g6")
    return buf.value.decode()


class DText:
    """One shard of pileup text parsed on the device (sid_dtext_*)."""

    def __init__(self, ctx: "Context", text: bytes = None, chunk: int = 0, stream=None, fd: int = None,
                 offset: int = 0, length: int = None, threads: int = 0):
        self.ctx = ctx
        h = C.c_void_p()
        off = C.c_uint64(0)
        if fd is not None:   # bytes [offset, offset+length) of an open file
            rc = lib().sid_dtext_parse_fd(ctx.h, fd, offset, length, threads, C.byref(h), C.byref(off), stream)
        else:
            buf = C.c_char_p(text)
            rc = lib().sid_dtext_parse(ctx.h, C.cast(buf, C.c_void_p), len(text), chunk, C.byref(h), C.byref(off),
                                       stream)
        if rc != 0:
            err = SidError(rc, "sid_dtext_parse")
            err.offset = off.value   # byte offset of the first malformed line
            raise err
        self.h = h

    def __len__(self):
        return lib().sid_dtext_count(self.h)

    @property
    def counts_ptr(self):
        return lib().sid_dtext_counts(self.h)

    def format(self, code_ptr, hom_ptr, het_ptr, conf_type="p_value", begin=0, end=None, stream=None) -> bytes:
        end = len(self) if end is None else end
        parts = []

        def w(_user, data, n):
            parts.append(C.string_at(data, n))
            return 0
        cb = WRITE_FN(w)
        check(lib().sid_dtext_format(self.ctx.h, self.h, begin, end, code_ptr, hom_ptr, het_ptr,
                                     conf_type.encode(), cb, None, stream), "sid_dtext_format")
        return b"".join(parts)

    def close(self):
        if getattr(self, "h", None):
            lib().sid_dtext_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_text(seed: int, n: int, depth: float = 30.0, first: int = 0,
               sites_per_chrom: int = 0, mapq: bool = False) -> bytes:
    """Synthetic pileup text; mapq=True adds the 7th (mapping quality) column."""
    L = lib()
    fn = L.sid_synth_text_mq if mapq else L.sid_synth_text
    ln = C.c_size_t(0)
    check(fn(seed, depth, first, n, sites_per_chrom, None, 0, C.byref(ln)), "synth")
    buf = C.create_string_buffer(max(ln.value, 1))
    check(fn(seed, depth, first, n, sites_per_chrom, buf, ln.value, C.byref(ln)), "synth")
    return buf.raw[: ln.value]


def synth_counts_host(seed: int, n: int, depth: float = 30.0, first: int = 0) -> np.ndarray:
    out = np.zeros((n, 4), np.uint16)
    check(lib().sid_synth_counts_host(seed, depth, first, n, _ptr(out)), "synth")
    return out


# ------------------------------------------------------------- device side --
class Context:
    """One sid_ctx (one device, one host thread)."""

    def __init__(self, device: int = 0, **opts):
        self.opts = make_opts(**opts)
        self.device = device
        h = C.c_void_p()
        check(lib().sid_create(device, C.byref(self.opts), C.byref(h)), "sid_create")
        self.h = h

    @classmethod
    def wrap(cls, handle, device: int = 0):
        """A non-owning view of a context another object owns (e.g. an engine's)."""
        c = cls.__new__(cls)
        c.opts, c.device, c.h, c._borrowed = None, device, C.c_void_p(handle), True
        return c

    def close(self):
        if getattr(self, "h", None) and not getattr(self, "_borrowed", False):
            lib().sid_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_prior(self, prior: float):
        check(lib().sid_set_prior(self.h, float(prior)), "sid_set_prior")

    # raw device-pointer entry points -------------------------------------
    def call_local(self, counts_ptr, n, code_ptr, hom_ptr, het_ptr, stream=None):
        check(lib().sid_call_local(self.h, counts_ptr, n, code_ptr, hom_ptr, het_ptr, stream),
              "sid_call_local")

    def timing_enable(self, on=True):
        check(lib().sid_timing_enable(self.h, int(bool(on))), "sid_timing_enable")

    def timing_read(self):
        """(calls, main kernel ms, fix-up kernel ms) averaged since the last read."""
        k, m, f = C.c_uint64(0), C.c_double(0), C.c_double(0)
        check(lib().sid_timing_read(self.h, C.byref(k), C.byref(m), C.byref(f)), "sid_timing_read")
        return k.value, m.value, f.value

    def lookup_sites(self, counts_ptr, n, code_ptr, hom_ptr, het_ptr, stream=None):
        check(lib().sid_lookup_sites(self.h, counts_ptr, n, code_ptr, hom_ptr, het_ptr, stream),
              "sid_lookup_sites")

    def profile_reset(self, stream=None):
        check(lib().sid_profile_reset(self.h, stream), "sid_profile_reset")

    def profile_accumulate(self, counts_ptr, n, stream=None):
        check(lib().sid_profile_accumulate(self.h, counts_ptr, n, stream), "sid_profile_accumulate")

    def profile_table(self):
        u = C.c_size_t(0)
        check(lib().sid_profile_table(self.h, None, None, 0, C.byref(u)), "sid_profile_table")
        keys = np.zeros(u.value, np.uint64)
        cnts = np.zeros(u.value, np.uint64)
        if u.value:
            check(lib().sid_profile_table(self.h, _ptr(keys), _ptr(cnts), u.value, C.byref(u)),
                  "sid_profile_table")
        return keys, cnts

    def profile_load(self, keys: np.ndarray, cnts: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        cnts = np.ascontiguousarray(cnts, np.uint64)
        check(lib().sid_profile_load(self.h, _ptr(keys), _ptr(cnts), len(keys)), "sid_profile_load")

    def lynch_setup(self) -> Estimate:
        e = Estimate()
        check(lib().sid_lynch_setup(self.h, C.byref(e)), "sid_lynch_setup")
        return e

    def lynch_objective(self, pi: float, eps: float) -> float:
        out = C.c_double(0)
        check(lib().sid_lynch_objective(self.h, pi, eps, C.byref(out)), "sid_lynch_objective")
        return out.value

    def lynch_prepare(self, verbose: bool = False) -> Estimate:
        e = Estimate()
        check(lib().sid_lynch_prepare(self.h, int(verbose), C.byref(e)), "sid_lynch_prepare")
        return e

    def synth_counts(self, seed, depth, first, n, counts_ptr, stream=None):
        check(lib().sid_synth_counts(self.h, seed, depth, first, n, counts_ptr, stream),
              "sid_synth_counts")

    def synth_text_device(self, seed, depth, first, n, out_ptr, cap, sites_per_chrom=0, stream=None) -> int:
        """The generator's text written on the device (sid_synth_text_device); returns its bytes."""
        ln = C.c_size_t(0)
        check(lib().sid_synth_text_device(self.h, seed, depth, first, n, sites_per_chrom, out_ptr, cap,
                                          C.byref(ln), stream), "sid_synth_text_device")
        return ln.value


HEADER = b"chrom,pos,label,gt,hom_conf,het_conf,conf_type\n"


class Engine:
    """The streaming engine (sid_engine_*): pileup text in, CSV out, in
    line-aligned chunks over one or more devices."""

    def __init__(self, method="local", devices=1, first_device=0, chunk_bytes=0, slots=0, hold_bytes=0,
                 retain_bytes=0, host_threads=0, verbose=False, device_sink=False, lanes=0, host_hold_bytes=0,
                 **opts):
        self.opts = make_opts(method=method, **opts)
        cfg = EngineCfg()
        lib().sid_engine_cfg_default(C.byref(cfg))
        cfg.devices, cfg.first_device, cfg.chunk_bytes, cfg.slots = devices, first_device, chunk_bytes, slots
        cfg.hold_bytes, cfg.retain_bytes, cfg.host_threads = hold_bytes, retain_bytes, host_threads
        cfg.verbose, cfg.device_sink, cfg.lanes = int(bool(verbose)), int(device_sink), lanes
        cfg.host_hold_bytes = host_hold_bytes
        self.cfg = cfg
        h = C.c_void_p()
        check(lib().sid_engine_create(C.byref(self.opts), C.byref(cfg), C.byref(h)), "sid_engine_create")
        self.h = h
        self._keep = None

    def close(self):
        if getattr(self, "h", None):
            lib().sid_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def context(self, i=0):
        return lib().sid_engine_context(self.h, i)

    def placement(self, i=0) -> dict:
        """Pipeline i's host placement: its GPU's NUMA node, the CPUs its
        threads are bound to, the NUMA nodes of its pinned host buffers."""
        p = Placement()
        check(lib().sid_engine_placement(self.h, i, C.byref(p)), "sid_engine_placement")
        return {"device": p.device, "pci": p.pci.decode(), "gpu_numa_node": p.gpu_numa_node, "cpus": p.cpus,
                "first_cpu": p.first_cpu, "arena_numa_node": p.arena_numa_node, "ring_numa_node": p.ring_numa_node}

    def source_text(self, text: bytes):
        self._keep = C.create_string_buffer(text, len(text)) if text else None
        check(lib().sid_engine_source_text(self.h, C.cast(self._keep, C.c_void_p) if text else None, len(text)),
              "source_text")

    def source_host_ptr(self, ptr: int, n: int, keep=None):
        self._keep = keep
        check(lib().sid_engine_source_text(self.h, ptr, n), "source_text")

    def source_file(self, fd: int, offset: int = 0, length: int = None):
        if length is None:
            length = os.fstat(fd).st_size - offset
        check(lib().sid_engine_source_file(self.h, fd, offset, length), "source_file")

    def source_device_text(self, ptr: int, n: int, keep=None):
        self._keep = keep
        check(lib().sid_engine_source_device_text(self.h, ptr, n), "source_device_text")

    def source_synth(self, seed, n, depth=30.0, first=0, sites_per_chrom=0, sites_per_chunk=0, on_device=True):
        check(lib().sid_engine_source_synth(self.h, seed, depth, first, n, sites_per_chrom, sites_per_chunk,
                                            int(bool(on_device))), "source_synth")

    def ingest(self) -> RunStats:
        st = RunStats()
        rc = lib().sid_engine_ingest(self.h, C.byref(st))
        if rc != 0:
            err = SidError(rc, "sid_engine_ingest")
            err.offset = st.err_offset
            err.stats = st
            raise err
        return st

    def estimate(self, given: Estimate = None) -> Estimate:
        out = Estimate()
        check(lib().sid_engine_estimate(self.h, C.byref(given) if given is not None else None, C.byref(out)),
              "sid_engine_estimate")
        return out

    def emit(self, header=HEADER, sink=None, stats: RunStats = None):
        """Records in file order: returned as bytes (sink None), written to a
        file descriptor (sink int), or dropped (the device-sink engine)."""
        parts = []

        def w(_user, data, n):
            try:
                if isinstance(sink, int):   # every byte, across partial writes
                    mv = memoryview(C.string_at(data, n))
                    while len(mv):
                        mv = mv[os.write(sink, mv):]
                else:
                    parts.append(C.string_at(data, n))
                return 0
            except Exception:   # the engine reports SID_EIO
                return -1
        cb = WRITE_FN(w)
        st = stats if stats is not None else RunStats()
        check(lib().sid_engine_emit(self.h, header, cb, None, C.byref(st)), "sid_engine_emit")
        return b"".join(parts), st

    def profile_table(self):
        """The merged unique-profile table of all pipelines (after ingest)."""
        u = C.c_size_t(0)
        check(lib().sid_engine_profile_table(self.h, None, None, 0, C.byref(u)), "sid_engine_profile_table")
        keys = np.zeros(u.value, np.uint64)
        cnts = np.zeros(u.value, np.uint64)
        if u.value:
            check(lib().sid_engine_profile_table(self.h, _ptr(keys), _ptr(cnts), u.value, C.byref(u)),
                  "sid_engine_profile_table")
        return keys, cnts

    def profile_load(self, keys: np.ndarray, cnts: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        cnts = np.ascontiguousarray(cnts, np.uint64)
        check(lib().sid_engine_profile_load(self.h, _ptr(keys), _ptr(cnts), len(keys)), "sid_engine_profile_load")

    def records(self, chunk: int):
        """(address, length) of a chunk's records in the host arena."""
        p, n = C.c_void_p(), C.c_uint64(0)
        check(lib().sid_engine_records(self.h, chunk, C.byref(p), C.byref(n)), "sid_engine_records")
        return p.value or 0, n.value

    def records_bytes(self, nchunks: int) -> bytes:
        """Every chunk's records from the host arena, in file order."""
        out = []
        for j in range(nchunks):
            p, n = self.records(j)
            out.append(C.string_at(p, n) if n else b"")
        return b"".join(out)

    def profile(self, enable=True):
        check(lib().sid_engine_profile(self.h, int(bool(enable))), "sid_engine_profile")

    def profile_read(self) -> dict:
        p = EngineProf()
        check(lib().sid_engine_profile_read(self.h, C.byref(p)), "sid_engine_profile_read")
        return {f: getattr(p, f) for f, _ in EngineProf._fields_}

    def run(self, header=HEADER, sink=None):
        st = self.ingest()
        est = self.estimate()
        out, st2 = self.emit(header, sink)
        st.bytes_out, st.emit_s, st.chunks_reloaded = st2.bytes_out, st2.emit_s, st2.chunks_reloaded
        st.estimate = est
        return out, st


def profile_key(counts: np.ndarray) -> np.ndarray:
    c = counts.astype(np.uint64)
    return (c[:, 0] << np.uint64(48)) | (c[:, 1] << np.uint64(32)) | (c[:, 2] << np.uint64(16)) | c[:, 3]
