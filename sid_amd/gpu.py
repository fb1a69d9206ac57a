"""Device-side conveniences over the C ABI (tests, bench, smoke).

Buffers are torch CUDA(=HIP) tensors used purely as device allocations; every
computation runs in libsid.so kernels.
"""
from __future__ import annotations

import numpy as np

from . import Context, Estimate, lib  # noqa: F401


def _torch():
    lib()  # torch is imported before libsid.so
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: sid_amd.gpu needs an MI355X")
    return torch


def device_buffers(n: int, device: int = 0):
    """counts (n,4) int16, code (n) uint8, hom/het (n) float64 on `device`."""
    torch = _torch()
    dev = torch.device("cuda", device)
    counts = torch.empty((max(n, 1), 4), dtype=torch.int16, device=dev)
    code = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    hom = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    het = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    return counts, code, hom, het


def stream_handle(device: int = 0):
    torch = _torch()
    return torch.cuda.current_stream(device).cuda_stream


class _CAI:
    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2}


def device_view(ptr: int, shape, typestr: str = "<i2", device: int = 0):
    """A torch tensor viewing library-owned device memory (no copy)."""
    torch = _torch()
    return torch.as_tensor(_CAI(ptr, shape, typestr), device=torch.device("cuda", device))


def to_device(counts_np: np.ndarray, device: int = 0):
    torch = _torch()
    a = np.ascontiguousarray(counts_np, np.uint16).view(np.int16)
    return torch.from_numpy(a.copy()).to(torch.device("cuda", device))


def run_local(counts_np: np.ndarray, device: int = 0, **opts):
    """-m local over host counts; returns (code, hom_conf, het_conf) numpy."""
    torch = _torch()
    n = len(counts_np)
    ctx = Context(device, method="local", **opts)
    d_counts = to_device(counts_np.reshape(-1, 4), device) if n else None
    _, code, hom, het = device_buffers(n, device)
    st = stream_handle(device)
    if n:
        ctx.call_local(d_counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st)
    torch.cuda.synchronize(device)
    ctx.close()
    return code[:n].cpu().numpy(), hom[:n].cpu().numpy(), het[:n].cpu().numpy()


def run_method(counts_np: np.ndarray, method: str = "local", device: int = 0, verbose=False, **opts):
    """Full method on host counts, as the CLI runs it on one device.

    Returns (code, hom_conf, het_conf, estimate-or-None)."""
    torch = _torch()
    n = len(counts_np)
    estimate_prior = bool(opts.get("estimate_prior", False))
    ctx = Context(device, method=method, **opts)
    d_counts = to_device(counts_np.reshape(-1, 4), device) if n else None
    _, code, hom, het = device_buffers(n, device)
    st = stream_handle(device)
    cptr = d_counts.data_ptr() if n else None
    est = None
    if method != "local" or estimate_prior:
        ctx.profile_reset(st)
        ctx.profile_accumulate(cptr, n, st)
        est = ctx.lynch_prepare(verbose)
        if method == "local":
            ctx.set_prior(est.heterozygosity)
    if n:
        if method == "local":
            ctx.call_local(cptr, n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st)
        else:
            ctx.lookup_sites(cptr, n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st)
    torch.cuda.synchronize(device)
    ctx.close()
    return code[:n].cpu().numpy(), hom[:n].cpu().numpy(), het[:n].cpu().numpy(), est


def synth_text_hbm(seed: int, depth: float, first: int, n: int, sites_per_chrom: int = 0, device: int = 0):
    """The generator's pileup text of sites [first, first + n) written into a
    device buffer by the device generator (sid_synth_text_device), followed by
    512 zero bytes: (tensor, text length).  bench.py's C2/C3 input."""
    torch = _torch()
    dev = torch.device("cuda", device)
    ctx = Context(device)
    cap = int(n * (24 + 2.9 * depth)) + (64 << 20)
    text = torch.empty(cap + 512, dtype=torch.uint8, device=dev)
    ln = ctx.synth_text_device(seed, depth, first, n, text.data_ptr(), cap, sites_per_chrom=sites_per_chrom)
    text[ln:ln + 512].zero_()
    torch.cuda.synchronize(dev)
    ctx.close()
    return text, ln
