#!/usr/bin/env python3
"""bench.py — genome sites/s of sid's pileup -> CSV path on MI355X.

Headline (BASELINE.json metric, configs[1] = "C2"): 50,000,000 synthetic 30x
diploid sites per GPU, `-m local`.  A step is one whole sid run over the
rank's pileup text, in host memory when the timed region starts, with the CSV
in host memory when it ends -- the reference's file-in / stdout-out path
(sid.cpp:84-105) without the file system:

    pinned host text -H2D-> line index -> parse (counts) -> per-site call
      -> CSV records formatted -D2H-> the engine's pinned host arena

i.e. readFile + callSiteMLError + the output loop (call.cpp:11-20, :213-289,
sid.cpp:102-105) through the streaming engine (include/sid.h sid_engine_*,
host-text source, 128 MiB chunks, host_hold_bytes: each chunk's records are
copied back while later chunks upload, so PCIe runs both ways at once).
Beside it, in the same line:

  device_path   the same run over the text already resident in HBM with the
                records left in HBM (device_sink 1): the kernels alone, per
                stage, with the roofline of the dominant stage
  kernel_local  sid_call_local alone over resident counts (25 B/site)
  cli           build/sid on the same text as a file, CSV to /dev/null (wall)
  cpu_baseline  the oracle CLI (the reference's path restated in C) on the
                same 50M-site text, 16 line-aligned shard processes, plus a
                1-core figure on a 4M-site sample (rank 0, N=1 only)

Configs (--config):
  C2  -m local, seed 2, 50M sites per GPU (weak scaling)           [default]
  C3  -R -m likelihood_ratio, seed 3, 50M sites per GPU (weak): ingest builds
      the profile histogram; N>1 all-gathers it over RCCL (device tensors,
      backend "nccl"), rank 0 runs the one Nelder-Mead estimate and broadcasts
      (pi, eps) over RCCL; then every rank formats its records
  C3B -m bayes, seed 3, 50M sites per GPU (weak): the Lynch path's other
      caller (call.cpp:145-211), as C3
  C4  -m local, seed 4, 3G sites in total = 24 chromosomes x 125M, quoted on
      8 GPUs: rank r takes the eighth [r*3G/8, (r+1)*3G/8) (375M sites, 30.4
      GB of text), so N = 8 runs the whole genome; the same step as C2 (host
      text -> CSV in host memory), device_path on the shard resident in HBM
  C5  -m local, seed 5, 200x, 500M sites in total, as C4 (62.5M sites, 26.6
      GB of text per eighth)

Multi-GPU: one rank per GPU.  Under torchrun (WORLD_SIZE set) each process is
a rank; without it, `--gpus N` (N > 1) starts N rank processes itself (before
anything touches a GPU) and relays rank 0's line.  -m local has no data-path
exchange; the Lynch path exchanges only the O(U) profile histogram.  Ranks
beyond the visible GPUs are refused unless --allow-shared-gpu (a rehearsal:
n_gpus then counts distinct devices and "oversubscribed" is set).  Each rank
pins its host buffers on its GPU's NUMA node (the PCI device's local CPUs).
"""
import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the copy engines (SDMA) for every host<->device copy, set before the HIP
# runtime starts: with the runtime's default, device->host copies ran at 30
# GB/s; with SDMA both directions reach ~57 GB/s at the same time
# (tools/debug/pcie_probe.cpp, profiles/pcie_probe_r03.jsonl)
os.environ.setdefault("HSA_ENABLE_SDMA", "1")

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
LOCAL_BYTES_PER_SITE = 25    # sid_call_local: 8 B counts in, 1 B code + 2 x 8 B confs out
METRIC = "genome sites/sec (whole node) on 30x synthetic pileup; 1/2/4/8 GPU scaling"

CONFIGS = {
    "C2": dict(method="local", R=False, seed=2, depth=30.0, per_gpu=50_000_000, total=None, spc=0,
               desc="-m local, 50M-site 30x synthetic pileup per GPU"),
    "C3": dict(method="likelihood_ratio", R=True, seed=3, depth=30.0, per_gpu=50_000_000, total=None, spc=0,
               desc="-R -m likelihood_ratio, 50M-site 30x synthetic pileup per GPU"),
    "C3B": dict(method="bayes", R=False, seed=3, depth=30.0, per_gpu=50_000_000, total=None, spc=0,
                desc="-m bayes, 50M-site 30x synthetic pileup per GPU"),
    "C4": dict(method="local", R=False, seed=4, depth=30.0, per_gpu=None, total=3_000_000_000, spc=125_000_000,
               desc="-m local, 3G-site whole-genome 30x pileup (24 x 125M), site-range shards"),
    "C5": dict(method="local", R=False, seed=5, depth=200.0, per_gpu=None, total=500_000_000, spc=125_000_000,
               desc="-m local, 500M-site 200x pileup, site-range shards"),
}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS))
    p.add_argument("--method", default=None, choices=["local", "likelihood_ratio", "bayes"],
                   help="alias: local = C2, likelihood_ratio = C3, bayes = C3B")
    p.add_argument("--sites", type=int, default=None, help="override: sites per GPU (C2/C3) or in total (C4/C5)")
    p.add_argument("--chunk-mib", type=int, default=0, help="engine chunk size (0 = the engine's default)")
    p.add_argument("--device-steps", type=int, default=0, help="device_path steps (0 = max(steps, 10))")
    p.add_argument("--slots", type=int, default=0, help="PCIe path: device text buffers per GPU (0 = the engine's 3)")
    p.add_argument("--pcie-chunk-mib", type=int, default=0, help="PCIe path chunk size (0 = the engine's 128 MiB)")
    p.add_argument("--no-extras", action="store_true", help="skip kernel_local, cli and cpu_baseline")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--device-only", action="store_true",
                   help="profiling: only the device_path leg (its line's value is then the device path's)")
    p.add_argument("--allow-shared-gpu", action="store_true",
                   help="rehearsal: more ranks than GPUs share them round-robin")
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
    p.add_argument("--dump-records", default=None, metavar="DIR",
                   help="after the timed PCIe leg (C2/C3): each rank writes its records (file order) to "
                        "DIR/rank<r>.csv and its estimate to DIR/rank<r>.json (parity tests)")
    p.add_argument("--no-node-cli", action="store_true", help="N > 1: skip the whole-node CLI leg")
    a = p.parse_args(argv)
    if a.config is None:
        a.config = {"likelihood_ratio": "C3", "bayes": "C3B"}.get(a.method, "C2")
    return a


# ------------------------------------------------------------- launcher ----
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a):
    """`--gpus N` without torchrun: N rank processes of this script, started
    before this process touches any GPU (device_count() does not initialise
    one on this image); rank 0's line goes to stdout.  Returns the exit code."""
    import torch
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    if a.gpus > ndev and not a.allow_shared_gpu:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but {ndev} GPU(s) visible; pass --allow-shared-gpu "
                         "for a rehearsal with ranks sharing GPUs")
    env = dict(os.environ, WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    for r in range(a.gpus):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        # stdout: only rank 0's JSON line (collective libraries print to stdout too)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    import threading

    def relay(f):
        for line in iter(f.readline, b""):
            if line.startswith(b'{"metric"'):
                sys.stdout.buffer.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.buffer.write(line)
    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:   # a failed rank leaves the others at a barrier: stop them
                    q.terminate()
        time.sleep(0.05)
    th.join(timeout=10)
    return rc


def numa_bind(torch, gpu):
    """Run this rank on its GPU's NUMA node (the PCI device's local CPUs, within
    the CPUs this process may use), so pinned host buffers are allocated there
    and the DMA does not cross sockets.  Returns {pci, gpu_numa_node, cpus
    (bound to; 0: not bound -- the GPU's local CPUs are none or all of this
    job's)}, or None when the GPU's PCI function cannot be read."""
    try:
        pr = torch.cuda.get_device_properties(gpu)
        bdf = "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
        try:
            node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        except (OSError, ValueError):
            node = None
        txt = open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip()
        cpus = set()
        for part in txt.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        mine = cpus & os.sched_getaffinity(0)
        if not mine or mine == os.sched_getaffinity(0):
            return {"pci": bdf, "gpu_numa_node": node, "cpus": 0}
        os.sched_setaffinity(0, mine)
        return {"pci": bdf, "gpu_numa_node": node, "cpus": len(mine)}
    except Exception:
        return None


def numa_nodes_of(t):
    """The NUMA nodes holding a pinned host tensor's pages (its first, middle
    and last byte): get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR), x86-64 syscall
    239 -- the node the kernel actually placed each page on."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.syscall.restype = ctypes.c_long
        out = []
        n = t.numel()
        for off in sorted({0, n // 2, max(0, n - 1)}):
            node = ctypes.c_int(-1)
            rc = libc.syscall(ctypes.c_long(239), ctypes.byref(node), ctypes.c_void_p(0), ctypes.c_ulong(0),
                              ctypes.c_void_p(t.data_ptr() + off), ctypes.c_ulong(3))
            out.append(node.value if rc == 0 else None)
        return out
    except Exception:
        return None


# ----------------------------------------------------------------- ranks ----
def fmt_kind(cfg):
    """The formatter the engine runs: "local" (-m local, the call fused into
    it) or "lynch" (likelihood_ratio / bayes pass 2, the class lookup fused
    into it)."""
    return "local" if cfg["method"] == "local" else "lynch"


def parse_quad(text_per_site):
    """Lines over 256 B on average are parsed by a quad of lanes each
    (textpath.hip sid_parse_quad_kernel)."""
    return text_per_site > 256


def tile_parse(fused, text_per_site=81.0):
    """-m local: the engine's tile parse (run.cpp, textpath.hip
    sid_chunk_tile_local; a lane per line at 30x, a quad of lanes per line at
    200x) -- the line index fused into the parse (the text read once), the
    record lengths, the fix-up and the writer's offsets in the parse stage; no
    index stage."""
    return fused == "local"


def stage_bytes(stage, text_per_site, csv_per_site, fused):
    """Algorithmic HBM bytes per site of each engine stage.
    fused: a fmt_kind, the call / lookup fused into the formatter (it reads
    the 8 B counts instead of the call kernel's 17 B code + confs)."""
    site_in = 8 if fused else 17
    if fused == "lynch" and stage == "parse":
        # the Lynch paths' first pass: the tile parse writes every site's
        # counts (8) and header pair (16) per slot, compacted into the buffer
        # kept for pass 2 (those read, line offsets (4), counts and pairs
        # written: textpath.hip sid_tile_compact_kernel)
        return text_per_site + 24 + 24 + 28
    if tile_parse(fused, text_per_site) and stage in ("parse", "fmt_write"):
        # the tile parse reads the text once and writes each site's slot
        # words, which the writer reads before writing the records
        # (textpath.hip sid_tile_parse_kernel, tile_wave_store): the lane
        # shape a 4 B compact class word a site and a 16 B entry a wave of 64
        # slots (a 20 KiB tile's lines, slots for 3 % more rounded up to 16:
        # ~0.32 B a site); the quad shape the 4 B word and the 16 B header pair
        slot = 4 + 16
        if not parse_quad(text_per_site):
            lines = 20480 / text_per_site
            slot = 4 + 16 * math.ceil(math.ceil((lines * 1.03 + 2) / 16) * 16 / 64) / lines
        return {"parse": text_per_site + slot, "fmt_write": slot + csv_per_site}[stage]
    return {
        "index": text_per_site + text_per_site / 8,    # text read once, line-start masks written
        # text read; line-start masks (1/8 of the text) read back, 4 B line
        # offsets written and read; counts (8) and the formatter's header pair
        # (16) written
        "parse": text_per_site + text_per_site / 8 + 4 + 4 + 8 + 16,
        "call": 8 + 17,                                # counts in, code + confs out (Lynch lookup, quality)
        "hist": 8,                                     # counts read
        # formatter: the site's counts (or code + confs) and header pair read
        # (the line offset only for chrom names over 8 bytes); record bytes per
        # 512-site block written (0.01 B/site); then the same reads again and
        # the records written
        "fmt_len": site_in + 16,
        "fmt_write": site_in + 16 + csv_per_site,
    }[stage]


def stage_kernels(stage, fused, text_per_site=81.0):
    tp = tile_parse(fused, text_per_site)
    return {
        "index": ["sid_index_count_kernel", "sid_scan_*"],
        "parse": (["sid_tile_parse_kernel", "sid_tile_serial_kernel", "sid_scan_*"] if tp else
                  ["sid_tile_parse_kernel", "sid_tile_serial_kernel", "sid_tile_compact_kernel", "sid_scan_*"]
                  if fused == "lynch" else
                  ["sid_index_emit_kernel", ("sid_parse_quad_kernel" if parse_quad(text_per_site) else
                                             "sid_parse_kernel"), "sid_parse_serial_kernel"]),
        "call": ["sid_lookup_rec_kernel"],
        "hist": ["sid_hist_dense_kernel", "sid_hist_reduce_kernel"],
        "fmt_len": {"local": ["sid_local_len_kernel", "sid_local_fixlen_kernel"],
                    "lynch": ["sid_lynch_len_kernel"]}.get(fused, ["sid_fmt_blen_kernel"]) + ["sid_scan_*"],
        "fmt_write": {"local": ["sid_local_put_kernel"], "lynch": ["sid_lynch_put_kernel"]}.get(
            fused, ["sid_fmt_put_kernel"]),
    }[stage]


class Rank:
    def __init__(self, a):
        self.a = a
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        import torch  # plumbing: device memory, events, process group
        self.torch = torch
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise SystemExit("bench.py: no HIP device visible")
        if self.local_rank >= ndev and not a.allow_shared_gpu:
            raise SystemExit(f"bench.py: rank {self.rank} (local {self.local_rank}) has no GPU of its own "
                             f"({ndev} visible); pass --allow-shared-gpu for a rehearsal")
        if self.world > 1 and a.gpus not in (1, self.world):
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {self.world}")
        self.gpu = self.local_rank % ndev
        torch.cuda.set_device(self.gpu)
        self.dev = torch.device("cuda", self.gpu)
        self.cpus0 = os.sched_getaffinity(0)   # before the NUMA binding (the node CLI leg runs unbound)
        self.numa = numa_bind(torch, self.gpu)
        self.dist = None
        self.backend = None
        self.last_table = None   # the Lynch paths' global unique-profile table (keys, counts) of the last step
        self.n_gpus, self.oversub = 1, False
        if self.world > 1:
            import torch.distributed as dist
            # RCCL takes one rank per GPU: a rehearsal with ranks sharing GPUs runs over gloo
            backend = a.backend or ("nccl" if self.world <= ndev else "gloo")
            dist.init_process_group(backend, rank=self.rank, world_size=self.world,
                                    device_id=self.dev if backend == "nccl" else None)
            ids = [None] * self.world
            dist.all_gather_object(ids, (socket.gethostname(), self.gpu))
            self.n_gpus = len(set(ids))
            self.oversub = self.n_gpus < self.world
            self.dist = dist
            self.backend = backend

    # -- timing harness: warmup, barrier + sync, K steps, barrier + sync, max over ranks
    def timed(self, step, steps, warmup):
        torch, dist = self.torch, self.dist
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(self.dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            res = step()
        torch.cuda.synchronize(self.dev)
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        return t1 - t0, res

    def max_over_ranks(self, vals):
        if not self.dist:
            return vals
        v = self.torch.tensor(vals, dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX)
        return v.tolist()

    def sum_over_ranks(self, x):
        if not self.dist:
            return x
        v = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(v, op=self.dist.ReduceOp.SUM)
        return int(v.item())

    def lynch_step_exchange(self, eng):
        """The one exchange of the Lynch path at N > 1: every rank's unique-
        profile table (O(U) x 16 B) all-gathered as device tensors over RCCL,
        loaded; rank 0 runs the one Nelder-Mead estimate, (pi, eps) broadcast
        over RCCL, the others classify with it."""
        import sid_amd
        from sid_amd import dist as sdist
        keys, cnts = eng.profile_table()
        keys, cnts = sdist.allgather_profile_table(keys, cnts, device=self.dev)
        eng.profile_load(keys, cnts)
        self.last_table = (keys, cnts)
        torch = self.torch
        if self.rank == 0:
            est = eng.estimate()
            vec = torch.tensor([est.heterozygosity, est.error_rate, float(est.iterations)], dtype=torch.float64,
                               device=self.dev)
        else:
            vec = torch.zeros(3, dtype=torch.float64, device=self.dev)
        self.dist.broadcast(vec, 0)
        if self.rank != 0:
            g = sid_amd.Estimate()
            g.heterozygosity, g.error_rate, g.iterations = float(vec[0]), float(vec[1]), int(vec[2])
            est = eng.estimate(given=g)
        return est

    def run_step(self, eng, lynch, capture=False):
        """One step.  capture (untimed, one process): also keep the Lynch
        paths' unique-profile table for the spot check (at N > 1 the exchange
        keeps the gathered one)."""
        st = eng.ingest()
        if lynch and self.dist is not None:
            est = self.lynch_step_exchange(eng)
        else:
            if lynch and capture:
                self.last_table = eng.profile_table()
            est = eng.estimate()
        _, st2 = eng.emit()
        return st, st2, est

    def gather(self, obj):
        """Every rank's obj, in rank order (one process: [obj])."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def placement(self, host):
        """This rank's host placement: its GPU, the GPU's PCI function and
        NUMA node, the CPUs it was bound to, and the NUMA nodes of its pinned
        text's pages (first, middle, last byte)."""
        return dict({"rank": self.rank, "gpu": self.gpu}, **(self.numa or {}), text_numa_nodes=numa_nodes_of(host))


def main():
    a = parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    R = Rank(a)
    cfg = dict(CONFIGS[a.config])
    if cfg["total"]:
        out, eng_keep = bench_strong(R, a, cfg)
    else:
        out, eng_keep = bench_weak(R, a, cfg)
    if R.rank == 0:
        print(json.dumps(out), flush=True)
    for e in eng_keep:
        e.close()
    if R.dist:
        R.dist.barrier()
        R.dist.destroy_process_group()


def bench_weak(R, a, cfg):
    """C2 / C3: 50M sites per GPU; value = the PCIe-inclusive run."""
    import sid_amd
    from sid_amd import gpu as G
    torch = R.torch
    n = a.sites or cfg["per_gpu"]
    first = R.rank * n
    lynch = cfg["method"] != "local" or cfg["R"]
    text, ln = G.synth_text_hbm(cfg["seed"], cfg["depth"], first, n, device=R.gpu)
    if a.device_only:
        dp = device_path(R, a, cfg, text, ln, lynch)
        return {"metric": METRIC, "value": dp["sites_per_s"], "unit": "sites/s", "n_gpus": R.n_gpus,
                "steps": dp["steps"], "ms_per_step": dp["ms_per_step"], "roofline": dp.pop("roofline"),
                "device_path": dp, "note": "--device-only (profiling): value is the device path's"}, []
    host = text[:ln].cpu().pin_memory()     # the rank's input, in host memory (its GPU's NUMA node)
    elapsed, st, st2, est, eng = pcie_leg(R, a, cfg, host, ln, n, lynch)
    sites_all = R.sum_over_ranks(st.sites)
    placement = R.gather(R.placement(host))
    if lynch and R.dist is None:   # (one untimed step more: the profile table for the spot check)
        R.run_step(eng, lynch, capture=True)
    # the first chunk's records from the host arena, for every rank's spot
    # check against the oracle (-m local: the records of a prefix of the text
    # do not depend on the rest; the Lynch paths: given the global profile
    # table, neither do they)
    spot = eng.records_bytes(1)
    if a.dump_records:
        os.makedirs(a.dump_records, exist_ok=True)
        with open(os.path.join(a.dump_records, f"rank{R.rank}.csv"), "wb") as f:
            for j in range(st.chunks):
                p, m = eng.records(j)
                if m:
                    f.write(__import__("ctypes").string_at(p, m))
        with open(os.path.join(a.dump_records, f"rank{R.rank}.json"), "w") as f:
            json.dump({"rank": R.rank, "world": R.world, "sites": st.sites, "first_site": first,
                       "pi": est.heterozygosity if lynch else None, "eps": est.error_rate if lynch else None,
                       "iterations": est.iterations if lynch else None,
                       "n_unique": est.n_unique if lynch else None}, f)
    pcie = pcie_stats(a, ln, st, st2, elapsed, lynch)
    eng.close()
    del host
    spot = spot_check_ranks(R, a, cfg, text, ln, spot, R.last_table if lynch else None)

    dp = device_path(R, a, cfg, text, ln, lynch)
    node_cli, node_cpu = None, None
    if R.world > 1 and not a.no_extras and not a.no_node_cli:
        holder = [text]
        text = None   # the rank's text is freed before the CLI takes the GPUs (the N = 1 extras do not run)
        node_cli, node_cpu = bench_cli_node(R, cfg, holder, ln, n)
    out = {
        "metric": METRIC,
        "value": sites_all * a.steps / elapsed,
        "unit": "sites/s",
        "n_gpus": R.n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (counter-based pileup generator, BASELINE.md): each rank's pileup text in pinned host "
                 "memory when the timed region starts, the CSV records in pinned host memory when it ends "
                 "(H2D, index, parse, call, format, D2H inside every step)"),
        "config": {"workload": f"{a.config}: {cfg['desc']}", "method": cfg["method"],
                   "estimate_prior": cfg["R"], "seed": cfg["seed"], "depth": cfg["depth"],
                   "sites_per_gpu": n, "sites_total": sites_all, "text_bytes_rank0": ln,
                   "csv_bytes_rank0": st2.bytes_out,
                   "parallelism": f"site-range shards x{R.world}" + (
                       (" + RCCL histogram all-gather" if R.backend == "nccl" else
                        f" + {R.backend} histogram all-gather (ranks sharing a GPU)")
                       if lynch and R.world > 1 else ""),
                   "ranks": R.world, "oversubscribed": R.oversub, "dist_backend": R.backend,
                   "rccl_world": R.world if R.dist is not None and R.backend == "nccl" else None,
                   "numa": placement},
        "pcie": pcie,
        "spot_check": spot,
        "roofline": dp.pop("roofline"),
        "device_path": dp,
    }
    if lynch:
        out["estimate"] = {"pi": est.heterozygosity, "eps": est.error_rate, "iterations": est.iterations,
                           "n_unique": est.n_unique}
    if node_cli is not None:
        out["cli"] = node_cli
    if node_cpu is not None and not a.no_cpu:
        out["cpu_baseline"] = node_cpu
    if R.world == 1 and not a.no_extras:
        out["kernel_local"] = bench_kernel_local(torch, R.dev, cfg, n)
        out["cli"] = bench_cli(cfg, text, ln, n)
        if not a.no_cpu:
            out["cpu_baseline"] = bench_cpu(cfg, text, ln, n, R.cpus0)
    return out, []


# C4 / C5 with the rank's shard resident in HBM: 4000 MiB chunks, the
# engine's default for resident text (C5 per shard: 13.74 vs 14.16 ms with
# 2 GiB chunks, profiles/ab_engine_r05.log; the device sink formats into a
# pooled buffer, so the records need no hold arena beside the text)
STRONG_RESIDENT_CHUNK_MIB = 4000


def device_engine(cfg, gpu, chunk_mib, device_sink=1, **kw):
    """The engine of the device path (text in HBM): one device, chunk_mib MiB
    chunks (0 = the engine's 2 GiB default for resident text), records left in
    HBM (device_sink 1).  tests/test_benchpath_gpu.py builds the same engine
    with device_sink 0 to read the records back."""
    import sid_amd
    return sid_amd.Engine(method=cfg["method"], estimate_prior=cfg["R"], devices=1, first_device=gpu,
                          chunk_bytes=chunk_mib << 20, device_sink=device_sink, **kw)


def device_path(R, a, cfg, text, ln, lynch, gen=None):
    """The same sid run over text resident in HBM, records left in HBM: the
    kernels' own rate (the timed steps as the product runs them), then the
    same steps again with HIP event pairs around every engine stage on the
    compute stream (timing events: each pair costs the stream a few us) for
    the stage split and the roofline of the dominant stage."""
    steps = a.device_steps or max(a.steps, 10)
    eng = device_engine(cfg, R.gpu, a.chunk_mib)
    if gen is None:
        eng.source_device_text(text.data_ptr(), ln, keep=text)
    else:
        eng.source_synth(cfg["seed"], gen[1], cfg["depth"], first=gen[0], sites_per_chrom=cfg["spc"],
                         on_device=True)
    eng.profile(False)

    def step():
        return R.run_step(eng, lynch)

    def pstep():
        eng.profile(True)
        return R.run_step(eng, lynch)
    for _ in range(2):
        R.run_step(eng, lynch)
    elapsed, (st, st2, _) = R.timed(step, steps, 0)
    eng.profile_read()
    elapsed_prof, _ = R.timed(pstep, steps, 0)
    prof = eng.profile_read()
    elapsed_prof = R.max_over_ranks([elapsed_prof])[0]
    eng.profile(False)
    eng.close()
    stages = {k[:-3]: v / steps for k, v in prof.items() if k.endswith("_ms")}
    fused = fmt_kind(cfg)
    vals = R.max_over_ranks([elapsed] + [stages[k] for k in sorted(stages)])
    elapsed = vals[0]
    stages = dict(zip(sorted(stages), vals[1:]))
    sites_rank = st.sites
    sites_all = R.sum_over_ranks(sites_rank)
    text_bytes = ln if gen is None else None
    tps = (text_bytes / sites_rank) if text_bytes else (24 + 2.7 * cfg["depth"])
    cps = st2.bytes_out / sites_rank if sites_rank else 0.0
    chunks = prof["chunks"] / steps
    per_launch_sites = sites_rank / max(1.0, chunks)
    roofs = {}
    for k, ms in stages.items():
        if not ms:
            continue
        launch_ms = ms / max(1.0, chunks)
        bps = stage_bytes(k, tps, cps, fused)
        ach = bps * per_launch_sites / (launch_ms * 1e-3) / 1e9
        roofs[k] = {"ms_per_step": ms, "launch_ms": launch_ms, "bytes_per_site": bps, "GBps": ach,
                    "frac": ach / HBM_PEAK_GBS}
    dom = max(roofs, key=lambda k: roofs[k]["ms_per_step"])
    d = roofs[dom]
    roofline = {"bound": "hbm", "achieved": d["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": d["frac"],
                "traffic": pmc_traffic(dom, per_launch_sites, stage_kernels(dom, fused, tps), a.config),
                "kernel": f"engine stage '{dom}'", "stage_kernels": stage_kernels(dom, fused, tps),
                "launch_ms": d["launch_ms"], "sites_per_launch": per_launch_sites, "bytes_per_site": d["bytes_per_site"],
                "valu": valu_issue(dom, per_launch_sites, d["launch_ms"], stage_kernels(dom, fused, tps), a.config),
                "source": "device_path: HIP event pairs around each engine stage on the compute stream"}
    return {"sites_per_s": sites_all * steps / elapsed, "ms_per_step": elapsed / steps * 1e3, "steps": steps,
            "ms_per_step_profiled": elapsed_prof / steps * 1e3,
            "stages_ms": stages, "stages_note": "HIP event pairs around every stage, in a second run of the same "
                                                "steps (ms_per_step_profiled)",
            "stage_roofline": roofs, "roofline": roofline,
            "chunks_per_step": chunks, "chunks_tiled_last_step": st.chunks_tiled,
            "tile_overflows_last_step": st.tile_overflows,
            "path": {"bytes_per_site": tps + cps, "text_per_site": tps, "csv_per_site": cps,
                     "GBps": (text_bytes + st2.bytes_out) / (elapsed / steps) / 1e9 if text_bytes else None,
                     "note": "text in + CSV out per step (the path's minimum HBM traffic) / ms_per_step"},
            "note": "text resident in HBM before the timed region, records formatted into HBM (device_sink 1)"}


STRONG_PARTS = 8   # C4 / C5 are quoted on 8 GPUs: a rank's shard is 1/8 of the config's sites


def host_hold_bytes(n):
    """The PCIe path's host arena for n sites: every chunk's records fit (the
    CSV is ~42.7 B/site at 30x and at 200x)."""
    return int(n * 48) + (64 << 20)


def pcie_engine(cfg, gpu, n, ln, chunk_mib=0, slots=0):
    """The engine of the `value` leg (C2 - C5): one device, host text in
    chunk_mib MiB chunks (0 = the engine's 128 MiB), each chunk's records
    copied into the pinned host arena during the ingest (device_sink 2: not
    written anywhere else; sid_engine_records reads them).
    tests/test_benchpath_gpu.py builds the same engine."""
    import sid_amd
    return sid_amd.Engine(method=cfg["method"], estimate_prior=cfg["R"], devices=1, first_device=gpu,
                          chunk_bytes=chunk_mib << 20, slots=slots, device_sink=2,
                          host_hold_bytes=host_hold_bytes(n))


def pcie_leg(R, a, cfg, host, ln, n, lynch):
    """The timed value leg over pinned host text of n sites: (elapsed, ingest
    stats, emit stats, estimate, engine) -- the engine still open, its
    records in its host arena."""
    eng = pcie_engine(cfg, R.gpu, n, ln, a.pcie_chunk_mib, a.slots)
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    elapsed, (st, st2, est) = R.timed(lambda: R.run_step(eng, lynch), a.steps, a.warmup)
    elapsed = R.max_over_ranks([elapsed])[0]
    if st2.bytes_out == 0 and st.sites:
        raise SystemExit("bench.py: no records came back")
    return elapsed, st, st2, est, eng


def pcie_stats(a, ln, st, st2, elapsed, lynch):
    pcie = {"text_bytes": ln, "csv_bytes": st2.bytes_out,
            "GBps_h2d": ln / (elapsed / a.steps) / 1e9, "GBps_d2h": st2.bytes_out / (elapsed / a.steps) / 1e9,
            "chunks": st.chunks, "chunks_held_in_host_arena": st.chunks_held, "ingest_s": st.ingest_s,
            "emit_s": st2.emit_s, "h2d_s_last_step": st.h2d_s, "chunks_tiled_last_step": st.chunks_tiled,
            "tile_overflows_last_step": st.tile_overflows,
            "h2d_GBps_last_step": st.h2d_bytes / st.h2d_s / 1e9 if st.h2d_s else None}
    pcie["ceiling"] = pcie_ceiling(ln, st2.bytes_out, lynch, elapsed / a.steps)
    return pcie


def bench_strong(R, a, cfg):
    """C4 / C5 on the metric's footing (in-memory pileup text
    -> CSV): each rank takes 1/8 of the config's sites (C4: 375M sites, 30.4 GB
    of text; C5: 62.5M sites at 200x, 26.6 GB), so N = 8 ranks run the whole
    config (3G / 500M sites) and N = 1 its first eighth.  The value leg is
    C2's step: the shard's text in pinned host memory on the GPU's NUMA node
    when the timed region starts -> H2D, index, parse, call, format -> the
    CSV records in the pinned host arena (sid.cpp:85-105, call.cpp:213-289).
    Beside it, device_path: the same shard resident in HBM (generated there
    before the timed region), records formatted into HBM -- the kernels'
    own rate."""
    torch = R.torch
    import sid_amd
    total = a.sites or cfg["total"]
    if R.world > STRONG_PARTS:
        raise SystemExit(f"bench.py: {a.config} is split into {STRONG_PARTS} shards; {R.world} ranks")
    per = total // STRONG_PARTS
    first, n = R.rank * per, per
    t0 = time.perf_counter()
    text, ln = generate_resident(torch, sid_amd, R.dev, R.gpu, cfg, first, n)
    gen_ms = (time.perf_counter() - t0) * 1e3
    lynch = cfg["method"] != "local" or cfg["R"]
    if a.device_only:
        a.chunk_mib = a.chunk_mib or STRONG_RESIDENT_CHUNK_MIB
        dp = device_path(R, a, cfg, text, ln, lynch)
        return {"metric": METRIC, "value": dp["sites_per_s"], "unit": "sites/s", "n_gpus": R.n_gpus,
                "steps": dp["steps"], "ms_per_step": dp["ms_per_step"], "roofline": dp.pop("roofline"),
                "device_path": dp, "note": "--device-only (profiling): value is the device path's"}, []
    host = torch.empty(ln, dtype=torch.uint8, pin_memory=True)   # on the GPU's NUMA node (numa_bind)
    host.copy_(text[:ln])
    torch.cuda.synchronize(R.dev)
    elapsed, st, st2, est, eng = pcie_leg(R, a, cfg, host, ln, n, lynch)
    sites_all = R.sum_over_ranks(st.sites)
    placement = R.gather(R.placement(host))
    spot = eng.records_bytes(1)
    pcie = pcie_stats(a, ln, st, st2, elapsed, lynch)
    eng.close()
    del host
    spot = spot_check_ranks(R, a, cfg, text, ln, spot, None)
    if not a.chunk_mib:
        a.chunk_mib = STRONG_RESIDENT_CHUNK_MIB
    dp = device_path(R, a, cfg, text, ln, lynch)
    out = {
        "metric": METRIC,
        "value": sites_all * a.steps / elapsed,
        "unit": "sites/s",
        "n_gpus": R.n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (counter-based pileup generator, BASELINE.md): each rank's 1/8 shard of the config's "
                 "text in pinned host memory when the timed region starts, the CSV records in pinned host memory "
                 "when it ends (H2D, index, parse, call, format, D2H inside every step)"),
        "config": {"workload": f"{a.config}: {cfg['desc']}; 1/{STRONG_PARTS} of its {total:,} sites per GPU "
                               f"({per:,} sites; {STRONG_PARTS} GPUs run the whole config)",
                   "method": cfg["method"], "seed": cfg["seed"], "depth": cfg["depth"], "sites_total": total,
                   "sites_per_gpu": per, "sites_all_ranks": sites_all, "first_site_rank0": 0,
                   "sites_per_chrom": cfg["spc"], "text_bytes_rank0": ln, "csv_bytes_rank0": st2.bytes_out,
                   "parallelism": f"site-range shards x{R.world}", "ranks": R.world,
                   "oversubscribed": R.oversub, "numa": placement},
        "pcie": pcie,
        "spot_check": spot,
        "roofline": dp.pop("roofline"),
        "device_path": dp,
        "generator": {"ms": gen_ms, "inside_step": False,
                      "note": "the shard's text generated into HBM (then copied to pinned host memory), before "
                              "the timed region"},
    }
    if R.world == 1 and not a.no_extras and not a.no_cpu:
        out["cpu_baseline"] = bench_cpu(cfg, text, ln, n, R.cpus0,
                                        sample_sites=50_000_000 if cfg["depth"] < 100 else 10_000_000)
    return out, []


def generate_resident(torch, sid_amd, dev, gpu, cfg, first, n):
    """The rank's shard of C4/C5 as text in HBM: one buffer sized to the
    text (the rest, at least a 24 GiB reserve, stays free for the engine's
    chunk workspace, pooled record buffers and hold arena), filled by the device generator in 50M-site pieces
    laid end to end (every line stands alone, so the pieces concatenate to the
    shard's text)."""
    free, _ = torch.cuda.mem_get_info(dev)
    need = int(n * (2.72 * cfg["depth"] + 2))   # ~81 B/site at 30x, ~564 at 200x (measured)
    cap = min(free - (24 << 30), int(need * 1.03) + (1 << 30))
    text = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = sid_amd.Context(gpu)
    ln, piece = 0, 50_000_000
    for lo in range(0, n, piece):
        m = min(piece, n - lo)
        ln += ctx.synth_text_device(cfg["seed"], cfg["depth"], first + lo, m, text.data_ptr() + ln,
                                    cap - 512 - ln, sites_per_chrom=cfg["spc"])
    text[ln:ln + 512].zero_()
    torch.cuda.synchronize(dev)
    ctx.close()
    return text, ln


# wave64 VALU instructions/s the chip issues: 1024 SIMDs x one per 3.53
# cycles at 2.33 GHz, measured (tools/debug/valu_rate_probe.hip,
# profiles/valu_rate_probe_r06.jsonl: 32-bit integer VALU streams at 8 waves
# a SIMD, the in-kernel clock).  A SIMD is 16 lanes wide: a wave64
# instruction holds it for 4 cycles (157.3 TF f32 = 1024 x 16 lanes x 2 FMA x
# 2 packed x 2.4 GHz).  (Round 5 priced one per 2 cycles at 2.4 GHz, 1.82x
# this, and so read the tile parse as half busy.)
VALU_ISSUE_PER_S = 1024 * 2.33e9 / 3.53
PMC_ROUND = os.environ.get("SID_PMC_ROUND", "r06")


def pcie_ceiling(text_bytes, csv_bytes, lynch, step_s):
    """The step's PCIe floor from the committed probe of these boxes
    (profiles/pcie_probe_r03.jsonl, tools/debug/pcie_probe.cpp): -m local
    overlaps the records' D2H with the upload (full duplex: the H2D at its
    duplex rate), the Lynch paths format after the estimate (H2D, then D2H)."""
    try:
        rows = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "pcie_probe_r03.jsonl")) if l.strip()]
    except OSError:
        return None
    best = {}
    for r in rows:
        best[r["probe"]] = max(best.get(r["probe"], 0.0), r["GBps"])
    h2d_duplex, h2d, d2h = best.get("duplex_h2d_part"), best.get("h2d_128MiB_pieces"), best.get("d2h_one_2GiB")
    if not (h2d_duplex and h2d and d2h):
        return None
    floor = (text_bytes / (h2d * 1e9) + csv_bytes / (d2h * 1e9)) if lynch else \
        max(text_bytes / (h2d_duplex * 1e9), csv_bytes / (d2h * 1e9))
    return {"floor_ms": floor * 1e3, "frac": floor / step_s, "GBps_h2d": h2d, "GBps_h2d_duplex": h2d_duplex,
            "GBps_d2h": d2h, "source": "profiles/pcie_probe_r03.jsonl (pinned copies, best of the probe's runs)"}


def pmc_file(stage, config="C2"):
    """The committed per-stage PMC file: the config's own (pmc_<stage>_<round>_<config>.json)
    before the C2 one."""
    names = ([f"pmc_{stage}_{PMC_ROUND}_{config.lower()}.json"] if config != "C2" else []) + \
        [f"pmc_{stage}_{r}.json" for r in (PMC_ROUND, "r02")]
    for n in names:
        p = os.path.join(ROOT, "profiles", n)
        if os.path.exists(p):
            return p
    return None


def valu_issue(stage, sites, launch_ms, kernels, config="C2"):
    """The stage's VALU work against the chip's VALU issue rate: SQ_INSTS_VALU
    per site of its kernels (the committed PMC pass, tools/gpu/profile.sh) x
    the sites of a launch, at one wave64 instruction per SIMD per 2 cycles
    (MI355X_MICROARCH.md); None when absent."""
    try:
        summ = None
        for n in [f"pmc_{config.lower()}_{PMC_ROUND}_summary.json"] + [f"pmc_c2_{r}_summary.json"
                                                                     for r in (PMC_ROUND, "r02")]:
            p = os.path.join(ROOT, "profiles", n)
            if os.path.exists(p):
                summ = p
                break
        pm = json.load(open(summ))
        sites_pmc = json.load(open(pmc_file(stage, config)))["sites_per_launch"]
    except Exception:
        return None
    insts = 0.0
    for k in kernels:
        found = False
        for name, r in pm.items():
            if name.startswith(k.rstrip("*")) and "SQ_INSTS_VALU" in r:
                insts += r["SQ_INSTS_VALU"] / sites_pmc
                found = True
        # a stage kernel the committed counters do not cover (another config's
        # kernels): no figure rather than a partial one (the rare-path helpers
        # excepted)
        if not found and not k.endswith("*") and not any(x in k for x in ("serial", "list", "fixlen")):
            return None
    if not insts:
        return None
    per_launch = insts * sites
    issue_ms = per_launch / VALU_ISSUE_PER_S * 1e3
    return {"insts_per_launch": per_launch, "issue_bound_ms": issue_ms, "frac": issue_ms / launch_ms,
            "note": "VALU instructions of the stage's kernels (PMC) at the chip's issue rate vs the measured launch"}


def pmc_traffic(stage, sites, kernels=None, config="C2"):
    """HBM bytes per launch of the stage from the committed PMC summary
    (tools/pmc_stages.py over separate FETCH_SIZE / WRITE_SIZE passes), scaled
    to this launch's sites; None when absent, or when the committed pass
    measured other kernels for this stage (the counters are C2's: a C3 line's
    parse stage runs sid_parse_kernel, not sid_parse_len_kernel)."""
    p = pmc_file(stage, config)
    try:
        d = json.load(open(p))
        measured = d.get("kernels", {})
        for k in kernels or []:
            if k.endswith("*") or any(x in k for x in ("serial", "list", "fixlen")):
                continue
            if not measured.get(k):
                return None
        return d["hbm_bytes_per_site"] * sites
    except Exception:
        return None


def bench_kernel_local(torch, dev, cfg, n):
    """sid_call_local alone over the counts of the same sites resident in HBM
    (the per-site arithmetic kernel: 25 B/site), HIP events on its stream."""
    import sid_amd
    ctx = sid_amd.Context(dev.index)
    st = torch.cuda.current_stream(dev)
    counts = torch.empty((n, 4), dtype=torch.int16, device=dev)
    code = torch.empty(n, dtype=torch.uint8, device=dev)
    hom = torch.empty(n, dtype=torch.float64, device=dev)
    het = torch.empty(n, dtype=torch.float64, device=dev)
    ctx.synth_counts(cfg["seed"], cfg["depth"], 0, n, counts.data_ptr(), st.cuda_stream)
    args = (counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
    for _ in range(3):
        ctx.call_local(*args)
    torch.cuda.synchronize(dev)
    K = 20
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for s, e in ev:
        s.record(st)
        ctx.call_local(*args)
        e.record(st)
    torch.cuda.synchronize(dev)
    ms = sum(s.elapsed_time(e) for s, e in ev) / K
    ctx.timing_enable(True)
    for _ in range(10):
        ctx.call_local(*args)
    torch.cuda.synchronize(dev)
    ctx.timing_enable(False)
    _, main_ms, fix_ms = ctx.timing_read()
    ctx.close()
    gbs = LOCAL_BYTES_PER_SITE * n / (ms * 1e-3) / 1e9
    pm = None
    try:
        pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_local_r01.json"))).get("hbm_bytes_per_launch")
    except Exception:
        pass
    return {"sites_per_s": n / (ms * 1e-3), "ms": ms, "GBps": gbs, "frac": gbs / HBM_PEAK_GBS,
            "split_ms": {"sid_local_table_p2": main_ms, "sid_local_fixup": fix_ms}, "bytes_per_site": 25,
            "traffic": pm, "note": "counts resident in HBM -> code + confs (the round-1 headline kernel)"}


def bench_cli(cfg, text, ln, n):
    """build/sid on the same text as a file in the page cache, CSV to
    /dev/null: wall clock (process start, HIP init, mapping, both PCIe legs,
    write) and the CLI's own clock."""
    cli = os.path.join(ROOT, "build", "sid")
    if not os.path.exists(cli):
        return None
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "c.plp")
        write_text_file(text, ln, path)
        flags = [] if cfg["method"] == "local" else (["-R"] if cfg["R"] else []) + ["-m", cfg["method"]]
        cli_runs = []
        for _ in range(6):   # the first warms the page cache and the code objects; the median of the other 5
            with open(os.devnull, "wb") as dn:
                u0 = time.time()
                t0 = time.perf_counter()
                r = subprocess.run([cli, "--stats"] + flags + [path], stdout=dn, stderr=subprocess.PIPE)
                dt = time.perf_counter() - t0
                u1 = time.time()
            if r.returncode != 0:
                return {"error": r.returncode, "stderr": r.stderr.decode()[-400:]}
            try:
                stt = json.loads(r.stderr.decode().strip().splitlines()[-1])
            except Exception:
                stt = {}
            if "main_entry_unix" in stt:   # the process's start-up (exec, loading) and teardown, apart
                stt["startup_s"] = stt["main_entry_unix"] - u0
                stt["teardown_s"] = u1 - stt["main_exit_unix"]
            cli_runs.append((dt, stt))
        dt, stt = sorted(cli_runs[1:], key=lambda x: x[0])[len(cli_runs[1:]) // 2]
        return {"wall_s": dt, "wall_s_is": "median of 5 runs after one warm-up",
                "sites_per_s_wall": n / dt, "sites_per_s_cli_clock": stt.get("sites_per_s"),
                "wall_s_runs": [x[0] for x in cli_runs], "cli_stats": stt,
                # main() entry to its last line, and its last line to the exit seen here (the
                # driver's teardown of a GPU process: 1 ms or 0.1-0.15 s, run to run)
                "main_s_median": statistics.median(x[1]["main_exit_unix"] - x[1]["main_entry_unix"]
                                                   for x in cli_runs[1:]) if all("main_entry_unix" in x[1] for x in cli_runs[1:]) else None,
                "teardown_s_runs": [x[1].get("teardown_s") for x in cli_runs],
                "note": "build/sid FILE > /dev/null, one GPU: wall = process start + HIP init + mmap + "
                        "H2D + parse/call/format + D2H + write; cli_clock = input mapping to last write; "
                        "startup_s = exec to main(), teardown_s = main's last line to the exit seen here"}


def bench_cli_node(R, cfg, holder, ln, n):
    """N > 1: the drop-in over the whole node.  Every rank writes its text
    into one file (the shards in rank order, each at its byte offset), frees
    its GPU memory and waits on the store (no collective runs on the GPUs
    meanwhile); rank 0 runs `build/sid --devices N --stats FILE > /dev/null`
    (one mapping, one uploader per device, chunks dealt round robin, one
    ordered writer: main.cpp, run.cpp) -- one warm-up, then the median of 3.
    The reference's whole-node shape is one sid process per chromosome
    (scripts/sid-pipeline/parallel-run-sid.sh:2); this is one process over
    every GPU."""
    import shutil
    from datetime import timedelta
    torch, dist = R.torch, R.dist
    cli = os.path.join(ROOT, "build", "sid")
    lens = [None] * R.world
    dist.all_gather_object(lens, int(ln))
    total = sum(lens)
    info = [None]
    if R.rank == 0 and os.path.exists(cli):
        for cand in (tempfile.gettempdir(), "/dev/shm"):
            try:
                if shutil.disk_usage(cand).free > total + (8 << 30):
                    d = tempfile.mkdtemp(prefix="sid_node_", dir=cand)
                    path = os.path.join(d, "node.plp")
                    with open(path, "wb") as f:
                        f.truncate(total)
                    info = [path]
                    break
            except OSError:
                pass
    dist.broadcast_object_list(info, 0)
    path = info[0]
    text = holder.pop()
    if path is not None:
        t0 = time.perf_counter()
        fd = os.open(path, os.O_WRONLY)
        off, step = sum(lens[:R.rank]), 256 << 20
        for lo in range(0, ln, step):
            os.pwrite(fd, text[lo:min(ln, lo + step)].cpu().numpy().tobytes(), off + lo)
        os.close(fd)
        write_s = time.perf_counter() - t0
    del text
    torch.cuda.synchronize(R.dev)
    torch.cuda.empty_cache()
    torch._C._host_emptyCache()
    dist.barrier()
    if path is None:
        return {"skipped": f"build/sid missing or no directory with {total / 1e9:.1f} GB free"}, None
    store = dist.distributed_c10d._get_default_store()
    res, cpu = None, None
    if R.rank == 0:
        try:
            # the CLI runs unbound (it places its own threads per GPU): this
            # thread's mask widened for the fork, which the child inherits, and
            # restored after (no preexec_fn: this process runs other threads)
            mask = os.sched_getaffinity(0)
            args = [cli, "--stats", "--devices", str(R.world)] + method_flags(cfg) + [path]

            def median_of(env):
                runs = []
                for _ in range(4):
                    with open(os.devnull, "wb") as dn:
                        os.sched_setaffinity(0, R.cpus0)
                        try:
                            t0 = time.perf_counter()
                            r = subprocess.run(args, stdout=dn, stderr=subprocess.PIPE, env=env)
                            dt = time.perf_counter() - t0
                        finally:
                            os.sched_setaffinity(0, mask)
                    if r.returncode != 0:
                        return {"error": r.returncode, "stderr": r.stderr.decode()[-400:]}, None
                    try:
                        stt = json.loads(r.stderr.decode().strip().splitlines()[-1])
                    except Exception:
                        stt = {}
                    runs.append((dt, stt))
                dt, stt = sorted(runs[1:], key=lambda x: x[0])[len(runs[1:]) // 2]
                return {"wall_s": dt, "wall_s_runs": [x[0] for x in runs], "cli_stats": stt}, dt
            # the uploads from registered pages (the default) and through the
            # runtime's pageable path (SID_UPLOAD_REGISTER=0), one after the other
            reg, dt = median_of(dict(os.environ, SID_UPLOAD_REGISTER="1"))
            if dt is None:
                res = reg
            else:
                pageable, dt0 = median_of(dict(os.environ, SID_UPLOAD_REGISTER="0"))
                sites = n * R.world
                stt = reg["cli_stats"]
                res = {"devices": R.world, "sites": sites, "text_bytes": total, "wall_s": dt,
                       "wall_s_is": "median of 3 runs after one warm-up", "sites_per_s_wall": sites / dt,
                       "sites_per_s_cli_clock": stt.get("sites_per_s"), "wall_s_runs": reg["wall_s_runs"],
                       "cli_stats": stt, "placement": stt.get("placement"), "file_write_s_rank0": write_s,
                       "upload_pageable": dict(pageable, sites_per_s_wall=sites / dt0 if dt0 else None),
                       "note": f"build/sid --devices {R.world} FILE > /dev/null on one file holding every "
                               "rank's shard (the whole node's drop-in: one process, every GPU); wall = "
                               "process start + HIP init + mapping + H2D + kernels + D2H + write; the uploads "
                               "from registered pages (the default), and in upload_pageable through the "
                               "runtime's pageable path (SID_UPLOAD_REGISTER=0)"}
                if cfg["method"] == "local" and dt is not None:
                    # the whole node's CPU path beside it: the oracle over the same file, one
                    # line-aligned shard process per CPU the job may use
                    P, share = cpu_share(R.cpus0)
                    dtc = oracle_shards(path, total, P, method_flags(cfg), R.cpus0)
                    cpu = {"value": sites / dtc if dtc else None, "unit": "sites/s", "cores": P, "kind": "port",
                           "seconds": dtc, "cpu_model": cpu_model(), "cpu_share": share,
                           "sample": f"the node file ({sites:,} sites, every rank's shard, {total / 1e9:.2f} GB), "
                                     f"{P} line-aligned byte ranges, one oracle/_build/sid_oracle process each, "
                                     "CSV to /dev/null, wall"}
                elif dt is not None:
                    # the Lynch paths: one estimate over every site, so one
                    # oracle process, on a bounded sample of the node file
                    sys.path.insert(0, os.path.join(ROOT, "oracle"))
                    import oracle
                    m = min(sites, 4_000_000)
                    dtc, rc = one_process([oracle.CLI] + method_flags(cfg), path, line_end(path, m))
                    cpu = {"value": m / dtc if rc == 0 else None, "unit": "sites/s", "cores": 1, "kind": "port",
                           "seconds": dtc, "cpu_model": cpu_model(), "cpu_share": cpu_share(R.cpus0)[1],
                           "sample": f"the first {m:,} sites of the node file (rank 0's shard), one "
                                     "oracle/_build/sid_oracle process (the Lynch estimate and BH are global: "
                                     "call.cpp:62-143), CSV to /dev/null, wall"}
        finally:
            store.set("sid_node_cli_done", "1")
            try:
                shutil.rmtree(os.path.dirname(path))
            except OSError:
                pass
    else:
        store.wait(["sid_node_cli_done"], timedelta(minutes=15))
    dist.barrier()
    return res, cpu


def spot_check_ranks(R, a, cfg, text, ln, spot, table):
    """Every rank checks its value leg's first chunk of records (from the
    engine's pinned host arena, after the timed steps) byte for byte against
    the oracle CLI over the same lines of its own text; for the Lynch paths
    the oracle is given the global unique-profile table the rank used
    (ORACLE_PROFILE_TABLE: the estimate and BH run over every rank's
    profiles, call.cpp:62-143).  Gathered in rank order; a rank whose records
    differ fails the bench on every rank (after the gather, so none hangs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    res = {"rank": R.rank, "records": spot.count(b"\n"), "bytes": len(spot), "equal": None}
    try:
        if not os.path.exists(oracle.CLI):
            oracle.build()
        if spot:
            # the text through the line of the chunk's last record (its chrom
            # and position are unique in the rank's text; sites after it in
            # the chunk, dropped by the Lynch paths' coverage filter, print
            # nothing)
            last = spot[:-1].rsplit(b"\n", 1)[-1]
            chrom, pos = last.split(b",", 2)[:2]
            key = chrom + b"\t" + pos + b"\t"
            want = ((a.pcie_chunk_mib or 128) + 8) << 20
            prefix = text[:min(ln, want)].cpu().numpy().tobytes()
            at = 0 if prefix.startswith(key) else prefix.find(b"\n" + key) + 1
            if at == 0 and not prefix.startswith(key):
                res["equal"] = False
                res["why"] = "the last record's line is not in the chunk's text"
            else:
                cut = prefix.index(b"\n", at) + 1
                with tempfile.TemporaryDirectory() as td:
                    path = os.path.join(td, "spot.plp")
                    with open(path, "wb") as f:
                        f.write(prefix[:cut])
                    env = dict(os.environ)
                    if table is not None:
                        import numpy as np
                        tp = os.path.join(td, "table.bin")
                        np.stack([np.asarray(table[0], np.uint64), np.asarray(table[1], np.uint64)], 1).tofile(tp)
                        env["ORACLE_PROFILE_TABLE"] = tp
                        res["profile_table_rows"] = int(len(table[0]))
                    r = subprocess.run([oracle.CLI] + method_flags(cfg) + [path], stdout=subprocess.PIPE,
                                       stderr=subprocess.PIPE, env=env)
                res["lines"] = prefix[:cut].count(b"\n")
                res["equal"] = r.returncode == 0 and r.stdout == b"chrom,pos,label,gt,hom_conf,het_conf,conf_type\n" + spot
                if r.returncode != 0:
                    res["why"] = f"oracle rc {r.returncode}: {r.stderr.decode()[-200:]}"
        else:
            res["equal"] = ln == 0
    except Exception as e:   # (reported, and fails the bench below)
        res["equal"] = False
        res["why"] = repr(e)[:300]
    ranks = R.gather(res)
    out = {"ranks_equal": all(x["equal"] for x in ranks), "ranks": ranks,
           "what": "each rank's timed PCIe leg, its first chunk of records (engine host arena) vs the oracle CLI "
                   "over the same lines of the rank's text" + (", given the global unique-profile table"
                                                                  if table is not None else "")}
    if not out["ranks_equal"]:
        raise SystemExit(f"bench.py: a rank's records differ from the oracle's (spot check): {ranks}")
    return out


def write_text_file(text, ln, path):
    """The resident text, copied back in 256 MiB pieces, as a file."""
    step = 256 << 20
    with open(path, "wb") as f:
        for lo in range(0, ln, step):
            f.write(text[lo:min(ln, lo + step)].cpu().numpy().tobytes())
    with open(path, "rb") as f:   # into the page cache
        while f.read(1 << 26):
            pass


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_share(cpus):
    """The CPUs this job may use: its affinity mask (before the rank's NUMA
    binding), capped by its cgroup's CPU quota (a GPU box's share of a larger
    machine: os.cpu_count() shows the whole machine there)."""
    n = len(cpus)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return n, {"affinity_cpus": len(cpus), "cgroup_quota_cpus": quota, "nproc": os.cpu_count()}


def line_cuts(path, ln, P):
    """P line-aligned byte ranges covering the file's first ln bytes."""
    cuts = [0]
    with open(path, "rb") as f:
        for k in range(1, P):
            c = max(cuts[-1], ln * k // P)
            f.seek(c)
            w = f.read(1 << 20)
            nl = w.find(b"\n")
            cuts.append(min(ln, c + nl + 1) if nl >= 0 else ln)
    cuts.append(ln)
    return [(cuts[k], cuts[k + 1] - cuts[k]) for k in range(P) if cuts[k + 1] > cuts[k]]


def oracle_shards(path, ln, P, flags, cpus, cmd=None):
    """The oracle CLI (or cmd, a command taking FILE last) in P processes over
    line-aligned byte ranges of one file (ORACLE_RANGE: the harness's byte
    range), CSV to /dev/null: wall seconds, or None when a process failed.
    -m local only: its sites are independent (the reference's whole-node
    shape, one sid per chromosome, scripts/sid-pipeline/parallel-run-sid.sh:2,
    is the same split)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    if cmd is None:
        if not os.path.exists(oracle.CLI):
            oracle.build()
        cmd = [oracle.CLI] + flags
    ranges = line_cuts(path, ln, P)
    # the processes run on every CPU of the job (this thread's mask, which
    # they inherit, widened from the rank's NUMA binding for the forks)
    mask = os.sched_getaffinity(0)
    os.sched_setaffinity(0, cpus)
    try:
        with open(os.devnull, "wb") as dn:
            t0 = time.perf_counter()
            procs = [subprocess.Popen(cmd + [path], stdout=dn, stderr=subprocess.DEVNULL,
                                      env=dict(os.environ, ORACLE_RANGE=f"{o}:{m}")) for o, m in ranges]
            rcs = [p.wait() for p in procs]
            dt = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, mask)
    return None if any(rcs) else dt


def one_process(cmd, path, c1):
    """cmd over the first c1 bytes of path in one process, CSV to /dev/null:
    (wall seconds, exit code)."""
    with open(os.devnull, "wb") as dn:
        t0 = time.perf_counter()
        r = subprocess.run(cmd + [path], stdout=dn, stderr=subprocess.DEVNULL, env=dict(os.environ, ORACLE_RANGE=f"0:{c1}"))
        return time.perf_counter() - t0, r.returncode


def line_end(path, m):
    """The byte offset after the file's first m lines."""
    base = 0
    with open(path, "rb") as f:
        while m:
            blk = f.read(1 << 24)
            if not blk:
                return base
            k = blk.count(b"\n")
            if k < m:
                m -= k
                base += len(blk)
                continue
            idx = -1
            for _ in range(m):
                idx = blk.find(b"\n", idx + 1)
            return base + idx + 1
    return base


def method_flags(cfg):
    return [] if cfg["method"] == "local" else (["-R"] if cfg["R"] else []) + ["-m", cfg["method"]]


def bench_cpu(cfg, text, ln, n, cpus, sample_sites=None):
    """The CPU path on the same text, bounded to sample_sites (default: all n),
    on this job's CPUs:
      value              the oracle CLI (reference sid.cpp/call.cpp/lynch/stats
                         restated in C, single-threaded): one line-aligned
                         shard process per CPU (-m local: sites are
                         independent), and one process on the first 4M sites;
                         the Lynch paths (a global estimate): one process
      reference_sources  -m local: oracle/_ref/ref_pileup local, the
                         reference's own pileup.cpp, countUniqueProfiles,
                         profile map and call.hpp iostream output (each unique
                         profile's GSL arithmetic from the oracle), timed
                         the same two ways (timing only: it pins nothing)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    if not os.path.exists(oracle.CLI):
        oracle.build()
    flags = method_flags(cfg)
    P, share = cpu_share(cpus)
    m_all = min(n, sample_sites or n)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sample.plp")
        # the sample as one file (256 MiB pieces from HBM), its cut after m_all lines
        step, cut = 256 << 20, 0
        with open(path, "wb") as f:
            need = m_all
            for lo in range(0, ln, step):
                seg = text[lo:min(ln, lo + step)].cpu().numpy().tobytes()
                k = seg.count(b"\n")
                if k >= need:
                    idx = -1
                    for _ in range(need):
                        idx = seg.find(b"\n", idx + 1)
                    f.write(seg[:idx + 1])
                    cut += idx + 1
                    need = 0
                    break
                f.write(seg)
                cut += len(seg)
                need -= k
        res = {"unit": "sites/s", "kind": "port", "cpu_model": cpu_model(), "cpu_share": share}
        shard_desc = (f"{m_all:,} sites of the {cfg['desc']} text ({cut / 1e9:.2f} GB), {P} line-aligned byte ranges "
                      f"of one file (one per CPU this job may use), one process each, CSV to /dev/null, wall")
        if cfg["method"] == "local":
            dt = oracle_shards(path, cut, P, flags, cpus)
            res.update({"value": m_all / dt if dt else None, "cores": P, "seconds": dt,
                        "sample": shard_desc.replace("one process each", "one oracle/_build/sid_oracle process each")})
        # one core on the first 4M sites
        m = min(m_all, 4_000_000)
        c1 = line_end(path, m)
        dt, rc = one_process([oracle.CLI] + flags, path, c1)
        single = {"value": m / dt if rc == 0 else None, "cores": 1, "seconds": dt,
                  "sample": f"the first {m:,} sites of the same text, one process" + (
                      " (the Lynch estimate is global: one process)" if cfg["method"] != "local" else "")}
        if "value" not in res:
            res.update(single)
            res["sample"] = single["sample"]
        else:
            res["single_core"] = single
        if cfg["method"] == "local" and not cfg["R"] and oracle.ref_pileup_available():
            cmd = [oracle.REF_PILEUP, "local"]
            dts, rcs = one_process(cmd, path, c1)
            dtp = oracle_shards(path, cut, P, flags, cpus, cmd=cmd)
            ref_p = m_all / dtp if dtp else None
            ref_1 = m / dts if rcs == 0 else None
            res["reference_sources"] = {
                "value": ref_p, "cores": P, "seconds": dtp, "sample": shard_desc,
                "single_core": {"value": ref_1, "cores": 1, "seconds": dts,
                                "sample": f"the first {m:,} sites, one process"},
                # the same box, the same sample: how much faster the port is
                "port_over_reference": {"cores": res["value"] / ref_p if ref_p and res.get("value") else None,
                                        "single_core": single["value"] / ref_1 if ref_1 and single["value"]
                                        else None},
                "binary": "oracle/_ref/ref_pileup local (built by oracle/Makefile from the reference's pileup.cpp "
                          "and call.hpp, unmodified, -O2 as its autotools default; -fopenmp dropped: readFile is "
                          "serial)",
                "what": "the reference's own -m local per-site work: ifstream + getline + parsePileupLine into "
                        "std::vector<PileupLine> (call.cpp:11-20), countUniqueProfiles (pileup.cpp:169-196), "
                        "std::map profile -> class (call.cpp:216-221, 274-285), records through call.hpp:29-38's "
                        "operator<< on synced iostreams (sid.cpp:102-105); each unique profile's arithmetic "
                        "(call.cpp:238-273, GSL) from the oracle, once per profile; timing only, output "
                        "byte-equal to the oracle's (tests/test_oracle_kat.py)"}
    return res


if __name__ == "__main__":
    main()
