#!/usr/bin/env python3
"""bench.py — RHO radix hash join (+ predicate scan) on MI355X, BASELINE.json's metric.

Step = one full RHO join (partition pass 1 + pass 2 + build/probe, count-only) over
|R| = |S| = 2^28 uniform tuples per GPU (BASELINE config 2; weak scaling: with N GPUs
the global relations are N * 2^28 and are radix-sharded with an RCCL all-to-all of
each relation in pieces, sgxamd.dist).  Inputs are resident in HBM before the timed region.

One JSON line (rank 0):
  value = probed tuples (|S|, all ranks) per second over the whole join, in millions;
  roofline = the dominant kernel's algorithmic bytes / its HIP-event time vs 8 TB/s;
  cpu_baseline = the oracle's restated reference RHO (oracle/rho_oracle.c, pthreads)
  on a bounded sample of reference-generated relations on this host's cores.
The scan (BASELINE config 3: 2^30 int32, 10 % selectivity) is measured in the same run
and reported under "scan".
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd")
sys.path.insert(0, os.path.join(PKG, "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
TABLE_STEPS = 3  # untimed full-timing steps after a timed region (per-kernel table)
METRIC = "M probed tuples/sec (RHO join) + scan GB/s vs HBM roofline, 1/2/4/8 MI355X"
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic_r06zm.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_topology() -> dict:
    """CPU model, sockets, cores, NUMA nodes and the cgroup CPU quota of this host."""
    info: dict = {}
    try:
        with open("/proc/cpuinfo") as f:
            txt = f.read()
        info["model"] = next((ln.split(":", 1)[1].strip() for ln in txt.splitlines()
                              if ln.startswith("model name")), None)
        info["sockets"] = len({ln.split(":", 1)[1].strip() for ln in txt.splitlines() if ln.startswith("physical id")})
        info["logical_cpus"] = os.cpu_count()
    except OSError:
        pass
    cores = set()
    for c in range(os.cpu_count() or 0):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                cores.add(f.read().strip())
        except OSError:
            break
    if cores:
        info["physical_cores"] = len(cores)
        if info.get("sockets"):
            info["cores_per_socket"] = len(cores) // info["sockets"]
    nodes = {}
    base = "/sys/devices/system/node"
    if os.path.isdir(base):
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(base, d, "cpulist")) as f:
                    nodes[int(d[4:])] = f.read().strip()
    info["numa_nodes"] = nodes
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    info["affinity_cpus"] = len(os.sched_getaffinity(0))
    return info


def cpu_mhz(cpus: list[int] | None = None) -> dict:
    """Current (mean over `cpus`, else all) and maximum core clock in MHz, from cpufreq or
    /proc/cpuinfo: the CPU baseline varies from box to box, and the clock it ran at is
    part of reading it."""
    out: dict = {"cur_mhz": None, "max_mhz": None}
    cur = []
    for c in (cpus or range(os.cpu_count() or 0)):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cpufreq/scaling_cur_freq") as f:
                cur.append(int(f.read()) / 1000.0)
        except (OSError, ValueError):
            break
    if not cur:
        try:
            with open("/proc/cpuinfo") as f:
                mhz = [float(ln.split(":", 1)[1]) for ln in f if ln.startswith("cpu MHz")]
            sel = [mhz[c] for c in cpus if c < len(mhz)] if cpus else mhz
            cur = sel or mhz
        except (OSError, ValueError):
            pass
    if cur:
        out["cur_mhz"] = round(sum(cur) / len(cur), 1)
    try:
        with open("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq") as f:
            out["max_mhz"] = round(int(f.read()) / 1000.0, 1)
    except (OSError, ValueError):
        pass
    return out


def _cpulist(text: str) -> list[int]:
    out = []
    for part in text.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def pinned_physical_cores(k: int) -> list[int]:
    """Up to k physical cores (one hardware thread each) of the first NUMA node this
    process may run on -- numactl --physcpubind=0-15 in the reference's runs.  The
    cores are dealt round-robin over the node's L3 domains: on chiplet CPUs (EPYC:
    8 cores per L3 / CCD) the first 16 core ids sit on two CCDs whose fabric links
    cap the memory bandwidth, while the reference's Xeon node is one die."""
    allowed = os.sched_getaffinity(0)
    base = "/sys/devices/system/node"
    nodes = []
    if os.path.isdir(base):
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(base, d, "cpulist")) as f:
                    nodes.append(_cpulist(f.read().strip()))
    if not nodes:
        nodes = [sorted(allowed)]

    def read(path: str, default: str) -> str:
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return default

    for cpus in nodes:
        domains: dict[str, list[int]] = {}
        for c in cpus:
            if c not in allowed:
                continue
            sib = read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list", str(c))
            if _cpulist(sib)[0] != c:
                continue  # a second hardware thread of a core already listed
            l3 = read(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", "all")
            domains.setdefault(l3, []).append(c)
        picked = []
        lists = list(domains.values())
        while len(picked) < k and any(lists):
            for lst in lists:
                if lst and len(picked) < k:
                    picked.append(lst.pop(0))
        if picked:
            return sorted(picked)
    return sorted(allowed)[:k]


class cpu_affinity:
    """Pins this thread (and the threads it creates) to `cpus` for the duration of a
    with-block; None leaves the affinity alone."""

    def __init__(self, cpus):
        self.cpus = cpus
        self.saved = None

    def __enter__(self):
        if self.cpus:
            self.saved = os.sched_getaffinity(0)
            os.sched_setaffinity(0, self.cpus)
        return self

    def __exit__(self, *exc):
        if self.saved is not None:
            os.sched_setaffinity(0, self.saved)
        return False


# mi355_rho_stats.layout (sgxamd/rho.h)
LAYOUTS = {
    0: "8-byte tuples, pass-1 histogram + cursors",
    1: "8-byte tuples, pooled pass 1 (per-workgroup block chains, no pass-1 histogram)",
    2: "pooled pass 1; a counting join moves 4-byte keys after reading the 8-byte input tuples "
       "(the payloads are never read by the count; SGXAMD_KEYS=0 moves whole tuples)",
    3: "pooled pass 1 of 4-byte keys with per-chain pass-2 digit histograms counted in LDS (no digit side "
       "stream; the pass-2 histogram sums whole chains' histograms and counts the cut chains' keys; "
       "SGXAMD_CHAIN_HIST=0 keeps the side stream)",
    4: "pooled pass 1 of a narrow plan writing the keys' 16-bit residuals and their pass-2 digit bytes (a narrow "
       "pool, 11 B per tuple; repeated as 4-byte keys when a residual does not fit); pass 2 places each segment "
       "in LDS (opt-in: SGXAMD_NARROW_POOL=1; measured equal to layout 2, r05j)",
}


def visible_gpus() -> int:
    """GPUs this process could use (torch.cuda.device_count(), which on ROCm goes through
    hipGetDeviceCount and so initialises the HIP runtime in this parent process).  That
    is harmless here: the rank processes are started with Popen (fresh processes, no
    fork of an initialised runtime), and this process never launches GPU work when it
    spawns ranks.  The sysfs KFD topology is not used instead: it lists every GPU of the
    host, including ones this container cannot open."""
    import torch

    return torch.cuda.device_count()


def launch_ranks(cmd: list[str], n: int, grace_s: float = 60.0, env_extra: dict | None = None) -> int:
    """Runs `cmd` as n rank processes with the torch.distributed.run environment (RANK,
    LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT).
    Rank 0's stdout is relayed to this process's stdout, every other rank's to stderr.
    When a rank fails, the others get `grace_s` seconds and are then terminated (a peer
    may wait in a collective the failed rank never reaches).  Returns 0 if every rank
    succeeded, else the worst status (a rank killed by signal k counts as 128 + k)."""
    import signal
    import socket
    import subprocess
    import threading

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0", **(env_extra or {}))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True))
    log(f"bench.py: started {n} rank processes (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")

    def pump(r, p):
        for line in p.stdout:
            if r == 0:
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                log(f"[rank {r} stdout] {line.rstrip()}")

    pumps = [threading.Thread(target=pump, args=(r, p), daemon=True) for r, p in enumerate(procs)]
    for t in pumps:
        t.start()
    failed_at = None
    while any(p.poll() is None for p in procs):
        rcs = [p.poll() for p in procs]
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.monotonic()
            log(f"bench.py: a rank failed (exit statuses {rcs}); the others get {grace_s:.0f} s to finish")
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for sig, wait_s in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 0.0)):
                for p in procs:
                    if p.poll() is None:
                        os.killpg(p.pid, sig)
                t_end = time.monotonic() + wait_s
                while time.monotonic() < t_end and any(p.poll() is None for p in procs):
                    time.sleep(0.1)
            for p in procs:
                p.wait()
            break
        time.sleep(0.1)
    for t in pumps:
        t.join(timeout=10)
    status = [p.returncode if p.returncode >= 0 else 128 - p.returncode for p in procs]
    if any(status):
        log(f"bench.py: rank exit statuses {status}")
    return max(status, default=0)


def spawn_ranks(args, argv: list[str]) -> int:
    """`--gpus N` without a launcher (no WORLD_SIZE in the environment): N fresh rank
    processes of this script, one per GPU, started before this process touches a GPU --
    the way the reference's join_init_run spawns its NTHREADS workers itself
    (radix_join.cpp:1531-1540, driven by paper-4-scaling.py:190-199 -> native -n T).
    With the RCCL backend every rank needs a GPU of its own: fewer visible GPUs is an
    error (exit 2), never a line for fewer GPUs.  The gloo backend is the one-GPU
    rehearsal of the multi-rank path (the ranks share the visible GPUs)."""
    n = args.gpus
    have = visible_gpus()
    if args.dist_backend == "nccl" and have < n:
        log(f"bench.py: --gpus {n} needs {n} visible GPUs (one RCCL rank per GPU), but {have} "
            f"{'is' if have == 1 else 'are'} visible; not running (--dist-backend gloo rehearses the "
            f"multi-rank path on fewer GPUs)")
        return 2
    return launch_ranks([sys.executable, os.path.abspath(__file__), *argv], n)


def algorithmic_bytes(kernel: str, nR: int, nS: int, passes: int = 2, pass2_bits: int = 8, elem: int = 8,
                      layout: int = 2, narrow: int = 0) -> int:
    """Bytes a kernel must move per launch (DESIGN.md 'Kernels and their rooflines').

    Two-pass plans: the pass-1 scatter also writes one pass-2 digit byte per tuple (the
    digit side stream) and the pass-2 histogram reads those bytes, not the tuples; with
    chain histograms (layout 3, the default for 7 + 6/7-bit key plans) pass 1 writes a
    histogram per chain instead and the pass-2 histogram reads those.
    elem: bytes per partitioned element after the input read — 8 (row_t tuples) or 4
    (counting joins move keys only: the pass-1 scatter reads 8-byte tuples and
    writes 4-byte keys, pass 2 and the build/probe read and write keys).
    narrow (mi355_rho_stats.narrow, bit 0 R / bit 1 S): that relation's final partitions
    hold 2-byte key residuals — its pass 2 writes 2 bytes per key, the build/probe reads 2.
    layout 4 (the narrow pool): pass 1 of a narrow relation writes the 2-byte residuals and
    the digit byte (11 B per tuple) and pass 2 reads both (5 B per key with its 2-byte
    output); a relation that is not narrow pays that pass 1 and its repeat as keys
    (`pass1_wide`, 13 B)."""
    n = nR if kernel.startswith("R_") else nS
    nar = bool(narrow & (1 if kernel.startswith("R_") else 2))
    # uses_digit_side(); layout 3 (chain histograms) writes and reads no side stream
    side = (passes == 2 and pass2_bits <= 8 and os.environ.get("SGXAMD_DIGIT_SIDE", "1") != "0" and layout != 3)
    if kernel.endswith("pass2_hist") and side:
        return n              # one digit byte per tuple
    if layout == 3 and (kernel.endswith("pass2_hist") or kernel.endswith("pass1_scatter")):
        # chain histograms: u32 [2^7 pass-1 digits][pass-1 segments][2^pass2_bits], written by
        # pass 1 and read by the pass-2 histogram (the cut chains' keys it also reads are
        # not counted: the side stream's plan has no such reads)
        segs = int(os.environ.get("SGXAMD_POOL_SEGS", "512"))
        seg = max(-(-(-(-n // segs)) // 4096) * 4096, 4096)
        chist = 4 * 128 * (-(-n // seg)) * (1 << pass2_bits)
        return chist if kernel.endswith("pass2_hist") else (8 + elem) * n + chist
    if kernel.endswith("_hist"):
        return 8 * n          # read every tuple once (key only used, AoS line read)
    if kernel.endswith("pass1_scatter"):
        if layout == 4:
            return 11 * n  # read the tuple, write its residual and digit byte
        return (8 + elem + (1 if side else 0)) * n  # read the tuple, write the element (+ its digit byte)
    if kernel.endswith("pass1_wide"):
        return 0 if (layout != 4 or nar) else (8 + elem + 1) * n  # the 4-byte pool's repeat
    if kernel.endswith("_scatter"):
        if layout == 4 and nar:
            return 5 * n  # read residual + digit byte, write the residual
        return (elem + (2 if nar else elem)) * n  # read + write every element
    if kernel.endswith("_wire_merge"):  # multi-GPU u16 wire: the senders' pieces gathered (read + write 2 B)
        return 4 * n
    if kernel == "join_build_probe":  # every partitioned element read once
        return (2 if narrow & 1 else elem) * nR + (2 if narrow & 2 else elem) * nS
    return 0


def plan_of(ls: dict) -> tuple:
    """algorithmic_bytes' plan arguments from a join's statistics."""
    return (ls.get("passes") or 2, ls.get("pass2_bits") or 0, ls.get("elem_bytes") or 8, ls.get("layout") or 0,
            ls.get("narrow") or 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2n", type=int, default=28, help="c2: per-GPU |R| = |S| = 2^log2n")
    ap.add_argument("--workload", choices=["c2", "c4", "c5"], default="c2",
                    help="BASELINE config: c2 = pk/fk 2^28 per GPU (weak), c4 = |R| 2^27 x |S| 2^30 "
                         "global (strong), c5 = Zipf 0.75 |R| = |S| = 2^28 global (strong)")
    ap.add_argument("--algorithm", choices=["RHO", "RHT"], default="RHO",
                    help="build/probe: RHO bucket chaining (headline) or RHT histogram join")
    ap.add_argument("--partition-overlap", type=int, choices=[0, 1], default=0,
                    help="1: R/S partition chains on two streams (timed region); 0: one stream")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = single-GPU rehearsal of the "
                         "multi-rank path (ranks share the visible GPUs, tuples staged through host memory)")
    ap.add_argument("--no-scan", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE config 4 / 5 sections")
    ap.add_argument("--zipf-source", choices=["host", "device"], default="host",
                    help="config 5's Zipf stream: host mt19937_64 seed 22222 staged to HBM (BASELINE.md row 5) "
                         "or the device generator")
    ap.add_argument("--no-tpch", action="store_true")
    ap.add_argument("--no-tuple-layout", action="store_true",
                    help="skip the whole-tuple comparison join (profiling passes: per-kernel PMC averages stay one layout)")
    ap.add_argument("--no-paper", action="store_true",
                    help="skip the runs at the shapes of the reference's own published numbers")
    ap.add_argument("--tpch-scale-milli", type=int, default=10000, help="TPC-H scale factor x 1000 (10000 = SF10)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="time budget per CPU baseline leg")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        rc = spawn_ranks(args, sys.argv[1:])
        sys.exit(rc if 0 <= rc < 256 else 1)

    import numpy as np
    import torch
    import torch.distributed as dist

    import sgxamd
    from sgxamd.dist import sharded_rho_join

    ROW_DT = np.dtype([("key", "<u4"), ("payload", "<u4")])  # row_t (data-types.h:44-47)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # never print a line whose n_gpus differs from the --gpus asked for
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure")
        sys.exit(2)
    if args.dist_backend == "gloo":  # rehearsal: ranks may share a device
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            from sgxamd.dist import stdout_to_stderr

            with stdout_to_stderr():
                dist.init_process_group("gloo")
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # bench-side collectives

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    stream = torch.cuda.current_stream().cuda_stream
    sgxamd.set_stream(stream)
    sgxamd.timing_enable(True)  # per-kernel HIP events on `stream` (roofline "achieved")

    # ---------------- RHO workloads: this rank's slice of the global relations
    def make_relations(workload: str):
        """Device-resident slices of BASELINE config 2, 4 or 5 (generation is untimed)."""
        if workload == "c2":  # weak: pk(N n) and fk(N n, maxid N n), n per GPU
            n = 1 << args.log2n
            gR = gS = n * world
            desc = f"RHO join |R|=|S|=2^{args.log2n} uniform per GPU (BASELINE config 2)"
        elif workload == "c4":  # strong: pk(2^27) and fk(2^30, maxid 2^27) = 8 shuffled copies
            gR, gS = 1 << 27, 1 << 30
            desc = "RHO join |R|=2^27 |S|=2^30 uniform, global (BASELINE config 4)"
        else:  # strong: pk(2^28) and Zipf(0.75) over 1..2^28
            gR = gS = 1 << 28
            desc = "RHO join |R|=|S|=2^28, S Zipf theta=0.75, global (BASELINE config 5)"
        if gR % world or gS % world:
            raise SystemExit("relation sizes must divide by the number of GPUs")
        nR_loc, nS_loc = gR // world, gS // world
        R = torch.empty(nR_loc, dtype=torch.int64, device=dev)
        S = torch.empty(nS_loc, dtype=torch.int64, device=dev)
        sgxamd.gen_pk_dev(R, nR_loc, rank * nR_loc, gR, 11111, stream)
        gen = "device pk/fk (keyed-bijection shuffles)"
        if workload == "c5" and args.zipf_source == "host":
            # one mt19937_64 (seed 22222) Zipf stream for alphabet and
            # draws (genzipf.cpp:87-144), generated once on the host, staged to HBM and
            # shared: rank 0 generates, the other ranks receive it by broadcast
            t_gen = time.perf_counter()
            full = torch.empty(gS, dtype=torch.int64, device=dev)
            if rank == 0:
                host = np.empty(gS, dtype=np.int64)
                sgxamd.gen_zipf(host, gS, gR, 0.75, 22222, args.cpu_threads)
                full.copy_(torch.from_numpy(host))
                del host
            if world > 1:
                if args.dist_backend == "nccl":
                    dist.broadcast(full, 0)
                else:
                    cpu_full = full.cpu()
                    dist.broadcast(cpu_full, 0)
                    full.copy_(cpu_full)
            S.copy_(full[rank * nS_loc:(rank + 1) * nS_loc])
            del full
            gen = (f"host Zipf(0.75) over 1..|R|, mt19937_64 seed 22222 (generator.cpp restating "
                   f"genzipf.cpp), staged to HBM in {time.perf_counter() - t_gen:.1f} s; R device pk")
        elif workload == "c5":
            sgxamd.gen_zipf_dev(S, nS_loc, rank * nS_loc, gR, 0.75, 22222, stream)
            gen = "device Zipf(0.75) over 1..|R| (counter-based draws, keyed-bijection alphabet)"
        else:
            sgxamd.gen_fk_dev(S, nS_loc, rank * nS_loc, gR, 22222, stream)
        torch.cuda.synchronize()
        return R, S, gR, gS, desc, gen

    def measure_rho(workload: str, R, S, gR: int, gS: int):
        """W untimed + K timed steps of the (sharded) join; max over ranks."""
        N_glob = gS  # every S tuple matches exactly one R tuple in all three configs

        def step():
            return sharded_rho_join(R, S, algorithm=args.algorithm)

        for _ in range(args.warmup):
            res = step()
            assert res.matches == N_glob, (workload, res.matches, N_glob)
        # the timed steps carry events only around R's pass-1 scatter and the build/probe
        # (sparse timing: each event between two kernels costs ~4.6 us of GPU time); the
        # other kernels' table comes from a full-timing pass after the timed region
        sgxamd.timing_enable("sparse")
        barrier()
        live: dict[str, list[float]] = {}
        results = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = step()
            results.append(res)
            for name, ms in sgxamd.timings():
                live.setdefault(name, []).append(ms)
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        sgxamd.timing_enable(True)
        ok = all(r.matches == N_glob for r in results)
        if not ok:
            raise SystemExit(f"{workload}: wrong match count {[r.matches for r in results]} != {N_glob}")
        per_kernel: dict[str, list[float]] = {}
        for _ in range(TABLE_STEPS):
            r_t = step()
            if r_t.matches != N_glob:
                raise SystemExit(f"{workload}: wrong match count {r_t.matches} != {N_glob}")
            for name, ms in sgxamd.timings():
                per_kernel.setdefault(name, []).append(ms)
        for name, v in live.items():  # the timed region's own spans replace the table's
            if name != "other":
                per_kernel[name] = v
        return results, per_kernel, elapsed

    def gather_multi(res) -> dict | None:
        """N > 1: every rank's exchange record (mi355_multi_stats of the C++ RCCL path, or
        the torch.distributed path's equivalent) gathered to every rank (collective)."""
        if world == 1:
            return None
        mine = dict(res.multi)
        mine.update(rank=rank, recv_r=res.recv_r, recv_s=res.recv_s, local_matches=res.local_matches)
        allm = [None] * world
        dist.all_gather_object(allm, mine)
        phases = ("ms_exchange_post", "ms_local", "ms_allreduce", "ms_tail")
        m0 = allm[0]
        return {"world": m0.get("world"), "transport": m0.get("transport"), "pieces": m0.get("pieces"),
                "elem_bytes": m0.get("elem_bytes"), "sent_bytes_total": sum(int(m.get("sent_bytes", 0)) for m in allm),
                **{k + "_max": round(max(float(m.get(k, 0.0)) for m in allm), 4) for k in phases},
                "per_rank": [{"rank": m["rank"], "recv_r": m["recv_r"], "recv_s": m["recv_s"],
                              "sent_bytes": int(m.get("sent_bytes", 0)), "local_matches": m["local_matches"],
                              **{k: round(float(m.get(k, 0.0)), 4) for k in phases}} for m in allm],
                "mi355_multi_stats_rank0": {k: v for k, v in m0.items() if k not in ("per_rank",)}}

    def load_report(res, nS: int) -> dict:
        """Per-GPU received S tuples and per-partition S sizes (SURVEY.md 8(e) skew report)."""
        ls = res.local_stats
        recv = [float(nS)]
        if world > 1:
            rs = torch.tensor([float(nS)], dtype=torch.float64, device=coll_dev)
            allr = [torch.zeros_like(rs) for _ in range(world)]
            dist.all_gather(allr, rs)
            recv = [float(x.item()) for x in allr]
        P = ls.get("num_partitions") or 1
        return {"recv_S_per_gpu": recv, "recv_S_per_gpu_max_over_mean": round(max(recv) / (sum(recv) / len(recv)), 4),
                "S_partition_max": ls.get("max_part_s"), "S_partition_mean": round(nS / P, 1),
                "S_partition_max_over_mean": round((ls.get("max_part_s") or 0) / max(nS / P, 1e-9), 2),
                "R_partition_max": ls.get("max_part_r"), "partitions": P, "build_probe_tasks": ls.get("num_tasks"),
                "radix_bits": ls.get("radix_bits"), "passes": ls.get("passes")}

    sgxamd.set_partition_overlap(bool(args.partition_overlap))
    R, S, gR, gS, workload, gen_desc = make_relations(args.workload)
    N_glob = gS
    results, per_kernel, elapsed = measure_rho(args.workload, R, S, gR, gS)
    ok = True
    value = N_glob * args.steps / elapsed / 1e6  # M probed tuples/s, all ranks
    ms_per_step = elapsed / args.steps * 1e3
    kernel_times = (f"R_pass1_scatter and join_build_probe: HIP events inside the timed region (sparse timing, "
                    f"4 events per step); the other kernels: a full-timing pass of {TABLE_STEPS} steps after it")
    if args.partition_overlap:
        # With two streams a kernel's event span includes the concurrent chain's
        # kernels; per-kernel durations for the roofline come from an untimed
        # pass with the chains serialised (same kernels, same inputs).
        iso_steps = max(3, min(args.steps, 5))
        sgxamd.set_partition_overlap(False)
        sharded_rho_join(R, S, algorithm=args.algorithm)
        per_kernel = {}
        for _ in range(iso_steps):
            r_iso = sharded_rho_join(R, S, algorithm=args.algorithm)
            ok = ok and r_iso.matches == N_glob
            for name, ms in sgxamd.timings():
                per_kernel.setdefault(name, []).append(ms)
        sgxamd.set_partition_overlap(True)
        kernel_times = f"isolation pass after the timed region: {iso_steps} steps, partition chains on one stream"

    # roofline of the dominant kernel (this rank's event times; rank 0 reports)
    nR = results[-1].recv_r
    nS = results[-1].recv_s
    avg = {k: statistics.mean(v) for k, v in per_kernel.items()}
    plan = plan_of(results[-1].local_stats)
    byte_kernels = {k: v for k, v in avg.items() if algorithmic_bytes(k, nR, nS, *plan) > 0}
    dom = max(byte_kernels, key=byte_kernels.get)
    achieved = algorithmic_bytes(dom, nR, nS, *plan) / (avg[dom] * 1e-3) / 1e9
    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        try:
            tf = json.load(open(TRAFFIC_FILE))
            if (args.workload == "c2" and tf.get("log2n") == args.log2n
                    and dom in tf.get("bytes_per_launch", {})):
                traffic = tf["bytes_per_launch"][dom]
        except (OSError, ValueError):
            traffic = None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "avg_ms": round(avg[dom], 4), "algorithmic_bytes": algorithmic_bytes(dom, nR, nS, *plan)}
    probe_gbs = algorithmic_bytes("join_build_probe", nR, nS, *plan) / (avg["join_build_probe"] * 1e-3) / 1e9
    phase = {k: round(v, 4) for k, v in sorted(avg.items())}
    ls = results[-1].local_stats
    # the north-star probe phase and the whole step as scalars of `roofline` (the block
    # the driver's record keeps): the build/probe launch priced at the bytes it reads,
    # and every kernel of one join at its algorithmic bytes over the measured step time
    step_bytes = sum(algorithmic_bytes(k, nR, nS, *plan) for k in avg)
    roofline.update({
        "probe_kernel": ("k_join_n" if (ls.get("narrow") or 0) and os.environ.get("SGXAMD_JOIN_N", "1") != "0"
                         else "k_join_x" if args.algorithm == "RHO" else "k_join_hist_big"),
        "probe_bytes": algorithmic_bytes("join_build_probe", nR, nS, *plan),
        "probe_avg_ms": round(avg["join_build_probe"], 4),
        "probe_frac": round(probe_gbs / HBM_PEAK_GBS, 4),
        "probe_frac_tuple_layout": None,
        "step_algorithmic_bytes": step_bytes,
        "step_frac": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    })
    rho_info = {
        "matches_ok": ok, "matches": results[-1].matches, "generator": gen_desc,
        "M_rec_per_s_reference_formula": round((gR + gS) * args.steps / elapsed / 1e6, 1),
        "probe_phase_M_probed_tuples_per_s": round(nS / (avg["join_build_probe"] * 1e-3) / 1e6, 1),
        "probe_roofline": {"achieved": round(probe_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(probe_gbs / HBM_PEAK_GBS, 4),
                           "bytes": algorithmic_bytes("join_build_probe", nR, nS, *plan),
                           "bytes_are": ("the bytes the build/probe reads: 2 per key of a narrow relation (16-bit "
                                         "residuals), 4 per key otherwise; BASELINE.md's probe-phase definition "
                                         "(8 B per tuple of R and S) is priced on the whole-tuple leg, "
                                         "rho.tuple_layout.probe_roofline")},
        "kernel_ms_avg": phase, "kernel_times_from": kernel_times,
        "partition_overlap": bool(args.partition_overlap),
        "radix_bits": ls.get("radix_bits"), "passes": ls.get("passes"),
        "partition_layout": LAYOUTS.get(ls.get("layout"), "unknown"),
        "narrow_partitions": {"R": bool((ls.get("narrow") or 0) & 1), "S": bool((ls.get("narrow") or 0) & 2),
                              "what": "final partitions hold 2-byte key residuals (key >> radix bits): every "
                                      "key's residual fits 16 bits (pass 1's largest key)"},
        "step_ms_breakdown": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in results[-1].ms.items()},
    }
    if args.workload == "c5":
        rho_info["load_report"] = load_report(results[-1], nS)
    multi_info = gather_multi(results[-1])

    # the same join moving whole 8-byte tuples (the reference's data movement), measured
    # beside the headline: the probe phase's HBM fraction on the tuple layout
    if (world == 1 and args.workload == "c2" and args.algorithm == "RHO" and ls.get("elem_bytes") == 4
            and not args.no_tuple_layout):
        sgxamd.set_key_layout(False)
        try:
            res_t, pk_t, el_t = measure_rho("c2", R, S, gR, gS)
        finally:
            sgxamd.set_key_layout(True)
        avg_t = {k: statistics.mean(v) for k, v in pk_t.items()}
        ls_t = res_t[-1].local_stats
        plan_t = plan_of(ls_t)
        pb_t = algorithmic_bytes("join_build_probe", nR, nS, *plan_t) / (avg_t["join_build_probe"] * 1e-3) / 1e9
        roofline["probe_frac_tuple_layout"] = round(pb_t / HBM_PEAK_GBS, 4)
        rho_info["tuple_layout"] = {
            "partition_layout": LAYOUTS.get(ls_t.get("layout"), "unknown"), "timed": "untimed for value; own K steps",
            "ms_per_step": round(el_t / args.steps * 1e3, 4),
            "M_probed_tuples_per_s": round(N_glob * args.steps / el_t / 1e6, 1),
            "probe_roofline": {"achieved": round(pb_t, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(pb_t / HBM_PEAK_GBS, 4)},
            "kernel_ms_avg": {k: round(v, 4) for k, v in sorted(avg_t.items())},
        }

    # the CPU baseline joins the relations the GPU joined (BASELINE config 2 at N = 1):
    # one device-to-host copy, outside every timed region
    cpu_rel = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "c2":
        cpu_rel = (R.cpu().numpy().view(ROW_DT), S.cpu().numpy().view(ROW_DT))
    del R, S
    torch.cuda.empty_cache()

    # BASELINE configs 4 and 5 in the same run (strong totals over the N GPUs), each
    # with its load report; the headline value stays config 2
    configs_info = {}
    cpu_cfg_rel = {}  # host copies of the c4 / c5 relations for their CPU legs (rank 0, N = 1)
    if args.workload == "c2" and not args.no_configs and args.dist_backend == "gloo" and world > 1:
        configs_info["skipped"] = ("configs 4 / 5 are not run in the gloo rehearsal (tuples staged through host "
                                   "memory; not a scaling number)")
    elif args.workload == "c2" and not args.no_configs:
        for wl in ("c4", "c5"):
            Rw, Sw, gRw, gSw, desc_w, gen_w = make_relations(wl)
            res_w, pk_w, el_w = measure_rho(wl, Rw, Sw, gRw, gSw)
            avg_w = {k: statistics.mean(v) for k, v in pk_w.items()}
            nRw, nSw = res_w[-1].recv_r, res_w[-1].recv_s
            ls_w = res_w[-1].local_stats
            plan_w = plan_of(ls_w)
            pb = algorithmic_bytes("join_build_probe", nRw, nSw, *plan_w) / (avg_w["join_build_probe"] * 1e-3) / 1e9
            configs_info[wl] = {
                "workload": desc_w, "generator": gen_w, "scaling": "strong", "global_R": gRw, "global_S": gSw,
                "matches": res_w[-1].matches, "matches_ok": True,
                "ms_per_step": round(el_w / args.steps * 1e3, 4),
                "M_probed_tuples_per_s": round(gSw * args.steps / el_w / 1e6, 1),
                "M_rec_per_s_reference_formula": round((gRw + gSw) * args.steps / el_w / 1e6, 1),
                "probe_roofline": {"achieved": round(pb, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(pb / HBM_PEAK_GBS, 4)},
                "kernel_ms_avg": {k: round(v, 4) for k, v in sorted(avg_w.items())},
                "step_ms_breakdown": {k: (round(v, 3) if isinstance(v, float) else v)
                                      for k, v in res_w[-1].ms.items()},
                "load_report": load_report(res_w[-1], nSw),
            }
            if world > 1:
                configs_info[wl]["multi"] = gather_multi(res_w[-1])
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                # the CPU baseline joins these same relations later (one device-to-host copy,
                # outside every timed region)
                cpu_cfg_rel[wl] = (Rw.cpu().numpy().view(ROW_DT), Sw.cpu().numpy().view(ROW_DT))
            del Rw, Sw
            torch.cuda.empty_cache()
        # config 2 on the reference's own relations (native.cpp:62-101: glibc rand() Knuth
        # shuffles, seeds 11111 / 22222, generated on the host by the restated generator
        # and staged to HBM), beside the device-generated headline: untimed for value
        if world == 1:
            n2 = 1 << args.log2n
            t_gen = time.perf_counter()
            Rh, Sh = sgxamd.reference_relations(n2, n2)
            gen_s = time.perf_counter() - t_gen
            Rr = torch.from_numpy(Rh.view(np.int64)).to(dev)
            Sr = torch.from_numpy(Sh.view(np.int64)).to(dev)
            del Rh, Sh
            res_r, pk_r, el_r = measure_rho("c2", Rr, Sr, n2, n2)
            avg_r = {k: statistics.mean(v) for k, v in pk_r.items()}
            ls_r = res_r[-1].local_stats
            configs_info["c2_reference_relations"] = {
                "workload": f"RHO join |R|=|S|=2^{args.log2n}, the reference's generators (BASELINE config 2)",
                "generator": f"host glibc-rand Knuth shuffles restated (generator.cpp:100-153), seeds 11111 / "
                             f"22222, {gen_s:.1f} s, staged to HBM",
                "timed": "untimed for value; own K steps", "matches": res_r[-1].matches, "matches_ok": True,
                "ms_per_step": round(el_r / args.steps * 1e3, 4),
                "M_probed_tuples_per_s": round(n2 * args.steps / el_r / 1e6, 1),
                "radix_bits": ls_r.get("radix_bits"), "passes": ls_r.get("passes"),
                "partition_layout": LAYOUTS.get(ls_r.get("layout"), "unknown"),
                "kernel_ms_avg": {k: round(v, 4) for k, v in sorted(avg_r.items())},
            }
            del Rr, Sr
            torch.cuda.empty_cache()
    # BASELINE config 1's shape (|R| = |S| = 2^20, reference generators) on one GPU: the
    # small-join latency next to the CPU number of the same config (cpu_baseline.rho.config1)
    c1_gpu = None
    if world == 1 and args.workload == "c2":
        c1 = 1 << 20
        R1h, S1h = sgxamd.reference_relations(c1, c1)
        R1 = torch.from_numpy(R1h.view(np.int64)).to(dev)
        S1 = torch.from_numpy(S1h.view(np.int64)).to(dev)
        # per-kernel events off: at this size each event record is a visible share of
        # the join; the call's device time (first to last kernel) is still recorded
        sgxamd.timing_enable(False)
        for _ in range(max(3, args.warmup)):
            assert sgxamd.rho_join(R1, c1, S1, c1, stream=stream).matches == c1
        barrier()
        reps1 = max(20, args.steps)
        dev_ms = []
        t1 = time.perf_counter()
        for _ in range(reps1):
            r1 = sgxamd.rho_join(R1, c1, S1, c1, stream=stream)
            dev_ms.append(r1.stat("ms_total"))  # one field: no stats dict in the timed loop
        barrier()
        el1 = (time.perf_counter() - t1) / reps1
        sgxamd.timing_enable(True)
        c1_gpu = {"ms_per_join_wall": round(el1 * 1e3, 4), "M_probed_tuples_per_s": round(c1 / el1 / 1e6, 1),
                  "device_ms_median": round(statistics.median(dev_ms), 4),
                  "M_probed_tuples_per_s_device": round(c1 / (statistics.median(dev_ms) * 1e-3) / 1e6, 1),
                  "radix_bits": r1.stats.get("radix_bits"), "passes": r1.stats.get("passes"),
                  "path": "three-launch small-join path (one-pass plan)"}
        del R1, S1, R1h, S1h

    # measured stream ceilings of this GPU, from the library's own probe
    # kernels (mi355_stream_probe: grid-stride 16-byte accesses over 2 GiB buffers) timed
    # with HIP events on the stream they run on, best of 5 per shape; the copy ceiling is
    # the best copy shape (read + write bytes), each big kernel is priced against it too
    nb = 1 << 31
    src = torch.empty(nb // 8, dtype=torch.int64, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1)
    cur = torch.cuda.Stream()  # a stream of its own (not the null stream: the library maps that to its own)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur.wait_stream(torch.cuda.current_stream())

    def probe_best(kind, **kw):
        sgxamd.stream_probe(kind, src, dst, nb, stream=cur.cuda_stream, **kw)
        best = float("inf")
        for _ in range(5):
            ev0.record(cur)
            sgxamd.stream_probe(kind, src, dst, nb, stream=cur.cuda_stream, **kw)
            ev1.record(cur)
            ev1.synchronize()
            best = min(best, ev0.elapsed_time(ev1))
        return (2 if kind == "copy" else 1) * nb / (best * 1e-3) / 1e9

    shapes = {}
    for ntl, nts in ((True, True), (True, False), (False, False)):
        for u in (4, 8):
            for grid in (2048, 8192, 32768):
                name = f"copy U{u} grid{grid}{' ntl' if ntl else ''}{' nts' if nts else ''}"
                shapes[name] = probe_best("copy", nt_load=ntl, nt_store=nts, loads_in_flight=u, grid=grid)
    read_ceiling = max(probe_best("read", nt_load=True, loads_in_flight=u, grid=g) for u in (4, 8) for g in (2048, 8192))
    write_ceiling = max(probe_best("write", nt_store=nts, loads_in_flight=4, grid=g) for nts in (True, False)
                        for g in (2048, 8192))
    best_shape = max(shapes, key=shapes.get)
    copy_ceiling = shapes[best_shape]
    # scalars: the driver's parser keeps the roofline's scalar fields only
    roofline["measured_copy_ceiling_GB_per_s"] = round(copy_ceiling, 1)
    roofline["measured_copy_ceiling_how"] = (
        f"in-tree streaming copy kernel (mi355_stream_probe, {best_shape}: 16-byte loads / stores, 2 GiB, read + "
        f"write bytes, HIP events on its stream, best of 5; best of {len(shapes)} shapes)")
    roofline["measured_read_ceiling_GB_per_s"] = round(read_ceiling, 1)
    roofline["measured_write_ceiling_GB_per_s"] = round(write_ceiling, 1)
    roofline["frac_of_copy_ceiling"] = round(roofline["achieved"] / copy_ceiling, 4)
    roofline["probe_frac_of_copy_ceiling"] = round(probe_gbs / copy_ceiling, 4)
    roofline["step_frac_of_copy_ceiling"] = round(step_bytes / (ms_per_step * 1e-3) / 1e9 / copy_ceiling, 4)
    rho_info["ceilings"] = {"copy_shapes_GB_per_s": {k: round(v, 1) for k, v in shapes.items()},
                            "read_GB_per_s": round(read_ceiling, 1), "write_GB_per_s": round(write_ceiling, 1)}
    # every big kernel of the step at its algorithmic bytes: GB/s, fraction of 8 TB/s and
    # of the measured copy ceiling
    rho_info["kernel_rooflines"] = {
        k: {"ms": round(v, 4), "GB_per_s": round(algorithmic_bytes(k, nR, nS, *plan) / (v * 1e-3) / 1e9, 1),
            "frac_of_peak": round(algorithmic_bytes(k, nR, nS, *plan) / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_of_copy_ceiling": round(algorithmic_bytes(k, nR, nS, *plan) / (v * 1e-3) / 1e9 / copy_ceiling, 4)}
        for k, v in sorted(avg.items()) if algorithmic_bytes(k, nR, nS, *plan) > 0 and v > 0.02}
    del src, dst
    torch.cuda.empty_cache()

    # ---------------- scan (BASELINE config 3): 2^30 int32, [0, 26] = 10 % (types.hpp:134)
    scan_info = None
    scan_col_host = None
    if not args.no_scan and args.workload == "c2":
        ns = 1 << 30
        col = torch.empty(ns, dtype=torch.int32, device=dev)
        sgxamd.gen_scan_dev(col, ns, 0, 0, "i32", stream)
        exp = ns // 256 * 27
        bv = torch.empty(ns // 64, dtype=torch.int64, device=dev)
        idx = torch.empty(exp, dtype=torch.int64, device=dev)
        scan_info = {"rows": ns, "dtype": "i32", "predicate": [0, 26], "matches": exp}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            scan_col_host = col.cpu().numpy()  # the CPU scan leg scans the column the GPU scanned
        for kind in ("count", "bitvector", "index"):
            def run():
                if kind == "count":
                    assert sgxamd.scan_count(0, 26, col, ns) == exp
                elif kind == "bitvector":
                    sgxamd.scan_bitvector(0, 26, col, ns, bv)
                else:
                    assert sgxamd.scan_index(0, 26, col, ns, idx, exp) == exp
            for _ in range(max(1, args.warmup)):
                run()
            barrier()
            kt = {}
            t1 = time.perf_counter()
            for _ in range(args.steps):
                run()
                for name, ms in sgxamd.timings():
                    kt.setdefault(name, []).append(ms)
            barrier()
            el = max_over_ranks(time.perf_counter() - t1)
            out_bytes = {"count": 0, "bitvector": ns // 8, "index": 8 * exp}[kind]
            scan_info[kind] = {
                "input_GB_per_s": round(world * 4 * ns * args.steps / el / 1e9, 1),
                "total_GB_per_s": round(world * (4 * ns + out_bytes) * args.steps / el / 1e9, 1),
                "ms_per_call": round(el / args.steps * 1e3, 4),
                "kernel_ms_avg": {k: round(statistics.mean(v), 4) for k, v in kt.items()},
            }
        pk = "scan_bitvector"
        k_ms = scan_info["bitvector"]["kernel_ms_avg"].get(pk)
        if k_ms:
            gbs = (4 * ns + ns // 8) / (k_ms * 1e-3) / 1e9
            scan_info["bitvector_kernel_roofline"] = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                                      "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
        # the seeded-uniform int32 variant of config 3: uniform random
        # values, the predicate [INT32_MIN, INT32_MIN + 27/256 * 2^32) — the same 10.55 %
        # selectivity without the periodic match pattern; exact counts from the GPU count
        # scan, checked against the index scan's
        sgxamd.gen_scan_dev(col, ns, 1, 42, "i32", stream)
        lo_u, hi_u = -(2**31), -(2**31) + (27 << 24) - 1
        exp_u = sgxamd.scan_count(lo_u, hi_u, col, ns)
        idx_u = torch.empty(max(exp_u, 1), dtype=torch.int64, device=dev)
        for _ in range(max(1, args.warmup)):
            assert sgxamd.scan_index(lo_u, hi_u, col, ns, idx_u, exp_u) == exp_u
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            assert sgxamd.scan_index(lo_u, hi_u, col, ns, idx_u, exp_u) == exp_u
        barrier()
        el = max_over_ranks(time.perf_counter() - t1) / args.steps
        scan_info["index_uniform_random"] = {
            "predicate": [lo_u, hi_u], "matches": exp_u, "ms_per_call": round(el * 1e3, 4),
            "input_GB_per_s": round(world * 4 * ns / el / 1e9, 1),
            "total_GB_per_s": round(world * (4 * ns + 8 * exp_u) / el / 1e9, 1)}
        del col, bv, idx, idx_u
        torch.cuda.empty_cache()

    # ---------------- the shapes of the reference's own published numbers (BASELINE.md §1,
    # Xeon Gold 6326, 16 threads, native): RHO at |R| = 13,107,200, |S| = 52,428,800
    # (scaling-perf.csv, 1493.97 M rec/s) and the uint8 scans of SimdScanMulti
    # (bitvector at 1 % selectivity 107.79 GiB/s, scale-up.csv; index list at 10 %
    # 48.37 GiB/s, write-rate.csv).  Context lines, not the headline metric.
    paper_info = None
    if not args.no_paper and world == 1 and args.workload == "c2":
        nRp, nSp = 13_107_200, 52_428_800
        Rp = torch.empty(nRp, dtype=torch.int64, device=dev)
        Sp = torch.empty(nSp, dtype=torch.int64, device=dev)
        sgxamd.gen_pk_dev(Rp, nRp, 0, nRp, 11111, stream)
        sgxamd.gen_fk_dev(Sp, nSp, 0, nRp, 22222, stream)  # 4 shuffled copies of 1..|R|
        torch.cuda.synchronize()
        for _ in range(max(1, args.warmup)):
            assert sgxamd.rho_join(Rp, nRp, Sp, nSp, stream=stream).matches == nSp
        barrier()
        # every call is synchronous (it returns the count): per-call wall times, their
        # median (the reference reports the median of its runs) beside the mean, and
        # the per-kernel event times and plan of the same calls
        call_ms, kt_p = [], {}
        t1 = time.perf_counter()
        for _ in range(args.steps):
            tc = time.perf_counter()
            rp = sgxamd.rho_join(Rp, nRp, Sp, nSp, stream=stream)
            call_ms.append((time.perf_counter() - tc) * 1e3)
            assert rp.matches == nSp
            for name, ms in sgxamd.timings():
                kt_p.setdefault(name, []).append(ms)
        barrier()
        med = statistics.median(call_ms) * 1e-3
        rho_p = round((nRp + nSp) / med / 1e6, 1)
        stp = rp.stats
        paper_info = {"rho": {"shape": "|R|=13,107,200 |S|=52,428,800 (100/400 MiB), pk/fk, count only",
                              "M_rec_per_s": rho_p, "ms": round(med * 1e3, 4), "ms_median": round(med * 1e3, 4),
                              "ms_mean": round(statistics.mean(call_ms), 4), "ms_min": round(min(call_ms), 4),
                              "ms_max": round(max(call_ms), 4), "calls": len(call_ms),
                              "device_ms_total_median": round(statistics.median(
                                  sum(v[i] for v in kt_p.values()) for i in range(len(call_ms))), 4)
                              if kt_p and all(len(v) == len(call_ms) for v in kt_p.values()) else None,
                              "plan": {k: stp.get(k) for k in ("radix_bits", "passes", "pass1_bits", "pass2_bits",
                                                               "num_partitions", "num_tasks", "max_part_r",
                                                               "max_part_s", "layout", "elem_bytes")},
                              "kernel_ms_avg": {k: round(statistics.mean(v), 4) for k, v in sorted(kt_p.items())},
                              "kernel_ms_max": {k: round(max(v), 4) for k, v in sorted(kt_p.items())},
                              "reference_M_rec_per_s": 1493.97,
                              "reference": "Xeon Gold 6326, 16 threads, native, UNROLL+FORCE_2_PHASES "
                                           "(scaling-perf.csv median)",
                              "ratio": round(rho_p / 1493.97, 1)}}
        del Rp, Sp
        torch.cuda.empty_cache()
        nu = 1 << 32  # uint8 entries (the reference's index-list runs use 2^32)
        col = torch.empty(nu, dtype=torch.uint8, device=dev)
        sgxamd.gen_scan_dev(col, nu, 0, 0, "u8", stream)  # i % 256 (Allocator.hpp)
        bvu = torch.empty(nu // 64, dtype=torch.int64, device=dev)
        # selectivity -> [0, round(sel / 100 * 255)] (types.hpp:134): 1 % -> [0, 3], 10 % -> [0, 26]
        k10 = nu // 256 * 27
        idxu = torch.empty(k10, dtype=torch.int64, device=dev)
        for kind, hi, ref, src in (("bitvector_1pct", 3, 107.79, "scale-up.csv, 2^34 entries"),
                                   ("index_10pct", 26, 48.37, "write-rate.csv, 2^32 entries")):
            def run():
                if kind.startswith("bitvector"):
                    sgxamd.scan_bitvector(0, hi, col, nu, bvu, "u8")
                else:
                    assert sgxamd.scan_index(0, hi, col, nu, idxu, k10, "u8") == k10
            for _ in range(max(1, args.warmup)):
                run()
            barrier()
            kt = {}
            t1 = time.perf_counter()
            for _ in range(args.steps):
                run()
                for name, ms in sgxamd.timings():
                    kt.setdefault(name, []).append(ms)
            barrier()
            el = (time.perf_counter() - t1) / args.steps
            gib = nu / el / 2**30
            k_avg = {k: round(statistics.mean(v), 4) for k, v in kt.items()}
            # the dominant kernel's roofline: column bytes + its output (bitvector n/8 B,
            # index list 8 B per match), over its HIP-event time
            main = "scan_bitvector" if kind.startswith("bitvector") else max(k_avg, key=k_avg.get, default=None)
            out_b = nu // 8 if kind.startswith("bitvector") else 8 * k10
            kroof = None
            if main and k_avg.get(main):
                gbs = (nu + out_b) / (k_avg[main] * 1e-3) / 1e9
                kroof = {"kernel": main, "bytes": nu + out_b, "ms": k_avg[main], "achieved": round(gbs, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
            paper_info[f"scan_u8_{kind}"] = {"entries": nu, "predicate": [0, hi], "GiB_per_s": round(gib, 1),
                                             "ms": round(el * 1e3, 4), "reference_GiB_per_s": ref,
                                             "reference": f"Xeon Gold 6326, 16 threads, native ({src})",
                                             "ratio": round(gib / ref, 1), "kernel_ms_avg": k_avg,
                                             "kernel_roofline": kroof}
        del col, bvu, idxu
        torch.cuda.empty_cache()

    # ---------------- TPC-H callers: Q3/Q10/Q12/Q19 on device-resident
    # synthetic tables, one GPU (the pipelines are single-device; skipped for N > 1)
    tpch_info = None
    if not args.no_tpch and world == 1 and args.workload == "c2":
        import sgxamd.tpch as T

        sm = args.tpch_scale_milli
        tb = T.generate_dev(sm, 42, device=dev, stream=stream)
        torch.cuda.synchronize()
        tpch_info = {"scale_factor": sm / 1000, "rows": dict(tb.sizes), "algorithm": args.algorithm,
                     "data": "synthetic TPC-H-shaped tables (tpch_gen.hpp, spec distributions), device-generated"}
        for q in (3, 10, 12, 19):
            fn = T.QUERIES[q]
            for _ in range(max(1, args.warmup)):
                fn(tb, args.algorithm)
            runs = []
            t1 = time.perf_counter()
            for _ in range(args.steps):
                runs.append(fn(tb, args.algorithm))
            el = (time.perf_counter() - t1) / args.steps
            ms = statistics.median(r["ms_total"] for r in runs)
            r = runs[-1]
            tpch_info[f"Q{q}"] = {
                "result": r["result"], "join_matches": r["join_matches"], "filtered": r["filtered"],
                "ms_total_device": round(ms, 4), "ms_wall_per_query": round(el * 1e3, 4),
                "ms_selection": [round(x, 4) for x in r["ms_selection"]],
                "ms_join": [round(x, 4) for x in r["ms_join"]], "ms_copy": round(r["ms_copy"], 4),
                "M_rec_per_s": round(r["input_tuples"] / (ms * 1e3), 1),
                "column_GB_per_s": round(r["column_bytes"] / (ms * 1e-3) / 1e9, 1),
            }
        if rank == 0 and not args.no_cpu_baseline:  # the oracle's tpch.cpp restatement, SF 1 host copy
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle

            host = T.to_numpy(T.generate_dev(1000, 42, device=dev, stream=stream))
            cpu_t = {}
            for q in (3, 10, 12, 19):
                t1 = time.perf_counter()
                oracle.tpch_query(q, host, nthreads=args.cpu_threads)
                el = time.perf_counter() - t1
                n_in = sum(host.n(t) for t in T.QUERY_TABLES[q])
                cpu_t[f"Q{q}"] = {"ms": round(el * 1e3, 2), "M_rec_per_s": round(n_in / el / 1e6, 1)}
            tpch_info["cpu_baseline"] = {"kind": "port", "cores": args.cpu_threads, "scale_factor": 1.0,
                                         "sample": "oracle tpch.cpp restatement (scalar filter_table, pthreads "
                                                   "RHO joins), one run per query", **cpu_t}
            del host
        del tb
        torch.cuda.empty_cache()

    # ---------------- CPU baselines on this host, rank 0 at N = 1: the
    # oracle's restated reference RHO on the relations the GPU joined, pinned to the
    # physical cores of one NUMA node (the reference's methodology, J/README.md:67-70),
    # plus an unpinned run over all CPUs the process may use; BASELINE config 1 (2^20,
    # reference generators); the scan leg on the config-3 column the GPU scanned
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        topo = host_topology()
        pinned = pinned_physical_cores(args.cpu_threads)
        n_all = min(len(os.sched_getaffinity(0)), int(topo.get("cgroup_cpu_quota") or 1 << 30))
        threads = len(pinned) or args.cpu_threads
        topo["pinned_node"] = next((nd for nd, lst in topo.get("numa_nodes", {}).items()
                                    if pinned and pinned[0] in _cpulist(lst)), None)
        cpu_info = {"host": topo, "pinned_cpus": pinned}

        def timed_rho(Rh, Sh, nthr, cpus, budget):
            exp_m = len(Sh)
            tp = []
            with cpu_affinity(cpus):
                t_start = time.perf_counter()
                while time.perf_counter() - t_start < budget and len(tp) < 30:
                    m, t = oracle.rho_join(Rh, Sh, nthr)
                    assert m == exp_m, (m, exp_m)
                    tp.append(t["s_total"])
            return statistics.median(tp), len(tp), t

        rho_cpu = {}
        if cpu_rel is not None:
            Rh, Sh = cpu_rel
            med, reps, t = timed_rho(Rh, Sh, threads, pinned, args.cpu_seconds)
            rho_cpu["pinned"] = {"threads": threads, "cpus": "physical cores of one NUMA node, one thread per core, "
                                                              "spread over the node's L3 domains",
                                 "M_probed_tuples_per_s": round(len(Sh) / med / 1e6, 1), "ms": round(med * 1e3, 2),
                                 "joins": reps, "radix_bits": t["radix_bits"], "passes": t["passes"]}
            med_a, reps_a, _ = timed_rho(Rh, Sh, n_all, None, args.cpu_seconds / 2)
            rho_cpu["all_cpus"] = {"threads": n_all, "cpus": f"unpinned over the {len(os.sched_getaffinity(0))} "
                                                              f"CPUs of this process (cgroup quota "
                                                              f"{topo.get('cgroup_cpu_quota')} CPUs)",
                                   "M_probed_tuples_per_s": round(len(Sh) / med_a / 1e6, 1),
                                   "ms": round(med_a * 1e3, 2), "joins": reps_a}
            del Rh, Sh, cpu_rel
        # BASELINE config 1: the reference App driver's CPU RHO, |R| = |S| = 2^20, generated by
        # the restated reference generators (native.cpp:62-101 seeds)
        c1 = 1 << 20
        R1, S1 = sgxamd.reference_relations(c1, c1)
        med1, reps1, t1 = timed_rho(R1, S1, threads, pinned, 2.0)
        rho_cpu["config1"] = {"R": c1, "S": c1, "threads": threads, "M_probed_tuples_per_s": round(c1 / med1 / 1e6, 1),
                              "M_rec_per_s_reference_formula": round(2 * c1 / med1 / 1e6, 1),
                              "ms": round(med1 * 1e3, 3), "joins": reps1, "radix_bits": t1["radix_bits"],
                              "passes": t1["passes"]}
        if configs_info is not None:
            configs_info["c1"] = {"workload": "RHO join |R|=|S|=2^20, reference generators (BASELINE config 1)",
                                  "cpu": rho_cpu["config1"], "gpu": c1_gpu}
        # BASELINE configs 4 and 5 on the host: the oracle RHO on the relations the GPU joined
        # (c4 pk 2^27 x fk 2^30, c5 pk 2^28 x the Zipf stream), the same pinned cores
        for wl, (Rh, Sh) in list(cpu_cfg_rel.items()):
            medw, repsw, tw = timed_rho(Rh, Sh, threads, pinned, args.cpu_seconds)
            cw = {"R": len(Rh), "S": len(Sh), "threads": threads, "kind": "port",
                  "M_probed_tuples_per_s": round(len(Sh) / medw / 1e6, 1),
                  "M_rec_per_s_reference_formula": round((len(Rh) + len(Sh)) / medw / 1e6, 1),
                  "ms": round(medw * 1e3, 2), "joins": repsw, "radix_bits": tw["radix_bits"], "passes": tw["passes"],
                  "sample": f"oracle RHO on the {wl} relations the GPU joined, {threads} threads pinned, median of "
                            f"{repsw} joins"}
            rho_cpu[wl] = cw
            if wl in configs_info:
                configs_info[wl]["cpu"] = cw
                gpu_v = configs_info[wl].get("M_probed_tuples_per_s")
                if gpu_v:
                    configs_info[wl]["gpu_over_cpu"] = round(gpu_v / cw["M_probed_tuples_per_s"], 1)
            del Rh, Sh
            cpu_cfg_rel.pop(wl)
        lead = rho_cpu.get("pinned") or rho_cpu["config1"]
        cpu = {"value": lead["M_probed_tuples_per_s"], "unit": "M probed tuples/s", "cores": threads, "kind": "port",
               "sample": (f"oracle RHO (radix_join.cpp restated, pthreads) on the 2^28 x 2^28 config-2 relations "
                          f"the GPU joined, {threads} threads pinned to NUMA node {topo.get('pinned_node')}'s "
                          f"physical cores, median of {lead['joins']} joins")
               if "pinned" in rho_cpu else "config 1 only (no config-2 copy)",
               "rho": rho_cpu, **cpu_info}
        # the host record as scalars beside the value (the driver's record keeps scalars)
        clk = cpu_mhz(cpu_info.get("pinned_cpus"))
        cpu.update({"host_model": topo.get("model"), "host_cur_mhz": clk["cur_mhz"], "host_max_mhz": clk["max_mhz"],
                    "host_cgroup_cpu_quota": topo.get("cgroup_cpu_quota"),
                    "host_numa_nodes": len(topo.get("numa_nodes") or {})})
        if scan_col_host is not None:  # config 3 on the host: count / bitvector / index, SIMD512 restated
            scan_cpu = {"rows": len(scan_col_host), "dtype": "i32", "predicate": [0, 26], "threads": threads,
                        "how": "oracle/cpu_baseline.c (SIMD512.cpp AVX-512 formulation, multithreadedscan.cpp "
                               "slicing, pinned one thread per core), per-call time averaged over threads"}
            for kind in ("count", "bitvector", "index"):
                secs, m = oracle.cpu_scan_bench(kind, scan_col_host, 0, 26, threads, pinned, reps=3)
                assert m == len(scan_col_host) // 256 * 27, (kind, m)
                out_b = {"count": 0, "bitvector": len(scan_col_host) // 8, "index": 8 * m}[kind]
                scan_cpu[kind] = {"ms_per_call": round(secs * 1e3, 3),
                                  "input_GB_per_s": round(4 * len(scan_col_host) / secs / 1e9, 2),
                                  "total_GB_per_s": round((4 * len(scan_col_host) + out_b) / secs / 1e9, 2)}
            if scan_info is not None:
                scan_info["cpu_baseline"] = scan_cpu
            del scan_col_host

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "M probed tuples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak" if args.workload == "c2" else "strong",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: device-generated pk (shuffled 1..|R|) and "
                    + ("Zipf(0.75) over 1..|R|" if args.workload == "c5" else "fk (shuffled copies of 1..|R|)")
                    + " relations, 8-byte {key, payload} tuples",
            "config": {"workload": workload, "algorithm": args.algorithm, "global_R": gR, "global_S": gS,
                       "parallelism": f"radix-shard{world}",
                       "partition_layout": rho_info["partition_layout"],
                       **({"exchange": results[-1].ms.get("impl", "torch.distributed all_to_all_single (sgxamd.dist)")}
                          if world > 1 else {}),
                       **({"dist_backend": "gloo (single-GPU rehearsal, not a scaling number)"}
                          if world > 1 and args.dist_backend == "gloo" else {})},
            "roofline": roofline, "cpu_baseline": cpu, "rho": rho_info, "scan": scan_info, "tpch": tpch_info,
            "reference_shapes": paper_info, "configs": configs_info,
        }
        if multi_info is not None:
            line["multi"] = multi_info
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
