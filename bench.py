#!/usr/bin/env python3
"""Benchmark: two-round SP5 x SP27 demultiplexing throughput on MI355X (BASELINE.json metric).

One "step" = the complete two-round demux (round 1: 5' SP5 adapters with --rc; round 2: 3'
SP27rc adapters with --rc on every round-1-matched read; bins, trim coordinates, per-bin counts)
of one resident batch of synthetic reads — the work of scripts/02_cutadapt_loop.sh:64-103.
Workload (default, BASELINE.json configs[1]): 10M synthetic ONT reads per GPU, lognormal
length mean 1.2 kb, synthetic 24 x 24 M13 panel, -e 0.1, --rc.

Multi-GPU: one process per GPU, started by torchrun (the driver) or, for `--gpus N` without
WORLD_SIZE, by this script itself (N child processes spawned before anything touches the GPU;
never an exec).  `--gpus` must equal WORLD_SIZE when both are given.  Reads are sharded by
contiguous range: by default every rank processes `--reads` reads (rank r takes reads
[r*N, (r+1)*N) of one seeded generation: weak scaling); with `--reads-total T` the T reads of
one generation are split over the ranks balanced on the sum of read lengths (BASELINE
configs[2], "10M reads sharded across 8 GPUs": strong scaling).  One RCCL all-reduce of the
per-bin counts per step inside libdmx (dmx_allreduce_counts on the library's stream; the only
exchange the path has).  torch.distributed (gloo) is the control plane only: it hands rank 0's
RCCL id to the other ranks, and carries the barrier and the max-over-ranks time.  At N=1 the
step runs the same all-reduce on a single-rank communicator.

Prints ONE JSON line on rank 0 (see README "Benchmark contract").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nanopore-barcoding-orc_amd"))


def host_cores() -> tuple[int, str]:
    """Physical host cores this process may use: min(physical cores of the CPUs in its affinity
    set, the affinity set, the cgroup CPU quota); with how each was found."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = list(range(os.cpu_count() or 1))
    phys = set()
    try:   # (package, core) of every allowed logical CPU
        for cpu in aff:
            base = f"/sys/devices/system/cpu/cpu{cpu}/topology/"
            with open(base + "physical_package_id") as a, open(base + "core_id") as b:
                phys.add((a.read().strip(), b.read().strip()))
    except OSError:
        phys = set()
    quota = None
    try:   # cgroup v2 cpu.max: "<quota> <period>" or "max <period>"
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    cands = [len(aff)] + ([len(phys)] if phys else []) + ([quota] if quota else [])
    n = max(1, min(cands))
    how = (f"{len(aff)} logical CPUs in the affinity set, "
           f"{len(phys) if phys else 'unknown'} physical cores among them, "
           f"cgroup quota {quota if quota else 'none'}")
    return n, how


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torchrun sets them) before this process touches the GPU, wait for
    them, and return the worst exit status.  Rank 0 prints the JSON line."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
                if codes[i] not in (None, 0):   # one rank failed: the others would hang
                    for q in procs:
                        if q.poll() is None:
                            q.send_signal(signal.SIGTERM)
        time.sleep(0.1)
    return max((abs(c) for c in codes), default=0)

METRIC = "Mreads/s two-round SP5×SP27 demux; % HBM roofline; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_LANES = 256 * 128                      # lane-ops per shader cycle: 256 CUs x 4 SIMD32
VALU_PEAK_TOPS = VALU_LANES * 2.4e9 / 1e12  # at the nominal 2.4 GHz, 32-bit lane-ops
VALU_CEILING_FILE = os.path.join(ROOT, "profiles", "r3_valu_ceiling.json")
if not os.path.exists(VALU_CEILING_FILE):
    VALU_CEILING_FILE = os.path.join(ROOT, "profiles", "r2_valu_ceiling.json")


def _valu_ceiling() -> float:
    """Measured VALU issue ceiling (tools/microbench/run_ceiling.sh -> profiles/)."""
    try:
        with open(VALU_CEILING_FILE) as fh:
            return float(json.load(fh)["bitop3_t_lane_ops_per_s"]) * 1e12
    except (OSError, ValueError, KeyError):
        return 50.5e12


VALU_CEILING = _valu_ceiling()   # dependent v_bitop3 chain x4 per lane at full occupancy
VALU_CEILING_WHAT = ("v_bitop3 dependency chains (each instruction uses the one before), four "
                     "per lane, at full occupancy (" + os.path.relpath(VALU_CEILING_FILE, ROOT) +
                     " 'bitop3_dependent_chain_t_lane_ops_per_s'); eight independent chains per "
                     "lane reach less, 'bitop3_independent_t_lane_ops_per_s'")


def survey_bytes_per_read(lengths: np.ndarray) -> np.ndarray:
    """SURVEY.md §8(d) algorithmic HBM bytes per read: B(read) = ceil(L/4) (2-bit packed read)
    + 8 (offset + length) + ceil(L/64) (N mask) + 24 (result record)."""
    L = lengths.astype(np.float64)
    return np.ceil(L / 4) + 8.0 + np.ceil(L / 64) + 24.0


def survey_bytes(lengths: np.ndarray) -> float:
    """Σ B(read) over the reads (views) one launch processes."""
    return float(np.sum(survey_bytes_per_read(lengths)))


def pmc_table(workload: str, reads: int):
    """The committed rocprofv3 PMC table of this exact workload (profiles/kernel_pmc.json,
    tools/kernel_table_from_pmc.py over tools/pmc_passes.sh), or None."""
    try:
        with open(os.environ.get("DMX_KERNEL_PMC") or
                  os.path.join(ROOT, "profiles", "kernel_pmc.json")) as fh:
            return json.load(fh).get(f"{workload}:{reads}")
    except (OSError, ValueError):
        return None


def pmc_valu_insts(workload: str, reads: int, kernel: str, last_only: bool = False,
                   first_only: bool = False):
    """SQ_INSTS_VALU of the kernel's launches in one PMC'd step (all launches, the last or the
    first)."""
    pmc = pmc_table(workload, reads)
    launches = (pmc or {}).get("kernels", {}).get(kernel, [])
    if not launches:
        return None
    if last_only:
        return launches[-1]["valu_insts"]
    if first_only:
        return launches[0]["valu_insts"]
    return sum(e["valu_insts"] for e in launches)


def pmc_clock(workload: str, reads: int, kernel: str, launch=None):
    """Effective shader clock (GHz) of the kernel's PMC'd launches: GRBM_GUI_ACTIVE / 8 XCDs /
    duration (MI355X_MICROARCH.md 'DVFS give-back'), time-weighted; None without the counter."""
    pmc = pmc_table(workload, reads)
    launches = (pmc or {}).get("kernels", {}).get(kernel, [])
    if launch is not None:
        launches = launches[launch:launch + 1]
    pts = [(e["clock_ghz"], e["ms"]) for e in launches if e.get("clock_ghz")]
    if not pts:
        return None
    return sum(c * m for c, m in pts) / sum(m for _, m in pts)


def valu_roof(rate, clk_ghz, what: str):
    """roofline['valu']: the dominant kernel's VALU issue rate against the peak at the clock it
    ran at (and the nominal 2.4 GHz peak)."""
    out = {"unit": "T lane-ops/s", "achieved": round(rate / 1e12, 3) if rate else None,
           "nominal_peak": round(VALU_PEAK_TOPS, 2),
           "measured_ceiling": round(VALU_CEILING / 1e12, 2), "what": what}
    if rate and clk_ghz:
        peak = VALU_LANES * clk_ghz * 1e9
        out.update({"clock_ghz": round(clk_ghz, 3), "peak_at_clock": round(peak / 1e12, 3),
                    "frac": round(rate / peak, 4),
                    "clock_source": "GRBM_GUI_ACTIVE / 8 / launch duration of the PMC'd launches "
                                    "(profiles/kernel_pmc.json); the ceiling's own clock is "
                                    "stamped in-kernel (profiles/r3_valu_ceiling.json)"})
    return out


def filter_layout_bytes(lengths: np.ndarray, n_windows: int) -> float:
    """Bytes of one filter launch in this build's layout: each read's 2-bit
    packed codes once (L/4 B) and its 1-bit no-match mask (L/8 B), its offset + length (12 B),
    plus the 40-B window records the launch writes.  Both orientations of a read are filtered
    from the same bytes.  Reported beside the §8(d) figure, never as roofline.achieved."""
    L = lengths.astype(np.float64)
    return float(np.sum(np.ceil(L / 4) + np.ceil(L / 8) + 12.0) + 40.0 * n_windows)


def pmc_traffic(workload: str, reads: int):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary (FETCH_SIZE and
    WRITE_SIZE passes, corrected per MI355X_MICROARCH.md), if one exists for this workload."""
    path = os.environ.get("DMX_FILTER_TRAFFIC") or os.path.join(ROOT, "profiles",
                                                                "filter_pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    key = f"{workload}:{reads}"
    if key not in d:
        return None, None
    return d[key]["bytes_per_launch"], d[key]["source"]


# the two-round pipeline's kernels and the live stage events that time them (per round).  With
# the piece screen the filter stage is the piece screen ("pieces": pscan +
# pcompact, or the per-part pscreen) followed by the task-driven filter ("ftask"); without it,
# the full-pass filter_kernel.
KERNEL_STAGES_PIECES = (("pscan_kernel+pcompact_kernel", "pieces"), ("dmx::ftask_kernel", "ftask"),
                        ("dmx::verify_kernel", "verify"), ("dmx::iscreen4_kernel", "screen"),
                        ("dmx::wscan_kernel<true>", "wscan"),
                        ("band_cand<0,3>+band_cand<4,5|7>+select_cand", "resolve"))
KERNEL_STAGES_FULL = (("dmx::filter_kernel", "filter"), ("dmx::verify_kernel", "verify"),
                      ("dmx::iscreen4_kernel", "screen"), ("dmx::wscan_kernel<true>", "wscan"),
                      ("band_cand<0,3>+band_cand<4,5|7>+select_cand", "resolve"))
PMC_NAMES = {"filter": ["filter_kernel"], "verify": ["verify_kernel"],
             "pieces": ["pscan_kernel<1>", "pscan_kernel<2>", "pscan_kernel<4>", "pcompact_kernel",
                        "pscreen_kernel<1>", "pscreen_kernel<2>", "pscreen_kernel<4>",
                        "read_view_kernel", "read_item_kernel"],
             "ftask": ["ftask_kernel"],
             "screen": ["iscreen4_kernel", "iscreen_kernel"], "wscan": ["wscan_kernel<true>"],
             "resolve": ["band_cand_kernel<0, 3>", "band_cand_kernel<4, 5>",
                         "band_cand_kernel<4, 7>", "select_cand_kernel"]}
# stages timed by HIP events around exactly one kernel (candidates for the roofline's kernel)
SINGLE_KERNEL = {"filter": "filter_kernel", "ftask": "ftask_kernel", "verify": "verify_kernel",
                 "screen": "iscreen4_kernel", "wscan": "wscan_kernel<true>"}


def stage_split(stage: dict) -> dict:
    """stage totals with the piece screen's share split out: ftaskN = filterN - piecesN."""
    out = dict(stage)
    for r in (0, 1):
        out[f"ftask{r}"] = max(0.0, stage[f"filter{r}"] - stage.get(f"pieces{r}", 0.0))
    return out


def pmc_kernel_bytes(workload: str, reads: int, kernel: str):
    """Mean HBM bytes per launch of `kernel` in the committed PMC table (FETCH_SIZE x 2 +
    WRITE_SIZE, separate passes; profiles/kernel_pmc.json), or None."""
    pmc = pmc_table(workload, reads)
    launches = (pmc or {}).get("kernels", {}).get(kernel, [])
    if not launches:
        return None, None
    return (sum(e["hbm_bytes"] for e in launches) / len(launches),
            f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {kernel}, mean of the "
            f"{len(launches)} launches of one step; FETCH_SIZE x2 (gfx950 wide-read correction); "
            + pmc["source"])


def kernel_table(workload: str, reads: int, stage: dict, K: int, step_ms: float,
                 stages=KERNEL_STAGES_FULL):
    """Per-kernel live time (HIP events around each stage of each round) with, where a committed
    rocprofv3 PMC table exists for this exact workload (profiles/kernel_pmc.json, written by
    tools/kernel_table_from_pmc.py), the VALU issue rate and HBM bytes of the same launches:
    instructions and bytes per launch are properties of the workload, the time is this run's."""
    pmc = pmc_table(workload, reads)
    out = {}
    for name, st in stages:
        ms = [stage[f"{st}{r}"] / K for r in (0, 1)]
        ent = {"ms_per_step": round(sum(ms), 3), "ms_per_round": [round(x, 3) for x in ms],
               "share_of_step": round(sum(ms) / step_ms, 4)}
        if pmc is not None:
            valu = hbm = 0.0
            clk = []
            for kn in PMC_NAMES[st]:
                for launch in pmc["kernels"].get(kn, []):
                    valu += launch["valu_insts"]
                    hbm += launch["hbm_bytes"]
                    if launch.get("clock_ghz"):
                        clk.append((launch["clock_ghz"], launch["ms"]))
            if sum(ms) > 0 and valu > 0:
                rate = valu * 64 / (sum(ms) / 1e3)
                ent["valu_lane_ops_per_s"] = rate
                ent["valu_frac_of_ceiling"] = round(rate / VALU_CEILING, 4)
                ent["hbm_gb_per_s"] = round(hbm / (sum(ms) / 1e3) / 1e9, 1)
                ent["hbm_frac"] = round(hbm / (sum(ms) / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                if clk:   # time-weighted effective clock of the PMC'd launches (GRBM_GUI_ACTIVE)
                    g = sum(c * m for c, m in clk) / sum(m for _, m in clk)
                    ent["clock_ghz"] = round(g, 3)
                    ent["valu_frac_of_peak_at_clock"] = round(rate / (VALU_LANES * g * 1e9), 4)
        out[name] = ent
    if pmc is not None:
        out["_source"] = (pmc["source"] + "; VALU ceiling " + os.path.relpath(VALU_CEILING_FILE,
                                                                               ROOT))
    return out


def cpu_baseline(workload: str, threads: int, cores_how: str, target_s: float = 12.0):
    """Oracle (CPU restatement of cutadapt 4.9, C, pthreads) on a bounded sample of the same
    workload, one thread per physical host core available.  rank 0, N=1 only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed CPU baseline only
    from dmx import synth
    linked = workload == "c5"
    mode, rc = (2, False) if linked else (1, True)
    pilot = synth.generate(workload, n=400 * threads, seed=99)
    p1 = oracle.Panel(pilot["sp5"], oracle.FRONT)
    p2 = oracle.Panel(pilot["sp27"], oracle.BACK)
    t = time.perf_counter()
    oracle.run_batch(p1, p2, pilot["blob"], pilot["offsets"], pilot["lengths"], mode, rc, threads)
    rate = len(pilot["lengths"]) / (time.perf_counter() - t)
    n = int(max(1000, min(2_000_000, rate * target_s)))
    d = synth.generate(workload, n=n, seed=98)
    t = time.perf_counter()
    oracle.run_batch(p1, p2, d["blob"], d["offsets"], d["lengths"], mode, rc, threads)
    dt = time.perf_counter() - t
    what = "linked -g F...R, no --rc" if linked else "two rounds, --rc"
    return {"value": n / dt / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "port",
            "sample": f"{n} reads of workload {workload} (seed 98), {what}, -e 0.1, "
                      f"{dt:.1f} s wall on {threads} host threads, one per physical core "
                      f"available ({cores_how}) (oracle/cutadapt_oracle.c, a C restatement of "
                      "cutadapt 4.9's Ukkonen-banded DP; cutadapt itself is not installed)"}


def chop_cpu_baseline(threads: int, cores_how: str, cutoff: float, target_s: float = 12.0):
    """Oracle primer-hit search (oracle/chop_oracle.c, plain O(mn) DP on pthreads) on a bounded
    sample of the chop workload.  rank 0, N=1 only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import chopper  # test infrastructure: timed CPU baseline only
    from dmx import chop, synth
    primers = chop.load_primers(chop.PRIMERS_FASTA)
    pilot = synth.generate("c2", n=40 * threads, seed=99)
    t = time.perf_counter()
    chopper.batch_hit_counts(primers, cutoff, pilot["blob"], pilot["offsets"], pilot["lengths"],
                             threads)
    rate = len(pilot["lengths"]) / (time.perf_counter() - t)
    n = int(max(500, min(2_000_000, rate * target_s)))
    d = synth.generate("c2", n=n, seed=98)
    t = time.perf_counter()
    chopper.batch_hit_counts(primers, cutoff, d["blob"], d["offsets"], d["lengths"], threads)
    dt = time.perf_counter() - t
    return {"value": n / dt / 1e6, "unit": "Mreads/s", "cores": threads, "kind": "port",
            "sample": f"{n} reads of config 2 (seed 98): hits of SP5, SP27 and their reverse "
                      f"complements at cutoff {cutoff}, {dt:.1f} s wall on {threads} host threads "
                      f"({cores_how}) (oracle/chop_oracle.c, a plain-DP restatement; pychopper / "
                      "edlib are not installed)"}


def reads_desc(args, what: str) -> str:
    if args.scaling == "strong":
        return (f"{args.total_reads} {what} in total, split over {len(args.shards)} GPU(s) by "
                "sum of read lengths")
    return f"{args.shards[0]} {what} per GPU"


def chop_line(args, world, K, value, elapsed, ms, lengths, n_hits, n_segs, cutoff, gen_s,
              label_lens):
    """pychopper-style reorientation (01_pychopper.sh).  Dominant kernel: dmx::chop_kernel."""
    L = lengths.astype(np.float64)
    alg_bytes = (float(np.sum(np.ceil(L / 4) + np.ceil(L / 8) + 12.0)) + 8.0 * len(L)
                 + 16.0 * (n_hits + n_segs))
    kern_ms = ms["chop"] / K
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    # Myers columns: every label over the read, plus m + k warm-up columns per later segment
    extra = np.maximum(np.ceil(L / 512) - 1, 0)
    cols = sum(float(np.sum(L + extra * (m + int(cutoff * m)))) for m in label_lens)
    traffic, traffic_src = pmc_traffic("chop", args.reads)
    vi = pmc_valu_insts("chop", args.reads, "chop_kernel", last_only=True)
    ops_col = vi * 64 / cols if vi else None
    return {
        "metric": "Mreads/s pychopper-style reorientation (01_pychopper.sh: -m edlib -p, "
                  "M13 SP5/SP27 primers)",
        "value": round(value, 4), "unit": "Mreads/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"chop: {reads_desc(args, 'synthetic ONT reads')} (config 2 "
                               "generator, both orientations), primers "
                               "M13_seqs_for_pychopper.fa, layout +:SP5,-SP27|-:SP27,-SP5, "
                               "-p, inputs resident in HBM",
                   "cutoff": cutoff, "reads_per_gpu": args.shards, "reads_total": args.total_reads,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": round(alg_bytes),
                     "kernel": "dmx::chop_kernel", "avg_launch_ms": round(kern_ms, 3),
                     "note": "VALU-bound bit-vector scan (DESIGN.md §8d)"},
        "valu": {"columns_per_s": cols / (kern_ms / 1e3),
                 "lane_ops_per_column": ops_col,
                 "lane_ops_per_s": cols / (kern_ms / 1e3) * ops_col if ops_col else None,
                 "frac_of_measured_ceiling": (cols / (kern_ms / 1e3) * ops_col / VALU_CEILING
                                              if ops_col else None),
                 "measured_ceiling_lane_ops_per_s": VALU_CEILING,
                 "measured_ceiling_what": VALU_CEILING_WHAT,
                 "source": "ops/column = SQ_INSTS_VALU x 64 of the PMC'd timed launch "
                           "(profiles/kernel_pmc.json 'chop:<reads>') / its Myers columns"},
        "stage_ms_per_step": {k: round(v / K, 3) for k, v in ms.items()},
        "hits_per_read": round(n_hits / max(1, len(L)), 4),
        "segments_per_read": round(n_segs / max(1, len(L)), 4),
        "gen_s": round(gen_s, 1),
    }


def two_round_line(args, world, K, value, elapsed, stage, lengths, ctx, counts, gen_s,
                   clusters, windows, windows_raw, resolved, traces, filter_tasks):
    st = stage_split(stage)
    pieces = st.get("pieces0", 0.0) > 0 or st.get("pieces1", 0.0) > 0
    stages = KERNEL_STAGES_PIECES if pieces else KERNEL_STAGES_FULL
    res = ctx.fetch()
    m2 = res["bin1"] >= 0
    n2 = int(m2.sum())
    len2 = (lengths[m2] - res["m1_rstop"][m2]).astype(np.int64)
    # roofline.achieved: SURVEY.md §8(d)'s B(read) over the views each launch of the kernel
    # processes (round 1: every read; round 2: the round-1-trimmed tails), averaged over the
    # round-1 and round-2 launches, / that kernel's live average launch time (HIP events)
    sb0, sb1 = survey_bytes(lengths), survey_bytes(len2)
    alg_bytes = (sb0 + sb1) / 2
    step_ms = elapsed / K * 1e3
    step_bytes = survey_bytes(lengths)   # §8(d): round 2 reuses the resident read
    # the dominant kernel: the single-kernel stage with the largest share of the step
    single = [k for k in SINGLE_KERNEL if f"{k}0" in st and (k != "filter" or not pieces)
              and (k != "ftask" or pieces)]
    dom = max(single, key=lambda k: st[f"{k}0"] + st[f"{k}1"])
    dom_kernel = SINGLE_KERNEL[dom]
    dom_ms = (st[f"{dom}0"] + st[f"{dom}1"]) / (2 * K)
    achieved = alg_bytes / (dom_ms / 1e3) / 1e9
    traffic, traffic_src = pmc_kernel_bytes(args.workload, args.reads, dom_kernel)
    if traffic is None and dom_kernel == "filter_kernel":
        traffic, traffic_src = pmc_traffic(args.workload, args.reads)
    vi = pmc_valu_insts(args.workload, args.reads, dom_kernel)
    dom_rate = vi * 64 / ((st[f"{dom}0"] + st[f"{dom}1"]) / K / 1e3) if vi else None
    A0, A1 = ctx.panel_sizes
    read_stream = None
    if pieces:   # the piece screen reads every base of every view (the old filter's role)
        pm = (st["pieces0"] + st["pieces1"]) / (2 * K)
        ps_traffic = None
        tr = [pmc_kernel_bytes(args.workload, args.reads, k)[0]
              for k in ("pscan_kernel<2>", "pscan_kernel<1>", "pscan_kernel<4>")]
        tr = [t for t in tr if t]
        if tr:
            ps_traffic = tr[0]
        read_stream = {
            "kernel": "dmx::pscan_kernel + dmx::pcompact_kernel (the piece screen: every base "
                      "of every view, DESIGN.md §3.12)",
            "avg_launch_ms": round(pm, 3), "achieved": round(alg_bytes / (pm / 1e3) / 1e9, 3),
            "frac": round(alg_bytes / (pm / 1e3) / 1e9 / HBM_PEAK_GBS, 6),
            "pscan_traffic_bytes_per_launch": ps_traffic,
            "what": "the same §8(d) bytes over the piece screen stage's live time (HIP events "
                    "from the round start to the filter tasks; its memsets included)"}
    return {
        "metric": METRIC, "value": round(value, 4), "unit": "Mreads/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"{args.workload}: {reads_desc(args, 'synthetic ONT reads')} "
                               "(SURVEY.md §8d), two-round SP5 x SP27 demux, -e 0.1 --rc, "
                               "inputs resident in HBM",
                   "panel": f"{A0}x{A1}", "reads_per_gpu": args.shards,
                   "reads_total": args.total_reads,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": round(alg_bytes),
                     "algorithmic_bytes_per_launch_r1_r2": [round(sb0), round(sb1)],
                     "algorithmic_bytes_rule": "SURVEY.md §8(d) B(read) = ceil(L/4) + 8 + "
                                               "ceil(L/64) + 24 over the launch's views, mean "
                                               "of the round-1 and round-2 launches",
                     "traffic_over_algorithmic": (round(traffic / alg_bytes, 3)
                                                  if traffic else None),
                     "per_step": {"bytes": round(step_bytes), "ms": round(step_ms, 3),
                                  "achieved_gbs": round(step_bytes / (step_ms / 1e3) / 1e9, 3),
                                  "frac": round(step_bytes / (step_ms / 1e3) / 1e9
                                                / HBM_PEAK_GBS, 6),
                                  "what": "§8(d) bytes of every read once per step (round 2 "
                                          "reuses the resident read) / ms_per_step"},
                     "kernel": "dmx::" + dom_kernel, "avg_launch_ms": round(dom_ms, 3),
                     "share_of_step": round(2 * dom_ms / step_ms, 4),
                     "note": "the dominant kernel (the single-kernel stage with the largest share "
                             "of the step, see 'kernels'); integer/bit work, VALU- or "
                             "latency-bound by construction (DESIGN.md §5): roofline.valu gives "
                             "its issue rate against the VALU peak at the clock it ran at",
                     "valu": valu_roof(dom_rate,
                                       pmc_clock(args.workload, args.reads, dom_kernel),
                                       f"dmx::{dom_kernel}, both rounds"),
                     "read_stream": read_stream},
        "kernels": kernel_table(args.workload, args.reads, st, K, elapsed / K * 1e3, stages),
        "stage_ms_per_step": {k: round(v / K, 3) for k, v in st.items()},
        "clusters_per_step": (clusters / K).tolist(),
        "filter_tasks_per_step": (filter_tasks / K).tolist(),
        "filter_windows_raw_per_step": (windows_raw / K).tolist(),
        "filter_windows_per_step": (windows / K).tolist(),
        "resolved_clusters_per_step": (resolved / K).tolist(),
        "tracebacks_per_step": (traces / K).tolist(),
        "reads_round2_per_gpu": n2,
        "unknown_round1": int(counts[0]) if counts is not None else None,
        "gen_s": round(gen_s, 1),
    }


def linked_line(args, world, K, value, elapsed, stage, lengths, ctx, counts, gen_s):
    """Config 5: linked primers.  Dominant kernel: round 1's full scan (every front primer over
    every consensus: one lane per (read, pair))."""
    res = ctx.fetch()
    trimmed = int((res["bin1"] >= 0).sum())
    scan_ms = stage["scan0"] / K
    A0, _ = ctx.panel_sizes
    L = lengths.astype(np.float64)
    alg_bytes = survey_bytes(lengths)   # SURVEY.md §8(d) B(read) over the consensuses
    layout_bytes = float(np.sum(np.ceil(L / 4) + np.ceil(L / 8) + 12.0))
    achieved = alg_bytes / (scan_ms / 1e3) / 1e9
    traffic, traffic_src = pmc_traffic("c5", args.reads)
    vi = pmc_valu_insts("c5", args.reads, "scan_kernel<true>", first_only=True)
    rate = vi * 64 / (scan_ms / 1e3) if vi else None
    return {
        "metric": "Mreads/s linked-primer trimming (config 5, cutadapt -g F...R per pair)",
        "value": round(value, 4), "unit": "Mreads/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"c5: {reads_desc(args, 'synthetic COI consensuses')} (SURVEY.md "
                               "§8d config 5), linked COI_primers.fa pairs, -e 0.1, no --rc, "
                               "inputs resident in HBM",
                   "pairs": A0, "reads_per_gpu": args.shards, "reads_total": args.total_reads,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": round(alg_bytes),
                     "algorithmic_bytes_rule": "SURVEY.md §8(d) B(read) = ceil(L/4) + 8 + "
                                               "ceil(L/64) + 24 over the launch's reads",
                     "layout_bytes_per_launch": round(layout_bytes),
                     "traffic_over_algorithmic": (round(traffic / alg_bytes, 3)
                                                  if traffic else None),
                     "kernel": "dmx::scan_kernel<true>", "avg_launch_ms": round(scan_ms, 3),
                     "note": "VALU-bound bit-vector scan (DESIGN.md §5); the round-1 launch "
                             "(every front primer over every consensus)",
                     "valu": valu_roof(rate, pmc_clock("c5", args.reads, "scan_kernel<true>", 0),
                                       "dmx::scan_kernel<true>, round 1 (fronts)")},
        "stage_ms_per_step": {k: round(v / K, 3) for k, v in stage.items()},
        "trimmed_fraction": round(trimmed / max(1, len(lengths)), 4),
        "gen_s": round(gen_s, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="number of ranks (one per GPU); default WORLD_SIZE or 1.  Without a "
                         "launcher, N > 1 starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=10)
    # (after a single warm-up the first timed step still ran ~1 ms slow)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2x24",
                    choices=["c2x24", "c2", "c4", "c1", "c5", "chop"],
                    help="c5 = config 5, linked COI primers (-g F...R) on consensus FASTA; "
                         "chop = pychopper-style reorientation (01_pychopper.sh) of config 2's "
                         "reads")
    ap.add_argument("--reads", type=int, default=10_000_000,
                    help="reads per GPU (weak scaling)")
    ap.add_argument("--reads-total", type=int, default=None,
                    help="strong scaling: this many reads in total, split over the ranks in "
                         "contiguous ranges balanced on the sum of read lengths (BASELINE "
                         "configs[2]: --reads-total 10000000 on 8 GPUs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the CPU baseline; default one per physical host core "
                         "available to this process")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the PCIe-inclusive dmx_run after the timed region")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))   # nothing has touched the GPU in this process
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher must start "
                 "one process per GPU (torchrun --nproc-per-node N), or run without a launcher")
    if args.gpus is not None and args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = local_rank
    # DMX_DIST_BACKEND=gloo: rehearse the N-rank path with several ranks sharing the GPUs of a
    # smaller box (RCCL refuses two ranks on one device: the counts then go over gloo); the
    # default is libdmx's RCCL all-reduce over xGMI.
    backend = os.environ.get("DMX_DIST_BACKEND", "nccl")
    if world > 1:
        import torch
        import torch.distributed as tdist
        dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        tdist.init_process_group("gloo")   # control plane: id hand-off, barrier, max time
        dist = tdist
    on_gpu = backend == "nccl"

    from dmx import lib, synth
    gen_threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    t0 = time.perf_counter()
    chop_mode = args.workload == "chop"
    gen_cfg = "c2" if chop_mode else args.workload
    if args.reads_total is not None:   # strong scaling: one generation split over the ranks
        bounds = synth.shard_bounds(gen_cfg, args.reads_total, world)
        first, n_local = bounds[rank], bounds[rank + 1] - bounds[rank]
        args.shards = [bounds[r + 1] - bounds[r] for r in range(world)]
        args.total_reads = args.reads_total
        args.scaling = "strong"
    else:                              # weak scaling: args.reads per rank
        first, n_local = rank * args.reads, args.reads
        args.shards = [args.reads] * world
        args.total_reads = args.reads * world
        args.scaling = "weak"
    args.reads = n_local               # this rank's reads (PMC tables are keyed by it)
    d = synth.generate(gen_cfg, n=n_local, first=first, threads=gen_threads)
    packed = lib.pack(d["blob"], d["offsets"], d["lengths"])
    tune = None
    if chop_mode:   # the CLI's autotune sample: the first 10000 reads
        nt = min(10000, len(d["lengths"]))
        tune = lib.pack(d["blob"], d["offsets"][:nt], d["lengths"][:nt])
    lengths = d["lengths"].copy()
    del d["blob"]
    gen_s = time.perf_counter() - t0

    linked = args.workload == "c5"
    ctx = lib.Context(dev)
    if on_gpu and not chop_mode:   # the per-bin count exchange: RCCL inside libdmx
        cid = [lib.comm_unique_id() if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(cid, src=0)
        ctx.comm_init_rank(cid[0], world, rank)
    if chop_mode:
        return chop_main(args, ctx, packed, tune, lengths, gen_s, world, rank, dist, on_gpu)
    if linked:   # 04_cleaning_primers.sh:377: -g F...R per pair, no --rc
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK, 0.1)
        ctx.set_mode(lib.MODE_LINKED)
    else:
        ctx.set_panel(0, d["sp5"], lib.DMX_FRONT | lib.DMX_RC, 0.1)
        ctx.set_panel(1, d["sp27"], lib.DMX_BACK | lib.DMX_RC, 0.1)
        ctx.set_mode(lib.MODE_TWO_ROUND)
    ctx.load(packed)
    # kept for the PCIe-inclusive run after the timed region (dmx_run from host memory)
    host_batch = packed if not linked else None
    del packed

    def allreduce_counts():
        if on_gpu:   # ncclAllReduce of the counts in HBM, ordered after the exec on its stream
            return ctx.allreduce_counts()
        from dmx import dist as ddist   # gloo rehearsal (ranks sharing a GPU)
        return ddist.allreduce_counts(ctx.counts())

    def barrier_sync():
        ctx.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):   # the whole step body, read-backs included (their first
        ctx.exec()                  # calls set up host staging: ~9 ms once on c5)
        ctx.sync()
        ctx.stats()
        allreduce_counts()

    stage = {k: 0.0 for k in ("scan0", "resolve0", "finalize0", "scan1", "resolve1",
                              "finalize1", "total", "filter0", "verify0", "filter1", "verify1",
                              "screen0", "wscan0", "screen1", "wscan1", "pieces0",
                              "pieces1")}
    clusters = np.zeros(2)
    windows = np.zeros(2)
    windows_raw = np.zeros(2)
    resolved = np.zeros(2)
    traces = np.zeros(2)
    filter_tasks = np.zeros(2)
    barrier_sync()
    t = time.perf_counter()
    counts = None
    flags = 0
    step_wall = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        ctx.exec()
        ctx.sync()
        st = ctx.stats()
        for k in stage:
            stage[k] += st["ms"][k]
        clusters += np.array(st["clusters"], dtype=np.float64)
        windows += np.array(st["windows"], dtype=np.float64)
        windows_raw += np.array(st["windows_raw"], dtype=np.float64)
        resolved += np.array(st["resolved"], dtype=np.float64)
        traces += np.array(st["traces"], dtype=np.float64)
        filter_tasks += np.array(st["filter_tasks"], dtype=np.float64)
        flags |= st["flags"]
        counts = allreduce_counts()
        step_wall.append((time.perf_counter() - ts) * 1e3)
    barrier_sync()
    elapsed = time.perf_counter() - t
    if flags:
        raise SystemExit(f"pipeline flags {flags}: cluster overflow or window violation")
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    K = args.steps
    value = args.total_reads * K / elapsed / 1e6
    if linked:
        out = linked_line(args, world, K, value, elapsed, stage, lengths, ctx, counts, gen_s)
    else:
        out = two_round_line(args, world, K, value, elapsed, stage, lengths, ctx, counts, gen_s,
                             clusters, windows, windows_raw, resolved, traces, filter_tasks)
    out["step_wall_ms"] = [round(x, 3) for x in step_wall]   # this rank's, for outliers
    pcie = None
    if host_batch is not None and not args.no_pcie:
        # the boundary's host-memory path: upload, both rounds, download of every result, with
        # copies overlapped with kernels (dmx_run's double-buffered chunks); not the headline.
        # Inputs as a resident host pipeline holds them: the no-match mask as its exceptions
        # (dmx_mask_exceptions, part of packing) and the batch buffers page-locked once
        # (dmx_host_register, as reused batch buffers are), both outside the timed region.
        def timed(fn):
            ctx.sync()
            barrier_sync()
            t1 = time.perf_counter()
            fn(host_batch)
            ctx.sync()
            barrier_sync()
            pe = time.perf_counter() - t1
            if dist is not None:
                import torch
                tt = torch.tensor([pe], dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                pe = float(tt.item())
            return pe
        pe_dense = timed(ctx.run)                    # dense mask, pageable memory
        exc_idx, exc_val = host_batch.exceptions()
        pinned = lib.host_register([host_batch.seq2b, host_batch.offsets, host_batch.lengths,
                                    exc_idx, exc_val])
        try:
            pe = timed(ctx.run_sparse)
        finally:
            lib.host_unregister(pinned)
        pcie = {"value": round(args.total_reads / pe / 1e6, 4), "unit": "Mreads/s",
                "ms": round(pe * 1e3, 3),
                "chunk_reads": int(os.environ.get("DMX_RUN_CHUNK", 1 << 21)),
                # 2-bit codes, the mask's nonzero words (index + value), offsets, lengths
                "h2d_bytes_per_gpu": int(host_batch.seq2b.nbytes + exc_idx.nbytes +
                                         exc_val.nbytes + host_batch.offsets.nbytes +
                                         host_batch.lengths.nbytes),
                "h2d_bytes_per_read": round((host_batch.seq2b.nbytes + exc_idx.nbytes +
                                             exc_val.nbytes + host_batch.offsets.nbytes +
                                             host_batch.lengths.nbytes) /
                                            max(1, host_batch.n_reads), 1),
                "d2h_bytes_per_gpu": int(args.reads * 40),   # dmx_result
                "pinned_buffers": len(pinned),
                "pageable_dense": {"value": round(args.total_reads / pe_dense / 1e6, 4),
                                   "ms": round(pe_dense * 1e3, 3),
                                   "h2d_bytes_per_gpu": int(
                                       host_batch.seq2b.nbytes +
                                       min(host_batch.nmask.nbytes,
                                           host_batch.seq2b.nbytes // 2 + 8) +
                                       host_batch.offsets.nbytes + host_batch.lengths.nbytes)},
                "note": "dmx_run_sparse from page-locked host memory (one call, inputs not "
                        "resident): uploads (2-bit codes + the no-match mask's nonzero words), "
                        "both rounds, download of every per-read result; the next chunk's "
                        "upload and the previous chunk's download overlap each chunk's kernels. "
                        "pageable_dense: dmx_run with the dense mask from pageable memory"}
        del host_batch

    if pcie is not None:
        out["pcie_inclusive"] = pcie
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores, how = host_cores()
        if args.cpu_threads:
            cores, how = args.cpu_threads, f"--cpu-threads {args.cpu_threads}; detected: {how}"
        out["cpu_baseline"] = cpu_baseline(args.workload, cores, how)
    if rank == 0:
        out["provenance"] = run_provenance()
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def run_provenance():
    """Which code produced this line (tools/provenance.py: commit of the build, SHA-256 of the
    loaded libraries and of the sources)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from provenance import provenance
    return provenance()


def chop_main(args, ctx, packed, tune, lengths, gen_s, world, rank, dist, on_gpu):
    """--workload chop: one step = dmx_chop_exec (primer hits, segments, read-order compaction)
    over the resident batch; the cutoff is tuned once beforehand the way bin/pychopper does."""
    from dmx import chop
    primers = chop.load_primers(chop.PRIMERS_FASTA)
    with open(chop.CONFIG_FILE) as fh:
        rules = chop.parse_config(fh.read(), [p[0] for p in primers])
    ch = chop.Chopper(ctx, primers, rules, True)
    ctx.load(tune)
    cutoff = ch.autotune(np.arange(tune.n_reads))
    ch.set_cutoff(cutoff)
    ctx.load(packed)
    del packed

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        ctx.chop_exec()
    ms = {"chop": 0.0, "order": 0.0}
    barrier_sync()
    t = time.perf_counter()
    tot = (0, 0)
    for _ in range(args.steps):
        tot = ctx.chop_exec()
        st = ctx.chop_stats()
        ms["chop"] += st["chop"]
        ms["order"] += st["order"]
    barrier_sync()
    elapsed = time.perf_counter() - t
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    K = args.steps
    value = args.total_reads * K / elapsed / 1e6
    out = chop_line(args, world, K, value, elapsed, ms, lengths, tot[0], tot[1], cutoff, gen_s,
                    [len(p[1]) for p in primers for _ in (0, 1)])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores, how = host_cores()
        if args.cpu_threads:
            cores, how = args.cpu_threads, f"--cpu-threads {args.cpu_threads}; detected: {how}"
        out["cpu_baseline"] = chop_cpu_baseline(cores, how, cutoff)
    if rank == 0:
        out["provenance"] = run_provenance()
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
