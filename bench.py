#!/usr/bin/env python3
"""Word-count throughput of the MI355X engine (BASELINE.json metric).

One step = one full pass of the hot path (reference: main.rs:16-22) over the
HBM-resident corpus: dictionary -> map -> shuffle -> reduce -> (word, count)
table in HBM; with N > 1 also the RCCL all-to-all exchange and the final
per-owner reduce.  The corpus is generated on the host (synthetic, seeded) and
copied to HBM before timing.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no torchrun environment, ONE process drives all N GPUs
through an engine group (mox_config.n_gpus, include/mox.h): a step is one
mox_run_shards call (local passes on all GPUs at once, the all-to-all as one
RCCL group over the members' communicators, per-owner reduce and bytewise sort
of every member's byte range on its own GPU, gather in member order).  Under torchrun (RANK / WORLD_SIZE
set) every rank is one process per GPU (mox_comm_init, mox_exchange,
mox_gather); rank 0 prints the line.

Default workload (N = 1): config C2 of BASELINE.json, 1 GiB Zipf(1.1)
English-like corpus.  N > 1: config C3, weak scaling with an 8 GiB byte-range
shard per GPU of the C3 corpus stream (rank r owns bytes [8r GiB, 8(r+1) GiB);
N = 8 is the 64 GiB corpus); a step is the local pass, the RCCL all-to-all
exchange, the final per-owner reduce and the gather of the result at rank 0.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "map-oxidize_amd"))

import numpy as np  # noqa: E402

import mox  # noqa: E402
from mox import corpus  # noqa: E402
from mox import dist as mdist  # noqa: E402

METRIC = "word-count input GB/s end-to-end at 1 and 8 MI355X; % of HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
HALO = 1 << 16

KIND_DESC = {corpus.ZIPF: "Zipf(1.1) English-like text", corpus.HICARD: "random 4-16 byte [a-z0-9] tokens",
             corpus.SKEW: "top-10 words 90% + Zipf(1.1) tail", corpus.UNICODE: "Zipf text with Unicode tokens"}
WORKLOADS = {
    # name: (kind, seed, bytes per rank, description)
    "C2": (corpus.ZIPF, 0x5EED0002, 1 << 30, "C2: 1 GiB Zipf(s=1.1) English-like corpus per GPU (map+sort+reduce)"),
    "C3": (corpus.ZIPF, 0x5EED0003, 8 << 30, "C3: 64 GiB Zipf corpus = 8 GiB shard per GPU at 8 GPUs"),
    "C4": (corpus.HICARD, 0x5EED0004, 16 << 30, "C4: 16 GiB high-cardinality random 4-16 B tokens per GPU"),
    "C5": (corpus.SKEW, 0x5EED0005, 16 << 30, "C5: 16 GiB heavy skew (top-10 words = 90%) per GPU"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # the GPU's first ~15 passes after the corpus upload run slower (a clock /
    # power transient: C2 k_map 750-800 us in passes 3-6, ~690 from pass ~15 on,
    # profiles/r05/bench_warmup_transient.txt); 20 untimed passes measure the
    # steady state (C2: warmup 3 -> 927-931 GB/s, 10 -> 965-969, 20 -> 974-976)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="", choices=[""] + sorted(WORKLOADS),
                    help="default: C2 at N = 1, C3 (8 GiB shard per GPU) at N > 1")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: leave the final tables on their owner ranks")
    ap.add_argument("--cpu-runs", type=int, default=3, help="CPU baseline: median of this many runs")
    ap.add_argument("--bytes-per-gpu", type=int, default=0, help="override the shard size")
    ap.add_argument("--cpu-sample-mib", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dict", action="store_true")
    ap.add_argument("--sample-pieces", type=int, default=0, help="dictionary sample pieces (0 = engine default)")
    ap.add_argument("--sync-passes", action="store_true", help="N = 1: synchronous passes (no async enqueue)")
    ap.add_argument("--xport", default="rccl", choices=["rccl", "host"],
                    help="exchange transport for N > 1 (host: gloo-staged, for ranks sharing one GPU)")
    ap.add_argument("--device", type=int, default=-1, help="override the GPU (default LOCAL_RANK)")
    ap.add_argument("--no-map-events", action="store_true",
                    help="diagnostics: no HIP events around k_map in the timed steps (no roofline.achieved)")
    ap.add_argument("--traffic-json", default=None,  # profiles/pmc_k_map.json (C2) or pmc_k_map_<workload>.json
                    help="PMC summary of the map kernel (tools/pmc_traffic.py) to report as roofline.traffic")
    return ap.parse_args()


def progress(msg):
    """A progress line on stderr (long runs keep writing, so a watchdog sees them alive)."""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, timeout=20).stdout.decode()
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


def cpu_baseline(kind, seed, sample_bytes, runs=3):
    """Faithful C++ restatement of the reference pipeline (oracle/build/meduce_ref),
    timed on a bounded sample of the same corpus: 8 map threads, 4 reduce
    threads (main.rs:12-13); median of ``runs`` runs."""
    exe = os.path.join(ROOT, "oracle", "build", "meduce_ref")
    if not os.path.exists(exe):
        return None
    data = corpus.fill(kind, seed, 0, sample_bytes)
    tmpdir = "/dev/shm" if os.path.isdir("/dev/shm") else None
    times = []
    with tempfile.TemporaryDirectory(dir=tmpdir) as d:
        path = os.path.join(d, "shakes.txt")
        data.tofile(path)
        del data
        for i in range(max(1, runs)):
            progress("cpu baseline run %d of %d (%d MiB)" % (i + 1, max(1, runs), sample_bytes >> 20))
            r = subprocess.run([exe, path, "--workdir", d, "--quiet", "--time"], capture_output=True, timeout=600)
            if r.returncode != 0:
                return None
            times.append(json.loads(r.stderr.decode().strip().splitlines()[-1])["hot_s"])
    hot = statistics.median(times)
    return {
        "value": round(sample_bytes / hot / 1e9, 4),
        "unit": "GB/s",
        "cores": 8,
        "kind": "port",
        "sample": "first %d MiB of the same corpus; oracle/build/meduce_ref (faithful C++ restatement of "
                  "main.rs: line round-robin into 8 chunks, 8 map threads, spill files on tmpfs, 4 reduce "
                  "threads behind one mutex), -O3, split+map+reduce wall time (main.rs:16-22), median of %d runs"
                  % (sample_bytes >> 20, len(times)),
        "hot_s_runs": [round(t, 4) for t in times],
        "threads": {"map": 8, "reduce": 4},
        "host_nproc": os.cpu_count(),
        "cpu_model": cpu_model(),
    }


def local_tokens(eng, d_buf, n, own_b, own_e, at_end):
    """Tokens of this rank's shard: one local pass (untimed, after the timed loop)."""
    eng.run_range(d_buf, n, own_b, own_e, at_end)
    return eng.stats()["tokens"]


def limiter_fields(workload):
    """What binds k_map for this workload, as measured (SQ counters) and recorded
    in profiles/limiter_<workload>.json; omitted when no measurement of this
    workload exists."""
    f = os.path.join(ROOT, "profiles", "limiter_%s.json" % workload)
    try:
        lj = json.load(open(f))
    except Exception:
        return {}
    if lj.get("workload") != workload:
        return {}
    return {"binding_unit": lj.get("binding_unit"), "limiter": lj.get("limiter"),
            "limiter_source": os.path.relpath(f, ROOT)}


def roofline_fields(per_rank, map_avg, workload, traffic_json):
    achieved = per_rank / (map_avg * 1e-3) / 1e9
    traffic = None
    if traffic_json is None:
        traffic_json = os.path.join(ROOT, "profiles", "pmc_k_map%s.json" % ("" if workload == "C2" else "_" + workload))
    if traffic_json and os.path.exists(traffic_json):
        try:
            tj = json.load(open(traffic_json))
            # PMC traffic is per launch of one workload and size: report it only for that one
            if tj.get("workload", "C2") == workload and tj.get("bytes_per_gpu", 1 << 30) == per_rank:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    r = {
        "kernel": "k_map",
        # priced against HBM (no dense contraction: the contract's "hbm" roofline);
        # the unit that actually binds k_map, where measured for this workload,
        # is in binding_unit / limiter (limiter_fields)
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": per_rank,
        "avg_launch_ms": round(map_avg, 4),
    }
    r.update(limiter_fields(workload))
    return r


def same_work_n1(eng, shard, per_rank, steps, warmup, n, value_n):
    """The N = 1 figure of an N > 1 line on the same per-GPU work (weak-scaling
    denominator): ONE GPU alone on the shard of rank / member 0 -- a synchronous
    pass plus the device bytewise sort of its table per step, the N > 1 step's
    local work without the exchange and the gather -- timed after the N > 1
    steps in the same run.  ``eng`` is a single-GPU engine with the sort flag."""
    d, blen, ob, oe, end = shard
    for _ in range(warmup):
        eng.run_range(d, blen, ob, oe, end)
        eng.sort_result()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.run_range(d, blen, ob, oe, end)
        eng.sort_result()
    eng.synchronize()
    el = time.perf_counter() - t0
    v1 = per_rank / (el / steps) / 1e9
    return {"value": round(v1, 3), "unit": "GB/s", "ms_per_step": round(el / steps * 1e3, 4),
            "scaling_efficiency": round(value_n / (n * v1), 4),
            "note": "one GPU alone on shard 0 of this run (%d MiB): synchronous pass + device bytewise sort of its "
                    "table per step (the N > 1 step's per-GPU work without exchange and gather), %d untimed + %d "
                    "timed steps after the N > 1 steps; scaling_efficiency = value / (n_gpus x this)"
                    % (per_rank >> 20, warmup, steps)}


def main_group(a):
    """--gpus N > 1 without torchrun: one process, one engine group over N GPUs.
    A timed step is one mox_run_shards call with MOX_F_SORT_BYTES: local passes,
    the sorted exchange (words owned by byte range), per-owner reduce and
    bytewise sort on every member's GPU, and the gather at GPU 0 in member
    order, which is then the sorted table (north_star: "a gather of the sorted
    result").  The same K steps without the sort (hash-owned exchange, gathered
    table in engine order) are timed before them and reported beside the value."""
    n = a.gpus
    if not a.workload:
        a.workload = "C3"
    kind, seed, per_rank, desc = WORKLOADS[a.workload]
    if a.bytes_per_gpu:
        per_rank = a.bytes_per_gpu
    total = per_rank * n
    devices = [a.device] * n if a.device >= 0 else None
    n_dev = len(set(devices)) if devices else n  # distinct GPUs (members may share one in tests)
    xport = mox.XPORT_COPY if a.xport == "host" else mox.XPORT_RCCL
    base_flags = (mox.MOX_F_NO_DICT if a.no_dict else 0) | mox.MOX_F_TIMING_MAP
    g = mox.Engine(n_gpus=n, transport=xport, devices=devices, flags=base_flags | mox.MOX_F_SORT_BYTES,
                   sample_pieces=a.sample_pieces, reserve_bytes=per_rank)
    shards, bufs = [], []
    for r in range(n):
        lo, hi, ob, oe, end = mdist.shard_range(total, n, r, per_rank=per_rank, halo=HALO)
        progress("%s: generating shard %d of %d (%d MiB)" % (a.workload, r + 1, n, (hi - lo) >> 20))
        host = corpus.fill(kind, seed, lo, hi - lo)
        m = g.member(r)
        d = m.alloc(hi - lo)
        m.h2d(d, host)
        del host
        bufs.append((m, d))
        shards.append((d, hi - lo, ob, oe, end))

    def timed(flags):
        g.set_flags(flags)
        for _ in range(a.warmup):
            g.run_shards(shards)
        g.synchronize()
        rows = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.run_shards(shards)  # synchronous: returns with the gathered table on GPU 0
            rows.append(g.stats())
        g.synchronize()  # member 0's stream drained: the last step's sort / gather tail is inside the clock
        return time.perf_counter() - t0, rows

    progress("shards in HBM; hash-order steps")
    el_hash, rows_hash = timed(base_flags)
    progress("sorted-result steps")
    elapsed, rows = timed(base_flags | mox.MOX_F_SORT_BYTES)  # the value: sorted result inside the step
    last = rows[-1]
    progress("same-work N = 1 steps (member 0's shard alone)")
    e1 = mox.Engine(device=devices[0] if devices else 0, flags=base_flags | mox.MOX_F_TIMING_MAP | mox.MOX_F_SORT_BYTES,
                    sample_pieces=a.sample_pieces, reserve_bytes=per_rank)
    n1 = same_work_n1(e1, shards[0], per_rank, a.steps, a.warmup, n, total / (elapsed / a.steps) / 1e9)
    e1.close()
    t = g.fetch()  # bytewise order (sorted on GPU 0 by the last timed step)
    counts, offs, raw = t.arrays()
    table_n, table_bytes, table_tokens = t.n, int(offs[-1]) if t.n else 0, t.tokens
    ok = int(counts.sum()) == t.tokens == last["tokens"]
    t.close()
    ms_step = elapsed / a.steps * 1e3
    gbs = total / (elapsed / a.steps) / 1e9
    map_avg = statistics.mean(r["ms_map"] for r in rows)
    b_alg = total + table_bytes + 8 * table_n
    mean = lambda rr, k: round(statistics.mean(r[k] for r in rr), 4)  # noqa: E731
    line = {
        "metric": METRIC,
        "value": round(gbs, 3),
        "unit": "GB/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: mox_corpus kind=%d seed=%#x (%s, host-generated, copied to HBM before timing)"
                % (kind, seed, KIND_DESC.get(kind, "?")),
        "config": {"workload": desc, "bytes_per_gpu": per_rank, "total_bytes": total,
                   "parallelism": "dp%d byte-range shards + %s all-to-all (byte-range owners) + bytewise sort per "
                                  "GPU + gather in member order at GPU 0 (one process, engine group%s)" % (
                                      n, "RCCL" if xport == mox.XPORT_RCCL else "device-copy",
                                      "" if n_dev == n else "; %d members on %d GPU(s)" % (n, n_dev))},
        "words_per_s": round(last["tokens"] / (elapsed / a.steps), 1),
        # against the HBM peak of the GPUs actually used (members sharing one GPU share its HBM)
        "pct_hbm_peak": round(100.0 * gbs / (HBM_PEAK_GBS * n_dev), 2),
        "algorithmic_bytes_per_step": b_alg,
        "roofline_end_to_end": {"achieved": round(b_alg / (elapsed / a.steps) / 1e9, 1), "peak": HBM_PEAK_GBS * n_dev,
                                "unit": "GB/s", "frac": round(b_alg / (elapsed / a.steps) / 1e9 / (HBM_PEAK_GBS * n_dev), 4)},
        "roofline": roofline_fields(per_rank, map_avg, a.workload, a.traffic_json),
        "pass_mode": "sync (mox_run_shards per step, MOX_F_SORT_BYTES)",
        "phases_ms": {"local_passes": mean(rows, "ms_local"), "map_mean_over_gpus": mean(rows, "ms_map"),
                      "exchange": mean(rows, "ms_exchange"), "gather": mean(rows, "ms_gather"),
                      "sort_bytes": mean(rows, "ms_sort"), "step_wall": mean(rows, "ms_run")},
        "hash_order": {"value": round(total / (el_hash / a.steps) / 1e9, 3), "ms_per_step": round(el_hash / a.steps * 1e3, 4),
                       "note": "the same steps without the bytewise sort (gathered table in engine order)",
                       "phases_ms": {"local_passes": mean(rows_hash, "ms_local"), "exchange": mean(rows_hash, "ms_exchange"),
                                     "gather": mean(rows_hash, "ms_gather"), "step_wall": mean(rows_hash, "ms_run")}},
        "stats": {k: last[k] for k in ("tokens", "uniques", "cold_records", "weighted_records")},
        "multi_gpu": {
            "mode": "engine group (one process)",
            "transport": "RCCL (ncclCommInitAll, one ncclGroupStart/End per all-to-all)" if xport == mox.XPORT_RCCL
                         else "device-to-device copies (hipMemcpyPeerAsync)",
            "devices": devices if devices else list(range(n)),
            "all_to_all_bytes": int(last["x_bytes_sent"]),
            "all_to_all_bytes_recv": int(last["x_bytes_recv"]),
            "exchange_ms": mean(rows, "ms_exchange"),
            "gather_ms": mean(rows, "ms_gather"),
            "gather_bytes": int(last["gather_bytes"]),
            "gathered_table": {"n": table_n, "bytes": table_bytes, "tokens": table_tokens,
                               "order": "bytewise (sorted exchange: each member sorts its byte range on its GPU "
                                        "inside the timed step; sort_bytes = the slowest member's sort)"},
            "note": "exchange_ms = the slowest member's splitters + counts + pack + payload copies + reduce-only "
                    "pass, without its bytewise sort (phases_ms.sort_bytes); step_wall ≈ local_passes + exchange "
                    "+ sort_bytes + gather",
        },
        "same_work_n1": n1,
        "check_sum_counts_eq_tokens": ok,
        "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)
    for m, d in bufs:
        m.free(d)
    g.close()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return main_group(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        world = a.gpus if world == 1 else world
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only (rendezvous, barrier, max-time)
        dist.init_process_group("gloo")
    if not a.workload:
        a.workload = "C2" if world == 1 else "C3"
    kind, seed, per_rank, desc = WORKLOADS[a.workload]
    if a.bytes_per_gpu:
        per_rank = a.bytes_per_gpu
    total = per_rank * world
    lo, hi, own_b, own_e, at_end = mdist.shard_range(total, world, rank, per_rank=per_rank, halo=HALO)

    base_flags = mox.MOX_F_NO_DICT if a.no_dict else 0
    # timed steps: HIP events around k_map only (each event record idles the
    # stream ~5.6 us); one diagnostic step after the timed region has them all
    map_flag = 0 if a.no_map_events else mox.MOX_F_TIMING_MAP
    eng = mox.Engine(device=local if a.device < 0 else a.device, flags=base_flags | map_flag,
                     sample_pieces=a.sample_pieces, reserve_bytes=per_rank)
    progress("%s: generating %d MiB of corpus" % (a.workload, (hi - lo) >> 20))
    host = corpus.fill(kind, seed, lo, hi - lo)
    d_buf = eng.alloc(hi - lo)
    eng.h2d(d_buf, host)
    del host
    progress("corpus in HBM; %d warmup + %d timed steps" % (a.warmup, a.steps))
    if world > 1 and a.xport == "rccl":
        uid = mox.comm_unique_id() if rank == 0 else b""
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(world, rank, obj[0])
    a2a = mdist.gloo_alltoallv() if world > 1 and a.xport == "host" else None

    # N = 1: passes are enqueued asynchronously (mox_run_range_async): each call
    # enqueues its pass, then completes (checks) the previous one, so the GPU
    # runs the passes back to back with no host round trip between them.
    # N > 1: the exchange needs the local result on the host side, so passes
    # run synchronously.
    use_async = world == 1 and not a.sync_passes

    gather = world > 1 and not a.no_gather
    if gather:
        # the sorted result (north_star: "a gather of the sorted result"): the
        # sorted exchange (MOX_F_SORT_BYTES: words owned by byte range, every
        # rank sorts its own range on its GPU), so the gather at rank 0 is
        # already in bytewise order and sort_result() there finds nothing to do
        eng.set_flags(base_flags | mox.MOX_F_TIMING_MAP | mox.MOX_F_SORT_BYTES)

    def step(sync=False, sort=True):
        if use_async and not sync:
            eng.run_range_async(d_buf, hi - lo, own_b, own_e, at_end)
            return
        eng.run_range(d_buf, hi - lo, own_b, own_e, at_end)
        if world > 1:
            if a2a:
                eng.exchange_host(world, rank, a2a)
            else:
                eng.exchange()
            if gather:  # the whole table at rank 0 (mox_gather: device to device) ...
                if a2a:
                    eng.gather_host(world, rank, a2a, root=0)
                else:
                    eng.gather(0)
                if sort and rank == 0:  # ... sorted bytewise on its GPU (north_star: "a gather of the sorted result")
                    eng.sort_result()

    for _ in range(a.warmup):
        step()
    eng.synchronize()  # completes (and checks) every queued pass
    progress("warmup done")
    if dist:
        dist.barrier()
    map_ms, xms, gms = [], [], []
    t0 = time.perf_counter()
    for i in range(a.steps):
        step()
        if (not use_async or i > 0) and map_flag:  # async: the call completed the previous pass
            map_ms.append(eng.ms_map())
        if world > 1:
            st = eng.stats()
            xms.append(st["ms_exchange"])
            gms.append(st["ms_gather"])
    eng.synchronize()
    if use_async and map_flag:
        map_ms.append(eng.ms_map())  # the last pass, completed by synchronize
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sort_ms = eng.stats()["ms_sort"] if gather else 0.0  # this rank's sort of its byte range (sorted exchange)
    el_hash = None
    if world > 1 and gather:  # the same steps without the sort, reported beside the value
        eng.set_flags(base_flags | mox.MOX_F_TIMING_MAP)  # hash-owned exchange, gathered table in engine order
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(a.steps):
            step(sort=False)
        eng.synchronize()
        if dist:
            dist.barrier()
        el_hash = time.perf_counter() - t1
    n1 = None
    if world > 1 and gather:
        # the same-work N = 1 figure: rank 0 alone on its shard while the others wait
        if dist:
            dist.barrier()
        if rank == 0:
            progress("same-work N = 1 steps (rank 0's shard alone)")
            eng.set_flags(base_flags | mox.MOX_F_TIMING_MAP | mox.MOX_F_SORT_BYTES)
            n1 = (hi - lo, own_b, own_e, at_end)
            n1 = same_work_n1(eng, (d_buf,) + n1, per_rank, a.steps, a.warmup, world, 0.0)
        if dist:
            dist.barrier()
    sorted_result = None
    if world == 1:
        # like-for-like with the N > 1 line (whose step ends in the bytewise
        # sort of the gathered table): the same K steps, each a synchronous pass
        # followed by the device bytewise sort of its table (mox_sort_result)
        eng.synchronize()
        sort_ms = []
        t1 = time.perf_counter()
        try:
            for i in range(a.steps):
                step(sync=True)
                eng.sort_result()
                sort_ms.append(eng.stats()["ms_sort"])
            eng.synchronize()
            el_sorted = time.perf_counter() - t1
            sorted_result = {"value": round(total / (el_sorted / a.steps) / 1e9, 3),
                             "ms_per_step": round(el_sorted / a.steps * 1e3, 4),
                             "sort_bytes_ms": round(statistics.mean(sort_ms), 4),
                             "note": "the same K steps as synchronous passes, each followed by the device bytewise "
                                     "sort of its table (mox_sort_result): the work of the N > 1 step's sorted "
                                     "result on one GPU"}
        except mox.MoxError as ex:  # e.g. a table past the device sort's 4 GiB of word bytes (C4)
            eng.synchronize()
            sorted_result = {"value": None, "note": "device bytewise sort not available for this table: %s" % ex}
    eng.set_flags(base_flags | mox.MOX_F_TIMING)  # untimed diagnostic step: per-phase events
    step(sync=True)
    eng.synchronize()
    phases = [eng.stats()]
    if dist:
        import torch
        t = torch.tensor([elapsed, el_hash or 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        el_hash = float(t[1].item()) if el_hash is not None else None
    last = eng.stats()
    t = eng.fetch()
    counts, offs, _ = t.arrays()
    ok = int(counts.sum()) == t.tokens
    table_n, table_bytes, table_tokens = t.n, int(offs[-1]) if t.n else 0, t.tokens
    t.close()
    xinfo = None
    if dist:
        import torch
        # per-rank tokens of the local pass (the diagnostic step's stats are the
        # exchange's; the local pass counted what this rank's shard holds)
        loc = torch.tensor([float(local_tokens(eng, d_buf, hi - lo, own_b, own_e, at_end)), last["x_bytes_sent"],
                            last["x_bytes_recv"], statistics.mean(xms) if xms else 0.0,
                            statistics.mean(gms) if gms else 0.0, sort_ms], dtype=torch.float64)
        rows = [torch.zeros_like(loc) for _ in range(world)]
        dist.all_gather(rows, loc)
        rows = [r.tolist() for r in rows]
        tokens_all = int(sum(r[0] for r in rows))
        if gather:  # rank 0 holds the whole table: its tokens are the corpus's
            ok = ok and (rank != 0 or table_tokens == tokens_all)
        okt = torch.tensor([int(ok)], dtype=torch.float64)
        dist.all_reduce(okt)
        ok = int(okt.item()) == world
        xinfo = {
            "per_rank_tokens": [int(r[0]) for r in rows],
            "all_to_all_bytes": int(sum(r[1] for r in rows)),
            "all_to_all_bytes_recv": int(sum(r[2] for r in rows)),
            "exchange_ms_max_over_ranks": round(max(r[3] for r in rows), 4),
            "gather_ms_max_over_ranks": round(max(r[4] for r in rows), 4) if gather else None,
            "gathered_table": {"n": table_n, "bytes": table_bytes, "tokens": table_tokens,
                               "order": "bytewise (sorted exchange: every rank sorts its byte range inside the timed "
                                        "step, the gather concatenates in rank order)"} if gather else None,
            "sort_bytes_ms_max_over_ranks": round(max(r[5] for r in rows), 4) if gather else None,
            "hash_order": {"value": round(total / (el_hash / a.steps) / 1e9, 3), "ms_per_step": round(el_hash / a.steps * 1e3, 4),
                           "note": "the same steps without the sort at rank 0"} if el_hash else None,
            "note": "exchange = sampled byte-range splitters + counts all-to-all + pack + payload all-to-all "
                    "(RCCL send/recv in one group) + reduce-only pass; sort_bytes = the rank's bytewise sort of its "
                    "range, after the exchange; "
                    "gather = every rank's sorted table to rank 0 (mox_gather) in rank order, inside the timed step",
        }
    else:
        tokens_all = last["tokens"]

    if rank == 0:
        ms_step = elapsed / a.steps * 1e3
        gbs = total / (elapsed / a.steps) / 1e9
        map_avg = statistics.mean(map_ms) if map_ms else float("nan")
        if n1:  # the efficiency against the max-over-ranks time (known only now)
            n1["scaling_efficiency"] = round(gbs / (world * n1["value"]), 4)
        # algorithmic bytes per step = input read once + the output
        # table written once (word bytes + a u64 count per distinct word)
        b_alg = total + (table_bytes + 8 * table_n if (world == 1 or gather) else 0)
        line = {
            "metric": METRIC,
            "value": round(gbs, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: mox_corpus kind=%d seed=%#x (%s, host-generated, "
                    "copied to HBM before timing)" % (kind, seed, KIND_DESC.get(kind, "?")),
            "config": {"workload": desc, "bytes_per_gpu": per_rank, "total_bytes": total,
                       "parallelism": "dp%d byte-range shards%s" % (
                           world, (" + %s all-to-all%s" % ("RCCL" if a.xport == "rccl" else "host/gloo",
                                                            " + gather at rank 0" if gather else "")) if world > 1 else "")},
            "words_per_s": round(tokens_all / (elapsed / a.steps), 1),
            "pct_hbm_peak": round(100.0 * gbs / (HBM_PEAK_GBS * world), 2),
            "algorithmic_bytes_per_step": b_alg,
            "roofline_end_to_end": {"achieved": round(b_alg / (elapsed / a.steps) / 1e9, 1),
                                    "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                                    "frac": round(b_alg / (elapsed / a.steps) / 1e9 / (HBM_PEAK_GBS * world), 4)},
            "roofline": roofline_fields(per_rank, map_avg, a.workload, a.traffic_json),
            "phases_note": "phases_ms: one untimed diagnostic step with per-phase HIP events",
            "pass_mode": "async (mox_run_range_async: back-to-back passes, each completed and checked)" if use_async else "sync",
            "phases_ms": {k: round(statistics.mean(p[k] for p in phases), 4)
                          for k in ("ms_run", "ms_dict", "ms_map", "ms_lanes", "ms_reduce", "ms_finalize",
                                    "ms_exchange", "ms_gather")},
            "stats": {k: last[k] for k in ("tokens", "uniques", "dict_words", "cold_records", "weighted_records",
                                           "unicode_tokens", "long_tokens", "chunks", "max_subpasses", "retries",
                                           "reduce_units", "split_partitions")},
            "multi_gpu": xinfo,
            "sorted_result": sorted_result,
            "same_work_n1": n1,
            "check_sum_counts_eq_tokens": ok,
            "cpu_baseline": None,
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(kind, seed, min(per_rank, a.cpu_sample_mib << 20), a.cpu_runs)
        print(json.dumps(line), flush=True)
    eng.free(d_buf)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
