#!/usr/bin/env python3
"""bench.py -- device-resident QPACK Huffman encode + decode throughput.

Metric (BASELINE.json): GB/s of device-resident QPACK Huffman enc+dec on a
1M-string batch per GPU.  One step = one encode pass over the rank's 1M-string
synthetic batch (config 2) + one decode pass over the Huffman payload of a
1M-string batch (config 3), both through the C-ABI (libqhuff.so).  value =
(raw bytes encoded + raw bytes decoded, summed over ranks) / wall time.

Run: python bench.py [--gpus N --steps K --warmup W].  One process per GPU:
under torch.distributed.run (WORLD_SIZE must equal --gpus), or, with no
launcher, bench.py starts the N rank processes itself before anything touches
the GPU (ranks beyond the visible GPUs share them round-robin).  Strings are
sharded, no collective on the data path: "scaling": "weak".

Input buffers are rotated over --copies device copies (default 4, > 512 MB
footprint) so a step does not re-read the previous step's bytes from the
256 MB Infinity Cache.  Ranks meet only at the timing barrier and the
max-over-ranks of the wall time, both over gloo on the host: no RCCL.

--config4: ONE process, one host thread + HIP
stream + qhuff context per GPU; a 16M-string batch is split by
qhuff_shard_cuts into G byte-balanced contiguous shards, each GPU encodes
and decodes its shard per step, and the shard outputs are stitched back
(shard bases added on the host) and checked against a single-GPU pass over
the whole batch.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

METRIC = ("GB/s device-resident QPACK Huffman enc+dec, 1M-string batch, "
          "1/2/4/8 MI355X")
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=1 << 20,
                    help="strings per GPU (default 1M)")
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--alphabet", default="token", choices=["token", "base64"])
    ap.add_argument("--cpu-seconds", type=float, default=2.0,
                    help="wall seconds per CPU-baseline leg (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline 'all' leg threads (0 = every CPU this "
                         "process may use: affinity, capped by the cgroup "
                         "CPU quota)")
    ap.add_argument("--config4", action="store_true",
                    help="one process, G = --gpus devices, 16M strings split "
                         "by qhuff_shard_cuts (no RCCL)")
    ap.add_argument("--n4", type=int, default=16 << 20,
                    help="--config4 total strings (default 16M)")
    ap.add_argument("--host-path", action=argparse.BooleanOptionalAction,
                    default=True,
                    help="also time the PCIe-inclusive host-memory path "
                         "(rank 0; never `value`)")
    ap.add_argument("--overlap", action=argparse.BooleanOptionalAction,
                    default=True,
                    help="also time the same steps with encode and decode on "
                         "two streams (two contexts), consecutive launches "
                         "overlapping (rank 0; never `value`)")
    ap.add_argument("--workloads", action=argparse.BooleanOptionalAction,
                    default=True,
                    help="also time the real-workload batches (QIF corpora, "
                         "base64, long-code alphabet C; rank 0; never "
                         "`value`)")
    ap.add_argument("--probe-launch", action="store_true",
                    help=argparse.SUPPRESS)   # tests: ranks meet, no GPU
    ap.add_argument("--time-every", type=int, default=10,
                    help="time every k-th encode / decode launch of the timed "
                         "region (dispatch-stamped events; each timed launch "
                         "adds ~4.6 us of queue time to its step)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles",
                                                  "pmc_latest.json"),
                    help="PMC traffic summary (tools/pmc_summary.py)")
    return ap.parse_args()


def cpu_model():
    """The host CPU model (report it beside the CPU baseline)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cpus():
    """What the CPU baseline can use: logical CPUs in the affinity mask,
    capped by the cgroup CPU quota (a GPU box shares its host), plus the
    machine's sockets / physical cores / SMT from /proc/cpuinfo."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    sockets, cores, logical = set(), set(), 0
    phys = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    logical += 1
                elif k == "physical id":
                    phys = v
                    sockets.add(v)
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"usable": usable, "affinity": aff,
            "cgroup_quota_cpus": quota, "nproc": os.cpu_count(),
            "sockets": len(sockets) or None,
            "physical_cores": len(cores) or None,
            "smt": (logical // len(cores)) if cores else None}


def free_port():
    """An unused TCP port on 127.0.0.1 for the gloo rendezvous."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_check(gpus, env):
    """--gpus against the launcher's WORLD_SIZE.  Returns None when bench.py
    must start the ranks itself (no launcher, --gpus > 1), the world size
    otherwise; raises SystemExit when the two disagree."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return None if gpus > 1 else 1
    if int(ws) != gpus:
        raise SystemExit("bench: WORLD_SIZE=%s but --gpus %d: one rank per "
                         "GPU, the two must agree" % (ws, gpus))
    return int(ws)


def launch_plan(gpus, env, port):
    """Environments of the --gpus ranks bench.py starts itself: the variables
    torch.distributed.run would set (rendezvous on 127.0.0.1)."""
    plan = []
    for r in range(gpus):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(gpus),
                  "LOCAL_WORLD_SIZE": str(gpus), "GROUP_RANK": "0",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        plan.append(e)
    return plan


def self_launch(gpus):
    """`bench.py --gpus N` without an outside launcher: start N rank
    processes (this process has not touched the GPU, and never does), wait
    for them, exit with the worst status.  Rank 0 prints the JSON line."""
    import subprocess
    plan = launch_plan(gpus, os.environ, free_port())
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)]
                              + sys.argv[1:], env=e) for e in plan]
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    sys.exit(bad[0] if bad else 0)


def main():
    args = parse()
    if args.config4:
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            sys.exit("bench: --config4 is one process driving --gpus devices "
                     "(one host thread each); do not start it per rank")
    elif rank_check(args.gpus, os.environ) is None:
        return self_launch(args.gpus)
    import numpy as np
    import torch
    import torch.distributed as dist
    import qhuff

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; more ranks than GPUs (a rehearsal on a small box)
    # share them round-robin
    local = local % max(1, torch.cuda.device_count())
    if args.config4:
        return run_config4(args, np, torch, qhuff)
    if world > 1:
        # timing barrier + max-over-ranks only: host-side gloo, no RCCL.
        # Gloo announces its connections on stdout; rank 0's stdout carries
        # only the JSON line, so its fd 1 points at stderr meanwhile.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if args.probe_launch:
        # (tests/test_bench_launch.py) the rank plumbing alone, on the CPU:
        # every rank reports its rank and planned device; rank 0 prints them
        me = torch.tensor([rank, local], dtype=torch.int64)
        got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        if world > 1:
            dist.all_gather(got, me)
            dist.destroy_process_group()
        else:
            got = [me]
        if rank == 0:
            print(json.dumps({"n_gpus": world, "gpus_arg": args.gpus,
                              "ranks": [int(g[0]) for g in got],
                              "devices": [int(g[1]) for g in got]}),
                  flush=True)
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    # ---- inputs: this rank's shard of an (world x n)-string batch --------------
    alpha = (qhuff.TOKEN_ALPHABET if args.alphabet == "token"
             else qhuff.BASE64_ALPHABET)
    seed = 0x9E3779B97F4A7C15 ^ (rank * 0x632BE59BD9B4E019)
    data, off = qhuff.synth_batch(args.n, seed=seed & 0xFFFFFFFFFFFFFFFF,
                                  alphabet=alpha)
    n = args.n
    raw_bytes = int(off[-1])
    codec = qhuff.Codec(local)

    d_in = [torch.from_numpy(data).to(dev) for _ in range(args.copies)]
    d_off = [torch.from_numpy(off.view(np.int32)).to(dev)
             for _ in range(args.copies)]
    enc_cap = qhuff.encode_bound(raw_bytes, n, 0)
    e_out = [torch.empty(enc_cap, dtype=torch.uint8, device=dev)
             for _ in range(args.copies)]
    e_off = [torch.empty(n + 1, dtype=torch.int32, device=dev)
             for _ in range(args.copies)]

    # decode inputs = the Huffman payloads (forced Huffman), made once
    h_out, h_off = codec.encode(d_in[0], d_off[0], 0)
    torch.cuda.synchronize()
    h_off_np = h_off.cpu().numpy().view(np.uint32)
    huff_bytes = int(h_off_np[-1])
    h_np = h_out[:huff_bytes].cpu().numpy()
    del h_out
    d_hin = [torch.from_numpy(h_np).to(dev) for _ in range(args.copies)]
    d_hoff = [torch.from_numpy(h_off_np.view(np.int32)).to(dev)
              for _ in range(args.copies)]
    dec_cap = qhuff.decode_bound(huff_bytes, n)
    d_out = [torch.empty(dec_cap, dtype=torch.uint8, device=dev)
             for _ in range(args.copies)]
    d_ooff = [torch.empty(n + 1, dtype=torch.int32, device=dev)
              for _ in range(args.copies)]
    d_st = [torch.empty(n, dtype=torch.uint8, device=dev)
            for _ in range(args.copies)]

    stream = torch.cuda.current_stream()

    def step(i):
        k = i % args.copies
        j = (i + args.copies // 2) % args.copies
        codec.encode_into(d_in[k], d_off[k], n, 0, e_out[k], e_off[k], stream)
        codec.decode_into(d_hin[j], d_hoff[j], n, d_out[j], d_ooff[j],
                          d_st[j], stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()

    # one correctness probe outside the timed region: round trip of copy 0
    codec.decode_into(d_hin[0], d_hoff[0], n, d_out[0], d_ooff[0], d_st[0],
                      stream)
    torch.cuda.synchronize()
    ok_dec = (torch.equal(d_out[0][:raw_bytes], d_in[0])
              and bool((d_st[0] == 0).all())
              and torch.equal(d_ooff[0], d_off[0]))

    # kernel durations for the roofline: every --time-every-th launch of each
    # kind in the timed region carries a HIP event pair stamped by its own
    # dispatch (qhuff_timing_*: hipExtLaunchKernel's start / stop events --
    # the kernel's device time, as rocprofv3's kernel trace measures it).
    # Sampled: a timed launch adds ~4.6 us of queue time to its step
    # (tools/timing_cost.py: 114.8 vs 105.6 us per step with every launch
    # timed / none, profiles/r04_tc), which would otherwise count in `value`
    codec.timing(True, every=args.time_every)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    timed = codec.timing_read()
    codec.timing(False)
    enc_t = [u for k, u in timed if k == qhuff.KIND_ENCODE]
    dec_t = [u for k, u in timed if k == qhuff.KIND_DECODE]
    enc_ms = sum(enc_t) / len(enc_t) * 1e-3
    dec_ms = sum(dec_t) / len(dec_t) * 1e-3
    # the kernels' sticky error word (look-back spin / offset range): a
    # launch that raised one produced no valid output
    dev_err = codec.device_error()

    if world > 1:
        t = torch.tensor([wall, 0.0 if ok_dec else 1.0, float(dev_err)],
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t[0])
        ok_dec = bool(t[1] < 0.5)
        dev_err = int(t[2])

    ms_per_step = wall * 1e3 / args.steps
    bytes_per_step = 2 * raw_bytes           # raw in (encode) + raw out (decode)
    value = world * bytes_per_step / (wall / args.steps) / 1e9

    # ---- roofline for the dominant kernel ---------------------------------------
    alg_enc = raw_bytes + huff_bytes + 8 * n       # in, out, in_off, out_off
    alg_dec = huff_bytes + raw_bytes + 9 * n       # + 1 B status
    if dec_ms >= enc_ms:
        kname, kms, alg = "qhuff_decode_kernel", dec_ms, alg_dec
    else:
        kname, kms, alg = "qhuff_encode_kernel", enc_ms, alg_enc
    achieved = alg / (kms * 1e-3) / 1e9
    # SURVEY 8(d)'s per-string figure counts separate in_len / out_len arrays
    # (16 B / 17 B per string for encode / decode); this ABI derives lengths
    # from the offsets (8 / 9 B).  Both fractions are reported.
    alg_survey = (huff_bytes + raw_bytes + 17 * n
                  if kname == "qhuff_decode_kernel"
                  else raw_bytes + huff_bytes + 16 * n)
    traffic = None
    pmc_src = None
    if os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            ent = pm.get("kernels", {}).get(kname)
            if ent and ent.get("n") == n:
                traffic = ent.get("hbm_bytes_per_launch")
                pmc_src = os.path.relpath(args.pmc, ROOT)
        except Exception:
            traffic = None
    roof = {"bound": "hbm", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "frac_survey": round(alg_survey / (kms * 1e-3) / 1e9
                                 / HBM_PEAK_GBS, 4),
            "alg_bytes_survey": alg_survey,
            "kernel": kname, "kernel_us": round(kms * 1e3, 2),
            "alg_bytes": alg,
            "timing": "mean over %d %s launches of the timed region (every "
                      "%d-th), each dispatched with HIP start/stop events "
                      "stamped by the dispatch itself (hipExtLaunchKernel)"
                      % (len(dec_t if kname == "qhuff_decode_kernel" else enc_t),
                         kname, max(1, args.time_every))}
    if pmc_src:
        roof["traffic_source"] = pmc_src

    # ---- header hashing, outside the timed step --------
    # the batch read as n/2 (name, value) headers: XXH32 name + name/value
    hh = n // 2
    h1 = torch.empty(hh, dtype=torch.int32, device=dev)
    h2 = torch.empty(hh, dtype=torch.int32, device=dev)
    # timed the way enc/dec are: each launch's own dispatch timestamps
    for i in range(10):
        codec.xxh32_headers_into(d_in[i % args.copies], d_off[i % args.copies],
                                 hh, qhuff.XXH_SEED, h1, h2, stream)
    codec.timing(True)
    nh = max(1, min(args.steps, 20))
    for i in range(nh):
        codec.xxh32_headers_into(d_in[i % args.copies], d_off[i % args.copies],
                                 hh, qhuff.XXH_SEED, h1, h2, stream)
    ht = [u for k, u in codec.timing_read() if k == qhuff.KIND_HASH]
    codec.timing(False)
    hash_ms = sum(ht) / len(ht) * 1e-3
    hash_bytes = int(off[2 * hh])
    hash_alg = hash_bytes + 4 * (2 * hh + 1) + 8 * hh
    hashing = {"kernel": "qhuff_hash_kernel", "headers": hh,
               "kernel_us": round(hash_ms * 1e3, 2),
               "timing": "mean over %d launches, dispatch-stamped HIP "
                         "events (hipExtLaunchKernel)" % len(ht),
               "payload_gbps": round(hash_bytes / (hash_ms * 1e-3) / 1e9, 2),
               "alg_bytes": hash_alg,
               "roofline_frac": round(hash_alg / (hash_ms * 1e-3) / 1e9
                                      / HBM_PEAK_GBS, 4),
               "traffic": None}
    if os.path.exists(args.pmc):
        try:
            ent = json.load(open(args.pmc)).get("kernels", {}).get(
                "qhuff_hash_kernel")
            if ent and ent.get("n") == hh:
                hashing["traffic"] = ent.get("hbm_bytes_per_launch")
        except Exception:
            pass

    overlap = None
    if args.overlap and rank == 0 and world == 1:
        overlap = run_overlap(args, np, torch, qhuff, dev, n, raw_bytes, d_in,
                              d_off, e_out, e_off, d_hin, d_hoff, d_out,
                              d_ooff, d_st, ms_per_step)

    work = None
    if args.workloads and rank == 0 and world == 1:
        work = run_workloads(args, np, torch, qhuff, codec, dev, stream, n,
                             raw_bytes, enc_ms, dec_ms,
                             (d_in[0], d_off[0], d_hin[0], d_hoff[0]))

    host = None
    if args.host_path and rank == 0:
        # result buffers allocated and faulted in once (a fresh np.zeros of
        # the bound per call would time page faults, not the library); the
        # first calls size the pinned / device staging buffers; time after
        eo = np.ones(enc_cap, dtype=np.uint8)
        eoo = np.ones(n + 1, dtype=np.uint32)
        do = np.ones(dec_cap, dtype=np.uint8)
        doo = np.ones(n + 1, dtype=np.uint32)
        dst = np.ones(n, dtype=np.uint8)
        codec.encode_host(data, off, 0, eo, eoo)
        codec.decode_host(h_np, h_off_np, do, doo, dst)
        t_e = t_d = 1e30
        for _ in range(5):
            t = time.perf_counter()
            codec.encode_host(data, off, 0, eo, eoo)
            t_e = min(t_e, time.perf_counter() - t)
            t = time.perf_counter()
            codec.decode_host(h_np, h_off_np, do, doo, dst)
            t_d = min(t_d, time.perf_counter() - t)
        ok_host = (np.array_equal(doo, off) and not dst.any()
                   and np.array_equal(do[:raw_bytes], data))
        host = {"enc_gbps": round(raw_bytes / t_e / 1e9, 3),
                "dec_gbps": round(raw_bytes / t_d / 1e9, 3),
                "enc_ms": round(t_e * 1e3, 3), "dec_ms": round(t_d * 1e3, 3),
                "roundtrip_ok": bool(ok_host),
                "note": "host buffers in and out: chunked pipeline of pinned "
                        "staging copies (copy workers) + hipMemcpyAsync in + "
                        "kernel + exact-size hipMemcpyAsync out, synchronous, "
                        "best of 5 after one sizing call"}
        # the same calls with every buffer registered (qhuff_host_register):
        # DMA straight from / into the caller's memory, no staging copy
        for a in (eo, eoo, do, doo, dst):
            a.fill(1)
        t = time.perf_counter()
        with qhuff.registered(data, off, h_np, h_off_np, eo, eoo, do, doo,
                              dst):
            t_reg = time.perf_counter() - t
            t_e = t_d = 1e30
            for _ in range(5):
                t = time.perf_counter()
                codec.encode_host(data, off, 0, eo, eoo)
                t_e = min(t_e, time.perf_counter() - t)
                t = time.perf_counter()
                codec.decode_host(h_np, h_off_np, do, doo, dst)
                t_d = min(t_d, time.perf_counter() - t)
        ok_reg = (np.array_equal(doo, off) and not dst.any()
                  and np.array_equal(do[:raw_bytes], data)
                  and np.array_equal(eoo, h_off_np)
                  and np.array_equal(eo[:int(eoo[-1])], h_np))
        host["registered"] = {
            "enc_gbps": round(raw_bytes / t_e / 1e9, 3),
            "dec_gbps": round(raw_bytes / t_d / 1e9, 3),
            "enc_ms": round(t_e * 1e3, 3), "dec_ms": round(t_d * 1e3, 3),
            "register_ms": round(t_reg * 1e3, 3), "roundtrip_ok": bool(ok_reg),
            "note": "all nine buffers registered once (register_ms, not in "
                    "the calls): hipMemcpyAsync from / into them directly"}

    # ---- CPU baseline (rank 0, N = 1 only), after every GPU leg: seconds of
    # an idle GPU before a leg slow its first launches (the hash leg's mean
    # read 16.5 us against rocprof's 12.5 when it ran after this one) -------
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, data, off, h_np, h_off_np, n, raw_bytes)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (xorshift64 %s alphabet, U[8,64] B strings)"
                    % args.alphabet,
            "config": {"workload": "config2+3: encode 1M strings + decode 1M "
                                   "Huffman strings per GPU per step",
                       "strings_per_gpu": n, "raw_bytes_per_gpu": raw_bytes,
                       "huff_bytes_per_gpu": huff_bytes,
                       "parallelism": "dp%d (independent string shards)" % world},
            "enc_kernel_us": round(enc_ms * 1e3, 2),
            "dec_kernel_us": round(dec_ms * 1e3, 2),
            "enc_payload_gbps": round(raw_bytes / (enc_ms * 1e-3) / 1e9, 2),
            "dec_payload_gbps": round(raw_bytes / (dec_ms * 1e-3) / 1e9, 2),
            "roundtrip_ok": bool(ok_dec),
            "device_error": dev_err,
            "xxh32_headers": hashing,
            "roofline": roof, "cpu_baseline": cpu,
        }
        if host:
            line["host_path"] = host
        if work:
            line["workloads"] = work
        if overlap:
            line["two_streams"] = overlap
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()
    if dev_err or not ok_dec:
        sys.exit("bench: device error %d / round trip %s: the line above is "
                 "not a valid measurement" % (dev_err, ok_dec))


def cpu_baseline(args, data, off, h_np, h_off_np, n, raw_bytes):
    """The oracle (a restatement of lsqpack_enc_enc_str(7, ..) and
    lsqpack_huff_decode's fast path) over the same batch: one thread, then
    every CPU this process may use.  `value` is the all-CPU
    leg."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    cpus = host_cpus()
    t_all = args.cpu_threads or cpus["usable"]

    def leg(buf, offs, op, threads):
        best, tot, reps = 1e30, 0.0, 0
        while tot < args.cpu_seconds or reps < 2:
            dt = oracle_lib.bench_pass(buf, offs, op, threads)
            best = min(best, dt)
            tot += dt
            reps += 1
        return raw_bytes / best / 1e9, reps

    legs = {}
    for name, threads in (("threads_1", 1), ("threads_all", t_all)):
        e, r1 = leg(data, off, 0, threads)
        d, r2 = leg(h_np, h_off_np, 1, threads)
        legs[name] = {"threads": threads, "enc_gbps": round(e, 3),
                      "dec_gbps": round(d, 3),
                      "gbps": round(2.0 / (1.0 / e + 1.0 / d), 3),
                      "passes": [r1, r2]}
    return {"value": legs["threads_all"]["gbps"], "unit": "GB/s",
            "cores": t_all, "kind": "port",
            "sample": ("full %d-string batch, oracle restatement of "
                       "lsqpack_enc_enc_str(7,..) + lsqpack_huff_decode (fast "
                       "path), best pass of >= %.0f s per leg, at 1 thread and "
                       "at every usable CPU" % (n, args.cpu_seconds)),
            "threads_1": legs["threads_1"], "threads_all": legs["threads_all"],
            "host": cpus, "cpu_model": cpu_model()}


def run_overlap(args, np, torch, qhuff, dev, n, raw, d_in, d_off, e_out,
                e_off, d_hin, d_hoff, d_out, d_ooff, d_st, ms_seq):
    """The timed steps again with encode on one stream and decode on another
    (a context each: one look-back workspace per context), no per-step sync,
    so one kernel's ramp and partial last round overlap the other's.  Never
    `value`: reported beside it, with the round trip checked."""
    ce, cd = qhuff.Codec(dev.index or 0), qhuff.Codec(dev.index or 0)
    se, sd = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def step(i):
        k = i % args.copies
        j = (i + args.copies // 2) % args.copies
        ce.encode_into(d_in[k], d_off[k], n, 0, e_out[k], e_off[k], se)
        cd.decode_into(d_hin[j], d_hoff[j], n, d_out[j], d_ooff[j], d_st[j],
                       sd)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    k = (args.warmup + args.steps - 1) % args.copies
    j = (args.warmup + args.steps - 1 + args.copies // 2) % args.copies
    ok = (torch.equal(d_out[j][:raw], d_in[j]) and not bool(d_st[j].any())
          and ce.device_error() == 0 and cd.device_error() == 0
          and torch.equal(e_off[k], d_hoff[k]))
    ce.close()
    cd.close()
    ms = wall * 1e3 / args.steps
    return {"ms_per_step": round(ms, 4),
            "gbps": round(2 * raw / (ms * 1e-3) / 1e9, 3),
            "vs_sequential": round(ms_seq / ms, 3), "roundtrip_ok": bool(ok),
            "note": "encode stream + decode stream, a context each, no "
                    "per-step synchronisation; not `value`"}


def run_workloads(args, np, torch, qhuff, codec, dev, stream, n, raw_syn,
                  enc_ms_syn, dec_ms_syn, syn):
    """Real-workload shapes, never `value`: 1M-string
    batches of the reference's QIF corpora (names and values in wire order,
    repeated), of the base64 alphabet and of the long-code alphabet C; each
    encoded and decoded K times with dispatch-stamped timing (kernel device
    time), the round trip checked, and the tile-path shares of each batch
    (qhuff/workload.py: slow tiles, variable arena slots, encode fallback).
    first_launch_us: each batch's first encode and
    first decode launch, timed right after 8 token launches of each kind on
    the same context -- no launch on the batch itself before it (its
    Huffman form is made on a second context; the code objects are loaded
    by the earlier legs).  Unhinted (the device-pointer calls' default,
    qhuff_host.cpp pick_full) that launch runs the full kernel (round 6;
    until round 5 decode went by a history of earlier launches and ran
    lean: 4.3x its warmed time on the corpus); hinted_*: the same with the
    variant hinted from the host's copy of the offsets (qhuff_batch_hint,
    as the host-memory calls do themselves)."""
    from qhuff import workload as W
    K = 10
    data_dir = os.path.join(ROOT, "tests", "golden", "data")
    s_in, s_off, s_h, s_hoff = syn
    s_eo = torch.empty(qhuff.encode_bound(int(s_in.numel()), n, 0),
                       dtype=torch.uint8, device=dev)
    s_eoo = torch.empty(n + 1, dtype=torch.int32, device=dev)
    s_do = torch.empty(qhuff.decode_bound(int(s_h.numel()), n),
                       dtype=torch.uint8, device=dev)
    s_doo = torch.empty(n + 1, dtype=torch.int32, device=dev)
    s_st = torch.empty(n, dtype=torch.uint8, device=dev)
    batches = [
        ("base64", "synthetic U[8,64], base64 alphabet",
         qhuff.synth_batch(n, alphabet=qhuff.BASE64_ALPHABET)),
        ("alphabet_c", "synthetic U[8,64], token alphabet + ~2 % long-code "
                       "bytes {1,2,6,92,141}", W.alphabet_c(n)),
        ("qif_corpus", "tests/golden/data/{fb-req,fb-resp,long-codes,netbsd}"
                       ".qif names and values in wire order, repeated",
         W.corpus_batch(n, data_dir)),
    ]
    syn_gbps = 2 * raw_syn / ((enc_ms_syn + dec_ms_syn) * 1e-3) / 1e9
    out = {"strings": n, "launches_per_kernel": K,
           "synthetic_token_gbps": round(syn_gbps, 1)}
    # each batch's Huffman form (the decode legs' input) made on a context
    # of its own: on `codec` that launch would be a launch on the batch
    # before its first-launch measurement
    prep = qhuff.Codec(dev.index or 0)
    for name, desc, (data, off) in batches:
        raw = int(off[-1])
        d = torch.from_numpy(data).to(dev)
        o = torch.from_numpy(off.view(np.int32)).to(dev)
        ecap = qhuff.encode_bound(raw, n, 0)
        eo = torch.empty(ecap, dtype=torch.uint8, device=dev)
        eoo = torch.empty(n + 1, dtype=torch.int32, device=dev)
        prep.encode_into(d, o, n, 0, eo, eoo, stream)
        torch.cuda.synchronize()
        hoff = eoo.cpu().numpy().view(np.uint32).copy()
        hb = int(hoff[-1])
        h = eo[:hb].clone()
        do = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8,
                         device=dev)
        doo = torch.empty(n + 1, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        # the first launch of each kind on this batch, after 8 token
        # launches of each kind, each waited for (the output is checked
        # with the others')
        for _ in range(8):
            codec.encode_into(s_in, s_off, n, 0, s_eo, s_eoo, stream)
            torch.cuda.synchronize()
        for _ in range(8):
            codec.decode_into(s_h, s_hoff, n, s_do, s_doo, s_st, stream)
            torch.cuda.synchronize()
        codec.timing(True)
        codec.encode_into(d, o, n, 0, eo, eoo, stream)
        torch.cuda.synchronize()
        first_e = [u for k, u in codec.timing_read() if k == qhuff.KIND_ENCODE]
        var_e = codec.kernel_variant(qhuff.KIND_ENCODE)
        codec.timing(False)
        for _ in range(8):
            codec.decode_into(s_h, s_hoff, n, s_do, s_doo, s_st, stream)
            torch.cuda.synchronize()
        codec.timing(True)
        codec.decode_into(h, eoo, n, do, doo, st, stream)
        torch.cuda.synchronize()
        first_d = [u for k, u in codec.timing_read() if k == qhuff.KIND_DECODE]
        var_d = codec.kernel_variant(qhuff.KIND_DECODE)
        codec.timing(False)
        first_ok = (torch.equal(do[:raw], d) and not bool(st.any()))
        # the same with the variant hinted from the host copy of the batch's
        # offsets (qhuff_batch_hint / qhuff_batch_needs_full, ABI 6)
        hint = qhuff.batch_needs_full(off)
        hint_d = qhuff.batch_needs_full(hoff)
        hinted = {}
        for kind, hv in ((qhuff.KIND_ENCODE, hint), (qhuff.KIND_DECODE, hint_d)):
            for _ in range(8):
                if kind == qhuff.KIND_ENCODE:
                    codec.encode_into(s_in, s_off, n, 0, s_eo, s_eoo, stream)
                else:
                    codec.decode_into(s_h, s_hoff, n, s_do, s_doo, s_st, stream)
                torch.cuda.synchronize()
            codec.timing(True)
            codec.batch_hint(kind, hv)
            if kind == qhuff.KIND_ENCODE:
                codec.encode_into(d, o, n, 0, eo, eoo, stream)
            else:
                codec.decode_into(h, eoo, n, do, doo, st, stream)
            torch.cuda.synchronize()
            hinted[kind] = [u for k, u in codec.timing_read() if k == kind][0]
            codec.timing(False)
        first_ok = first_ok and torch.equal(do[:raw], d) and not bool(st.any())
        for _ in range(2):
            codec.encode_into(d, o, n, 0, eo, eoo, stream)
            codec.decode_into(h, eoo, n, do, doo, st, stream)
        torch.cuda.synchronize()
        codec.timing(True)
        for _ in range(K):
            codec.encode_into(d, o, n, 0, eo, eoo, stream)
        for _ in range(K):
            codec.decode_into(h, eoo, n, do, doo, st, stream)
        tm = codec.timing_read()
        codec.timing(False)
        eu = [u for k, u in tm if k == qhuff.KIND_ENCODE]
        du = [u for k, u in tm if k == qhuff.KIND_DECODE]
        e_us, d_us = sum(eu) / len(eu), sum(du) / len(du)
        ok = (torch.equal(do[:raw], d) and not bool(st.any())
              and np.array_equal(doo.cpu().numpy().view(np.uint32), off))
        gbps = 2 * raw / ((e_us + d_us) * 1e-6) / 1e9
        ent = {"data": desc, "raw_bytes": raw, "huff_bytes": hb,
               "enc_kernel_us": round(e_us, 2), "dec_kernel_us": round(d_us, 2),
               "enc_payload_gbps": round(raw / (e_us * 1e-6) / 1e9, 1),
               "dec_payload_gbps": round(raw / (d_us * 1e-6) / 1e9, 1),
               "enc_dec_gbps": round(gbps, 1),
               "vs_synthetic_token": round(gbps / syn_gbps, 3),
               "first_launch_us": {"enc": round(first_e[0], 2),
                                   "dec": round(first_d[0], 2),
                                   "enc_vs_mean": round(first_e[0] / e_us, 3),
                                   "dec_vs_mean": round(first_d[0] / d_us, 3),
                                   "full_kernel": [var_e, var_d],
                                   "hinted_enc": round(hinted[qhuff.KIND_ENCODE], 2),
                                   "hinted_dec": round(hinted[qhuff.KIND_DECODE], 2),
                                   "hinted_vs_mean": [
                                       round(hinted[qhuff.KIND_ENCODE] / e_us, 3),
                                       round(hinted[qhuff.KIND_DECODE] / d_us, 3)],
                                   "hint": [hint, hint_d],
                                   "roundtrip_ok": bool(first_ok)},
               "roundtrip_ok": bool(ok)}
        ent.update(W.tile_shares(data, off, hoff))
        out[name] = ent
        del d, o, eo, eoo, h, do, doo, st
    del s_eo, s_eoo, s_do, s_doo, s_st
    prep.close()
    return out


def run_config4(args, np, torch, qhuff):
    """Config 4: one batch of --n4 strings over G GPUs of one process,
    through the C-ABI's multi-context entry (include/qhuff.h
    qhuff_encode_batch_multi / qhuff_decode_batch_multi: one host thread per
    context inside the library, every shard's out_off rebased on its device
    to the stitched batch's offsets)."""
    G = args.gpus
    # one device per shard; more shards than visible GPUs (a rehearsal on a
    # small box) share them round-robin
    ndev = max(1, torch.cuda.device_count())
    alpha = (qhuff.TOKEN_ALPHABET if args.alphabet == "token"
             else qhuff.BASE64_ALPHABET)
    N = args.n4
    data, off = qhuff.synth_batch(N, seed=0x9E3779B97F4A7C15, alphabet=alpha)
    cuts = qhuff.shard_cuts(off, G)
    from qhuff import shard as S
    copies = max(1, min(args.copies, 2))
    codecs, enc_sh, dec_sh, info = [], [[] for _ in range(copies)], \
        [[] for _ in range(copies)], []
    for g in range(G):
        dev = torch.device("cuda", g % ndev)
        torch.cuda.set_device(dev)
        sd, soff, _ = S.shard_view(data, off, cuts, g)
        n = len(soff) - 1
        raw = int(soff[-1])
        codec = qhuff.Codec(g % ndev)
        codecs.append(codec)
        st = torch.cuda.Stream(device=dev)
        d_in = torch.from_numpy(np.ascontiguousarray(sd)).to(dev)
        d_off = torch.from_numpy(soff.view(np.int32)).to(dev)
        ecap = qhuff.encode_bound(raw, n, 0)
        # decode input: this shard's Huffman payloads (shard-local offsets)
        h_out, h_off = codec.encode(d_in, d_off, 0)
        torch.cuda.synchronize(dev)
        hb = int(h_off[-1].item())
        dcap = qhuff.decode_bound(hb, n)
        for k in range(copies):
            enc_sh[k].append(dict(
                in_=d_in if k == 0 else d_in.clone(),
                in_off=d_off if k == 0 else d_off.clone(), n=n,
                out=torch.empty(ecap, dtype=torch.uint8, device=dev),
                out_off=torch.empty(n + 1, dtype=torch.int32, device=dev),
                stream=st))
            dec_sh[k].append(dict(
                in_=h_out[:hb].clone(), in_off=h_off.clone(), n=n,
                out=torch.empty(dcap, dtype=torch.uint8, device=dev),
                out_off=torch.empty(n + 1, dtype=torch.int32, device=dev),
                status=torch.empty(max(n, 1), dtype=torch.uint8, device=dev),
                stream=st))
        info.append({"n": n, "raw": raw, "huff": hb, "device": g % ndev})
        del h_out
    for g in range(G):
        torch.cuda.synchronize(g % ndev)

    def step(i):
        k = i % copies
        eb = qhuff.batch_multi(codecs, enc_sh[k], True, 0, rebase=True)
        db = qhuff.batch_multi(codecs, dec_sh[k], False, rebase=True)
        return eb, db

    for i in range(args.warmup):
        step(i)
    t0 = time.perf_counter()
    for i in range(args.steps):
        eb, db = step(args.warmup + i)
    wall = time.perf_counter() - t0       # (the calls are synchronous)
    raw_total = int(off[-1])
    value = 2 * raw_total * args.steps / wall / 1e9

    # stitched output (the last step's) == one pass over the whole batch on
    # GPU 0; its decode == the input
    k = (args.warmup + args.steps - 1) % copies
    cat = lambda parts: np.concatenate(parts) if parts else np.zeros(0)
    enc_m = cat([s["out"][:eb[g + 1] - eb[g]].cpu().numpy()
                 for g, s in enumerate(enc_sh[k])])
    enc_moff = cat([s["out_off"].cpu().numpy().view(np.uint32)[:-1]
                    for s in enc_sh[k]] + [np.array([eb[-1]], np.uint32)])
    dec_m = cat([s["out"][:db[g + 1] - db[g]].cpu().numpy()
                 for g, s in enumerate(dec_sh[k])])
    dec_moff = cat([s["out_off"].cpu().numpy().view(np.uint32)[:-1]
                    for s in dec_sh[k]] + [np.array([db[-1]], np.uint32)])
    status_ok = all(not s["status"][:s["n"]].cpu().numpy().any()
                    for s in dec_sh[k])
    dev_err = max(c.device_error() for c in codecs)
    for c in codecs:
        c.close()
    torch.cuda.set_device(0)
    c0 = qhuff.Codec(0)
    d_all = torch.from_numpy(data).cuda(0)
    o_all = torch.from_numpy(off.view(np.int32)).cuda(0)
    ref_out, ref_off = c0.encode(d_all, o_all, 0)
    torch.cuda.synchronize()
    ref_off = ref_off.cpu().numpy().view(np.uint32)
    stitched_ok = (np.array_equal(enc_moff.astype(np.uint32), ref_off)
                   and np.array_equal(enc_m,
                                      ref_out[:int(ref_off[-1])].cpu().numpy()))
    roundtrip_ok = (np.array_equal(dec_moff.astype(np.uint32), off)
                    and np.array_equal(dec_m, data) and status_ok)
    c0.close()
    shard_bytes = [r["raw"] for r in info]
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GB/s",
        "n_gpus": G, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (xorshift64 %s alphabet, U[8,64] B strings)"
                % args.alphabet,
        "config": {"workload": "config4", "strings": N,
                   "raw_bytes": raw_total,
                   "parallelism": "%d GPUs through qhuff_encode_batch_multi / "
                                  "qhuff_decode_batch_multi (one host thread "
                                  "+ stream + qhuff_ctx per shard, "
                                  "qhuff_shard_cuts byte-balanced shards, "
                                  "offsets rebased on device, no "
                                  "collective)" % G,
                   "shard_strings": [r["n"] for r in info],
                   "shard_raw_bytes": shard_bytes,
                   "shard_devices": [r["device"] for r in info],
                   "shard_byte_balance": round(max(shard_bytes)
                                               / max(1, min(shard_bytes)), 6)},
        "step": "encode call (all shards, synchronous) + decode call (all "
                "shards, synchronous)",
        "stitched_equals_single_pass": bool(stitched_ok),
        "roundtrip_ok": bool(roundtrip_ok), "device_error": dev_err,
    }
    print(json.dumps(line), flush=True)
    if dev_err or not stitched_ok or not roundtrip_ok:
        sys.exit("config4: check failed")


if __name__ == "__main__":
    main()
