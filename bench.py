"""Benchmark: weights quantized GB/s for Llama-2-7B 4-bit g=128 pseudo_quantize_tensor (BASELINE.json
metric / configs[1]) on MI355X, one process per GPU.

One step = one pass of the hot path over one batch of synthetic input: ALL 224 Linear weights of a
Llama-2-7B (32 x {q,k,v,o: 4096x4096, gate,up: 11008x4096, down: 4096x11008}, 6.476e9 fp16
weights = 12.95 GB) quantized INT4 g=128 asymmetric (quant_funcs.pseudo_quantize_tensor defaults
zero_point=True, out-of-place) in ONE persistent multi-tensor launch, writing the dequantized fp16
weights plus fp16 scales/zeros.  Inputs are generated on the device (oracle/synth.py's counter
generator) and resident in HBM before the timed region.

Multi-GPU, one rank per GPU: `python bench.py --gpus N` with no WORLD_SIZE in the environment spawns
N fresh rank processes itself (before any GPU call); under torchrun the ranks come from the
environment.  The model's 224 (7B) / 560 (70B) weights are bin-packed by bytes over the ranks
(shard.plan_shards) and every rank quantizes its bin with ONE batched launch: strong scaling, no
data-path collective (the layers are independent).  value = the model's fp16 input
bytes / max-over-ranks time.  For the 7B model at N > 1 the weak-scaling figure (every rank
quantizes a full 7B) is reported beside it ("weak").

Also reported: "roofline" for the quantize kernel (algorithmic bytes / measured HIP-event time vs
8 TB/s), "traffic" from a committed rocprofv3 PMC summary stamped with the kernel sources' hash
(dropped when the sources changed since), and "cpu_baseline": the reference's CPU arithmetic
(oracle/torch_ref.py, pinned to the reference) timed on a bounded sample on rank 0.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "weights quantized GB/s + PPL delta, Llama-2-7B 4-bit g=128 at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MODEL_NAME = {"llama2-7b": "Llama-2-7B", "llama2-70b": "Llama-2-70B", "opt-125m": "OPT-125M"}



class Marks:
    """--mark-file: the host-clock interval of every timed region (synchronized on both sides), so a
    rocprofv3 --kernel-trace of the same run can be cut into the regions afterwards
    (tools/trace_sections.py): per region, the kernels that ran in it and their average duration, to set
    beside the number bench.py reports for it.  No-op (no extra synchronization) without the flag."""

    def __init__(self):
        self.rows = None

    def enable(self):
        self.rows = []

    def region(self, name, **info):
        import contextlib
        if self.rows is None:
            return contextlib.nullcontext({})

        @contextlib.contextmanager
        def cm():
            rec = {"region": name, **info}
            torch.cuda.synchronize()
            rec["t0"] = {"boot": time.clock_gettime_ns(time.CLOCK_BOOTTIME), "mono": time.monotonic_ns(),
                         "real": time.time_ns()}
            yield rec
            torch.cuda.synchronize()
            rec["t1"] = {"boot": time.clock_gettime_ns(time.CLOCK_BOOTTIME), "mono": time.monotonic_ns(),
                         "real": time.time_ns()}
            self.rows.append(rec)
        return cm()

    def write(self, path, rank):
        if self.rows is None or not path:
            return
        with open(path if rank == 0 else f"{path}.rank{rank}", "w") as f:
            for r in self.rows:
                f.write(json.dumps(r) + "\n")


MARKS = Marks()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--symmetric", action="store_true")
    ap.add_argument("--model", default="llama2-7b", choices=["llama2-7b", "llama2-70b", "opt-125m"],
                    help="the model's Linear weights are bin-packed over the ranks (strong scaling); "
                         "llama2-7b = configs[1], llama2-70b = configs[3]")
    ap.add_argument("--weak", action="store_true",
                    help="headline = weak scaling instead: every rank quantizes the full model")
    ap.add_argument("--no-weak", action="store_true", help="7B at N > 1: skip the secondary weak-scaling figure")
    ap.add_argument("--gather", action="store_true",
                    help="(default at N > 1, kept for old command lines) time the rooted gather of the packed "
                         "codes + scales/zeros to rank 0 over RCCL, reported separately (never in value)")
    ap.add_argument("--no-collectives", action="store_true",
                    help="N > 1: skip the separately timed RCCL gather / scatter (gather_ms, scatter_ms)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank plumbing (spawn, shard plan, rooted gather) over gloo; "
                         "no GPU, no kernels, no timing")
    ap.add_argument("--scatter", action="store_true",
                    help="strong scaling of the chosen model: its weights start on rank 0 and are scattered to "
                         "their owners over RCCL point-to-point first (timed separately as scatter_ms, never in value)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ppl", action="store_true", help="skip the PPL-harness plumbing run (random-init OPT-125M)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--traffic-70b-file", default=os.path.join(ROOT, "profiles", "traffic_70b.json"))
    ap.add_argument("--variant", type=int, default=0, help="kernel tuning variant for the timed run")
    ap.add_argument("--variants", default="", help="A/B: comma list of variants timed in interleaved rounds")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--inplace", action="store_true",
                    help="time the in-place form instead: dequantized weights over the inputs "
                         "(QuantLinear.quantize_weight / quantize_model semantics, quant_linear.py:949)")
    ap.add_argument("--ramp-seconds", type=float, default=1.0,
                    help="untimed clock ramp before the copy-ceiling probe and the W warmup steps")
    ap.add_argument("--no-shapes", action="store_true",
                    help="skip the cold single-tensor calls per Llama shape (4096x4096, 11008x4096, 4096x11008)")
    ap.add_argument("--no-sections", action="store_true",
                    help="skip the configs[2] fused-forward, configs[4] format and configs[3] 70B sections")
    ap.add_argument("--no-70b", action="store_true", help="skip the configs[3] Llama-2-70B section")
    ap.add_argument("--mark-file", default="",
                    help="write the host-clock interval of every timed region (JSONL) for tools/trace_sections.py "
                         "(cuts a rocprofv3 kernel trace of this run into the bench's rows)")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: start N fresh rank processes of this same command (one
    per GPU, rendezvous on 127.0.0.1) and return the first failing exit code (0 if all succeed).
    Nothing here touches the GPU, and the children are new interpreters (no fork of a process
    with HIP state, no exec).  If a rank fails, the others are stopped by PID, not left waiting in
    a collective."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def init_dist(args):
    """Rank setup.  Returns (world, rank, local_rank, n_devices): one rank per GPU over RCCL; with
    IWQ_DIST_BACKEND=gloo more ranks than GPUs rehearse the multi-rank path on a 1-GPU box (ranks
    share devices round-robin, and n_devices says so).  --dry-run: gloo on the CPU, no device."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"bench.py: world size {ws} != --gpus {args.gpus}")
    if args.dry_run:
        if ws > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        return ws, rank, local, 0
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        raise SystemExit("bench.py: no ROCm GPU visible")
    if ws > 1:
        import torch.distributed as dist
        backend = os.environ.get("IWQ_DIST_BACKEND", "nccl")
        if backend == "nccl" and local >= n_dev:
            raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but only {n_dev} are visible "
                             "(one rank per GPU over RCCL)")
        dev = local % n_dev
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        # distinct devices over all ranks (each rank's device index, gathered)
        t = torch.tensor([dev], dtype=torch.int64, device=coll_device())
        devs = [torch.zeros_like(t) for _ in range(ws)]
        dist.all_gather(devs, t)
        devs = [int(d.item()) for d in devs]
        if backend == "nccl" and len(set(devs)) != ws:
            raise SystemExit(f"bench.py: ranks share GPUs {devs}; one rank per GPU is required over RCCL")
        return ws, rank, local, len(set(devs))
    torch.cuda.set_device(0)
    return ws, rank, local, 1


def coll_device():
    import torch.distributed as dist
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, ws):
    if ws == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_weights(model, rank, world, weak=False):
    """This rank's synthetic weights: its bin-packed shard of the model (strong scaling; seeds = the
    weight's global index, so the union over ranks is the N=1 model) or, weak, a full model per rank
    (seeds offset by rank)."""
    from iron_weight_only_quant_amd import kernels, shard
    shapes = shard.model_linear_shapes(model)
    if not weak:
        owned = shard.plan_shards(shapes, world)[rank]
        seed_base = 0
    else:
        owned = list(range(len(shapes)))
        seed_base = 1_000_000 * rank
    ws, names = [], []
    for i in owned:
        name, (r, c) = shapes[i]
        t = torch.empty((r, c), dtype=torch.float16, device="cuda")
        kernels.fill_synthetic(t, seed=seed_base + i)
        ws.append(t)
        names.append(name)
    return ws, names, shapes


def scatter_weights(model, rank, world):
    """--scatter (strong scaling): the whole model's fp16 weights start on rank 0 (one flat buffer
    per destination rank, synthetic) and are sent to their owners over RCCL point-to-point (all
    sends in flight together: rank 0's xGMI links to every other GPU run in parallel), timed alone
    (max over ranks).  Returns this rank's weights as views into its received buffer."""
    from iron_weight_only_quant_amd import kernels, shard
    shapes = shard.model_linear_shapes(model)
    bins = shard.plan_shards(shapes, world)
    layouts = [shard.bin_layout(shapes, b) for b in bins]
    index = {n: i for i, (n, _) in enumerate(shapes)}
    sends, recv = None, None
    if rank == 0:
        sends = []
        for lay, tot in layouts:
            flat = torch.empty(tot, dtype=torch.float16, device="cuda")
            for name, off, (r, c) in lay:
                kernels.fill_synthetic(flat[off: off + r * c].view(r, c), seed=index[name])
            sends.append(flat)
    else:
        recv = torch.empty(layouts[rank][1], dtype=torch.float16, device="cuda")
    # warm: one small transfer per peer through the same path, so the timed scatter does not pay
    # RCCL's lazy point-to-point connection setup
    small = [torch.zeros(1 << 19, dtype=torch.float16, device="cuda") for _ in range(world)] if rank == 0 else None
    shard.scatter_from_rank0(small, None if rank == 0 else torch.empty(1 << 19, dtype=torch.float16, device="cuda"))
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    mine = shard.scatter_from_rank0(sends, recv)
    torch.cuda.synchronize()
    barrier(world)
    ms = max_over_ranks((time.perf_counter() - t0) * 1e3, world)
    if rank == 0:
        sends = [mine]  # drop the other ranks' copies on rank 0
    views = shard.views_of(mine, layouts[rank][0])
    names = [n for n, _, _ in layouts[rank][0]]
    nbytes = 2 * sum(layouts[r][1] for r in range(1, world))  # fp16 bytes that left rank 0
    return [views[n] for n in names], names, shapes, round(ms, 3), nbytes


def ppl_plumbing(bits, group, symmetric, chunks=8, seqlen=2048):
    """Second half of the metric, as far as it can be measured offline: the SequentialPPLEvaluator
    arithmetic (main.py:42-140) before and after quantize_model on a RANDOM-INIT OPT-125M-shaped
    model with synthetic tokens (no weights / datasets exist here).  Exercises the harness and the
    module swap; the perplexities themselves carry no quality information."""
    try:
        import copy
        from types import SimpleNamespace
        import transformers
        from iron_weight_only_quant_amd.ppl import SequentialPPLEvaluator
        from iron_weight_only_quant_amd.quant_wrapper import quantize_model
        torch.manual_seed(0)
        base = transformers.OPTForCausalLM(transformers.OPTConfig()).half().cuda().eval()
        toks = torch.randint(0, base.config.vocab_size, (1, chunks * seqlen), generator=torch.Generator().manual_seed(1))
        p0, ntok, _ = SequentialPPLEvaluator(base, device="cuda", seqlen=seqlen, tokens=toks).calculate_ppl("wikitext")
        q = copy.deepcopy(base)
        quantize_model(q, SimpleNamespace(w_bit=bits, a_bit=16, w_group_size=group, w_symmetric=symmetric,
                                          w_format="int", quant_dim=0), verbose=False)
        p1, _, _ = SequentialPPLEvaluator(q, device="cuda", seqlen=seqlen, tokens=toks).calculate_ppl("wikitext")
        del base, q
        torch.cuda.empty_cache()
        return {"model": "random-init OPT-125M-shaped (transformers OPTConfig defaults; no weights offline)",
                "tokens": "synthetic", "num_tokens": ntok, "seqlen": seqlen, "ppl_fp16": round(p0, 3),
                "ppl_quant": round(p1, 3), "delta": round(p1 - p0, 3),
                "note": "plumbing check of the PPL half of the metric; not a quality measurement"}
    except Exception as e:  # transformers missing etc.: report, do not fail the bench
        return {"error": f"{type(e).__name__}: {e}"}


def host_cpus():
    """(usable CPUs, description): the smallest of os.cpu_count(), this process's affinity mask and
    the cgroup CPU quota (on the GPU box os.cpu_count() is the whole machine while the job's share is
    a quota), plus the CPU model from /proc/cpuinfo."""
    n_os = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = n_os
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(n for n in (n_os, n_aff, quota) if n)
    return usable, {"os_cpu_count": n_os, "affinity": n_aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def cpu_baseline(weights, bits, group, symmetric, budget_s, model_name):
    """Reference CPU arithmetic on whole tensors of the same workload until the budget is spent, on
    every host CPU this job may use (torch intra-op threads = usable CPUs, recorded)."""
    from oracle.torch_ref import minmax_fake_quant_cpu
    usable, info = host_cpus()
    prev = torch.get_num_threads()
    torch.set_num_threads(usable)
    threads = torch.get_num_threads()
    done_bytes, spent, n = 0, 0.0, 0
    try:
        for w in weights:
            x = w.cpu()
            t0 = time.perf_counter()
            minmax_fake_quant_cpu(x, bits, not symmetric, group)
            spent += time.perf_counter() - t0
            done_bytes += x.numel() * 2
            n += 1
            if spent >= budget_s:
                break
    finally:
        torch.set_num_threads(prev)
    return {"value": round(done_bytes / spent / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "host": info,
            "sample": f"{n} of this rank's {model_name} weight tensors ({done_bytes / 1e9:.2f} GB fp16) through "
                      f"oracle/torch_ref.py (reference quant_funcs.py:16-38 op sequence, torch CPU, "
                      f"{threads} threads on {info['cpu_model']}), {spent:.1f} s"}


def time_gather(plan, names, all_shapes, args, ws_n):
    """Rooted gather of the packed results (codes + scales/zeros) to rank 0 over RCCL, timed alone.
    Returns (ms, bytes received by rank 0)."""
    from iron_weight_only_quant_amd import shard
    import torch.distributed as dist
    res = shard.ShardResult(list(names), list(plan.codes), list(plan.scales), list(plan.zeros))
    bins = shard.plan_shards(all_shapes, ws_n)
    names_per_rank = [[all_shapes[i][0] for i in b] for b in bins]
    shp = dict(all_shapes)
    shard.gather_to_rank0(res, shp, names_per_rank, args.bits, args.group, args.symmetric)  # warm
    torch.cuda.synchronize()
    dist.barrier()
    stats = {}
    t0 = time.perf_counter()
    shard.gather_to_rank0(res, shp, names_per_rank, args.bits, args.group, args.symmetric, stats=stats)
    torch.cuda.synchronize()
    dist.barrier()
    ms = max_over_ranks((time.perf_counter() - t0) * 1e3, ws_n)
    return round(ms, 3), stats.get("recv_bytes", 0)


def gather_section(plan, names, all_shapes, args, ws_n):
    """N > 1, default: the packed results of this rank's bin (codes + scales/zeros, what a rank would
    hand back) produced by one codes-writing launch over the same weights (outside the headline's
    timed region), then the rooted gather to rank 0 timed alone (shard.gather_to_rank0: one
    point-to-point send per rank, every receive posted together on rank 0)."""
    from iron_weight_only_quant_amd import kernels
    gplan = kernels.BatchPlan(plan.weights, args.bits, args.group, args.symmetric, outs=plan.outs, want_codes=True)
    gplan.run()
    torch.cuda.synchronize()
    ms, nbytes = time_gather(gplan, names, all_shapes, args, ws_n)
    del gplan
    torch.cuda.empty_cache()
    return {"gather_ms": ms, "gather_bytes_to_rank0": nbytes,
            "gather_GBps": round(nbytes / ms / 1e6, 1) if ms else None}


def scatter_section(model, rank, ws_n):
    """N > 1, default (bounded): the whole model's fp16 weights from rank 0 to their owners
    (shard.scatter_from_rank0 over RCCL, one send per destination, all in flight), timed alone after
    a small warm-up transfer; the received buffers are dropped again."""
    _, _, _, ms, nbytes = scatter_weights(model, rank, ws_n)
    torch.cuda.empty_cache()
    return {"scatter_ms": ms, "scatter_bytes_from_rank0": nbytes,
            "scatter_GBps": round(nbytes / ms / 1e6, 1) if ms else None,
            "scatter_model": MODEL_NAME[model]}


def dry_run(args, ws_n, rank):
    """--dry-run: the multi-rank plumbing without a GPU (CPU tests): every rank builds zero-filled
    packed results of its bin's sizes, the rooted gather moves them to rank 0, and rank 0 prints the
    bench record (per-rank roofline from stand-in kernel times, the CPU baseline) with the bytes that
    crossed (each non-root bin exactly once) next to the plan's totals."""
    from iron_weight_only_quant_amd import shard
    shapes = shard.model_linear_shapes(args.model)
    bins = shard.plan_shards(shapes, ws_n)
    mine = bins[rank]
    nb = lambda shp: shard.packed_nbytes(shp, args.bits, args.group, args.symmetric)  # noqa: E731
    names, codes, scales, zeros = [], [], [], []
    for i in mine:
        name, (r, c) = shapes[i]
        G = shard.n_groups(r, c, args.group)
        names.append(name)
        codes.append(torch.zeros(r * (c // 2) if args.bits <= 4 else r * c, dtype=torch.uint8))
        scales.append(torch.zeros(G, dtype=torch.float16))
        zeros.append(None if args.symmetric else torch.zeros(G, dtype=torch.float16))
    res = shard.ShardResult(names, codes, scales, zeros)
    sent, recv, got = 0, 0, 0
    coll = {}
    if ws_n > 1 and not args.no_collectives:
        import torch.distributed as dist
        stats = {}
        dist.barrier()
        t0 = time.perf_counter()
        out = shard.gather_to_rank0(res, dict(shapes), [[shapes[i][0] for i in b] for b in bins], args.bits,
                                    args.group, args.symmetric, stats=stats)
        dist.barrier()
        gather_ms = max_over_ranks((time.perf_counter() - t0) * 1e3, ws_n)
        t = torch.tensor([stats["sent_bytes"], stats["recv_bytes"]], dtype=torch.int64)
        dist.all_reduce(t)
        sent, recv = int(t[0]), int(t[1])
        got = len(out) if out is not None else 0
        # the scatter of the model's fp16 bins from rank 0 (CPU buffers over gloo; bin r filled with
        # the value r + 1 so every receiver checks it got its own bin)
        layouts = [shard.bin_layout(shapes, b) for b in bins]
        sends = [torch.full((tot,), float(r + 1), dtype=torch.float16) for r, (_, tot) in enumerate(layouts)] \
            if rank == 0 else None
        rbuf = None if rank == 0 else torch.empty(layouts[rank][1], dtype=torch.float16)
        dist.barrier()
        t0 = time.perf_counter()
        got_bin = shard.scatter_from_rank0(sends, rbuf)
        dist.barrier()
        scatter_ms = max_over_ranks((time.perf_counter() - t0) * 1e3, ws_n)
        ok = torch.tensor([int(got_bin.numel() == layouts[rank][1] and bool((got_bin == rank + 1).all()))])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        sbytes = 2 * sum(tot for _, tot in layouts[1:])
        coll = {"gather_ms": round(gather_ms, 3), "gather_bytes_to_rank0": recv,
                "gather_GBps": round(recv / gather_ms / 1e6, 3),
                "scatter_ms": round(scatter_ms, 3), "scatter_bytes_from_rank0": sbytes,
                "scatter_GBps": round(sbytes / scatter_ms / 1e6, 3), "scatter_model": MODEL_NAME[args.model],
                "scatter_verified": bool(ok.item())}
    # the record's multi-rank plumbing with stand-in timings (no GPU): per-rank statistics gathered
    # over gloo, the roofline over ranks, the CPU baseline on rank 0 (a small CPU sample)
    kernel_ms = 1.0 + 0.25 * rank  # stand-in: rank r "took" 1 + r/4 ms
    numel = sum(shapes[i][1][0] * shapes[i][1][1] for i in mine)
    alg = numel * 4 + (numel // args.group) * 2 * (1 if args.symmetric else 2)
    ceil = 5000.0 - 100.0 * rank  # stand-in: each rank's own in-run copy ceiling
    per_rank = gather_per_rank([kernel_ms, alg, ceil], ws_n)
    roof = roofline_record(per_rank, "k_group<f16,128,asym,batched,RW256>", None, "dry run: no PMC",
                           {"GBps": ceil, "forms": {"stand-in": ceil}})
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.synth import synth
        sample = [torch.from_numpy(synth(900 + i, (256, 1024), "float16")) for i in range(4)]
        cpu = cpu_baseline(sample, args.bits, args.group, args.symmetric, 0.2, MODEL_NAME[args.model] + " (stand-in)")
    total = all_ranks_sum(numel, ws_n)
    if rank == 0:
        rec = build_record(args, ws_n, 0, args.weak, shapes, total, None, roof, {
            "dry_run": True, "world": ws_n, "model": args.model, "tensors": len(shapes),
            "tensors_at_rank0": got,
            "plan_packed_bytes_per_rank": [sum(nb(shapes[i][1]) for i in b) for b in bins],
            "gather_sent_bytes": sent, "gather_recv_bytes": recv, "cpu_baseline": cpu, **coll})
        rec["note"] = ("dry run over gloo on the CPU: stand-in kernel timings, no GPU; gather / scatter times are "
                       "gloo over loopback")
        print(json.dumps(rec), flush=True)


def kernel_sources_sha():
    """Hash of the sources that define the headline kernel (k_group): profiles/traffic.json is only
    trusted while it carries the same hash."""
    import hashlib
    h = hashlib.sha256()
    for rel in ("iron_weight_only_quant_amd/csrc/iwq_minmax.hip", "iron_weight_only_quant_amd/csrc/iwq_minmax.cuh",
                "iron_weight_only_quant_amd/csrc/iwq_common.cuh", "include/iwq.h"):
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def committed_traffic(path, numel, bits, group, placement="out-of-place"):
    """HBM bytes per launch from the committed PMC record, if it was measured on this workload (and
    placement) AND on the current kernel sources; (bytes or None, reason)."""
    rel = os.path.relpath(path, ROOT)
    if not os.path.exists(path):
        return None, f"no PMC record ({rel})"
    try:
        tf = json.load(open(path))
    except (OSError, ValueError):
        return None, f"unreadable PMC record ({rel})"
    if (tf.get("workload_numel") != numel or tf.get("bits") != bits or tf.get("group") != group
            or tf.get("placement", "out-of-place") != placement):
        return None, f"PMC record {rel} is for another workload"
    if tf.get("kernel_sources_sha") != kernel_sources_sha():
        return None, f"PMC record {rel} predates the current kernel sources"
    return tf.get("hbm_bytes_per_launch"), f"{rel} (rocprofv3 FETCH_SIZE/WRITE_SIZE, same sources)"


def clock_ramp(plan, seconds):
    """Untimed back-to-back launches until `seconds` of wall time have passed: a few warmup steps
    (23 ms at W=5) leave the GPU below its sustained clock and cost up to ~15 % on a fresh box."""
    stream = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(10):
            plan.run(stream)
        torch.cuda.synchronize()


CEILING_PROBES = {100: "copy, nt 16-B load + nt store, grid-stride",
                  101: "copy, plain 16-B load + store, grid-stride",
                  102: "copy, 4 x 16 B in flight per lane (nt), grid-stride",
                  118: "k_group's own (region) walk and load/store stream, no arithmetic (same grid, same units)"}


def copy_ceiling(plan, steps=5, rounds=3):
    """In-run ceiling for a read+write stream of the same bytes: the best of several copy forms
    (read w, write out; in place: w onto itself, values unchanged), interleaved over `rounds`.
    The kernel's achieved rate is compared with the BEST of them.  Overwrites plan.outs; call before
    the timed warmup."""
    stream = torch.cuda.current_stream()
    nbytes = plan.numel * 4
    best = {}
    for v in CEILING_PROBES:
        plan.run(stream, variant=v)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for v in CEILING_PROBES:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(steps):
                plan.run(stream, variant=v)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / steps
            best[v] = min(best.get(v, ms), ms)
    forms = {CEILING_PROBES[v]: round(nbytes / (ms / 1e3) / 1e9, 1) for v, ms in best.items()}
    return {"GBps": max(forms.values()), "forms": forms}


def fresh_ceiling(plan, steps=5, rounds=2):
    """The box's copy rate on buffers that are NOT the plan's (box speed and the plan's
    placement reported apart): a fresh input and output allocated for every weight of the plan (the
    same shapes, the same number of allocations -- a single large buffer is its own placement draw,
    profiles/r06_ab_placement_2x2.jsonl), timed with the guide's grid-stride 16-B copy (probe 100)
    and the headline kernel's walk without arithmetic (118).  The contents are never read as
    numbers, so the buffers are left unfilled."""
    from iron_weight_only_quant_amd import kernels
    stream = torch.cuda.current_stream()
    need = plan.numel * plan.weights[0].element_size() * 2
    if torch.cuda.mem_get_info()[0] < need * 1.15:  # (the 70B run in place: no room for a second model)
        return None
    ins = [torch.empty_like(w) for w in plan.weights]
    fp = kernels.BatchPlan(ins, plan.n_bits, plan.group, plan.symmetric)
    nbytes = plan.numel * 4
    best = {}
    for v in (100, 118):
        fp.run(stream, variant=v)
        torch.cuda.synchronize()
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(steps):
                fp.run(stream, variant=v)
            e1.record(stream)
            torch.cuda.synchronize()
            best[v] = max(best.get(v, 0.0), nbytes / (e0.elapsed_time(e1) / steps / 1e3) / 1e9)
    del fp, ins
    torch.cuda.empty_cache()
    forms = {CEILING_PROBES[v]: round(g, 1) for v, g in best.items()}
    return {"GBps": max(forms.values()), "forms": forms,
            "basis": "fresh input + output per weight of the plan (same shapes, not the plan's buffers)"}


def launch_floor_us(reps=32):
    """Per-call device time of the smallest kernel of this library (iwq_fill_synthetic on 16
    elements: one wave, no memory traffic to speak of) in the same hipGraph replay form as the cold
    single calls: the per-kernel floor of a dependent launch on this box (dispatch, end-of-kernel
    release, next dispatch; profiles/r05_launch_floor.jsonl: 1.6 us).  Reported beside every
    per-call figure so the kernel's own share can be read off (never subtracted from `value`)."""
    from iron_weight_only_quant_amd import kernels as K
    t = torch.empty(16, dtype=torch.float16, device="cuda")
    return _graph_ms([(lambda: K.fill_synthetic(t, 1))] * reps, region="launch_floor") * 1e3


def per_shape(plan, names, ws_n, args, reps=32, rounds=5):
    """Single-tensor drop-in calls (kernels.quantize_minmax == pseudo_quantize_tensor's device path)
    per Llama weight shape, COLD: `reps` consecutive calls on distinct resident instances of the
    shape (>= 1 GB per replay, so the 256 MB MALL holds none of it), captured in one hipGraph and
    replayed; device time per call = event time / reps (includes the inter-kernel boundary).
    value per shape = all ranks' fp16 input bytes / max-over-ranks time."""
    from iron_weight_only_quant_amd import kernels as K
    floor = launch_floor_us()
    by_shape = {}
    for i, w in enumerate(plan.weights):
        by_shape.setdefault(tuple(w.shape), []).append(i)
    out = {}
    for shp in sorted(by_shape):
        idx = by_shape[shp][:reps]
        fns = [(lambda i=i: K.quantize_minmax(plan.weights[i], args.bits, args.group, args.symmetric, 0,
                                              out=plan.outs[i])) for i in idx]
        for f in fns:
            f()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for f in fns:
                f()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for f in fns:
                f()
        g.replay()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ts = []
        with MARKS.region(f"shapes/{shp[0]}x{shp[1]}", calls_per_replay=len(idx), replays=rounds) as mk:
            for _ in range(rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                g.replay()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / len(idx) * 1e-3)
        ts.sort()
        mk["bench_us_per_call"] = round(ts[len(ts) // 2] * 1e6, 3)
        t = max_over_ranks(ts[len(ts) // 2], ws_n)
        n = shp[0] * shp[1]
        alg = n * 4 + (n // args.group) * 2 * (1 if args.symmetric else 2)
        kt = t - floor * 1e-6
        out[f"{shp[0]}x{shp[1]}"] = {
            "us_per_call": round(t * 1e6, 2), "weights_GBps": round(ws_n * n * 2 / t / 1e9, 1),
            "achieved_GBps_per_gpu": round(alg / t / 1e9, 1), "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
            "calls": len(idx), "cold": True, "launch_floor_us": round(floor, 3),
            "frac_beyond_launch_floor": round(alg / kt / 1e9 / HBM_PEAK_GBS, 4) if kt > 0 else None}
        del g
    return out


def other_placement_kernel(weights, plan, args, steps=10):
    """The same launch in the other placement, HIP-event time on its stream, reported beside the
    headline: in place (QuantLinear.quantize_weight writes the dequantized weight back into the weight
    storage, quant_linear.py:949) when the headline is out of place, and vice versa.  Its inputs are
    copies, so the headline plan's inputs are untouched.  Which placement is faster depends on the box
    (DESIGN.md §5): the headline stays pseudo_quantize_tensor's default, out of place."""
    from iron_weight_only_quant_amd import kernels
    if args.inplace:
        other = kernels.BatchPlan(weights, args.bits, args.group, args.symmetric)
    else:
        copies = [w.clone() for w in weights]
        other = kernels.BatchPlan(copies, args.bits, args.group, args.symmetric, outs=copies)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        other.run(stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        other.run(stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    numel = other.numel
    alg = numel * 4 + (numel // args.group) * 2 * (1 if args.symmetric else 2)
    del other
    torch.cuda.empty_cache()
    return {"placement": "out-of-place" if args.inplace else "in-place", "kernel_ms": round(ms, 4),
            "achieved_GBps": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4)}


def ab_variants(plan, variants, args):
    """Interleaved in-process A/B of kernel variants (cdna_hip_programming.md §5.4 rule 24)."""
    stream = torch.cuda.current_stream()
    plan.run(stream, variant=0)
    torch.cuda.synchronize()
    ref = [o.clone() for o in plan.outs[:3]]
    times = {v: [] for v in variants}
    for v in variants:  # warm + correctness vs variant 0 (probes >= 100 are not quantizers; in place
        plan.run(stream, variant=v)  # the inputs change every run, so only out of place compares)
        torch.cuda.synchronize()
        if v < 100 and not args.inplace:
            for o, r in zip(plan.outs[:3], ref):
                assert torch.equal(o.view(torch.int16), r.view(torch.int16)), f"variant {v} differs"
    for _ in range(args.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.steps):
                plan.run(stream, variant=v)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.steps)
    numel = plan.numel
    for v in variants:
        t = sorted(times[v])
        med = t[len(t) // 2]
        nbytes = numel * (2 if v in (103, 104) or 106 <= v <= 111 else 4)
        print(f"[ab] variant {v}: median {med:.4f} ms  min {t[0]:.4f} ms  -> {nbytes / med / 1e6:.1f} GB/s moved",
              file=sys.stderr, flush=True)


def timed_steps(plan, args, ws_n, stream, region="headline"):
    """W untimed warmup steps, then EXACTLY K steps bracketed by barrier + synchronize on both sides.
    Returns (kernel ms per launch from HIP events on the launch stream, max-over-ranks wall ms per step)."""
    return _timed_steps(plan, args, ws_n, stream, region)


def _timed_steps(plan, args, ws_n, stream, region):
    for _ in range(args.warmup):
        plan.run(stream, variant=args.variant)
    torch.cuda.synchronize()
    assert plan.nan_flag.item() == 0
    barrier(ws_n)
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    with MARKS.region(region, launches=args.steps) as mk:  # exactly the K timed launches
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(args.steps):
            plan.run(stream, variant=args.variant)
        ev1.record(stream)
        torch.cuda.synchronize()
        barrier(ws_n)
        wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    mk["bench_kernel_ms"] = round(kernel_ms, 5)
    return kernel_ms, max_over_ranks(wall, ws_n) / args.steps * 1e3


def all_ranks_sum(x, ws_n):
    if ws_n == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.int64, device=coll_device())
    dist.all_reduce(t)
    return int(t.item())


def weak_secondary(args, ws_n, rank):
    """7B at N > 1: every rank quantizes a full 7B (weak scaling), timed like the headline.  With
    shapes: the cold single-tensor calls per Llama shape on the same full copy, every rank running its
    own calls at once (per_shape: max over ranks, aggregate = N x one GPU's calls) -- the north star's
    per-shape GB/s at N GPUs.  Every rank holds every shape, so the per-shape collectives line up."""
    from iron_weight_only_quant_amd import kernels
    weights, names, _ = make_weights(args.model, rank, ws_n, weak=True)
    plan = kernels.BatchPlan(weights, args.bits, args.group, args.symmetric)
    stream = torch.cuda.current_stream()
    clock_ramp(plan, 0.2)
    kernel_ms, ms = timed_steps(plan, args, ws_n, stream, region="weak")
    total = all_ranks_sum(plan.numel, ws_n)
    shapes = None if args.no_shapes else per_shape(plan, names, ws_n, args)
    del plan, weights
    torch.cuda.empty_cache()
    return {"scaling": "weak", "value": round(total * 2 / (ms / 1e3) / 1e9, 2), "ms_per_step": round(ms, 4),
            "kernel_ms_rank0": round(kernel_ms, 4), "fp16_weights_total": total,
            "workload": f"every rank quantizes all {len(make_shapes(args.model))} Linear weights of "
                        f"{MODEL_NAME[args.model]}"}, shapes


def shard_bin_elems(model, world):
    """Elements of each rank's flat bin buffer (shard.bin_layout) for the model over `world` ranks."""
    from iron_weight_only_quant_amd import shard
    shapes = shard.model_linear_shapes(model)
    return [shard.bin_layout(shapes, b)[1] for b in shard.plan_shards(shapes, world)]


def make_shapes(model):
    from iron_weight_only_quant_amd import shard
    return shard.model_linear_shapes(model)


# ---------------------------------------------------------------------------------------------
# Per-rank statistics and the JSON record (shared by the GPU run and the --dry-run rehearsal)
# ---------------------------------------------------------------------------------------------
def gather_per_rank(vals, ws_n):
    """[[v0, v1, ...] of rank 0, of rank 1, ...]: every rank's float statistics, on every rank."""
    if ws_n == 1:
        return [list(vals)]
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device=coll_device())
    out = [torch.zeros_like(t) for _ in range(ws_n)]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu()] for o in out]


def roofline_record(per_rank, kernel_name, traffic, traffic_src, ceiling=None, other=None):
    """HBM roofline of the headline kernel over all ranks.  per_rank = [kernel_ms, alg_bytes(,
    ceiling_GBps)] per rank (HIP-event time of its launch on its stream; its algorithmic bytes per
    launch; the in-run copy ceiling of its own GPU).  `achieved` is per GPU: the mean algorithmic
    bytes per rank over the SLOWEST rank's kernel time (what the max-over-ranks step time sees);
    `per_rank` gives each rank's own rate, fraction and kernel / ceiling ratio.  At N > 1 the top-level
    `kernel_over_ceiling` is the lowest rank's ratio."""
    kmax = max(p[0] for p in per_rank)
    mean_bytes = sum(p[1] for p in per_rank) / len(per_rank)
    achieved = mean_bytes / (kmax / 1e3) / 1e9 if kmax > 0 else None
    rows = []
    for r, p in enumerate(per_rank):
        k, b = p[0], p[1]
        row = {"rank": r, "kernel_ms": round(k, 4), "alg_bytes": int(b),
               "frac": (round(b / (k / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if k > 0 else None)}
        if len(p) > 2 and p[2] > 0 and k > 0:
            row["ceiling_GBps"] = round(p[2], 1)
            row["kernel_over_ceiling"] = round(b / (k / 1e3) / 1e9 / p[2], 4)
        rows.append(row)
    rec = {"bound": "hbm", "achieved": None if achieved is None else round(achieved, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
           "traffic": traffic, "traffic_source": traffic_src, "kernel": kernel_name,
           "kernel_ms": round(kmax, 4), "kernel_ms_basis": "max over ranks" if len(per_rank) > 1 else "rank 0",
           "alg_bytes_per_launch": int(round(mean_bytes)) if len(per_rank) > 1 else int(per_rank[0][1]),
           "per_rank": rows}
    if ceiling is not None:
        if len(per_rank) == 1:
            rec["ceiling"] = ceiling
            rec["kernel_over_ceiling"] = round(achieved / ceiling["GBps"], 4) if achieved else None
        else:
            ratios = [row["kernel_over_ceiling"] for row in rows if "kernel_over_ceiling" in row]
            rec["ceiling"] = {"GBps": round(min(row.get("ceiling_GBps", 0) for row in rows), 1),
                              "basis": "lowest rank's in-run ceiling (each rank's in per_rank)",
                              "forms_rank0": ceiling.get("forms")}
            rec["kernel_over_ceiling"] = min(ratios) if ratios else None
    if other is not None:
        rec["other_placement"] = other
    return rec


# ---------------------------------------------------------------------------------------------
# Extra sections of the default run: BASELINE configs[2] (fused forward), configs[4] (FP formats),
# configs[3] (Llama-2-70B) -- bounded, after the headline's timed region
# ---------------------------------------------------------------------------------------------
MFMA_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA (MI355X_MICROARCH.md chip table; never the sparse figure)
FF_SHAPES = (("q_proj", 4096, 4096), ("gate_proj", 11008, 4096), ("down_proj", 4096, 11008))
# fused_proj.fuse_projections' row concatenations of one layer's siblings: q/k/v and gate/up
DECODE_FUSED_SHAPES = (("qkv_fused", 3 * 4096, 4096), ("gate_up_fused", 2 * 11008, 4096))


def _interleaved_ms(arms, reps=5, rounds=7, region=None):
    """Median ms per call of each arm: every round times each arm once (reps calls back to back, HIP
    events on the current stream -- the stream every arm launches on), arms in rotating order
    (cdna_hip_programming.md §5.4 rule 24).  With --mark-file each arm's timed calls are a region of
    their own (`region`/<arm>), so the kernel trace can be cut per arm."""
    st = torch.cuda.current_stream()
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    keys = list(arms)
    times = {k: [] for k in keys}
    for rd in range(rounds):
        for k in keys[rd % len(keys):] + keys[:rd % len(keys)]:
            with MARKS.region(f"{region}/{k}", calls=reps, round=rd) as mk:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    arms[k]()
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / reps)
            mk["bench_ms_per_call_this_round"] = round(times[k][-1], 5)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def _graph_ms(calls, rounds=5, region=None):
    """Median device ms per call of `calls` captured in ONE hipGraph and replayed (no host launch cost
    in the time; the calls rotate over distinct resident buffers, so they run cold)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for c in calls:
            c()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    out = []
    with MARKS.region(region or "graph", calls_per_replay=len(calls), replays=rounds) as mk:
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / len(calls))
    del g
    mk["bench_ms_per_call"] = round(sorted(out)[len(out) // 2], 6)
    return sorted(out)[len(out) // 2]


def fused_forward_section(rot_bytes=1 << 30):
    """BASELINE configs[2]: Llama-2-7B INT4 per channel (and g=128) QuantLinear forward on the packed
    codes (kernels.w4a16_gemm: MFMA dequant->GEMM) against the reference forward F.linear(x, W_deq)
    (hipBLASLt on the resident fp16 weight, quant_linear.py:960-972) timed in the same run.
    M = 8192 (the PPL batch 4 x 2048, main.py:117-128): interleaved, MFMA-bound -> TF/s and fraction
    of the dense fp16 MFMA peak.  M = 1 (decode): cold (each call reads a different resident copy,
    >= 1 GiB per replay, hipGraph) -> packed-weight GB/s and fraction of 8 TB/s.  `auto` = which path
    QuantLinear(fused_forward="auto") takes at that M (kernels.auto_fused_preferred)."""
    from iron_weight_only_quant_amd import kernels as K
    F = torch.nn.functional
    out = []
    gen = torch.Generator(device="cuda").manual_seed(1234)
    floor = launch_floor_us()

    def decode_row(name, N, Kd, r, group, gname, M=1):
        """M = 1, cold (each call reads a different resident copy, >= rot_bytes per replay, hipGraph),
        codes in the decode tile layout (what QuantLinear "auto" keeps) vs F.linear on rotated fp16."""
        x = (torch.randn(M, Kd, device="cuda", generator=gen) * 0.5).half()
        y = torch.empty(M, N, dtype=torch.float16, device="cuda")
        tiled = K.tile_codes(r.codes, N, Kd)
        cb = r.codes.numel()
        copies = [tiled] + [tiled.clone() for _ in range(int(rot_bytes // cb))]
        wbytes = cb + r.scales.numel() * 2 + (r.zeros.numel() * 2 if r.zeros is not None else 0)
        t_f = _graph_ms([(lambda c=c: K.w4a16_gemm(x, c, r.scales, r.zeros, 4, group, N, tiled=True, out=y))
                         for c in copies], region=f"fused_forward/{name}/{gname}/M1/fused")
        refs = [r.out] + [r.out.clone() for _ in range(int(rot_bytes // (N * Kd * 2)))]
        t_r = _graph_ms([(lambda wt=wt: F.linear(x, wt)) for wt in refs],
                        region=f"fused_forward/{name}/{gname}/M1/F.linear")
        gbs = wbytes / (t_f / 1e3) / 1e9
        kt = t_f - floor / 1e3
        row = {"shape": name, "N": N, "K": Kd, "weights": gname, "M": M, "bound": "hbm",
               "fused_ms": round(t_f, 5), "F_linear_ms": round(t_r, 5),
               "packed_weight_GBps": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
               "launch_floor_us": round(floor, 3),
               "frac_beyond_launch_floor": round(wbytes / (kt / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if kt > 0 else None,
               "fused_vs_F_linear": round(t_r / t_f, 3), "cold_copies": len(copies),
               "auto": "fused" if K.auto_fused_preferred(M, N, Kd, group) else "F.linear"}
        del x, y, tiled, copies, refs
        torch.cuda.empty_cache()
        return row
    for name, N, Kd in FF_SHAPES:
        w = torch.empty(N, Kd, dtype=torch.float16, device="cuda")
        K.fill_synthetic(w, 7)
        for group in (-2, 128):
            r = K.quantize_minmax(w, 4, group, False, 0, want_codes=True)
            gname = "per-channel" if group == -2 else f"g{group}"
            M = 8192
            x = (torch.randn(M, Kd, device="cuda", generator=gen) * 0.5).half()
            y = torch.empty(M, N, dtype=torch.float16, device="cuda")
            nib = K.nib_codes(r.codes, N, Kd)
            # QuantLinear(fused_forward=True)'s call: grouped weights also pass the group-major copies
            # of their parameters (IWQ_FLAG_GROUP_MAJOR); "fused_ref_order" = the same kernel reading
            # the reference's [N, K/g] parameter order
            sgm, zgm = K.group_major_params(r.scales, r.zeros, N, Kd, group) if group != -2 else (None, None)
            arms = {"fused": lambda: K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, out=y,
                                                  scales_gm=sgm, zeros_gm=zgm),
                    "fused_nib": lambda: K.w4a16_gemm(x, nib, r.scales, r.zeros, 4, group, N, out=y, nib=True,
                                                      scales_gm=sgm, zeros_gm=zgm),
                    "F.linear": lambda: F.linear(x, r.out)}
            if group != -2:
                arms["fused_ref_order"] = lambda: K.w4a16_gemm(x, r.codes, r.scales, r.zeros, 4, group, N, out=y)
            t = _interleaved_ms(arms, region=f"fused_forward/{name}/{gname}/M{M}")
            tf = 2.0 * M * N * Kd / (t["fused"] / 1e3) / 1e12
            tfn = 2.0 * M * N * Kd / (t["fused_nib"] / 1e3) / 1e12
            out.append({"shape": name, "N": N, "K": Kd, "weights": gname, "M": M, "bound": "mfma",
                        "fused_ms": round(t["fused"], 4), "F_linear_ms": round(t["F.linear"], 4),
                        "fused_TFLOPs": round(tf, 1), "frac_of_mfma_peak": round(tf / MFMA_PEAK_TFLOPS, 4),
                        "F_linear_TFLOPs": round(2.0 * M * N * Kd / (t["F.linear"] / 1e3) / 1e12, 1),
                        "fused_vs_F_linear": round(t["F.linear"] / t["fused"], 3),
                        "fused_nib_ms": round(t["fused_nib"], 4), "fused_nib_TFLOPs": round(tfn, 1),
                        "fused_nib_vs_F_linear": round(t["F.linear"] / t["fused_nib"], 3),
                        "auto": "fused" if K.auto_fused_preferred(M, N, Kd, group) else "F.linear"})
            if group != -2:
                out[-1].update(fused_ref_order_ms=round(t["fused_ref_order"], 4),
                               fused_ref_order_vs_F_linear=round(t["F.linear"] / t["fused_ref_order"], 3))
            del x, y, nib, sgm, zgm
            out.append(decode_row(name, N, Kd, r, group, gname))
            del r
        del w
        torch.cuda.empty_cache()
    # the decode GEMV as QuantLinear "auto" runs it after fused_proj.fuse_projections: ONE launch over
    # the row-concatenated q/k/v (and gate/up) codes of a layer, which amortises the per-launch floor
    for name, N, Kd in DECODE_FUSED_SHAPES:
        w = torch.empty(N, Kd, dtype=torch.float16, device="cuda")
        K.fill_synthetic(w, 7)
        r = K.quantize_minmax(w, 4, -2, False, 0, want_codes=True)
        out.append(decode_row(name, N, Kd, r, -2, "per-channel"))
        del r, w
        torch.cuda.empty_cache()
    return {"config": "BASELINE configs[2]: Llama-2-7B INT4 fused dequant+GEMM QuantLinear forward (packed codes) "
                      "vs F.linear on the dequantized fp16 weight, same run",
            "kernels": "M=8192: row-major codes k_w4a16_b16w (per channel 151, grouped 150), NIB codes "
                       "(QuantLinear nib_prefill) k_w4a16_b16p (persistent, 172) / b16w 152 (iwq_prefill16.hip); "
                       "grouped: group-major parameter copies (IWQ_FLAG_GROUP_MAJOR, what QuantLinear keeps), "
                       "fused_ref_order = the reference's parameter order; M=1: k_w4a16_gemv(_ct) on tile-layout codes "
                       "(qkv_fused / gate_up_fused: the fused_proj concatenations, one launch per layer input)",
            "mfma_peak_TFLOPs": MFMA_PEAK_TFLOPS, "launch_floor_us": round(floor, 3), "rows": out}


def formats_section(rows=11008, cols=4096, copies=16):
    """BASELINE configs[4]: FP8 E4M3 and FP4 (E2M1 codec, and the fp4_quantize_cpu.py E2M1 grid)
    weight formats as pack (fake-quant + codes) / unpack (codes -> fp16) kernels on a Llama-2-7B
    gate_proj weight, cold (the calls rotate over `copies` distinct resident weights, hipGraph)."""
    from iron_weight_only_quant_amd import kernels as K
    n, g = rows * cols, 128
    G = n // g
    ws = []
    for c in range(copies):
        t = torch.empty(rows, cols, dtype=torch.float16, device="cuda")
        K.fill_synthetic(t, 100 + c)
        ws.append(t)
    outs = [torch.empty_like(t) for t in ws]
    paths = []
    for fname, e, m, sym in (("fp8_e4m3_g128_sym", 4, 3, True), ("fp8_e4m3_g128_asym", 4, 3, False),
                             ("fp4_e2m1_g128_asym", 2, 1, False)):
        cb = n if 1 + e + m > 4 else n // 2
        par = 2 * G * (1 if sym else 2)
        packs = [K.quantize_fp(w, e, m, g, sym, 0, out=o, want_codes=True) for w, o in zip(ws, outs)]
        paths.append((fname + "_pack", [(lambda w=w, o=o, e=e, m=m, sym=sym:
                                         K.quantize_fp(w, e, m, g, sym, 0, out=o, want_codes=True))
                                        for w, o in zip(ws, outs)], 4 * n + cb + par))
        paths.append((fname + "_unpack", [(lambda p=p, o=o, e=e, m=m:
                                           K.dequant_fp_packed(p.codes, p.scales, p.zeros, e, m, g, rows, cols, out=o))
                                          for p, o in zip(packs, outs)], 2 * n + cb + par))
    grids = [K.fp4_grid(w, g, want_codes=True) for w in ws]
    paths.append(("e2m1_grid_g128_pack", [(lambda w=w: K.fp4_grid(w, g, want_codes=True)) for w in ws],
                  4 * n + n // 2 + 2 * G))
    paths.append(("e2m1_grid_g128_unpack", [(lambda p=p, o=o: K.dequant_fp_packed(p.codes, p.scales, None, 2, 1, g,
                                                                                  rows, cols, out=o))
                                            for p, o in zip(grids, outs)], 2 * n + n // 2 + 2 * G))
    res = []
    for name, calls, alg in paths:
        t = _graph_ms(calls, region=f"formats/{name}") / 1e3
        res.append({"path": name, "us": round(t * 1e6, 2), "alg_bytes": int(alg),
                    "achieved_GBps": round(alg / t / 1e9, 1), "frac_of_hbm_peak": round(alg / t / 1e9 / HBM_PEAK_GBS, 4)})
    del ws, outs, grids
    torch.cuda.empty_cache()
    return {"config": f"BASELINE configs[4]: FP8 / FP4 weight formats, pack (fake-quant + codes) and unpack "
                      f"(codes -> fp16) on [{rows}, {cols}] fp16, cold over {copies} resident copies",
            "kernels": "pack: k_fp_group_lut / fp4 grid (iwq_fp.hip); unpack: iwq_fpunpack.hip", "rows": res}


def model70b_section(args, ws_n, rank, steps=5, warmup=2):
    """BASELINE configs[3]: Llama-2-70B INT4 g=128, all 560 Linear weights (137 GB fp16) bin-packed
    over the ranks, quantized IN PLACE (QuantLinear semantics; one GPU holds the whole model) with one
    batched launch per rank per step.  value = 70B fp16 bytes / max-over-ranks step time."""
    from iron_weight_only_quant_amd import kernels
    weights, _, shapes = make_weights("llama2-70b", rank, ws_n)
    plan = kernels.BatchPlan(weights, args.bits, args.group, args.symmetric, outs=weights)
    stream = torch.cuda.current_stream()
    a = argparse.Namespace(warmup=warmup, steps=steps, variant=0)
    kernel_ms, ms = timed_steps(plan, a, ws_n, stream, region="llama2_70b")
    numel = plan.numel
    alg = numel * 4 + (numel // args.group) * 2 * (1 if args.symmetric else 2)
    per_rank = gather_per_rank([kernel_ms, alg], ws_n)
    total = all_ranks_sum(numel, ws_n)
    if ws_n == 1:
        traffic, src = committed_traffic(args.traffic_70b_file, numel, args.bits, args.group, "in-place")
    else:
        traffic, src = None, "the committed 70B PMC record is the 1-GPU launch's; at N > 1 each rank runs its own bin"
    del plan, weights
    torch.cuda.empty_cache()
    return {"config": f"BASELINE configs[3]: Llama-2-70B {len(shapes)} Linear weights bin-packed over {ws_n} GPU(s), "
                      f"INT{args.bits} g={args.group} {'sym' if args.symmetric else 'asym'}, in place",
            "value": round(total * 2 / (ms / 1e3) / 1e9, 2), "unit": "GB/s", "ms_per_step": round(ms, 4),
            "steps": steps, "warmup": warmup, "fp16_weights_total": total, "scaling": "strong",
            "roofline": roofline_record(per_rank, "k_group<f16,128,asym,batched,RW256> in place", traffic, src)}


def build_record(args, ws_n, n_dev, weak, all_shapes, total_numel, ms_per_step, roofline, extra):
    placement = "in-place" if args.inplace else "out-of-place"
    if weak:
        workload = f"{MODEL_NAME[args.model]} all {len(all_shapes)} Linear weights on every GPU "
    else:
        workload = f"{MODEL_NAME[args.model]} {len(all_shapes)} Linear weights bin-packed over {ws_n} GPU(s) "
    value = total_numel * 2 / (ms_per_step / 1e3) / 1e9 if ms_per_step else None
    rec = {
        "metric": METRIC, "value": None if value is None else round(value, 2), "unit": "GB/s", "n_gpus": n_dev,
        "ranks": ws_n, "n_devices": n_dev, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None if ms_per_step is None else round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak" if weak else "strong", "vs_baseline": None, "dtype": "fp16",
        "data": "synthetic",
        "config": {"workload": workload + f"({total_numel} fp16 weights in all), INT{args.bits} g={args.group} "
                               f"{'sym' if args.symmetric else 'asym'} pseudo_quantize_tensor, "
                               f"{placement} dequant + scales/zeros, one batched launch per rank per step",
                   "model": args.model, "bits": args.bits, "group": args.group,
                   "parallelism": f"layer-shard x{ws_n} (no collective)"},
        "roofline": roofline,
    }
    rec.update(extra)
    if n_dev < ws_n:
        rec["note"] = f"{ws_n} ranks shared {n_dev} GPU(s) (gloo rehearsal): one GPU's bandwidth, not a scaling point"
    rec["summary"] = summary_of(rec)
    return rec


def summary_of(rec):
    """The record's key figures in a few hundred bytes, emitted as the LAST key of the line: the
    driver keeps only the tail of stdout, which otherwise ends inside the long sections."""
    def g(d, *ks):
        for k in ks:
            d = d.get(k) if isinstance(d, dict) else None
        return d
    r = rec.get("roofline") or {}
    s = {"frac": r.get("frac"), "kernel_over_ceiling": r.get("kernel_over_ceiling"),
         "fresh_ceiling_GBps": g(r, "fresh_ceiling", "GBps"), "kernel_over_fresh_ceiling": r.get("kernel_over_fresh_ceiling"),
         "other_placement": [g(r, "other_placement", "placement"), g(r, "other_placement", "frac")], "traffic_over_alg": (
             round(r["traffic"] / r["alg_bytes_per_launch"], 4) if r.get("traffic") and r.get("alg_bytes_per_launch") else None)}
    if rec.get("shapes"):
        s["shapes_frac"] = {k: [v.get("frac"), v.get("frac_beyond_launch_floor")] for k, v in rec["shapes"].items()}
    if rec.get("fused_forward"):
        s["fused_vs_F_linear"] = {f"{x['shape']}/{'pc' if x['weights'] == 'per-channel' else x['weights']}/M{x['M']}":
                                  x.get("fused_vs_F_linear") for x in rec["fused_forward"].get("rows", [])}
    if rec.get("formats"):
        s["formats_frac"] = {x["path"]: x.get("frac_of_hbm_peak") for x in rec["formats"].get("rows", [])}
    if rec.get("llama2_70b"):
        s["llama2_70b_frac"] = g(rec["llama2_70b"], "roofline", "frac")
    cpu = rec.get("cpu_baseline")
    if cpu:
        s["cpu_baseline_GBps"] = cpu.get("value")
    return s


def main():
    args = parse()
    if args.mark_file:
        MARKS.enable()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    ws_n, rank, _, n_dev = init_dist(args)
    if args.dry_run:
        dry_run(args, ws_n, rank)
        if ws_n > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    from iron_weight_only_quant_amd import kernels

    weak = args.weak
    # 70B fp16 = 137 GB: in place (QuantLinear semantics) so N=1 fits in 288 GB; --scatter likewise
    if args.model == "llama2-70b" or args.scatter:
        args.inplace = True
    scatter_ms = None
    if args.scatter and ws_n > 1:
        weak = False
        weights, names, all_shapes, scatter_ms, _ = scatter_weights(args.model, rank, ws_n)
    else:
        weights, names, all_shapes = make_weights(args.model, rank, ws_n, weak=weak)
    numel = sum(w.numel() for w in weights)
    plan = kernels.BatchPlan(weights, args.bits, args.group, args.symmetric,
                             outs=weights if args.inplace else None)
    stream = torch.cuda.current_stream()
    if args.variants:
        ab_variants(plan, [int(v) for v in args.variants.split(",")], args)
    clock_ramp(plan, args.ramp_seconds)
    ceiling = copy_ceiling(plan)  # every rank: its own GPU's ceiling (roofline.per_rank)
    fresh = fresh_ceiling(plan)   # and the box's, on buffers that are not the plan's
    kernel_ms, ms_per_step = timed_steps(plan, args, ws_n, stream)

    other = None
    if ws_n == 1 and not args.inplace:
        other = other_placement_kernel(weights, plan, args)

    shapes_rec = None
    if not args.no_shapes and ws_n == 1 and not args.inplace:
        shapes_rec = per_shape(plan, names, ws_n, args)

    coll = {"gather_ms": None, "gather_bytes_to_rank0": None, "scatter_ms": scatter_ms}
    if ws_n > 1 and not args.no_collectives:
        coll.update(gather_section(plan, names, all_shapes, args, ws_n))

    total_numel = all_ranks_sum(numel, ws_n)
    groups = numel // args.group
    alg_bytes = numel * 2 + numel * 2 + groups * 2 * (1 if args.symmetric else 2)  # read w, write deq, s(,z)
    per_rank = gather_per_rank([kernel_ms, alg_bytes, ceiling["GBps"]], ws_n)
    if ws_n == 1:
        if args.model == "llama2-70b":
            traffic, traffic_src = committed_traffic(args.traffic_70b_file, numel, args.bits, args.group, "in-place")
        else:
            traffic, traffic_src = committed_traffic(args.traffic_file, numel, args.bits, args.group,
                                                     "in-place" if args.inplace else "out-of-place")
    else:
        traffic, traffic_src = None, ("the committed PMC record is the 1-GPU workload's; at N > 1 every rank runs "
                                      "a different bin (profiles/traffic.json: +0.07 % over algorithmic at N = 1)")
    roofline = roofline_record(per_rank, "k_group<f16,128,asym,batched,RW256>", traffic, traffic_src, ceiling, other)
    fresh_g = gather_per_rank([fresh["GBps"] if fresh else 0.0], ws_n)
    roofline["fresh_ceiling"] = (fresh if ws_n == 1 or not fresh else
                                 {**fresh, "GBps_per_rank": [round(f[0], 1) for f in fresh_g]})
    if roofline.get("achieved") and min(f[0] for f in fresh_g) > 0:
        lo = min(f[0] for f in fresh_g)
        roofline["kernel_over_fresh_ceiling"] = round(roofline["achieved"] / lo, 4)
        roofline["plan_ceiling_over_fresh_ceiling"] = round(min(p[2] for p in per_rank) / lo, 4)

    if ws_n > 1 and not args.no_collectives and not args.scatter:
        # bounded: the headline model's fp16 weights scattered from rank 0 (its own buffers are freed
        # first: rank 0 briefly holds every rank's bin)
        del plan
        plan = weights = None
        torch.cuda.empty_cache()
        coll.update(scatter_section(args.model, rank, ws_n))
    elif args.scatter and scatter_ms is not None:
        coll["scatter_bytes_from_rank0"] = 2 * sum(shard_bin_elems(args.model, ws_n)[1:])

    weak_rec = None
    if ws_n > 1 and not weak and args.model == "llama2-7b" and not args.no_weak and not args.scatter:
        plan = weights = None
        torch.cuda.empty_cache()
        weak_rec, shapes_rec = weak_secondary(args, ws_n, rank)
    if weights is None:  # the CPU baseline samples this rank's bin
        weights, _, _ = make_weights(args.model, rank, ws_n) if (rank == 0 and not args.no_cpu_baseline) else (None, 0, 0)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(weights, args.bits, args.group, args.symmetric, args.cpu_seconds, MODEL_NAME[args.model])
    plan = weights = None
    torch.cuda.empty_cache()

    ppl = None
    if rank == 0 and ws_n == 1 and not args.no_ppl:
        ppl = ppl_plumbing(args.bits, args.group, args.symmetric)

    # BASELINE configs[2] / [4] (one GPU: the driver's N = 1 run) and configs[3] (every N)
    fused = formats = m70 = None
    if ws_n == 1 and not args.no_sections:
        fused = fused_forward_section()
        formats = formats_section()
    if args.model == "llama2-7b" and not args.no_sections and not args.no_70b:
        m70 = model70b_section(args, ws_n, rank)

    if rank == 0:
        rec = build_record(args, ws_n, n_dev, weak, all_shapes, total_numel, ms_per_step, roofline, {
            "shapes": shapes_rec,
            "shapes_scaling": (None if shapes_rec is None else "single GPU" if ws_n == 1 else
                               f"weak: each of {ws_n} ranks runs its own cold calls at once; weights_GBps = "
                               "all ranks' input bytes / max-over-ranks time"),
            "weak": weak_rec,
            "cpu_baseline": cpu,
            "ppl_delta": None,
            "ppl_plumbing": ppl,
            **coll,
            "fused_forward": fused,
            "formats": formats,
            "llama2_70b": m70,
        })
        print(json.dumps(rec), flush=True)
    MARKS.write(args.mark_file, rank)
    if ws_n > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
