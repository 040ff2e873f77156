"""Benchmark: device-resident JPEG -> RGB224 on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic 480x640 q90 4:2:0 baseline JPEGs
(~110 KB, BASELINE.md §2 generator), batch 256 per GPU, already resident in
HBM; each step decodes the whole batch to RGB 224x224 u8 with the reference
CPU path's filter semantics (scale bicubic, force_original_aspect_ratio=
decrease, centred black pad, rgb24) -- the output load_image_batch(width=224,
height=224) produces.  One process per GPU; images are independent, so each
rank decodes its own 256-image slice with no collective on the data path
(weak scaling).  A barrier + MAX all-reduce of the elapsed time is the only
cross-rank traffic.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: either launched by torch.distributed.run (one rank per GPU), or
  started plainly, in which case bench.py spawns the N rank processes itself
  before any GPU call.  The barrier and the MAX-over-ranks reduction of the
  elapsed time go over gloo (host); nothing crosses xGMI.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# --hw-queues Q: HIP initialised (through torch) with GPU_MAX_HW_QUEUES=Q
# before spdl_amd is imported (the regime of a drop-in imported after the
# trainer touched the GPU).  Without it HIP takes the environment's value
# (its own default: 4).  The lanes' low-priority streams make the rate
# independent of Q; the record carries the rate at the other setting too.
if "--hw-queues" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[sys.argv.index("--hw-queues") + 1]
    import torch  # noqa: E402

    torch.cuda.init()
import spdl_amd  # noqa: E402,F401

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spdl_amd import _lib  # noqa: E402
from spdl_amd._lib import Output  # noqa: E402
from spdl_amd.distributed import (  # noqa: E402
    bind_rank_cpus,
    barrier,
    contiguous_shard,
    init_host_group,
    launched_world,
    reduce_max,
    spawn_ranks,
)
from spdl_amd.synthetic import synthetic_slice  # noqa: E402

METRIC = "images/sec device-resident JPEG→RGB224, 1/2/4/8×MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# Per-launch HBM-side bytes and SQ issue/wait shares per kernel from the
# committed rocprofv3 --pmc passes of this same command (tools/pmc_round.sh:
# tools/pmc_traffic.py, tools/pmc_issue.py): counters cannot be read from
# inside the timed process.
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06", "final")
PMC_TRAFFIC = os.path.join(PROFILE_DIR, "traffic.json")
PMC_ISSUE = os.path.join(PROFILE_DIR, "issue.json")
# rocprofv3 --kernel-trace --stats of this command (tools/profile_round.sh)
# union of each kernel's launch intervals per step in the kernel traces of
# the KSTATS runs (tools/kernel_busy.py)
BUSY = os.path.join(PROFILE_DIR, "kernel_busy.json")
KSTATS = {4: os.path.join(PROFILE_DIR, "kernel_stats_lanes4.csv"),
          1: os.path.join(PROFILE_DIR, "kernel_stats_lanes1.csv")}
# bench stage -> kernels launched in it
STAGE_KERNELS = {
    "parse": ["hj::parse_kernel"],
    "destuff": ["hj::destuff_count_kernel", "hj::destuff_prefix_kernel", "hj::destuff_write_kernel"],
    "entropy": ["hj::entropy_kernel<"],
    "idct": ["hj::idct_kernel<"],
    "output": ["hj::sws_kernel", "hj::csc_kernel"],
}


def _pmc(path: str, stage: str, batch: int) -> dict | None:
    """The committed PMC record of `stage`'s kernel(s) for this batch size
    (None when absent or recorded for another batch size)."""
    try:
        with open(path) as f:
            rec = json.load(f)
    except OSError:
        return None
    if rec.get("batch") not in (None, batch):
        return None
    hits = [v for name, v in rec["kernels"].items()
            if any(name.startswith(k) for k in STAGE_KERNELS.get(stage, []))]
    return hits[0] if len(hits) == 1 else None


def _rocprof_ms(lanes: int, stage: str) -> float | None:
    """Average duration (ms) of `stage`'s kernel in the committed rocprofv3
    kernel-trace summary of the bench at `lanes` lanes (None if absent)."""
    import csv

    try:
        with open(KSTATS[lanes]) as f:
            rows = list(csv.DictReader(f))
    except (KeyError, OSError):
        return None
    for r in rows:
        name = r["Name"].replace("void ", "")
        if any(name.startswith(k) for k in STAGE_KERNELS.get(stage, [])):
            return float(r["AverageNs"]) / 1e6
    return None


def _kernel_busy_ms(lanes: int, stage: str) -> float | None:
    """The device time per bench step during which `stage`'s kernel runs (the
    union of its launches' intervals / steps) in the committed kernel trace
    of the bench at `lanes` lanes (tools/kernel_busy.py)."""
    try:
        with open(BUSY) as f:
            rec = json.load(f)
    except OSError:
        return None
    for name, v in rec.get(str(lanes), {}).items():
        if any(name.startswith(k) for k in STAGE_KERNELS.get(stage, [])):
            return v["busy_ms_per_step"]
    return None


def _lib_hash() -> str | None:
    """sha256 of the loaded decode library (the build a profile belongs to)."""
    import hashlib

    try:
        with open(_lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except (OSError, AttributeError):
        return None


def _profile_build_match() -> bool | None:
    """Whether the committed profile set was taken on the library now loaded
    (PROFILE_DIR/lib_sha256.txt, written by tools/profile_round.sh); None
    when the profile set records no hash."""
    try:
        with open(os.path.join(PROFILE_DIR, "lib_sha256.txt")) as f:
            want = f.read().split()[0]
    except (OSError, IndexError):
        return None
    return want == _lib_hash()


def _limiter(issue: dict | None, hbm_frac: float | None) -> str:
    """What bounds the dominant kernel, derived from its measured shares
    (SQ counters, tools/pmc_issue.py; HBM traffic over the kernel's time):
    HBM when its traffic runs at >= 60 % of peak, VALU issue when its waves
    issue VALU >= 50 % of their cycles, latency when they wait >= 40 %,
    otherwise mixed issue."""
    if not issue:
        return "unmeasured (no PMC record for this configuration)"
    v, w = issue["valu_share"], issue["wait_share"]
    shares = (f"waves issue VALU {v:.0%} and wait {w:.0%} of their cycles; {issue['waves']} "
              f"waves per launch; {issue['lds_conflict_per_lds_inst']:.2f} LDS bank-conflict "
              f"cycles per LDS instruction"
              + (f"; PMC HBM traffic at {hbm_frac:.1%} of peak" if hbm_frac is not None else ""))
    if hbm_frac is not None and hbm_frac >= 0.6:
        kind = "HBM bandwidth"
    elif v >= 0.5:
        kind = "VALU issue"
    elif w >= 0.4:
        kind = "latency (dependent LDS / VALU chains, barriers)"
    else:
        kind = "instruction issue (VALU, SALU and LDS mixed)"
    return f"{kind}: {shares}"


BATCH = 256
OUT_SPEC = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease",
                  pad_w=224, pad_h=224)
# configs[3]: examples/imagenet_classification.py's filter chain (scale 256
# decrease + pad 256 + centre crop 224) with its Preprocessing fused:
# (x/255 - mean)/std in fp32 -> fp16 (or bf16), NCHW.
IMAGENET_SPEC = Output(pix_fmt="rgb", resize=True, fit_w=256, fit_h=256, aspect="decrease",
                       pad_w=256, pad_h=256, crop_w=224, crop_h=224, normalize=True)
FULLRES_SPEC = Output(pix_fmt="rgb24", resize=False)
WORKLOADS = {
    "fullres": ("configs[1] full resolution: synthetic 480x640 q90 4:2:0 baseline JPEG resident in "
                "HBM -> RGB 480x640 u8 (rgb24, load_image's format=rgb24 chain)"),
    "pad224": ("configs[1]: synthetic 480x640 q90 4:2:0 baseline JPEG resident in HBM -> RGB "
               "224x224 u8 (scale bicubic decrease + centred pad, rgb24)"),
    "imagenet": ("configs[3]: synthetic 480x640 q90 4:2:0 baseline JPEG resident in HBM -> "
                 "scale 256 decrease + pad 256 + crop 224, (x/255-mean)/std fused, NCHW {dt}"),
    "mixed": ("heterogeneous ImageNet-shaped batch resident in HBM (spdl_amd.synthetic.mixed_spec: "
              "0.02-12 MP log-normal around 0.19 MP, 4:2:0/4:2:2/4:4:4, q60-95, 30% optimised "
              "Huffman tables, 10% restart intervals) -> RGB 224x224 u8 pad"),
    "big1": ("one 4000x3000 q90 4:2:0 JPEG (~4 MB) + 255 configs[1] images resident in HBM -> "
             "RGB 224x224 u8 pad (size-adaptive entropy decode)"),
}


def _args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=BATCH)
    p.add_argument("--distinct", type=int, default=32)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline threads (0: every core this process may use)")
    p.add_argument("--cpu-images", type=int, default=2048,
                   help="CPU baseline sample per run (RGB224; half that for full-res)")
    p.add_argument("--cpu-runs", type=int, default=5)
    p.add_argument("--oracle-check", type=int, default=32,
                   help="images of the last timed batch compared with the oracle")
    p.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                   help="extra decoder parameter (spdl_hj_set_param), for A/B runs")
    p.add_argument("--debug-mask", type=int, default=0,
                   help="kernel phase ablations for timing (outputs are wrong; no oracle check); "
                        "needs a library built with -DHJ_ABLATIONS=1 (SPDL_AMD_LIB)")
    p.add_argument("--lanes1-steps", type=int, default=20,
                   help="synchronous one-lane batches timed for the dominant kernel's own "
                        "duration (0: skip)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="run every rank on device 0 (a one-GPU rehearsal of the N-rank launch; "
                        "the record says so -- not a multi-GPU measurement)")
    p.add_argument("--bind", choices=["node", "split", "none"], default="node",
                   help="N > 1: each rank's threads on the cores of its GPU's NUMA node (node), on "
                        "its own disjoint share of them (split), or left alone (none)")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU-only rehearsal of the multi-rank launch and timing reduction")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--sub-bits", type=int, default=0)
    p.add_argument("--entropy-threads", type=int, default=0)
    p.add_argument("--entropy-lds-pad", type=int, default=-1,
                   help="extra dynamic LDS bytes per entropy workgroup (-1: library default)")
    p.add_argument("--warm-slots", type=int, default=-1,
                   help="entropy round-0 warm-up slots before each run (-1: library default)")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="pad224")
    p.add_argument("--piece-bytes", type=int, default=-1,
                   help="entropy_piece_bytes (size-adaptive entropy decode; 0: off; -1: library "
                        "default)")
    p.add_argument("--mixed-skip", default="",
                   help="A/B: comma-separated mixed-set images left out of --workload mixed")
    p.add_argument("--norm-dtype", choices=["float16", "bfloat16"], default="float16")
    p.add_argument("--inflight", type=int, default=0, choices=range(0, 11),
                   help="batches submitted ahead before waiting the oldest (0: lanes + 2; the ring holds 10)")
    p.add_argument("--lanes", type=int, default=0,
                   help="concurrent decode pipelines in the context (1-8; 0: the library default)")
    p.add_argument("--hw-queues", type=int, default=0,
                   help="initialise HIP with this many hardware queues before importing spdl_amd "
                        "(the late-import regime of a drop-in)")
    p.add_argument("--no-queue-compare", action="store_true",
                   help="skip the child run at the other GPU_MAX_HW_QUEUES setting (4 <-> 16)")
    p.add_argument("--sync-steps", action="store_true",
                   help="one synchronous call per step (no overlap of host work)")
    p.add_argument("--with-copies", action="store_true",
                   help="also time the host-bytes path (pinned H2D + D2H of the output)")
    p.add_argument("--warmup-mode", choices=["sync", "pipelined"], default="pipelined",
                   help="warmup steps one synchronous batch at a time, or submitted as the timed "
                        "steps are (the device is busy up to the timed region)")
    p.add_argument("--timed-events", choices=["dominant", "stages", "off"], default="dominant",
                   help="HIP events in the timed steps: around the dominant kernel's stage only "
                        "(found by an untimed profiled pass first), around every stage, or none "
                        "(A/B); the per-stage breakdown then comes from as many profiled steps "
                        "after the timed region")
    return p.parse_args()


def _param_or_none(dec, name: str):
    """A decoder parameter, or None when the loaded library predates it (A/B
    runs of older builds)."""
    try:
        return dec.get_param(name)
    except ValueError:
        return None


def _pack_device(datas: list[bytes], device: torch.device):
    offs, sizes, total = [], [], 0
    for d in datas:
        offs.append(total)
        sizes.append(len(d))
        total += (len(d) + 64 + 255) // 256 * 256
    host = np.zeros(total, np.uint8)
    for o, d in zip(offs, datas):
        host[o : o + len(d)] = np.frombuffer(d, np.uint8)
    dev = torch.from_numpy(host).to(device)
    infos = [_lib.get_image_info(d) for d in datas]
    # marshalled once: the step loop passes the same arrays every time
    return (dev, np.asarray(offs, np.int64), np.asarray(sizes, np.int64),
            (_lib.ImageInfo * len(infos))(*infos))


def _cpu_cores() -> dict:
    """Host cores this process may use: the CPU affinity mask, capped by a
    cgroup v2 CPU quota when one is set (a GPU box's share of a large host),
    plus os.cpu_count() and the CPU model for the record."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = max(1, min(usable, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"usable": usable, "nproc": os.cpu_count(), "model": model}


def _mean_ci95(xs):
    """Mean and 95 % confidence half-width (Student t) of repeated runs, as
    the reference's examples/benchmark_utils.py:204-345 reports them."""
    from scipy import stats

    x = np.asarray(xs, np.float64)
    if len(x) < 2:
        return float(x.mean()), 0.0
    half = stats.t.ppf(0.975, len(x) - 1) * x.std(ddof=1) / np.sqrt(len(x))
    return float(x.mean()), float(half)


def _cpu_baseline(datas, threads: int, n224: int, nfull: int, runs: int) -> dict:
    """The oracle (CPU restatement of the reference FFmpeg path: mjpeg
    simple_idct + swscale) on the host cores, one decoder per thread, over
    bounded samples of the same workload: warmup, then `runs` timed runs,
    mean +- 95 % CI.  RGB224 pad (the metric's output) and full-resolution
    rgb24 are both timed."""
    from oracle import oracle as O

    rs = O.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)

    def timed(fn, n):
        sample = [datas[i % len(datas)] for i in range(n)]
        fn(sample[: min(64, n)])  # warmup
        rates = []
        for _ in range(runs):
            t0 = time.perf_counter()
            failed = fn(sample)
            rates.append(n / (time.perf_counter() - t0))
            assert failed == 0
        return _mean_ci95(rates)

    m224, c224 = timed(lambda s: O.decode_resize_batch(s, rs, "rgb24", nthreads=threads)[2], n224)
    mfull, cfull = timed(lambda s: O.decode_rgb_batch(s, "rgb24", nthreads=threads)[2], nfull)
    cores = _cpu_cores()
    return {
        "value": round(m224, 1),
        "ci95": round(c224, 1),
        "unit": "images/sec",
        "cores": threads,
        "kind": "port",
        "fullres_value": round(mfull, 1),
        "fullres_ci95": round(cfull, 1),
        "host": {"nproc": cores["nproc"], "usable_cores": cores["usable"], "cpu": cores["model"]},
        "sample": f"{runs} runs (after warmup) of {n224} images 480x640 q90 4:2:0 -> RGB224 pad "
                  f"(bicubic swscale) and {runs} of {nfull} -> full-res rgb24; {threads} threads, "
                  f"one decoder per thread; oracle/jpeg_oracle.c (CPU restatement of the "
                  f"src/libspdl FFmpeg path); mean +- 95% CI",
    }


def _oracle_check(datas, out: torch.Tensor, spec: Output, n_check: int) -> str:
    """Bit-exact check of the first `n_check` images of a timed batch
    against the oracle, outside the timed region."""
    from oracle import oracle as O

    host = out[:n_check].cpu()
    kw = dict(fit_w=spec.fit_w, fit_h=spec.fit_h, aspect=spec.aspect, pad_w=spec.pad_w,
              pad_h=spec.pad_h, crop_w=spec.crop_w, crop_h=spec.crop_h, filter=spec.filter)
    for i in range(n_check):
        if not spec.resize:  # full resolution: the format=rgb24 chain
            ref = O.decode_rgb(datas[i], O.IDCT_SIMPLE, spec.pix_fmt)
        else:
            ref = O.decode_resize(datas[i], O.Resize(**kw), pix_fmt=spec.pix_fmt,
                                  normalize=spec.normalize, norm_dtype=spec.norm_dtype)
        hyp = host[i]
        if spec.normalize:
            hyp = hyp.view(torch.int16).numpy().view(np.uint16)
            ref = ref.view(np.uint16)
        else:
            hyp = hyp.numpy()
        if not np.array_equal(hyp, ref):
            raise AssertionError(f"timed batch image {i} differs from the oracle")
    return f"{n_check} images of the last timed batch bit-exact vs oracle"


def _dry_run(a, rank: int, world: int) -> None:
    """CPU-only rehearsal of the launch/partition/timing plumbing (tests):
    the same rank slicing and MAX-over-ranks reduction, no GPU."""
    import torch.distributed as dist

    from spdl_amd.distributed import barrier, contiguous_shard, reduce_max

    sl = contiguous_shard(world * a.batch, rank, world)
    barrier()
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))
    barrier()
    elapsed = reduce_max(time.perf_counter() - t0)
    slices = [None] * world
    if world > 1:
        dist.all_gather_object(slices, [sl.start, sl.stop])
    else:
        slices = [[sl.start, sl.stop]]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "global_batch": world * a.batch,
                          "slices": slices, "elapsed": elapsed}), flush=True)


def main():
    a = _args()
    rank, world, local = launched_world()
    if a.gpus > 1 and world == 1:
        # one process per GPU, started before anything touches a device
        # (reference examples/image_dataloading.py:291-317)
        raise SystemExit(spawn_ranks(a.gpus, [os.path.abspath(__file__), *sys.argv[1:]]))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    init_host_group()
    if a.dry_run:
        _dry_run(a, rank, world)
        return
    device = torch.device("cuda", 0 if a.rehearse_one_gpu else local)
    torch.cuda.set_device(device)
    bind = None
    if world > 1 and a.bind != "none":
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        devices = [0] * lw if a.rehearse_one_gpu else list(range(lw))
        bind = bind_rank_cpus(device.index, devices, local, a.bind)

    # this rank's contiguous slice of the global batch (configs[2]: 2048 -> 8 x 256)
    sl = contiguous_shard(world * a.batch, rank, world)
    if a.workload == "mixed":
        from spdl_amd.synthetic import mixed_jpeg

        cache: dict[int, bytes] = {}
        datas = []
        skip = {int(x) for x in a.mixed_skip.split(",") if x}
        keep = [j for j in range(64) if j not in skip]
        for i in sl:  # 64 distinct images of the mixed set, cycled
            j = keep[i % len(keep)]
            if j not in cache:
                cache[j] = mixed_jpeg(j)
            datas.append(cache[j])
    elif a.workload == "big1":
        from spdl_amd.synthetic import big_batch

        datas = big_batch(a.batch, a.distinct)
    else:
        datas = synthetic_slice(sl, distinct=a.distinct)
    dev, offs, sizes, infos = _pack_device(datas, device)
    dec = _lib.Decoder(device.index)
    if a.sub_bits:
        dec.set_param("sub_bits", a.sub_bits)
    if a.entropy_threads:
        dec.set_param("entropy_threads", a.entropy_threads)
    if a.entropy_lds_pad >= 0:
        dec.set_param("entropy_lds_pad", a.entropy_lds_pad)
    if a.warm_slots >= 0:
        dec.set_param("warmup_slots", a.warm_slots)
    if a.piece_bytes >= 0:
        dec.set_param("entropy_piece_bytes", a.piece_bytes)
    dec.set_param("lanes", a.lanes)  # (0: the library's choice for the queues in effect)
    a.lanes = dec.get_param("lanes")
    if a.inflight == 0:
        a.inflight = min(10, max(2, a.lanes + 2))
    for kv in a.param:
        k, v = kv.split("=", 1)
        dec.set_param(k, int(v))
    if a.debug_mask:
        try:
            dec.set_param("debug_mask", a.debug_mask)
        except ValueError:
            raise SystemExit("--debug-mask needs an HJ_ABLATIONS build of the library "
                             "(make -C spdl_amd/csrc variant NAME=abl DEFS=-DHJ_ABLATIONS=1; "
                             "SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_abl.so)") from None
    if a.workload == "imagenet":
        spec = Output(**{**IMAGENET_SPEC.__dict__, "norm_dtype": a.norm_dtype})
        outs = [torch.empty((a.batch, 3, 224, 224), dtype=spec.torch_dtype, device=device)
                for _ in range(max(3, a.inflight))]
    elif a.workload == "fullres":
        spec = FULLRES_SPEC
        outs = [torch.empty((a.batch, 480, 640, 3), dtype=torch.uint8, device=device)
                for _ in range(max(3, a.inflight))]
    else:  # pad224, mixed, big1
        spec = OUT_SPEC
        outs = [torch.empty((a.batch, 224, 224, 3), dtype=torch.uint8, device=device)
                for _ in range(max(3, a.inflight))]
    out = outs[0]
    stream = torch.cuda.current_stream(device)
    nbytes_out = out.numel() * out.element_size()
    nsub = [0]

    def submit(sync: bool) -> int:
        # output buffer per in-flight batch (up to three)
        o = outs[nsub[0] % len(outs)]
        nsub[0] += 1
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                o.data_ptr(), nbytes_out, stream=stream, sync=sync)
        return dec.last_ticket()

    # Steps are submitted asynchronously through the decoder's ring (up to
    # --inflight batches, executing on the context's two lanes): host-side
    # layout and launches overlap the kernels, as in a data loader.  Each
    # batch is waited for (statuses checked) and its per-stage HIP-event
    # timings collected.
    stages = {}

    def collect(ticket: int):
        st = dec.wait(ticket, a.batch)
        assert not any(st), st
        for k, v in dec.last_timings().items():
            stages[k] = stages.get(k, 0.0) + v

    def run_steps(k: int) -> float:
        """k steps, up to --inflight batches in flight; returns the host time
        spent inside the asynchronous submissions."""
        pending = []
        host = 0.0
        for _ in range(k):
            if a.sync_steps:
                submit(True)
                for kk, v in dec.last_timings().items():
                    stages[kk] = stages.get(kk, 0.0) + v
                continue
            ts = time.perf_counter()
            pending.append(submit(False))
            host += time.perf_counter() - ts
            if len(pending) > a.inflight - 1:  # wait the oldest (the ring holds 10)
                collect(pending.pop(0))
        for t in pending:
            collect(t)
        return host

    # warmup: every lane's workspace sized and its kernels loaded; pipelined
    # (the default), so the device runs at its working clocks up to the
    # barrier that opens the timed region
    if a.warmup_mode == "sync" or a.sync_steps:
        for _ in range(a.warmup):
            submit(True)
    else:
        for _ in range(min(a.warmup, a.lanes)):
            submit(True)
        run_steps(max(0, a.warmup - a.lanes))
    stages.clear()
    dom_stage = None
    if a.timed_events == "dominant":
        # which stage dominates: an untimed pass with every stage timed
        dec.set_profiling(True)
        run_steps(max(8, a.inflight))
        ks = {k: v for k, v in stages.items() if k not in ("h2d", "d2h_status")}
        dom_stage = max(ks, key=ks.get)
        stages.clear()
        dec.set_profiling(True, stages=[dom_stage])
    else:
        dec.set_profiling(a.timed_events == "stages")

    torch.cuda.synchronize(device)
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    host_submit = run_steps(a.steps)  # host time inside the asynchronous submissions
    torch.cuda.synchronize(device)
    own = time.perf_counter() - t0
    barrier()
    torch.cuda.synchronize(device)
    elapsed = reduce_max(time.perf_counter() - t0)
    timed_stages = dict(stages)  # the HIP-event times of the timed steps
    if a.timed_events != "stages":
        # the per-stage breakdown: as many profiled steps after the timed region
        stages.clear()
        dec.set_profiling(True)
        run_steps(a.steps)
    dec.set_profiling(False)

    # correctness outside the timed region: the last timed batch against
    # the oracle (every distinct image of the slice)
    last = outs[(nsub[0] - 1) % len(outs)]
    checked = ("skipped (--debug-mask ablation)" if a.debug_mask else
               _oracle_check(datas, last, spec, min(a.batch, a.distinct, a.oracle_check)))

    stages_ms = {k: v / a.steps / 1000.0 for k, v in stages.items()}
    kernels = {k: v for k, v in stages_ms.items() if k not in ("h2d", "d2h_status")}
    dominant = dom_stage or max(kernels, key=kernels.get)
    # the dominant kernel's launch time inside the timed region (its own HIP
    # events on its lane streams); with --timed-events off, from the
    # profiled steps after it
    timed_ms = {k: v / a.steps / 1000.0 for k, v in timed_stages.items()}
    kernel_ms = timed_ms.get(dominant, kernels[dominant])
    comp_bytes = float(np.mean(sizes))
    # §8(d): compressed in + RGB224 out (u8: 150,528 B; fp16/bf16: 301,056 B)
    per_image_bytes = comp_bytes + nbytes_out / a.batch
    launch_bytes = per_image_bytes * a.batch

    # The dominant kernel alone: with several lanes its launches share the CUs
    # with the other lanes' kernels, so the per-launch time above is a shared
    # wall time.  One lane, synchronous batches, the same HIP-event stages.
    lanes1 = None
    if a.lanes1_steps > 0 and not a.debug_mask:
        dec1 = _lib.Decoder(device.index)
        dec1.set_param("lanes", 1)
        if a.piece_bytes >= 0:
            dec1.set_param("entropy_piece_bytes", a.piece_bytes)
        dec1.set_profiling(True)
        acc = {}
        for i in range(a.lanes1_steps + 2):
            dec1.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                     out.data_ptr(), nbytes_out, stream=stream, sync=True)
            if i >= 2:
                for k, v in dec1.last_timings().items():
                    acc[k] = acc.get(k, 0.0) + v
        th1 = dec1.get_param("entropy_threads")
        dec1.close()
        ms1 = acc[dominant] / a.lanes1_steps / 1000.0
        ach1 = launch_bytes / (ms1 / 1000.0) / 1e9
        r1 = _rocprof_ms(1, dominant) if a.workload == "pad224" and a.batch == BATCH else None
        lanes1 = {"kernel_ms": round(ms1, 4), "achieved": round(ach1, 3),
                  "frac": round(ach1 / HBM_PEAK_GBS, 6), "steps": a.lanes1_steps,
                  "entropy_threads": th1, "kernel_ms_rocprof": r1}

    # per-rank record: each rank's own rate and device (the driver's 8-GPU
    # run shows N distinct devices working)
    props = torch.cuda.get_device_properties(device)
    mine = {"rank": rank, "device": device.index,
            "pci_bus_id": getattr(props, "pci_bus_id", None),
            "slice": [sl.start, sl.stop],
            "images_per_sec": round(a.batch * a.steps / own, 1),
            "oracle_check": checked, **(bind or {})}
    if world > 1:
        import torch.distributed as dist

        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]

    copies = None
    if a.with_copies and rank == 0:
        host_out = torch.empty_like(out, device="cpu").pin_memory()
        t1 = time.perf_counter()
        nrep = max(5, a.steps // 4)
        for _ in range(nrep):
            dec.decode_batch(datas, spec, out.data_ptr(), nbytes_out, stream=stream, sync=True)
            host_out.copy_(out, non_blocking=True)
            torch.cuda.synchronize(device)
        copies = a.batch * nrep / (time.perf_counter() - t1)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.workload == "pad224":
        threads = a.cpu_threads or _cpu_cores()["usable"]
        cpu = _cpu_baseline(datas, threads, a.cpu_images, a.cpu_images // 2, a.cpu_runs)

    # the same bench in a child process whose HIP starts with the other
    # hardware-queue count (4 <-> 16): the record carries both rates
    queues = None
    hwq = dec.get_param("hw_queues")
    if (rank == 0 and world == 1 and not a.no_queue_compare and not a.debug_mask
            and a.workload == "pad224"):
        other = 16 if hwq != 16 else 4
        cmd = [sys.executable, os.path.abspath(__file__), "--hw-queues", str(other),
               "--steps", str(a.steps), "--warmup", str(a.warmup), "--batch", str(a.batch),
               "--lanes", str(a.lanes), "--no-cpu-baseline", "--lanes1-steps", "0",
               "--no-queue-compare", "--oracle-check", "8"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        child = [json.loads(line) for line in r.stdout.splitlines() if line.startswith('{"metric"')]
        if r.returncode != 0 or not child:
            raise SystemExit(f"queue-compare child failed ({r.returncode}): {r.stderr[-2000:]}")
        c = child[-1]
        queues = {"this_run": {"hw_queues": hwq, "value": None},
                  "other": {"hw_queues": c["config"]["hw_queues"], "value": c["value"],
                            "lanes": c["config"]["lanes"], "steps": c["steps"],
                            "oracle_check": c["oracle_check"]}}

    traffic = issue = rocprof_ms = None
    if a.workload == "pad224" and a.lanes in KSTATS and a.batch == BATCH:
        rocprof_ms = _rocprof_ms(a.lanes, dominant)
    if a.workload == "pad224" and a.lanes == 4:  # the configuration the PMC passes ran
        traffic = _pmc(PMC_TRAFFIC, dominant, a.batch)
        issue = _pmc(PMC_ISSUE, dominant, a.batch)
    # `achieved` and `frac` from this run's own HIP-event duration of the
    # dominant kernel (events recorded on the lane streams the kernel runs
    # on), so a kernel change shows in the headline fields at once.  The
    # committed rocprofv3 summary of this configuration rides along under
    # `profile`, with whether it was taken on this very library build.
    achieved = launch_bytes / (kernel_ms / 1e3) / 1e9
    prof_match = _profile_build_match()
    # (the PMC traffic per launch over this run's launch duration: the same
    # time base as `achieved` / `frac`)
    hbm_frac = (traffic["traffic_bytes"] / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS
                if traffic else None)
    busy = _kernel_busy_ms(a.lanes, dominant) if a.workload == "pad224" else None
    if rank == 0:
        value = world * a.batch * a.steps / elapsed
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000.0, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8" if a.workload in ("pad224", "fullres", "mixed", "big1") else
                     {"float16": "f16", "bfloat16": "bf16"}[a.norm_dtype] + " out (int decode, f32 normalise)",
            "data": "synthetic",
            "config": {
                "workload": WORKLOADS[a.workload].format(dt=a.norm_dtype),
                "global_batch": world * a.batch,
                "per_gpu_batch": a.batch,
                "mean_jpeg_bytes": round(comp_bytes, 1),
                "distinct_images": a.distinct,
                "parallelism": f"{world} ranks (one process per GPU), contiguous slices of the "
                               f"global batch, no collective on the data path",
                "lanes": dec.get_param("lanes"),
                "hw_queues": dec.get_param("hw_queues"),
                "entropy_threads": dec.get_param("entropy_threads"),
                "entropy_piece_bytes": _param_or_none(dec, "entropy_piece_bytes"),
                "compressed_GBps": round(world * float(np.sum(sizes)) * a.steps / elapsed / 1e9, 3),
                **({"rehearsal": f"{world} ranks sharing ONE GPU (launch-path check, not a "
                                 f"multi-GPU rate)"} if a.rehearse_one_gpu else {}),
            },
            "roofline": {
                # the roofline the path is priced against (no MFMA work); what
                # the counters say limits the kernel is `limiter`
                "bound": "hbm",
                "kernel": dominant,
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic["traffic_bytes"] if traffic else None,
                "traffic_source": (f"{os.path.relpath(PMC_TRAFFIC, ROOT)}: "
                                   f"{traffic['correction']} (tools/fetch_calib.hip)")
                                  if traffic else None,
                "algorithmic_bytes_per_image": round(per_image_bytes, 1),
                "launch_images": a.batch,
                "formula": "achieved = algorithmic_bytes_per_image x launch_images / kernel_ms; "
                           "frac = achieved / peak",
                "kernel_ms": round(kernel_ms, 4),
                "time_source": ("HIP events around the kernel's launches in the timed steps "
                                "(this run)" if a.timed_events != "off" else
                                "HIP events in profiled steps after the timed region (A/B mode)"),
                "timed_events": a.timed_events,
                # the committed rocprofv3 kernel-trace average of this
                # configuration; with several lanes a launch's duration is a
                # shared wall time (it waits for CUs the other lanes hold), so
                # it can exceed ms_per_step; the device time per step the
                # kernel occupies is the union of its launches' intervals
                "profile": {
                    "dir": os.path.relpath(PROFILE_DIR, ROOT),
                    "build_match": prof_match,
                    "kernel_ms_rocprof": round(rocprof_ms, 4) if rocprof_ms else None,
                    "frac_rocprof": (round(launch_bytes / (rocprof_ms / 1e3) / 1e9
                                           / HBM_PEAK_GBS, 6) if rocprof_ms else None),
                    "source": (os.path.relpath(KSTATS[a.lanes], ROOT) if rocprof_ms else None),
                },
                "kernel_busy_ms_per_step": busy,
                "kernel_busy_source": (f"{os.path.relpath(BUSY, ROOT)}: union of the kernel's "
                                       f"launch intervals in the rocprofv3 kernel trace / steps"
                                       if busy is not None else None),
                "limiter": _limiter(issue, hbm_frac),
                # the limiter's HBM share divides the committed PMC traffic by the
                # same duration as `frac`
                "limiter_time_base": "kernel_ms",
                "pipeline_GBps": round(launch_bytes / (elapsed / a.steps) / 1e9, 3),
                "lanes1": lanes1,
            },
            "stages_ms": {k: round(v, 4) for k, v in stages_ms.items()},
            "stages_source": ("HIP events of every stage in the timed steps"
                              if a.timed_events == "stages" else
                              "HIP events of every stage in as many profiled steps after the "
                              "timed region (" + ("the timed steps bracket the dominant kernel "
                                                  "only)" if a.timed_events == "dominant" else
                                                  "the timed steps record no events)")),
            # host time of one asynchronous batch submission (layout, pinned
            # staging, launches): the device-resident path's host budget
            "host_submit_ms": round(host_submit / a.steps * 1000.0, 4) if not a.sync_steps else None,
            "oracle_check": checked,
            "ranks": ranks,
            "cpu_baseline": cpu,
        }
        if queues is not None:
            queues["this_run"]["value"] = rec["value"]
            queues["other_over_this"] = round(queues["other"]["value"] / rec["value"], 4)
            rec["hw_queue_regimes"] = queues
        if copies is not None:
            rec["with_copies_images_per_sec"] = round(copies, 1)
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
