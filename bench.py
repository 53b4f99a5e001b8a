"""Benchmark: depth maps/s of the cascade forward on MI355X (BASELINE.json metric), ms per stage,
roofline of the dominant kernel and the CPU baseline — one JSON line on rank 0.

  python bench.py [--gpus N --steps K --warmup W] [--config cfgC] [--batch B] [--no-cpu-baseline]
                  [--shard depth|rows|gather [--emulate P]] [--no-shard-latency]

Workload (BASELINE.json configs[2]): DTU 1600x1184, 5 views, 3-stage 48/32/8 hypotheses, bf16 storage
on 1x MI355X; synthetic seeded images/cameras, synthetic weights with calibrated BN statistics
(no checkpoints or datasets exist offline). One step = one full CascadeMVSNet forward
(front-end + 3 x (hypotheses, [GeoFeatureFusion], DepthNet)) over one batch per GPU, inputs resident
in HBM. Multi-GPU: one process per GPU, each processing its own batch (reference views are
independent units: weak scaling, no collective in the data path); timing = max over ranks. With N > 1 the
depth-sharded latency mode (damvsnet_amd/sharded.py: one map's cost volumes over all N GPUs) is timed
after the throughput steps and reported as "depth_sharded"; ``--shard`` makes it the measured mode
(``--emulate P``: P ranks as threads on one GPU, a functional rehearsal, not a speed figure).

Roofline (damvsnet_amd/costmodel.py): HIP events recorded inside damvs_stage_forward
(damvs_stage_forward_probed) around the warp, the U-Net and the regression of every stage of the timed
steps give the in-pipeline kernel-group times; the headline roofline kernel is the stage-2 warp as the
product runs it. MFMA utilisation of the U-Net / front-end conv kernels comes from the committed
rocprofv3 PMC summary (tools/pmc_mfma.py) when present.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    # name: (H, W, views, ndepths, dtype, description)
    "cfgA": (256, 320, 3, (48, 32, 8), torch.float32, "DTU 320x256, ref+2 src, fp32"),
    "cfgB": (512, 640, 5, (48, 32, 8), torch.float32, "DTU 640x512, 5 views, 3-stage 48/32/8, fp32"),
    "cfgC": (1184, 1600, 5, (48, 32, 8), torch.bfloat16, "DTU 1600x1184, 5 views, 3-stage 48/32/8, bf16"),
    "cfgD": (1184, 1600, 7, (64, 32, 8), torch.bfloat16, "DTU 1600x1184, 7 views, 3-stage 64/32/8, bf16"),
    "cfgE": (1056, 1920, 11, (64, 32, 8), torch.bfloat16, "T&T 1920x1056, 11 views, 3-stage 64/32/8, bf16"),
}
SHARD_GUARD_S = 240  # N > 1: seconds the depth-sharded blocks may take before the line goes out without them
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def coll_device(device):
    """Where collective tensors live: the GPU under RCCL ("nccl"), the host under gloo (tests/bench_dryrun.py runs
    this script's N > 1 path as a CPU gloo job)."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend() != "nccl":
        return torch.device("cpu")
    return device


def build_model(ndepths, dtype, device, frontend="hip"):
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.weights import synthetic_state_dict, apply_bn_stats
    net = CascadeMVSNet(ndepths=list(ndepths), compute_dtype=dtype,
                        frontend_dtype=torch.bfloat16 if dtype == torch.bfloat16 else None, frontend_impl=frontend)
    sd = synthetic_state_dict(net.state_dict(), 0)
    g = np.load(os.path.join(REPO, "tests", "golden", "forward_cfgB_640x512.npz"))
    sd = apply_bn_stats(sd, {k[4:]: g[k] for k in g.files if k.startswith("bn::")})
    net.load_state_dict(sd)
    return net.to(device).eval(), sd


def make_inputs(B, N, H, W, device=None, seed=0):
    from damvsnet_amd import synth
    proj, ins, dv = synth.cameras(B, N, H, W)
    imgs = torch.from_numpy(synth.images(B, N, H, W, seed=seed))
    proj = {k: torch.from_numpy(v) for k, v in proj.items()}
    ins = {k: torch.from_numpy(v) for k, v in ins.items()}
    dv = torch.from_numpy(dv)
    if device is not None:
        imgs, dv = imgs.to(device), dv.to(device)
        proj = {k: v.to(device) for k, v in proj.items()}
        ins = {k: v.to(device) for k, v in ins.items()}
    return imgs, proj, dv, ins


class StageTimer:
    """Records a HIP event on the current stream at every phase boundary (no host sync)."""

    def __init__(self):
        self.marks = []

    def __call__(self, name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.marks.append((name, e))

    def per_phase_ms(self):
        out = {}
        for (n0, e0), (_, e1) in zip(self.marks, self.marks[1:]):
            out.setdefault(n0, []).append(e0.elapsed_time(e1))
        return out


class ProbeRecorder:
    """DepthNet.probe: 4 events per stage call (before / after the warp, after the U-Net, after the
    regression), recorded by the library on the launch stream (damvs_stage_forward_probed)."""

    def __init__(self):
        self.calls = []

    def __call__(self, stage_idx):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        self.calls.append((stage_idx, ev))
        return ev

    def per_stage_ms(self):
        out = {}
        for s, ev in self.calls:
            d = out.setdefault(s, {"warp": [], "unet": [], "regress": []})
            d["warp"].append(ev[0].elapsed_time(ev[1]))
            d["unet"].append(ev[1].elapsed_time(ev[2]))
            d["regress"].append(ev[2].elapsed_time(ev[3]))
        return {s: {k: statistics.mean(v) for k, v in d.items()} for s, d in sorted(out.items())}


def hot_path_roofline(per_stage_ms, H, W, N, nd, B, dtype_name):
    """Per stage and per map: algorithmic bytes / FLOPs (costmodel) against the in-pipeline times."""
    from damvsnet_amd import costmodel as CM
    e = 2 if dtype_name == "bf16" else 4
    cost = CM.cascade_cost(H, W, N, nd, e)
    stages, t_meas, t_roof = {}, 0.0, 0.0
    for s, ms in per_stage_ms.items():
        groups = {}
        for g in ("warp", "unet", "regress"):
            nbytes, flops = (B * x for x in cost[s][g])
            t = ms[g] * 1e-3
            groups[g] = {"ms": round(ms[g], 4), "GB/s": round(nbytes / t / 1e9, 1), "TFLOP/s": round(flops / t / 1e12, 2),
                         "hbm_frac": round(nbytes / t / CM.HBM_PEAK, 4),
                         "mfma_frac": round(flops / t / CM.MFMA_PEAK[dtype_name], 4),
                         **({"mfma_frac_vs_exact_f32": round(flops / t / CM.MFMA_PEAK["f32_exact"], 4)}
                            if dtype_name == "f32" else {}),
                         "roofline_frac": round(CM.roofline_time(nbytes, flops, dtype_name) / t, 4)}
        sb = sum(B * cost[s][g][0] for g in groups)
        sf = sum(B * cost[s][g][1] for g in groups)
        ts = sum(ms[g] for g in groups) * 1e-3
        tr = CM.roofline_time(sb, sf, dtype_name)
        stages["stage%d" % (s + 1)] = {"ms": round(ts * 1e3, 4), "roofline_ms": round(tr * 1e3, 4),
                                        "roofline_frac": round(tr / ts, 4), "kernels": groups}
        t_meas += ts
        t_roof += tr
    return {"per_stage": stages, "per_map": {"ms": round(t_meas * 1e3 / B, 4), "roofline_ms": round(t_roof * 1e3 / B, 4),
                                              "roofline_frac": round(t_roof / t_meas, 4)}}


def pmc_mfma(config, batch, dtype=None):
    """MFMA utilisation per kernel family from the committed rocprofv3 PMC summary
    (profiles/<round>/pmc_mfma_<config>_b<batch>[_f32].json, tools/pmc_mfma.py), or None."""
    import glob
    sfx = "_f32" if dtype == "f32" else ""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_mfma_%s_b%d%s.json" % (config, batch, sfx))))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return {"source": os.path.relpath(files[-1], REPO), "kernels": d.get("summary", d)}


def sharded_latency(net, H, W, N, device, comm=None, emulate=1, warp="depth", steps=5, warmup=2):
    """One depth map (B=1) with every stage's DepthNet over the ranks (damvsnet_amd/sharded.py): ms per map
    (max over ranks) and rank 0's per-phase times of the last step."""
    from damvsnet_amd.sharded import DepthShardedDepthNet, ThreadGroup
    imgs, proj, dv, ins = make_inputs(1, N, H, W, device, seed=0)  # every rank: the same map
    world = comm.world if comm is not None else emulate

    def step(c, hook=None):
        return net(imgs, proj, dv, ins, depthnet=DepthShardedDepthNet(net, c, warp=warp, hook=hook))

    def run_all(hook=None):
        if comm is not None:
            step(comm, hook)
        else:
            ThreadGroup(emulate).run(lambda c: step(c, hook if c.rank == 0 else None))

    with torch.no_grad():
        net(imgs, proj, dv, ins)  # folded front-end and stage engines exist before any rank thread starts
        for _ in range(warmup):
            run_all()
        torch.cuda.synchronize()
        if comm is not None:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            run_all()
        torch.cuda.synchronize()
        if comm is not None:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        timer = StageTimer()
        res = {}

        def checked(c, hook=None):  # one sharded forward, every stage bitwise against the unsharded one
            out = step(c, hook)
            if c.rank == 0:
                ref = net(imgs, proj, dv, ins)
                res["bitwise_vs_unsharded"] = all(
                    torch.equal(out[st][k], ref[st][k]) for st in ("stage1", "stage2", "stage3")
                    for k in ("depth", "photometric_confidence", "variance", "prob_volume"))
        if comm is not None:
            checked(comm, timer)
        else:
            ThreadGroup(emulate).run(lambda c: checked(c, timer if c.rank == 0 else None))
        torch.cuda.synchronize()
    from damvsnet_amd.dist import max_over_ranks
    el = max_over_ranks(el, device=coll_device(device)) if comm is not None else el
    return {"ms_per_map": round(el / steps * 1e3, 3), "ranks": world, "warp": warp,
            "transport": "rccl" if comm is not None else "threads on one GPU (rehearsal)",
            "bitwise_vs_unsharded": res.get("bitwise_vs_unsharded"),
            "phases_rank0_ms": {k: round(sum(v), 3) for k, v in timer.per_phase_ms().items()}}


def latency_b1(net, imgs, proj, dv, ins, steps=10):
    """Single-view latency (SURVEY.md 8(d) 'B=1 for latency'): the first batch element alone, HIP
    events around each step and phase; reported beside the throughput line, never as `value`."""
    one = lambda x: x[:1] if torch.is_tensor(x) else {k: v[:1] for k, v in x.items()}
    imgs, proj, dv, ins = one(imgs), one(proj), one(dv), one(ins)
    with torch.no_grad():
        for _ in range(2):
            net(imgs, proj, dv, ins)
        torch.cuda.synchronize()
        timer = StageTimer()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            net(imgs, proj, dv, ins, stage_hook=timer, check_range=False)
        e1.record()
        torch.cuda.synchronize()
        net.DepthNet.check_range()
    return {"ms_per_map": round(e0.elapsed_time(e1) / steps, 3),
            "ms_per_stage": {k: round(statistics.mean(v), 3) for k, v in timer.per_phase_ms().items()}}


def warp_roofline(net, imgs, proj, dv, stage, dtype, iters=20):
    """Time the product-path fused warp+aggregation kernel of one stage alone (HIP events on the
    stream it is launched on): features in the stage's gather layout, cameras and the pipeline's hypotheses
    (stage >= 1: refined from the previous stage's depth and variance) prepared outside the loop.

    Algorithmic bytes per launch: e * (N*C*h*w [features, read
    once] + C*D*h*w [volume write]) + 4*D*h*w [fp32 hypotheses] + 4*B*(N-1)*12 [cameras].
    """
    from damvsnet_amd import _capi
    from damvsnet_amd.depthnet import to_nhwc
    from damvsnet_amd.engine import hypotheses, proj_prepare, block_channels, warp_blocked
    name = "stage%d" % (stage + 1)
    B, N, _, H, W = imgs.shape
    scale = (4, 2, 1)[stage]
    with torch.no_grad():
        feats = net.extract_features(imgs)
        fs = [f[name].to(dtype).contiguous() if net.frontend_impl == "hip" else to_nhwc(f[name], dtype)
              for f in feats]
        blocked = warp_blocked(fs[0].shape[-1], fs[0].element_size())
        fb = block_channels(fs) if blocked else fs
        layout = _capi.DAMVS_LAYOUT_CBLOCK if blocked else _capi.DAMVS_LAYOUT_NHWC
        if stage == 0:
            hyps = hypotheses(dv, net.ndepths[stage], H, W, scale)
        else:  # the pipeline's hypotheses: refined around the previous stage's depth by its uncertainty
            prev = net(imgs, proj, dv)["stage%d" % stage]
            hyps = hypotheses(dv, net.ndepths[stage], H, W, scale, prev["depth"], prev["variance"])
        rt = proj_prepare(proj[name])
        eng = net.DepthNet.engine(stage, net.cost_regularization[stage], imgs.device)
        eng.warp_aggregate(fb, None, hyps, rt=rt, layout=layout)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            eng.warp_aggregate(fb, None, hyps, rt=rt, layout=layout)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    D = net.ndepths[stage]
    h, w, C = fs[0].shape[1], fs[0].shape[2], fs[0].shape[3]
    return ms, warp_alg_bytes(B, N, C, D, h, w, 2 if dtype == torch.bfloat16 else 4)


def pmc_traffic(config, batch, kernel_substr="warp_aggregate", dtype=None):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC summary
    (profiles/<round>/pmc_*.json, produced by tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE,
    the gfx950 correction of MI355X_MICROARCH.md), or None."""
    import glob
    # preferred: the kernel as the pipeline runs it (tools/pmc_warp_inpipe.py: FETCH_SIZE x2 + WRITE_SIZE of the
    # in-pipeline launches, whose per-pixel hypotheses scatter the gathers far more than kbench's)
    sfx = "_f32" if dtype == "f32" else ""
    inpipe = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_warp_inpipe_%s_b%d%s.json" % (config, batch, sfx))))
    if inpipe and kernel_substr == "warp_aggregate":
        with open(inpipe[-1]) as f:
            p = json.load(f)["summary"]["pipeline"]
        if "fetch_bytes_x2_gfx950" in p and "write_bytes" in p:
            return {"bytes": int(p["fetch_bytes_x2_gfx950"] + p["write_bytes"]),
                    "raw_bytes": int(p["fetch_bytes_raw"] + p["write_bytes"]),
                    "read_bytes_by_request_size": int(p["read_bytes_by_request_size"]) if "read_bytes_by_request_size" in p
                    else None,
                    "source": os.path.relpath(inpipe[-1], REPO) + " (in-pipeline launches)"}
    if dtype == "f32":
        return None
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_%s_%s_b%d.json" % (kernel_substr, config, batch))))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return {"bytes": int(d["hbm_bytes_per_launch"]), "source": os.path.relpath(files[-1], REPO)}


def cpu_baseline(cfg, budget_s=60.0):
    """The oracle (PyTorch CPU restatement of the reference forward, fp32) on this host's cores."""
    from oracle import mvs_oracle as O
    H, W, N, nd, _, _ = CONFIGS[cfg]
    # the GPU box's CPU share is what OMP_NUM_THREADS says (affinity shows the whole machine)
    cores = int(os.environ.get("OMP_NUM_THREADS") or min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.weights import synthetic_state_dict, apply_bn_stats
    sd = synthetic_state_dict(CascadeMVSNet(ndepths=list(nd)).state_dict(), 0)
    g = np.load(os.path.join(REPO, "tests", "golden", "forward_cfgB_640x512.npz"))
    sd = apply_bn_stats(sd, {k[4:]: g[k] for k in g.files if k.startswith("bn::")})
    imgs, proj, dv, _ = make_inputs(1, N, H, W)
    times = []
    t_start = time.time()
    with torch.no_grad():
        O.cascade_forward(sd, imgs, proj, dv, nd, "adaptive")  # warm-up (allocator, thread pool), not timed
        t_warm = time.time() - t_start
        while True:  # the median of at least 3 timed forwards (more while the budget allows)
            t0 = time.time()
            O.cascade_forward(sd, imgs, proj, dv, nd, "adaptive")
            times.append(time.time() - t0)
            if len(times) >= 3 and time.time() - t_start + times[-1] > budget_s:
                break
            if len(times) >= 5:
                break
    t = statistics.median(times)
    return {"value": round(1.0 / t, 5), "unit": "depth maps/s", "cores": cores, "kind": "port",
            "sample": "1 warm-up + %d timed full forwards at %s (B=1, fp32, PyTorch CPU restatement of the reference), "
                      "median %.2f s (min %.2f, max %.2f; warm-up %.2f s)"
                      % (len(times), cfg, t, min(times), max(times), t_warm)}


def warp_alg_bytes(B, N, C, D, h, w, es):
    """Algorithmic bytes of one warp + aggregation launch: features read once, the volume written
    once, fp32 hypotheses, cameras."""
    return es * (N * C * h * w * B + C * D * h * w * B) + 4 * D * h * w * B + 4 * B * (N - 1) * 12


def parity_path(args, nd, device, imgs, proj, dv, ins, world, steps=20, warmup=3):
    """The fp32 path (fp32 storage and regression, conv products as split-f16 MFMAs) timed like the headline steps:
    the path that holds north_star's 1e-3 per-pixel depth gate and the fp32 parity suites (tests/test_gpu_parity.py
    fp32 gates incl. the end-to-end conditioning gates, tests/test_gpu_fullsize.py fp32 at cfgC/D/E). Its own
    rooflines come from a one-stream attribution pass after the timed steps (HIP events inside
    damvs_stage_forward_probed), priced at the split-f16 ceiling (2.5 PFLOP/s / 3) for the MFMA-bound groups."""
    from damvsnet_amd.dist import max_over_ranks
    net, _ = build_model(nd, torch.float32, device, args.frontend)
    with torch.no_grad():
        for _ in range(warmup):
            net(imgs, proj, dv, ins, **stream_kw(args))
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):  # the range status accumulates over the steps and is read once after them
            net(imgs, proj, dv, ins, check_range=False, **stream_kw(args))
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        elapsed = max_over_ranks(time.perf_counter() - t0, device=coll_device(device))
        net.DepthNet.check_range()  # raises DamvsRangeError if any timed forward produced non-finite maps
        probes = ProbeRecorder()
        net.DepthNet.probe = probes
        for _ in range(3):
            net(imgs, proj, dv, ins, check_range=False)
        torch.cuda.synchronize()
        net.DepthNet.check_range()
        net.DepthNet.probe = None
    del net
    torch.cuda.empty_cache()
    maps = steps * args.batch * world
    H, W, N = imgs.shape[3], imgs.shape[4], imgs.shape[1]
    per_stage = probes.per_stage_ms()
    hp = hot_path_roofline(per_stage, H, W, N, nd, args.batch, "f32")
    from damvsnet_amd import costmodel as CM
    D2, h2, w2 = nd[1], H // 2, W // 2
    warp_ms = per_stage[1]["warp"]
    alg = warp_alg_bytes(args.batch, N, 16, D2, h2, w2, 4)
    unet_ms = per_stage[1]["unet"]
    unet_flops = args.batch * CM.stage_cost(N, 16, D2, h2, w2, 4)["unet"][1]
    tr = pmc_traffic(args.config, args.batch, dtype="f32")
    mf = pmc_mfma(args.config, args.batch, dtype="f32")
    roof = {"kernel": "warp_split_kernel<float, 16> stage 2 (fused homography warp + adaptive aggregation, 4 lanes per "
                      "voxel: 64-byte fp32 pixels), in-pipeline launch time (HIP events inside "
                      "damvs_stage_forward_probed, one-stream attribution pass)",
            "bound": "hbm", "achieved": round(alg / (warp_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / (warp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ms_per_launch": round(warp_ms, 4),
            "algorithmic_bytes": int(alg), "traffic": tr["bytes"] if tr else None,
            "traffic_raw": tr.get("raw_bytes") if tr else None,
            "traffic_source": ("committed PMC profile " + tr["source"]) if tr else None}
    mroof = {"kernel": "stage-2 CostRegNet (10 conv layers, split-f16 MFMAs), in-pipeline time",
             "bound": "mfma", "achieved": round(unet_flops / (unet_ms * 1e-3) / 1e12, 2),
             "peak": CM.MFMA_PEAK["f32"] / 1e12, "unit": "TFLOP/s",
             "frac": round(unet_flops / (unet_ms * 1e-3) / CM.MFMA_PEAK["f32"], 4), "ms": round(unet_ms, 4),
             "algorithmic_flops": int(unet_flops),
             "peak_note": "split-f16 ceiling: every fp32 product is three f16 MFMAs, 2.5 PFLOP/s dense f16 / 3"}
    return {"value": round(maps / elapsed, 4), "unit": "depth maps/s", "ms_per_step": round(elapsed / steps * 1e3, 3),
            "steps": steps, "warmup": warmup, "dtype": "f32", "streams": args.streams, "stream_offset": eff_offset(args, "f32"),
            "batch_per_gpu": args.batch,
            "range_status": "ok: every stage of every timed forward finite (damvs_stage_status, read after the steps)",
            "compute": "fp32 storage, fp32 warp / aggregation / regression; every conv product as split-f16 MFMAs "
                       "(x = hi + lo, hi*hi + hi*lo + lo*hi, fp32 accumulation; damvsnet_amd/csrc/damvs_device.h)",
            "gates": "north_star: depth within 1e-3 relative at every pixel on identical inputs "
                     "(tests/test_gpu_fullsize.py fp32 at cfgC/D/E, tests/test_gpu_parity.py stage-isolated), and the "
                     "end-to-end fp32-vs-fp64 conditioning gates (tests/test_gpu_parity.py _check_forward_e2e)",
            "roofline": roof, "mfma_roofline": mroof, "hot_path_roofline": hp, "mfma_utilisation": mf}


def eff_offset(args, dname):
    """The sub-batch stream offset a forward of this dtype runs with (CascadeMVSNet.forward stream_offset="auto")."""
    if args.streams < 2:
        return None
    if args.stream_offset:
        return None if args.stream_offset == "none" else args.stream_offset
    return "stage1.hypotheses" if dname == "f32" else None


def stream_kw(args):
    """The forward's sub-batch stream arguments (the offset only when given)."""
    kw = {"streams": args.streams}
    if args.stream_offset:
        kw["stream_offset"] = None if args.stream_offset == "none" else args.stream_offset
    return kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfgC", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=4,
                    help="depth maps (reference views) per GPU per step; default 4 = the reference's own "
                         "test batch (scripts/test.sh:25 --batch_size=4), SURVEY.md 8(d) 'B=4 for throughput'")
    ap.add_argument("--stream-offset", default=None,
                    help="start sub-batch i + 1 when sub-batch i reaches this stage-hook point (e.g. stage1.hypotheses, "
                         "'none'); default: the model's (fp32: stage1.hypotheses, bf16: none)")
    ap.add_argument("--streams", type=int, default=2,
                    help="sub-batches of the per-GPU batch on concurrent HIP streams in the timed steps "
                         "(bitwise the one-stream result; ms_per_stage / rooflines come from a one-stream pass)")
    ap.add_argument("--dtype", choices=["bf16", "f32"], default=None,
                    help="override the config's compute dtype (cfgC is bf16 in BASELINE.json; f32 = the parity path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-path", action="store_true",
                    help="bf16 runs: skip the fp32 parity-path block (20 timed steps of the fp32 forward)")
    ap.add_argument("--frontend", default="hip", choices=["hip", "torch"], help="2D front-end implementation")
    ap.add_argument("--cpu-budget", type=float, default=60.0,
                    help="seconds of CPU-baseline forwards beyond the warm-up and the 3 timed ones")
    ap.add_argument("--shard", choices=["depth", "rows", "gather"], default=None,
                    help="measure the depth-sharded latency mode (one map over all ranks) instead of replicas")
    ap.add_argument("--emulate", type=int, default=1, help="with --shard on one GPU: P ranks as threads")
    ap.add_argument("--no-shard-latency", action="store_true",
                    help="N > 1: skip the depth-sharded latency block after the throughput steps")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import datetime
        torch.cuda.set_device(local)
        # a finite collective timeout: a rank that fails inside the depth-sharded block cannot leave its peers
        # waiting in a P2P exchange forever (the NCCL watchdog aborts the group instead)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local),
                                             timeout=datetime.timedelta(seconds=300))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    H, W, N, nd, dtype, desc = CONFIGS[args.config]
    if args.dtype:
        dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
        desc = desc.rsplit(",", 1)[0] + ", " + args.dtype
    dname = "bf16" if dtype == torch.bfloat16 else "f32"
    net, _ = build_model(nd, dtype, device, args.frontend)
    if args.shard:
        from damvsnet_amd.sharded import TorchComm
        res = sharded_latency(net, H, W, N, device, comm=TorchComm() if world > 1 else None, emulate=args.emulate,
                              warp=args.shard, steps=args.steps, warmup=args.warmup)
        if rank == 0:
            ms = res["ms_per_map"]
            print(json.dumps({
                "metric": "depth maps/sec (full CascadeMVSNet forward, one map over all ranks)",
                "value": round(1e3 / ms, 4), "unit": "depth maps/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
                "vs_baseline": None, "dtype": dname, "data": "synthetic",
                "config": {"workload": "%s: %s" % (args.config, desc), "batch_per_gpu": 1, "global_batch": 1,
                           "height": H, "width": W, "views": N, "ndepths": list(nd),
                           "parallelism": "depth-sharded x%d (%s warp)" % (res["ranks"], args.shard)},
                "depth_sharded": res}), flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    imgs, proj, dv, ins = make_inputs(args.batch, N, H, W, device, seed=rank)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    pp = None
    # DAMVS_BENCH_PARITY_FIRST=1 (A/B of the in-process order): the parity path before the headline steps
    parity_first = os.environ.get("DAMVS_BENCH_PARITY_FIRST", "0") == "1"
    if parity_first and dtype == torch.bfloat16 and not args.no_parity_path:
        pp = parity_path(args, nd, device, imgs, proj, dv, ins, world)
    with torch.no_grad():
        for _ in range(args.warmup):
            net(imgs, proj, dv, ins, **stream_kw(args))
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):  # the range status accumulates over the steps and is read once after them
            net(imgs, proj, dv, ins, check_range=False, **stream_kw(args))
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        net.DepthNet.check_range()  # raises DamvsRangeError if any timed forward produced non-finite maps
        # attribution pass, one stream (per-phase and per-kernel-group times are not separable when sub-batches
        # overlap): HIP events at the phase boundaries and inside damvs_stage_forward_probed
        timer = StageTimer()
        probes = ProbeRecorder()
        net.DepthNet.probe = probes
        for _ in range(min(args.steps, 5)):
            net(imgs, proj, dv, ins, stage_hook=timer, check_range=False)
        torch.cuda.synchronize()
        net.DepthNet.check_range()
        net.DepthNet.probe = None
    from damvsnet_amd.dist import max_over_ranks
    elapsed = max_over_ranks(elapsed, device=coll_device(device))
    maps = args.steps * args.batch * world
    if not parity_first and dtype == torch.bfloat16 and not args.no_parity_path:  # every rank takes part (max over ranks)
        pp = parity_path(args, nd, device, imgs, proj, dv, ins, world)
    phases = {k: round(statistics.mean(v), 3) for k, v in timer.per_phase_ms().items()}

    result = None
    if rank == 0:
        lat = latency_b1(net, imgs, proj, dv, ins)
        per_stage = probes.per_stage_ms()
        hp = hot_path_roofline(per_stage, H, W, N, nd, args.batch, dname)
        iso_ms, alg = warp_roofline(net, imgs, proj, dv, 1, dtype)
        pipe_ms = per_stage[1]["warp"]
        achieved = alg / (pipe_ms * 1e-3) / 1e9
        tr = pmc_traffic(args.config, args.batch, dtype=dname)  # committed PMC profiles of this dtype
        result = {
            "metric": "depth maps/sec (full CascadeMVSNet forward)",
            "value": round(maps / elapsed, 4),
            "unit": "depth maps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dname,
            "data": "synthetic (seeded DTU-like images/cameras, synthetic weights with calibrated BN stats)",
            "config": {"workload": "%s: %s" % (args.config, desc), "batch_per_gpu": args.batch,
                       "frontend": args.frontend,
                       "global_batch": args.batch * world, "height": H, "width": W, "views": N,
                       "ndepths": list(nd), "streams": args.streams, "stream_offset": eff_offset(args, dname),
                       "parallelism": "replicas x%d (reference views sharded over ranks)" % world},
            "ms_per_stage": phases,
            "latency_b1": lat,
            "roofline": {"kernel": "warp_split_kernel stage2 (fused homography warp + adaptive aggregation, 2 lanes "
                                   "per voxel), in-pipeline launch time (HIP events inside damvs_stage_forward_probed)",
                         "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr["bytes"] if tr else None,
                         "traffic_raw": tr.get("raw_bytes") if tr else None,
                         "traffic_note": "traffic = FETCH_SIZE x 2 + WRITE_SIZE per launch: on gfx950 every L2 read "
                                         "request is a 128-B line fill counted as 64 B, for streaming reads and for "
                                         "16/32/64-B record gathers alike (profiles/r03/pmc_fetch_calibration.json); "
                                         "traffic_raw = FETCH_SIZE + WRITE_SIZE as rocprofv3 reports them",
                         "traffic_source": ("committed PMC profile " + tr["source"]) if tr else None,
                         "ms_per_launch": round(pipe_ms, 4), "launch": "whole batch (B=%d) on one stream, the "
                         "attribution pass after the timed steps; rocprof check: tools/prof_roofline_kernel.py" % args.batch,
                         "algorithmic_bytes": int(alg),
                         "isolated_ms_per_launch": round(iso_ms, 4),
                         "isolated_frac": round(alg / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "hot_path_roofline": hp,
            "range_status": "ok: every stage of every timed forward finite (damvs_stage_status, read after the steps)",
            "mfma_utilisation": pmc_mfma(args.config, args.batch, dtype=dname),
        }
        if pp is not None:
            result["parity_path"] = pp
    import threading
    guard, printed = None, threading.Event()
    if world > 1 and not args.no_shard_latency:
        torch.distributed.barrier()  # rank 0's line is built: every rank starts its guard from here
        # The depth-sharded modes below are the run's only RCCL P2P traffic. Should one of them hang (the NCCL
        # watchdog would abort the process at the collective timeout, losing the throughput line), a timer prints
        # rank 0's line without them (unless it is out already) and ends the process with status 3.
        line = json.dumps(dict(result, depth_sharded={"error": "timed out after %d s" % SHARD_GUARD_S})) if rank == 0 else None

        def _guard():  # a hung exchange is a failed run: the line goes out, the exit status says so
            if line is not None and not printed.is_set():
                print(line, flush=True)
            os._exit(3)
        guard = threading.Timer(SHARD_GUARD_S, _guard)
        guard.daemon = True
        guard.start()
    shard_blocks = {}
    if world > 1 and not args.no_shard_latency:  # every rank takes part
        from damvsnet_amd.sharded import TorchComm
        # "depth": the recommended all-to-all + H-slab U-Net; "gather": north_star's literal volume all-gather
        for key, mode in (("depth_sharded", "depth"), ("depth_sharded_gather", "gather")):
            err, blk = None, None
            try:
                blk = sharded_latency(net, H, W, N, device, comm=TorchComm(), warp=mode)
            except Exception as ex:  # reported, never fatal for the throughput line
                err = repr(ex)[:300]
            # every rank leaves the block knowing whether any rank failed (a failure after the last exchange would
            # otherwise go unnoticed by the peers); a failure before an exchange ends at the collective timeout
            flag = torch.tensor([1 if err else 0], device=coll_device(device))
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.SUM)
            if int(flag.item()):
                blk = {"error": err or "failed on %d other rank(s)" % int(flag.item()), "failed_ranks": int(flag.item())}
            shard_blocks[key] = blk

    if rank == 0:
        result.update(shard_blocks)
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.config, args.cpu_budget)
        printed.set()
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    if guard is not None:
        guard.cancel()


if __name__ == "__main__":
    main()
