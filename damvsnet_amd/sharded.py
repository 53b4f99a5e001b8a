"""Depth-sharded execution: one depth map's cascade stage over the P GPUs of a group (BASELINE.json north_star,
SURVEY.md section 8(e)). The throughput mode stays replicas (damvsnet_amd.dist); this is the latency mode for
one reference view.

Per stage (DepthNet.forward, models/cas_mvsnet.py:18-134), on rank r of P:

1. Cost volume sharded along the depth-hypothesis axis (``warp="depth"``, the north-star partitioning): rank r
   builds the aggregated volume of planes [d0_r, d1_r) over the whole image. The warp + aggregation is per voxel
   (models/cas_mvsnet.py:42-87): no communication; every rank holds all N feature maps.
2. All-to-all re-shard to H-slabs: rank q receives from every rank its planes of rows [y0_q - 8, y1_q + 8) of the
   image (its slab plus an 8-row halo). The U-Net cannot run D-sharded: its 3x3x3 kernels and three stride-2
   levels couple all depth planes, and D/P is not a multiple of 8 at stages 2-3.
3. CostRegNet (models/module.py:510-541) on the haloed slab, layer by layer. Halos of 8 / 4 / 2 / 1 rows at levels
   0-3 keep the stride-2 row parity of every level aligned with the whole-image U-Net, so each layer is the
   whole-tensor kernel unchanged (damvs_costreg_layer); after every layer the halo rows are refreshed from the
   neighbouring slabs (P2P) and zeroed outside the image (the whole-image convolution's zero padding). The batch
   runs as two halves so one half's halo transfer overlaps the other half's layer (_costreg_sharded).
4. Prob conv + softmax regression (models/cas_mvsnet.py:105-124) locally: the softmax is over D, per pixel.
5. All-gather of the slabs' depth / confidence / variance rows (and prob volume), one collective
   (all_gather_into_tensor over RCCL) of slabs padded to the tallest: every rank then holds the stage output, which
   the next stage's hypotheses and GeoFeatureFusion read whole.

``warp="rows"`` builds each rank's haloed slab of the volume directly (damvs_warp_aggregate_rows) and skips the
all-to-all: the same voxels, with redundant warp work on the halo rows instead of communication.

``warp="gather"`` is north_star's literal partitioning: the D-sharded volumes of step 1 are all-gathered along D
(one all_gather_into_tensor over RCCL) before the U-Net, which then runs replicated on the whole volume, followed by
the regression; no further communication. Only the warp is divided by P, the volume crosses xGMI once per rank
(7/8 of it received at P = 8), and every rank ends with the stage output.

Results equal the unsharded stage: every voxel of the warp and every output of a layer is computed by the same
kernel arithmetic from the same inputs (tests/test_sharded.py, tests/test_gpu_sharded.py). The front-end
(FeatureNet, GeoFeatureFusion) and the hypotheses run replicated on every rank.

fp32 magnitude slots (include/damvs.h DAMVS_AMAX_SLOT_BYTES): the fp32 path splits every activation tensor at a
scale set by its largest magnitude, which the unsharded stage records with atomics as its kernels store. Sharded, each
rank measures the part of a tensor it owns (its depth planes of the volume, or its slab's rows without the halos, which
hold partial sums until they are refreshed) and one all-gather of those maxima gives every rank the whole tensor's:
the same scale, so the same bits as the unsharded stage.

Communication goes through a ``Comm``: ``TorchComm`` (torch.distributed; backend "nccl" = RCCL over xGMI, "gloo"
for CPU tests) or ``ThreadGroup`` (P ranks as threads of one process: single-device rehearsal and tests).
"""
from __future__ import annotations

import threading

import torch

from . import _capi

HALO = 8  # level-0 halo rows; level l carries HALO >> l (the U-Net has three stride-2 levels)
# U-Net schedule: (layer, input tensor, output tensor, output level); "v" = volume, "cN" = convN output
_STEPS = ((0, "v", 0, 0), (1, 0, 1, 1), (2, 1, 2, 1), (3, 2, 3, 2), (4, 3, 4, 2), (5, 4, 5, 3), (6, 5, 6, 3),
          (7, 6, 4, 2), (8, 4, 2, 1), (9, 2, 0, 0))
# fp32 magnitude slot of each layer's input and output (capi.cpp kLayerSlots): 0 = volume, 1..7 = c0..c6, 8 / 9 = the
# conv7 / conv9 skip sums; conv11's output feeds the exact-fp32 prob conv (no slot)
_SLOTS = ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, None))


def _new_slots(eng, B):
    """Zeroed magnitude slots [tensor][batch element][words] of an fp32 engine (None: bf16, or an engine without
    slots)."""
    if getattr(eng, "dtype", None) != torch.float32 or not hasattr(eng, "new_slots"):
        return None
    return eng.new_slots(B)


def _fold_owned(comm: "Comm", slots, parts):
    """slots[b] := max |x[b]| over every rank's ``parts`` (the [B, ...] tensor pieces this rank owns; None entries
    skipped): one all-gather of the per-rank, per-sample maxima. A slot holds the float's bits in its first word."""
    B, dev = slots.shape[0], slots.device
    m = torch.zeros(B, dtype=torch.float32, device=dev)
    for p in parts:
        if p is not None and p.numel():
            m = torch.maximum(m, p.abs().reshape(B, -1).amax(1).float())
    got = comm.all_gather(m.view(torch.int32))
    slots.zero_()
    slots[:, 0].copy_(torch.stack([g.to(dev) for g in got]).amax(0))


def slab_rows(h: int, P: int):
    """Row boundaries [y_0 = 0, ..., y_P = h] of the P H-slabs: multiples of 8 rows (whole level-3 rows), as
    even as possible. Needs h / 8 >= P."""
    n8 = h // 8
    base, extra = divmod(n8, P)
    if h % 8 or base < 1:
        raise ValueError("h = %d must be a multiple of 8 with at least 8 rows per rank (P = %d)" % (h, P))
    ys = [0]
    for r in range(P):
        ys.append(ys[-1] + 8 * (base + (1 if r < extra else 0)))
    return ys


def depth_planes(D: int, P: int):
    """Plane boundaries [0, ..., D] of the P depth shards (as even as possible; a shard may be empty)."""
    base, extra = divmod(D, P)
    ds = [0]
    for r in range(P):
        ds.append(ds[-1] + base + (1 if r < extra else 0))
    return ds


# ----------------------------------------------------------------------------- communicators

class Comm:
    """Point-to-point exchange between the ranks of a group. ``exchange(ops)``: ops = [(peer, send or None,
    recv or None)]; all of them complete (stream-ordered for device tensors) before it returns. A rank's op list
    holds at most one send and one receive per peer; peer == rank copies send into recv."""
    rank = 0
    world = 1

    def exchange(self, ops):
        raise NotImplementedError

    def exchange_start(self, ops):
        """Start ``exchange(ops)``; the returned handle's ``wait()`` completes it (stream-ordered for device tensors).
        Communicators without asynchronous transfers complete it here."""
        self.exchange(ops)
        return _Done()

    def all_gather(self, t):
        """Every rank's ``t`` (one shape on all ranks) as a list indexed by rank."""
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.exchange([(q, t, outs[q]) for q in range(self.world)])
        return outs


class _Done:
    def wait(self):
        pass


class _TorchPending:
    def __init__(self, works, back):
        self.works, self.back = works, back

    def wait(self):
        for work in self.works:
            work.wait()  # NCCL / RCCL: the current stream waits for the transfer (the host does not block)
        for dst, src in self.back:
            dst.copy_(src)


class TorchComm(Comm):
    """torch.distributed over the default group: batched isend/irecv (RCCL groups them into one launch; the
    all-to-all of step 2 is one such batch). With gloo, device tensors are staged through host memory."""

    def __init__(self):
        import torch.distributed as dist
        self._dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self._host = dist.get_backend() == "gloo"

    def exchange(self, ops):
        self.exchange_start(ops).wait()

    def exchange_start(self, ops):
        dist = self._dist
        p2p, back = [], []
        for peer, send, recv in ops:
            if peer == self.rank:
                if recv is not None:
                    recv.copy_(send)
                continue
            if send is not None:
                p2p.append(dist.P2POp(dist.isend, send.cpu() if self._host and send.is_cuda else send, peer))
            if recv is not None:
                r = recv
                if self._host and recv.is_cuda:
                    r = torch.empty(recv.shape, dtype=recv.dtype)
                    back.append((recv, r))
                p2p.append(dist.P2POp(dist.irecv, r, peer))
        return _TorchPending(dist.batch_isend_irecv(p2p) if p2p else [], back)

    def all_gather(self, t):
        """One collective: all_gather_into_tensor (RCCL ring over xGMI) into a [world, ...] buffer; gloo gathers
        host copies."""
        dist = self._dist
        t = t.contiguous()
        src = t.cpu() if self._host and t.is_cuda else t
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src)  # ranks concatenated along dim 0
        return [p.to(t.device) for p in out.chunk(self.world, 0)]


class ThreadGroup:
    """P ranks as P threads of one process sharing a device: tensors travel through a mailbox. Kernels of all
    ranks go to the same stream, so a copy enqueued after the barrier is ordered after its producer."""

    def __init__(self, world: int):
        self.world = world
        self._barrier = threading.Barrier(world)
        self._lock = threading.Lock()
        self._box = {}

    def comm(self, rank: int) -> "ThreadComm":
        return ThreadComm(self, rank)

    def run(self, fn):
        """Run fn(comm) on every rank (one thread each); returns the per-rank results, re-raises a failure."""
        out, err = [None] * self.world, []

        def body(r):
            try:
                out[r] = fn(self.comm(r))
            except BaseException as e:  # noqa: BLE001 - propagated below
                err.append(e)
                self._barrier.abort()

        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if err:
            raise err[0]
        return out


class ThreadComm(Comm):
    def __init__(self, group: ThreadGroup, rank: int):
        self.group, self.rank, self.world = group, rank, group.world

    def exchange(self, ops):
        g = self.group
        with g._lock:
            for peer, send, _ in ops:
                if send is not None and peer != self.rank:
                    g._box[(self.rank, peer)] = send
        g._barrier.wait()
        for peer, send, recv in ops:
            if recv is not None:
                if peer == self.rank:
                    recv.copy_(send)
                else:
                    with g._lock:
                        src = g._box.pop((peer, self.rank))
                    recv.copy_(src)
        g._barrier.wait()


# ----------------------------------------------------------------------------- one sharded stage

def _halo_start(comm: Comm, t: torch.Tensor, hl: int):
    """Start refreshing the hl-row halos of a slab tensor [B][D][rows][w][C] from the neighbouring slabs; the
    returned callable completes it (and zeroes the halo rows that lie outside the image: first / last rank)."""
    r, P = comm.rank, comm.world
    R = t.shape[2]
    ops, top, bot = [], None, None
    if r > 0:
        top = torch.empty_like(t[:, :, :hl])
        ops.append((r - 1, t[:, :, hl:2 * hl].contiguous(), top))
    if r < P - 1:
        bot = torch.empty_like(t[:, :, :hl])
        ops.append((r + 1, t[:, :, R - 2 * hl:R - hl].contiguous(), bot))
    pending = comm.exchange_start(ops) if ops else _Done()

    def finish():
        pending.wait()
        del ops[:]  # the staged send buffers live until the transfer has completed
        if top is None:
            t[:, :, :hl].zero_()
        else:
            t[:, :, :hl].copy_(top)
        if bot is None:
            t[:, :, R - hl:].zero_()
        else:
            t[:, :, R - hl:].copy_(bot)
    return finish


def _costreg_sharded(comm: Comm, eng, vol, c, D: int, R: int, w: int, slots=None, rows: int = 0):
    """The U-Net on the haloed slab with each layer's halo exchange overlapped: the batch runs as two halves, and
    a half's halo transfer is in flight while the other half's layer computes (the next layer of a half waits
    only for that half's halos). Same kernels per voxel as one whole-batch launch: identical results. fp32
    (``slots``): after a layer, its output's magnitude over every rank's owned rows (``rows`` at level 0) sets the
    slot the next layer reads."""
    B = vol.shape[0]
    halves = [(0, B // 2), (B // 2, B)] if B >= 2 else [(0, B)]
    pending = [None] * len(halves)
    for (layer, src, dst, level), (sin, sout) in zip(_STEPS, _SLOTS):
        for i, (b0, b1) in enumerate(halves):
            if pending[i] is not None:
                pending[i]()  # this half's halos of the previous layer's output
            x = vol if src == "v" else c[src]
            if slots is None:
                eng.unet_layer(layer, D, R, w, x[b0:b1], c[dst][b0:b1])
            else:
                eng.unet_layer(layer, D, R, w, x[b0:b1], c[dst][b0:b1], in_slot=slots[sin][b0:b1])
            pending[i] = _halo_start(comm, c[dst][b0:b1], HALO >> level)
        if slots is not None and sout is not None:
            hl = HALO >> level
            _fold_owned(comm, slots[sout], [c[dst][:, :, hl:hl + (rows >> level)]])
    for fin in pending:
        fin()


def sharded_stage(comm: Comm, eng, feats, layout, rt, hyps, h: int, w: int, warp: str = "depth",
                  want_prob: bool = True, hook=None):
    """One DepthNet stage of B depth maps over the group: see the module docstring.

    eng     StageEngine of the stage (or any object with its warp_aggregate / warp_aggregate_rows / unet_layer /
            unet_buffers / regress_c0 methods)
    feats   the N feature maps as the engine takes them (whole images, every rank), ``layout`` their layout
    rt      proj_prepare output [B][N-1][12];  hyps: [B][D][h][w] float (every rank)
    Returns (depth, conf, var, prob) whole-image [B][h][w] (prob [B][D][h][w] or None) on every rank."""
    hook = hook or (lambda name: None)
    if warp not in ("depth", "rows", "gather"):
        raise ValueError("warp must be 'depth', 'rows' or 'gather'")
    r, P = comm.rank, comm.world
    B, D = hyps.shape[:2]
    C = eng.C
    dev, dt = hyps.device, eng.dtype
    if warp == "gather":
        return _gathered_stage(comm, eng, feats, layout, rt, hyps, h, w, want_prob, hook)
    ys = slab_rows(h, P)
    y0, y1 = ys[r], ys[r + 1]
    R = (y1 - y0) + 2 * HALO
    lo, hi = max(0, y0 - HALO), min(h, y1 + HALO)  # image rows inside my haloed window
    top = lo - (y0 - HALO)                          # ... start at this slab row
    n = hi - lo

    slots = _new_slots(eng, B)
    hyps_s = torch.empty(B, D, R, w, device=dev, dtype=hyps.dtype)
    hyps_s[:, :, :top].zero_()
    hyps_s[:, :, top + n:].zero_()
    hyps_s[:, :, top:top + n].copy_(hyps[:, :, lo:hi])
    vol = torch.empty(B, D, R, w, C, device=dev, dtype=dt)
    vol[:, :, :top].zero_()
    vol[:, :, top + n:].zero_()

    hook("warp")
    if warp == "rows":
        eng.warp_aggregate_rows(feats, rt, hyps_s, h, lo, n, top, vol, layout=layout)
        if slots is not None:  # the rows this rank computed (halo rows too: exact volume rows)
            _fold_owned(comm, slots[0], [vol[:, :, top:top + n]])
    else:
        ds = depth_planes(D, P)
        d0, d1 = ds[r], ds[r + 1]
        part = None
        if d1 > d0:
            part = eng.warp_aggregate(feats, None, hyps[:, d0:d1].contiguous(), rt=rt, layout=layout)
        if slots is not None:  # this rank's depth planes
            _fold_owned(comm, slots[0], [part])
        hook("all_to_all")
        ops, recvs = [], []
        for q in range(P):
            qlo, qhi = max(0, ys[q] - HALO), min(h, ys[q + 1] + HALO)
            nq = ds[q + 1] - ds[q]
            recv = torch.empty(B, nq, n, w, C, device=dev, dtype=dt) if nq > 0 else None
            send = part[:, :, qlo:qhi].contiguous() if part is not None else None
            ops.append((q, send, recv))
            recvs.append(recv)
        comm.exchange(ops)
        for q in range(P):
            if recvs[q] is not None:
                vol[:, ds[q]:ds[q + 1], top:top + n].copy_(recvs[q])

    hook("costreg")
    c = eng.unet_buffers(B, D, R, w)
    _costreg_sharded(comm, eng, vol, c, D, R, w, slots, y1 - y0)

    hook("regress")
    depth, conf, var, prob = eng.regress_c0(c[0], hyps_s, want_prob=want_prob)

    hook("all_gather")
    core = slice(HALO, HALO + (y1 - y0))
    parts = [depth[:, None, core], conf[:, None, core], var[:, None, core]]
    if want_prob:
        parts.append(prob[:, :, core])
    # one all-gather of equal-size buffers (slabs differ by at most 8 rows: padded to the tallest)
    rmax = max(ys[q + 1] - ys[q] for q in range(P))
    K = 3 + (prob.shape[1] if want_prob else 0)
    mine = torch.zeros(B, K, rmax, w, device=dev, dtype=depth.dtype)  # [B][3 (+D)][rows][w]
    mine[:, :, :y1 - y0].copy_(torch.cat(parts, 1))
    got = comm.all_gather(mine)
    full = torch.cat([got[q][:, :, :ys[q + 1] - ys[q]] for q in range(P)], 2)
    depth, conf, var = full[:, 0].contiguous(), full[:, 1].contiguous(), full[:, 2].contiguous()
    prob = full[:, 3:].contiguous() if want_prob else None
    hook("end")
    return depth, conf, var, prob


def _gathered_stage(comm: Comm, eng, feats, layout, rt, hyps, h: int, w: int, want_prob: bool, hook):
    """warp="gather": D-sharded warp, all-gather of the volume along D, U-Net + regression replicated."""
    r, P = comm.rank, comm.world
    B, D = hyps.shape[:2]
    ds = depth_planes(D, P)
    d0, d1 = ds[r], ds[r + 1]
    dmax = max(ds[q + 1] - ds[q] for q in range(P))
    hook("warp")
    # equal-size buffers for one collective: every shard padded to the deepest, planes outermost so a shard is
    # one contiguous block ([dmax][B][h][w][C])
    mine = torch.zeros(dmax, B, h, w, eng.C, device=hyps.device, dtype=eng.dtype)
    if d1 > d0:
        part = eng.warp_aggregate(feats, None, hyps[:, d0:d1].contiguous(), rt=rt, layout=layout)
        mine[:d1 - d0].copy_(part.transpose(0, 1))
        del part
    hook("all_gather")
    got = comm.all_gather(mine)
    vol = torch.cat([got[q][:ds[q + 1] - ds[q]] for q in range(P)], 0).transpose(0, 1).contiguous()
    del got, mine
    hook("costreg")
    c = eng.unet_buffers(B, D, h, w)
    slots = _new_slots(eng, B)
    if slots is None:
        for layer, src, dst, _level in _STEPS:
            eng.unet_layer(layer, D, h, w, vol if src == "v" else c[src], c[dst])
    else:  # every rank holds the whole volume: the kernels' own magnitude records are the whole tensors'
        eng.tensor_amax(vol, slots[0])
        for (layer, src, dst, _level), (sin, sout) in zip(_STEPS, _SLOTS):
            eng.unet_layer(layer, D, h, w, vol if src == "v" else c[src], c[dst], in_slot=slots[sin],
                           out_slot=None if sout is None else slots[sout])
    hook("regress")
    depth, conf, var, prob = eng.regress_c0(c[0], hyps, want_prob=want_prob)
    hook("end")
    return depth, conf, var, prob


class DepthShardedDepthNet:
    """Drop-in stage runner for CascadeMVSNet.forward(..., depthnet=...): the HIP engine of the model's DepthNet,
    features prepared as damvs_stage_forward prepares them (compute dtype, channel blocking), then
    sharded_stage over ``comm``."""

    def __init__(self, net, comm: Comm, warp: str = "depth", want_prob: bool = True, hook=None):
        self.net, self.comm, self.warp, self.want_prob, self.hook = net, comm, warp, want_prob, hook

    def __call__(self, stage_idx, feats_nhwc, proj_matrices, depth_values, cost_regularization):
        from .engine import block_channels, proj_prepare, warp_blocked
        dn = self.net.DepthNet
        dev = depth_values.device
        eng = dn.engine(stage_idx, cost_regularization, dev)
        feats = [f if f.dtype == dn.compute_dtype and f.is_contiguous() else f.to(dn.compute_dtype).contiguous()
                 for f in feats_nhwc]
        B, h, w, C = feats[0].shape
        layout = _capi.DAMVS_LAYOUT_NHWC
        if warp_blocked(C, feats[0].element_size(), len(feats)):
            feats, layout = block_channels(feats), _capi.DAMVS_LAYOUT_CBLOCK
        hyps = depth_values.float().contiguous()
        rt = proj_prepare(proj_matrices.float().contiguous())
        depth, conf, var, prob = sharded_stage(self.comm, eng, feats, layout, rt, hyps, h, w, self.warp,
                                               self.want_prob, self.hook)
        return {"depth": depth, "photometric_confidence": conf, "variance": var, "prob_volume": prob,
                "depth_values": depth_values}
