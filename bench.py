"""Headline benchmark: fields-of-view/sec of the 2080x2080x5ch illum -> seg -> feat pipeline.

Workload (BASELINE.json configs[1]): one 384-well plate, 1 FOV/well, 2080x2080x5ch synthetic,
processed in steps of --batch FOVs that are resident in HBM when the timed region starts.  One
step = flat-field + QC (PercentMaximal, PowerLogLogSlope) -> Cellpose-restated segmentation
(CPnet at the fp32 network's precision on split-fp16 MFMA kernels + HIP
post-processing) -> Cells/Cytoplasm -> object tables -> shape/intensity/texture
features for Nuclei, Cells, Cytoplasm -> results copied to the host.  Multi-GPU: one process per
GPU, FOVs (wells) sharded by rank, no data-path collective (scaling "weak").

  python bench.py [--gpus N --steps K --warmup W --batch B]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3     # f32-input MFMA = f32 vector peak (MI355X_MICROARCH.md)
LDS_ATOMICS_PER_CU_CLK = 64 / 7.59  # no-return ds_add on random words (tools/micro/lds_atomic.hip, r05p)
CLOCK_HZ = 2.4e9            # the clock the LDS rates are quoted at (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=48, help="FOVs per step per GPU (384-well plate = 8 steps)")
    ap.add_argument("--pool", type=int, default=8,
                    help="distinct synthetic batches cycled per GPU (8 x 48 = the 384 wells of configs[1])")
    ap.add_argument("--size", type=int, default=2080)
    ap.add_argument("--channels", type=int, default=5)
    ap.add_argument("--weights", default=None, help="CPnet state_dict (default: seeded random init)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stage-steps", type=int, default=3, help="instrumented steps after timing (>= 1)")
    ap.add_argument("--pipes", type=int, default=2,
                    help="pipelines (own libcpx context, buffers and HIP stream) per GPU: step i "
                         "runs on pipeline i %% pipes, so that many batches are in flight")
    ap.add_argument("--cu-split", choices=("auto", "none", "interleave", "halves"), default=None,
                    help="each pipeline's stream restricted to its own share of the CUs "
                         "(cpx.device.pipeline_streams; default auto: halves for "
                         "two pipelines)")
    ap.add_argument("--cpnet-precision", choices=("f16x3", "bf16", "fp32"), default="f16x3",
                    help="CPnet arithmetic: f16x3 = native split-fp16 MFMA kernels at the fp32 network's "
                         "accuracy (default: the reference's precision, masks and IDs identical to the fp32 "
                         "CPU network, DESIGN §6); bf16 = native bf16 MFMA (IDs differ); fp32 = eager PyTorch")
    ap.add_argument("--host-inputs", action="store_true",
                    help="PCIe-inclusive variant (not the headline): the synthetic batches live in "
                         "pinned host memory and every step copies its planes to the GPU inside the "
                         "timed region (on the pipeline's stream, so the other pipeline overlaps it)")
    ap.add_argument("--scheduler", choices=("queue", "static"), default="queue",
                    help="N > 1: 'queue' (default, the product's scheduler: every rank claims the next batch "
                         "of the job's steps x N batches from one shared counter, cpx.plate.WorkQueue, as "
                         "cpx.launch ranks do) or 'static' (each rank runs exactly --steps batches)")
    ap.add_argument("--zstack", type=int, default=0,
                    help="configs[4] variant: Z planes per channel, z-max projected on the GPU "
                         "inside every step (default size 2048); not the headline workload")
    return ap.parse_args()


def main():
    a = parse()
    a.stage_steps = max(1, a.stage_steps)
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # development rehearsal of the multi-rank path on a one-GPU box: every rank on this device
    if os.environ.get("CPX_BENCH_DEVICE"):
        local = int(os.environ["CPX_BENCH_DEVICE"])
    # the CPU baseline's worker processes fork from a server started before this process
    # touches the GPU (no fork or exec of a GPU-initialised process)
    cpu_ctx = _cpu_pool_context() if (rank == 0 and world == 1 and not a.no_cpu_baseline) else None
    torch.cuda.set_device(local)
    if world > 1:
        # barrier + max/sum reductions of two host scalars only: gloo (no RCCL on the data path)
        dist.init_process_group("gloo")

    from cpx import shard
    from cpx.cpnet import count_flops
    import ctypes as ct

    from cpx.device import Device, as_numpy
    from cpx.pipeline import OBJECT_SETS, FovPipeline, PipelineConfig
    from cpx.synth import synth_fovs, synth_illum, synth_zstack

    Z = a.zstack
    if Z > 1 and a.size == 2080:
        a.size = 2048  # configs[4]: 2048x2048x5ch x 7 z-planes
    H = W = a.size
    C, B = a.channels, a.batch
    dev = Device(local)
    td = dev.torch_device
    weights = a.weights
    if weights is None:
        cand = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
        weights = cand if os.path.exists(cand) else None
    cfg = PipelineConfig(H=H, W=W, C=C, batch=B, weights=weights, cpnet_precision=a.cpnet_precision)
    illum = synth_illum(C, H, W, seed=1)
    # P pipelines, each with its own libcpx context (workspaces), buffers and HIP stream: the
    # kernels of one batch fill the gaps of the other (many post-processing / feature kernels
    # do not fill 256 CUs on their own)
    from cpx.device import pipeline_streams
    streams = pipeline_streams(td, max(1, a.pipes), a.cu_split)
    pipes = []
    for p_i, st in enumerate(streams):
        with torch.cuda.stream(st):
            pipes.append(FovPipeline(dev if p_i == 0 else Device(local), cfg, illum))
    pipe = pipes[0]
    # this rank's wells (well w -> rank w % world); the synthetic batches are seeded
    # by the rank's own FOV keys, so ranks never share inputs and exchange nothing
    mine = shard.shard(shard.plate_fovs(n_wells=384), rank, world)
    if Z > 1:
        pool = [synth_zstack(B, C, Z, H, W, td, seed=shard.fov_seed(mine[(i * B) % len(mine)]) + 7919 * i)
                for i in range(a.pool)]
    else:  # (+ 7919 i: distinct batches even when a rank's wells wrap around)
        pool = [synth_fovs(B, C, H, W, td, seed=shard.fov_seed(mine[(i * B) % len(mine)]) + 7919 * i)
                for i in range(a.pool)]

    if a.host_inputs:  # pinned host copies of the batches; each pipeline gets its own device planes
        pool = [x.cpu().pin_memory() for x in pool]
        for q in pipes:
            q.raw = torch.empty_like(pool[0], device=td)

    def run_step(i, k=None):
        """Enqueue this rank's step i (input batch k, default i) on pipeline i % P (its
        stream); returns (pipeline, result slot)."""
        q = pipes[i % len(pipes)]
        i_in = i if k is None else k
        with torch.cuda.stream(streams[i % len(pipes)]):
            if Z > 1:  # a5: z-max projection into the pipeline's raw planes, then the hot path
                src = pool[i_in % a.pool]
                if a.host_inputs:
                    src = src.to(td, non_blocking=True)
                q.dev.zmax(src, q.raw)
                slot = q.run()
            elif a.host_inputs:  # H2D of the step's planes, then the hot path on the same stream
                q.raw.copy_(pool[i_in % a.pool], non_blocking=True)
                slot = q.run()
            else:
                slot = q.run(pool[i_in % a.pool])
        return q, slot
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def run_steps(batches, record=None):
        """One step per batch index of `batches` (an iterable: a range, or the claims from the
        shared work queue), every step's results fetched to the host.  Up to P + 1 steps are
        enqueued ahead of the oldest unfetched one; a fetch waits for its own step only and
        copies on a side stream, so the GPU never idles on the host.  Returns the step count."""
        pend = []
        done = 0

        def fetch_oldest():
            q, slot = pend.pop(0)
            res = q.fetch(slot)
            if record is not None:
                record.append([int(res.hdr[s]["n_objects"].sum()) for s in ("Nuclei", "Cells", "Cytoplasm")])
        for k in batches:
            pend.append(run_step(done, k))
            done += 1
            if len(pend) > len(pipes):
                fetch_oldest()
        while pend:
            fetch_oldest()
        return done

    queue = None
    if world > 1 and a.scheduler == "queue":
        # the product's multi-GPU scheduler (cpx.launch -> cpx.plate.WorkQueue): one shared counter
        # over the job's steps x N batches, each rank claiming the next one when it can take it.
        # The counter is a file in rank 0's /tmp: every rank must be on rank 0's host (one node)
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if lws != world:
            raise SystemExit(f"bench.py --scheduler queue needs a single-node job (LOCAL_WORLD_SIZE {lws} != "
                             f"WORLD_SIZE {world}); use --scheduler static across nodes")
        import tempfile
        from cpx.plate import WorkQueue
        qd = [tempfile.mkdtemp(prefix="cpx_benchq_") if rank == 0 else None]
        dist.broadcast_object_list(qd, src=0)
        queue = WorkQueue(qd[0], "bench", token=os.path.basename(qd[0]))  # the same token on every rank

    def claims(total):
        while True:
            k = queue.take()
            if k >= total:
                return
            yield k

    n_obj = []
    run_steps(range(a.warmup))
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_done = run_steps(claims(a.steps * world) if queue is not None else range(a.steps), n_obj)
    torch.cuda.synchronize()
    barrier()
    dt = shard.max_over_ranks(time.perf_counter() - t0)
    total_fovs = shard.sum_over_ranks(n_done * B)
    value = total_fovs / dt

    # ---- instrumented steps (outside the timed region): per-stage device time by HIP events on
    # the stream every stage is launched on (torch's current stream; libcpx is bound to it)
    stages = ["illum_qc", "segment", "objects_features"]
    acc = {s: 0.0 for s in stages}
    sub = {"illum": 0.0, "qc_rps": 0.0, "seg_prep": 0.0, "cpnet": 0.0, "seg_post": 0.0, "cells": 0.0,
           "features": 0.0}
    if Z > 1:
        sub["zmax"] = 0.0
    glcm = {"ms": 0.0, "atomics": 0, "items": 0}
    segt = {"follow_ms": 0.0, "item_steps": 0.0, "fe_reg_ms": 0.0}

    def glcm_acc(p):
        # GLCM device time of this step (HIP events around k_tex_band and the k_tex_glcm redo
        # pass) and its LDS work: per staged (object, channel) item and angle, one LDS atomic per
        # pair slot of the crop (rows - dr) x crop_stride(bw) (masked and background slots go to a
        # sink counter: atomics too) and one scan of the 65 x 512-byte band table
        ms, nl = ct.c_double(), ct.c_int()
        dev.lib.cpx_debug_glcm_ms(dev.h, ct.byref(ms), ct.byref(nl))
        dev.lib.cpx_debug_glcm_timing(dev.h, 0)
        glcm["ms"] += ms.value
        for s in OBJECT_SETS:
            objs = as_numpy(p.objects[s], "object").reshape(B, -1)
            nobj = as_numpy(p.hdr[s], "hdr")["n_objects"]
            for b in range(B):
                bb = objs[b, :nobj[b]]["bbox"].astype(np.int64)
                bh, bw = bb[:, 2] - bb[:, 0], bb[:, 3] - bb[:, 1]
                st = bh * bw <= 65535
                stride = (bw + 7) & ~7
                for dr in (0, 2, 3, 2):
                    glcm["atomics"] += int(C * np.sum(np.maximum(bh - dr, 0) * stride * st))
                glcm["items"] += int(C * st.sum())

    for i in range(a.stage_steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
        if Z > 1:
            ez = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ez[0].record()
            dev.zmax(pool[i % a.pool].to(td) if a.host_inputs else pool[i % a.pool], pipe.raw)
            ez[1].record()
        src = pipe.raw if (Z > 1 or a.host_inputs) else pool[i % a.pool]
        ev[0].record()
        dev.illum_correct(src, pipe.illum, C, pipe.corr, pipe.stats)
        ev[1].record()
        dev.qc_rps(src, pipe.illum, C, pipe.stats, pipe.qc)
        ev[2].record()
        pipe.seg.prepare(pipe.corr)
        ev[3].record()
        pipe.seg._run_net()
        ev[4].record()
        dev.lib.cpx_debug_seg_timing(dev.h, 1)
        pipe.seg.postprocess(pipe.labels["Nuclei"])
        ev[5].record()
        pipe.stage_cells()
        ev[6].record()
        dev.lib.cpx_debug_glcm_timing(dev.h, 1)
        pipe.stage_features()
        ev[7].record()
        torch.cuda.synchronize()
        glcm_acc(pipe)
        fm, isteps, fe = ct.c_double(), ct.c_double(), ct.c_double()
        dev.lib.cpx_debug_seg_stats(dev.h, ct.byref(fm), ct.byref(isteps), ct.byref(fe), None)
        dev.lib.cpx_debug_seg_timing(dev.h, 0)
        segt["follow_ms"] += fm.value
        segt["item_steps"] += isteps.value
        segt["fe_reg_ms"] += fe.value
        sub["illum"] += ev[0].elapsed_time(ev[1])
        sub["qc_rps"] += ev[1].elapsed_time(ev[2])
        sub["seg_prep"] += ev[2].elapsed_time(ev[3])
        sub["cpnet"] += ev[3].elapsed_time(ev[4])
        sub["seg_post"] += ev[4].elapsed_time(ev[5])
        acc["illum_qc"] += ev[0].elapsed_time(ev[2])
        acc["segment"] += ev[2].elapsed_time(ev[5])
        acc["objects_features"] += ev[5].elapsed_time(ev[7])
        sub["cells"] += ev[5].elapsed_time(ev[6])
        sub["features"] += ev[6].elapsed_time(ev[7])
        if Z > 1:
            sub["zmax"] += ez[0].elapsed_time(ez[1])
    per_step_ms = {k: v / a.stage_steps for k, v in acc.items()}
    sub_ms = {k: v / a.stage_steps for k, v in sub.items()}
    N = H * W
    n_tiles = pipe.seg.geom.n_tiles
    # algorithmic bytes / flops per launch (one batch of B FOVs)
    illum_bytes = B * C * N * (2 + 4 + 4)                # raw u16 + illum f32 in, fp32 plane out
    # the C fp32 planes once per step plus one int32 label image per object set
    feat_bytes = B * (C * 4 * N + 3 * 4 * N)
    # Cells watershed: Nuclei labels + the fp32 cell channel in, Cells + Cytoplasm labels out
    cells_bytes = B * (4 * N + 4 * N + 2 * 4 * N)
    cpnet_flops = B * n_tiles * count_flops(pipe.seg.geom.by)
    # QC spectrum: the raw u16 plane and the fp32 flat-field read once per channel (6 B/px)
    qc_bytes = B * C * N * (2 + 4)
    # segmentation post-processing: the full-resolution flows (dY, dX fp32) written
    # and read once + the int32 labels written once
    seg_post_bytes = B * N * (2 * 4 + 4)
    kernels = {
        "illum": dict(bound="hbm", work=illum_bytes, ms=sub_ms["illum"]),
        "qc_rps": dict(bound="hbm", work=qc_bytes, ms=sub_ms["qc_rps"]),
        "cpnet": dict(bound="mfma", work=cpnet_flops, ms=sub_ms["cpnet"]),
        "seg_post": dict(bound="hbm", work=seg_post_bytes, ms=sub_ms["seg_post"]),
        "cells": dict(bound="hbm", work=cells_bytes, ms=sub_ms["cells"]),
        "features": dict(bound="hbm", work=feat_bytes, ms=sub_ms["features"]),
    }
    if Z > 1:  # Z u16 planes in, one u16 plane out per channel group
        kernels["zmax"] = dict(bound="hbm", work=B * C * N * (2 * Z + 2), ms=sub_ms["zmax"])

    # the committed PMC traffic was measured on the headline workload; not valid for variants
    pmc, pmc_src = (pmc_traffic(B, a.cpnet_precision) if (Z <= 1 and H == 2080 and not a.host_inputs)
                    else ({}, None))

    def roof(k):
        d = kernels[k]
        traffic = pmc.get(k)
        if d["bound"] == "hbm":
            ach = d["work"] / (d["ms"] * 1e-3) / 1e9
            return {"kernel": k, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": pmc_src if traffic else None,
                    "algorithmic_bytes_per_launch": d["work"], "avg_launch_ms": round(d["ms"], 4)}
        ach = d["work"] / (d["ms"] * 1e-3) / 1e12
        # f16x3 forms each fp32-network product from three dense fp16 MFMA products: its peak in
        # network FLOP/s is the dense f16 peak / 3
        peak = {"bf16": BF16_PEAK_TFLOPS, "f16x3": BF16_PEAK_TFLOPS / 3.0}.get(a.cpnet_precision, F32_PEAK_TFLOPS)
        out = {"kernel": k, "bound": "mfma", "achieved": round(ach, 1), "peak": round(peak, 1),
               "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic,
               "traffic_source": pmc_src if traffic else None,
               "algorithmic_flops_per_launch": d["work"], "avg_launch_ms": round(d["ms"], 4)}
        if a.cpnet_precision == "f16x3":
            out["note"] = ("fp32-network FLOPs; executed as 3 fp16 MFMA products each: "
                           f"{round(3 * ach, 1)} TFLOP/s of f16 MFMA vs the {BF16_PEAK_TFLOPS} dense peak")
        return out

    # measured copy bandwidth of this HBM (report next to the vendor peak):
    # 2 GiB device-to-device copy, read + write bytes over the mean copy time
    src_b = torch.empty(1 << 31, dtype=torch.uint8, device=td)
    dst_b = torch.empty_like(src_b)
    dst_b.copy_(src_b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        dst_b.copy_(src_b)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * (1 << 31) * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src_b, dst_b

    # the GLCM against its LDS floor: the no-return LDS atomic rate on random
    # addresses, 64 / 7.59 per CU-cycle (tools/micro/lds_atomic.hip, profiles/r05p_lds_atomic.log),
    # and the 4 band-table scans (65 x 512 B) per item at 256 B per CU-cycle, at 2.4 GHz on every CU
    n_cu = torch.cuda.get_device_properties(td).multi_processor_count
    glcm_ms = glcm["ms"] / a.stage_steps
    atomics = glcm["atomics"] / a.stage_steps
    items = glcm["items"] / a.stage_steps
    atomic_peak = n_cu * LDS_ATOMICS_PER_CU_CLK * CLOCK_HZ
    floor_ms = (atomics / LDS_ATOMICS_PER_CU_CLK + items * 4 * 65 * 512 / 256) / (n_cu * CLOCK_HZ) * 1e3
    # flow following (k_dyn_follow): each step of a trajectory is two 16-byte gathers
    # of the float2 field returned through the CU's L1 at 64 B per clock, i.e. 2 item-steps per
    # CU-clock; item-steps = items per round x steps per round (an upper bound: a trajectory at an
    # exact fixed point stops early) over the follow rounds' device time
    follow_ms = segt["follow_ms"] / a.stage_steps
    isteps = segt["item_steps"] / a.stage_steps
    follow_peak = n_cu * 2.0 * CLOCK_HZ
    follow_roof = {"kernel": "k_dyn_follow", "bound": "l1_return", "unit": "G item-steps/s",
                   "achieved": round(isteps / (follow_ms * 1e-3) / 1e9, 1) if follow_ms else None,
                   "peak": round(follow_peak / 1e9, 1),
                   "frac": round(isteps / (follow_ms * 1e-3) / follow_peak, 4) if follow_ms else None,
                   "item_steps_per_step": int(isteps), "avg_launch_ms": round(follow_ms, 4),
                   "note": "item-steps are an upper bound (items per round x steps per round)"}
    # the register flow-error screening kernels (k_flow_error_reg*): VALU-issue bound —
    # instructions from the committed SQ_INSTS_VALU pass (profiles/r*_sq_flow_error.json, scaled
    # to the batch), 2 cycles per wave64 VALU instruction on 4 SIMDs per CU, over their live time
    fe_ms = segt["fe_reg_ms"] / a.stage_steps
    fe_valu, fe_src = sq_flow_error(B) if (Z <= 1 and H == 2080) else (None, None)
    fe_peak = n_cu * 4 * CLOCK_HZ / 2.0  # wave-instructions per second
    fe_roof = {"kernel": "k_flow_error_reg*", "bound": "valu_issue", "unit": "G wave-instr/s",
               "achieved": round(fe_valu / (fe_ms * 1e-3) / 1e9, 1) if fe_valu and fe_ms else None,
               "peak": round(fe_peak / 1e9, 1),
               "frac": round(fe_valu / (fe_ms * 1e-3) / fe_peak, 4) if fe_valu and fe_ms else None,
               "valu_wave_instr_per_step": int(fe_valu) if fe_valu else None, "valu_source": fe_src,
               "avg_launch_ms": round(fe_ms, 4)}
    glcm_roof = {"kernel": "k_tex_band", "bound": "lds_atomic", "achieved": round(atomics / (glcm_ms * 1e-3) / 1e9, 1),
                 "peak": round(atomic_peak / 1e9, 1), "unit": "Gatomic/s",
                 "frac": round(atomics / (glcm_ms * 1e-3) / atomic_peak, 4) if glcm_ms else None,
                 "lds_floor_ms": round(floor_ms, 4), "floor_frac": round(floor_ms / glcm_ms, 4) if glcm_ms else None,
                 "atomics_per_step": int(atomics), "items_per_step": int(items), "avg_launch_ms": round(glcm_ms, 4),
                 "peak_source": "tools/micro/lds_atomic.hip (random 32K-word no-return atomics), profiles/r05p_lds_atomic.log"}

    dominant = max(kernels, key=lambda k: kernels[k]["ms"])
    line = {
        "metric": "fields-of-view/sec, 2080x2080x5ch illum+seg+feat pipe",
        "value": round(value, 2),
        "unit": "FOV/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp32 planes / fp64 QC+features / " +
                  {"f16x3": "fp32 CPnet (split-fp16 MFMA, f16x3)", "bf16": "bf16 CPnet",
                   "fp32": "fp32 CPnet (eager PyTorch)"}[a.cpnet_precision]),
        "data": (f"synthetic ({'pinned-host uint16 plates copied to the GPU inside every step (PCIe-inclusive)' if a.host_inputs else 'HBM-resident uint16 plates'}, "
                 f"Poisson background, Gaussian nuclei + halos; "
                 f"{a.pool} distinct batches = {a.pool * B} distinct FOVs per GPU, cycled)"),
        "config": {"workload": ("configs[1]: 384-well plate, 1 FOV/well, 2080x2080x5ch, illum->seg->feat"
                                if Z <= 1 else
                                f"configs[4] variant: {H}x{W}x{C}ch x {Z} z-planes, z-max->illum->seg->feat"),
                   "fovs_per_step": B * world, "batch_per_gpu": B, "H": H, "W": W, "C": C,
                   "cellpose_model": cfg.model, "diameter": cfg.diameter,
                   "cpnet_weights": os.path.basename(weights) if weights else "seeded-random-init",
                   "tiles_per_fov": n_tiles, "parallelism": f"fov-sharded x{world}",
                   "scheduler": ("shared work queue (cpx.plate.WorkQueue)" if queue is not None
                                 else "static per-rank steps"),
                   "steps_this_rank": n_done,
                   "batches_in_flight_per_gpu": len(pipes)},
        "objects_per_fov": ([round(x / (B * world) * world, 1) for x in np.mean(np.array(n_obj), axis=0)]
                            if n_obj else None),
        "stage_ms_per_step": {k: round(v, 3) for k, v in {**per_step_ms, **sub_ms}.items()},
        "roofline": roof(dominant),
        "roofline_all": {**{k: roof(k) for k in kernels}, "glcm": glcm_roof, "follow": follow_roof,
                         "flow_error_reg": fe_roof},
        "hbm_copy_measured_GBs": round(copy_gbs, 1),
    }
    if cpu_ctx is not None:
        line["cpu_baseline"] = cpu_baseline(cpu_ctx, pipe.raw if (Z > 1 or a.host_inputs) else pool[0], illum,
                                            C, H, W, cfg)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()
        if queue is not None and rank == 0:
            import shutil
            shutil.rmtree(os.path.dirname(queue.path), ignore_errors=True)
        dist.destroy_process_group()


def pmc_traffic(batch, precision):
    """HBM bytes per launch (one pipeline step of `batch` FOVs) per stage, from the newest
    profiles/r*_pmc_traffic.json (tools/pmc_traffic.py: separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes over this bench, FETCH_SIZE doubled per the gfx950 correction).  Counters
    cannot be read inside a timed run, so the committed measurement of the same workload is
    used; {} if none is present."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.json")))
    # only a pass over the same CPnet precision describes this run (files record "cpnet_precision";
    # older ones were bf16)
    files = [f for f in files if json.load(open(f)).get("cpnet_precision", "bf16") == precision]
    if not files:
        return {}, None
    d = json.load(open(files[-1]))
    scale = batch / float(d.get("fovs_per_step", batch))
    fam = d["per_family_bytes_per_step"]
    out = {k: int(v["total"] * scale) for k, v in fam.items()}
    if "cpnet" in fam:
        out.setdefault("cpnet", int(fam["cpnet"]["total"] * scale))
    return out, os.path.relpath(files[-1], REPO)


def sq_flow_error(batch):
    """SQ_INSTS_VALU (wave-instructions) of the register flow-error kernels per step of `batch`
    FOVs, from the newest profiles/r*_sq_flow_error.json (tools/pmc_sq.py --json over a
    rocprofv3 --pmc pass of this bench); (None, None) if none is present."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_sq_flow_error.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d["valu_per_step"] * batch / float(d["fovs_per_step"]), os.path.relpath(files[-1], REPO)


CPU_BASELINE_MAX_CORES = 16  # the GPU box's CPU share per GPU (os.cpu_count() shows the host)


def _cpu_pool_context():
    """multiprocessing "forkserver" context whose server is started now, before any GPU call,
    with one thread per worker (OMP_NUM_THREADS=1) and oracle/ on its path."""
    import multiprocessing as mp
    from multiprocessing import forkserver
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    ctx = mp.get_context("forkserver")
    ctx.set_forkserver_preload(["numpy"])
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MKL_NUM_THREADS", "OPENBLAS_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        forkserver.ensure_running()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return ctx


def cpu_baseline(ctx, pool_batch, illum, C, H, W, cfg):
    """SURVEY 8(d) CPU baseline: the CPU restatement of the whole per-FOV path
    (oracle/cpu_pipeline.run_fov: QC, fp32 CPnet on the CPU, full-resolution dynamics, Cells /
    Cytoplasm, features) on `cores` FOVs of the same synthetic plate, one FOV per worker
    process, all workers concurrent, one thread each.  value = FOVs / the slowest worker's
    compute time (worker start-up and input transfer excluded)."""
    import tempfile
    import numpy as np
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    cores = max(1, min(aff, CPU_BASELINE_MAX_CORES))
    B = pool_batch.shape[0] // C
    raw = pool_batch.cpu().numpy().view(np.uint16).reshape(B, C, H, W)
    n = cores
    with tempfile.TemporaryDirectory(prefix="cpx_cpu_") as td:
        ill_path = os.path.join(td, "illum.npy")
        np.save(ill_path, illum)
        jobs = []
        for i in range(n):
            path = os.path.join(td, f"fov{i}.npy")
            np.save(path, raw[i % B])
            jobs.append((path, ill_path, cfg.weights, cfg.seed, cfg.model, cfg.diameter, cfg.cell_expand,
                         cfg.cells, cfg.ws_channel()))
        t0 = time.perf_counter()
        with ctx.Pool(cores) as pool:
            out = pool.map(_cpu_worker, jobs, chunksize=1)
        wall = time.perf_counter() - t0
    worst = max(o["total"] for o in out)
    mean = {k: float(np.mean([o[k] for o in out])) for k in out[0]}
    return {"value": round(n / worst, 5), "unit": "FOV/s", "cores": cores, "kind": "port",
            "sample": f"{n} FOVs of the same synthetic plate ({H}x{W}x{C}), one per worker process "
                      f"(multiprocessing forkserver Pool({cores}), OMP_NUM_THREADS=1), "
                      f"oracle/cpu_pipeline.run_fov = the CPU restatement (QC, fp32 CPnet, "
                      f"full-resolution dynamics with the C oracle loops, Cells by the heap watershed in C, features); value = FOVs / "
                      f"slowest worker; wall incl. start-up {wall:.1f} s; mean stage seconds: " +
                      ", ".join(f"{k}={v:.2f}" for k, v in mean.items())}


def _cpu_worker(job):
    """One FOV of the CPU baseline (runs in a forkserver child; never touches the GPU)."""
    import numpy as np
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_pipeline
    from cpx.cpnet import build_cpnet
    path, ill_path, weights, seed, model, diameter, expand, cells, cell_ch = job
    raw = np.load(path)
    illum = np.load(ill_path, mmap_mode="r")
    net = build_cpnet(seed=seed, model=model, state_dict_path=weights)
    tm = {}
    cpu_pipeline.run_fov(raw, np.asarray(illum), net, expand, model, diameter, timings=tm, cells=cells,
                         cell_channel=cell_ch)
    return tm


if __name__ == "__main__":
    main()
